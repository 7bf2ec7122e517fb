// pcshell_common.h -- helpers shared by the PCSHELL implementations (pcshell_fft3d.cpp,
// wave_system.cpp): cfp error -> PETSc error, and device views of Vecs (device arrays used in
// place, host arrays staged through a temporary device buffer).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/circulant_fft.h"
#include "../../include/petsc_mini.h"

namespace cfp_pc {

inline PetscErrorCode cfp_err(int rc, const char* where) {
  if (rc == CFP_SUCCESS) return PETSC_SUCCESS;
#ifndef CFP_WITH_PETSC
  return PetscErrorSet(rc, where, cfp_last_error());
#else
  SETERRQ(PETSC_COMM_SELF, rc, "%s: %s", where, cfp_last_error());
#endif
}

// The stream an apply on device Vecs is ordered on, and whether it must be waited for: the
// stand-in's Vec stream, stream-ordered like PETSc's VECHIP operations (the next Vec operation,
// e.g. GMRES's VecMAXPY, queues behind the apply; a host read synchronises), so PCApply costs no
// host round trip.  Built against a real PETSc: the default stream, waited for.
inline void device_stream(void** st, bool* wait) {
#ifdef CFP_WITH_PETSC
  *st = nullptr;
  *wait = true;
#else
  VecMiniGetStream(st);
  *wait = false;
#endif
}

// Device view of a Vec for the duration of one solve: device arrays are used in place,
// host arrays are staged through a temporary device buffer (PCIe-inclusive path).
struct DevIn {
  Vec v = nullptr;
  const PetscScalar* arr = nullptr;
  PetscMemType mt = PETSC_MEMTYPE_HOST;
  void* tmp = nullptr;
  const double* ptr() const { return tmp ? (const double*)tmp : (const double*)arr; }
  PetscErrorCode get(Vec vec, PetscInt n) {
    v = vec;
    PetscCall(VecGetArrayReadAndMemType(v, &arr, &mt));
    if (mt == PETSC_MEMTYPE_HOST) {
      PetscCheck(hipMalloc(&tmp, sizeof(PetscScalar) * (size_t)n) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_MEM,
                 "staging buffer");
      PetscCheck(hipMemcpy(tmp, arr, sizeof(PetscScalar) * (size_t)n, hipMemcpyHostToDevice) == hipSuccess,
                 PETSC_COMM_SELF, PETSC_ERR_LIB, "host to device copy");
    }
    return PETSC_SUCCESS;
  }
  PetscErrorCode put() {
    if (tmp) hipFree(tmp);
    tmp = nullptr;
    return VecRestoreArrayReadAndMemType(v, &arr);
  }
};
struct DevOut {
  Vec v = nullptr;
  PetscScalar* arr = nullptr;
  PetscMemType mt = PETSC_MEMTYPE_HOST;
  void* tmp = nullptr;
  PetscInt n = 0;
  double* ptr() const { return tmp ? (double*)tmp : (double*)arr; }
  PetscErrorCode get(Vec vec, PetscInt nn) {
    v = vec;
    n = nn;
    PetscCall(VecGetArrayWriteAndMemType(v, &arr, &mt));
    if (mt == PETSC_MEMTYPE_HOST)
      PetscCheck(hipMalloc(&tmp, sizeof(PetscScalar) * (size_t)n) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_MEM,
                 "staging buffer");
    return PETSC_SUCCESS;
  }
  PetscErrorCode put() {
    if (tmp) {
      hipDeviceSynchronize();
      PetscCheck(hipMemcpy(arr, tmp, sizeof(PetscScalar) * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess,
                 PETSC_COMM_SELF, PETSC_ERR_LIB, "device to host copy");
      hipFree(tmp);
      tmp = nullptr;
    }
    return VecRestoreArrayWriteAndMemType(v, &arr);
  }
};

inline PetscErrorCode check_size(Vec v, PetscInt n, const char* name) {
  PetscInt m;
  PetscCall(VecGetLocalSize(v, &m));
  PetscCheck(m == n, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ, name);
  return PETSC_SUCCESS;
}

}  // namespace cfp_pc

#define CFPCALL(expr) PetscCall(cfp_pc::cfp_err((expr), __func__))
