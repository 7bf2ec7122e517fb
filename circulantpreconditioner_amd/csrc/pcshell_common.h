// pcshell_common.h -- helpers shared by the PCSHELL implementations (pcshell_fft3d.cpp,
// wave_system.cpp): cfp error -> PETSc error, and device views of Vecs (device arrays used in
// place, host arrays staged through a temporary device buffer).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/circulant_fft_dist.h"
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

// ------------------------------------------------------------------ slab plans on a communicator
// The z-slab plan behind an FFT matrix of several ranks (the complex build, pcshell_fft3d.cpp, and
// the real-scalar build, pcshell_fft3d_real.cpp): the reference's MATFFTW on PETSC_COMM_WORLD
// (src/PCSHELLFft_3D.cxx:34-35).
#ifdef CFP_WITH_PETSC
// Exchange piece over a real MPI communicator (cfp_dist_exchange_fn): host-staged
// MPI_Alltoall of the [size][count] pieces.
struct MpiExchange {
  MPI_Comm comm;
  int size;
  std::vector<char> hs, hr;
};
inline int mpi_exchange(void* user, const double* src, double* dst, int64_t chunk, int64_t off, int64_t count,
                        void* stream) {
  MpiExchange* m = (MpiExchange*)user;
  const size_t bytes = 16 * (size_t)count, pitch = 16 * (size_t)chunk;
  if (bytes > (size_t)INT32_MAX) return 1;
  m->hs.resize(bytes * m->size);
  m->hr.resize(bytes * m->size);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemcpy2DAsync(m->hs.data(), bytes, src + 2 * off, pitch, bytes, m->size, hipMemcpyDeviceToHost, st) ||
      hipStreamSynchronize(st))
    return 1;
  if (MPI_Alltoall(m->hs.data(), (int)bytes, MPI_BYTE, m->hr.data(), (int)bytes, MPI_BYTE, m->comm)) return 1;
  if (hipMemcpy2DAsync(dst + 2 * off, pitch, m->hr.data(), bytes, bytes, m->size, hipMemcpyHostToDevice, st) ||
      hipStreamSynchronize(st))
    return 1;
  return 0;
}
#endif

// max over the ranks of an FFT matrix' communicator (one rank: itself)
inline PetscErrorCode comm_max(MPI_Comm comm, int nranks, double* v, int n) {
  if (nranks == 1) return PETSC_SUCCESS;
#ifdef CFP_WITH_PETSC
  PetscCallMPI(MPI_Allreduce(MPI_IN_PLACE, v, n, MPI_DOUBLE, MPI_MAX, comm));
#else
  PetscCall(PetscMiniAllreduce(comm, v, n, PETSCMINI_OP_MAX));
#endif
  return PETSC_SUCCESS;
}

// This rank's slab plan of the nx x ny x nz grid, its exchanges over `comm`: an RCCL communicator
// of the stand-in -> grouped ncclSend / ncclRecv on it; a callback communicator -> the caller's
// collectives, host-staged; a real MPI communicator -> host-staged MPI_Alltoall.  *resolved: the
// communicator to release (stand-in: PETSC_COMM_WORLD resolved, retained); *mx: the MPI exchange
// state (CFP_WITH_PETSC).
struct SlabBacking {
  cfp_dist_plan_t plan = nullptr;
  MPI_Comm comm = PETSC_COMM_SELF;
  void* mx = nullptr;
};
inline PetscErrorCode slab_create(MPI_Comm comm, int nranks, int rank, const PetscInt dims[3], int dev,
                                  SlabBacking* sb) {
#ifdef CFP_WITH_PETSC
  PetscCall(cfp_err(cfp_dist_plan_create_external(&sb->plan, dims[0], dims[1], dims[2], nranks, rank, dev), __func__));
  MpiExchange* m = new MpiExchange{comm, nranks, {}, {}};
  sb->mx = m;
  sb->comm = comm;
  PetscCall(cfp_err(cfp_dist_plan_set_exchange(sb->plan, mpi_exchange, m), __func__));
#else
  MPI_Comm c;
  PetscCall(PetscMiniCommResolve(comm, &c));
  void* nccl = nullptr;
  PetscCall(PetscMiniCommGetNCCL(c, &nccl));
  if (nccl) {
    PetscCall(cfp_err(cfp_dist_plan_create_with_comm(&sb->plan, dims[0], dims[1], dims[2], nranks, rank, nccl, dev),
                      __func__));
  } else {
    PetscCall(cfp_err(cfp_dist_plan_create_external(&sb->plan, dims[0], dims[1], dims[2], nranks, rank, dev), __func__));
    PetscCall(cfp_err(cfp_dist_plan_set_exchange(sb->plan, PetscMiniCommExchange, (void*)(intptr_t)c), __func__));
  }
  PetscCall(PetscMiniCommRetain(c));  // PetscMiniCommDestroy refuses until slab_destroy releases it
  sb->comm = c;
#endif
  return PETSC_SUCCESS;
}
inline void slab_destroy(SlabBacking* sb) {
  if (sb->plan) {
    cfp_dist_plan_destroy(sb->plan);
#ifndef CFP_WITH_PETSC
    PetscMiniCommRelease(sb->comm);
#endif
  }
#ifdef CFP_WITH_PETSC
  delete (MpiExchange*)sb->mx;
#endif
  sb->plan = nullptr;
  sb->mx = nullptr;
}

inline PetscErrorCode check_size(Vec v, PetscInt n, const char* name) {
  PetscInt m;
  PetscCall(VecGetLocalSize(v, &m));
  PetscCheck(m == n, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ, name);
  return PETSC_SUCCESS;
}

}  // namespace cfp_pc

#define CFPCALL(expr) PetscCall(cfp_pc::cfp_err((expr), __func__))
