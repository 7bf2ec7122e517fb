// petsc_mini.cpp -- stand-in for the PETSc subset declared in include/petsc_mini.h.
//
// PETSc is not installed in this image or on the GPU box, so the PCSHELL
// boundary would otherwise be untestable.  This file gives Vec (host VECSEQ and device
// VECSEQHIP with PETSc's offload-mask semantics), Mat (MATSHELL, MATSEQAIJ, the FFT shell)
// and PC (PCSHELL, PCNONE) objects with PETSc's names and argument conventions.  It is
// compiled out when building against a real PETSc (-DCFP_WITH_PETSC).
#ifndef CFP_WITH_PETSC
#include <hip/hip_runtime.h>

#include <atomic>
#include <sys/time.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pcshell_fft3d.h"
#include "../../include/petsc_mini.h"
#include "cfp_blas.h"
#include "cfp_internal.h"

using cfp::cd;
using cfp::i64;

static thread_local std::string g_perr;
static hipStream_t g_stream = nullptr;

extern "C" PetscErrorCode PetscErrorSet(PetscErrorCode code, const char* func, const char* msg) {
  g_perr = std::string(func ? func : "?") + ": " + (msg ? msg : "");
  return code;
}
extern "C" const char* PetscErrorLastMessage(void) { return g_perr.c_str(); }
extern "C" PetscErrorCode PetscTime(PetscLogDouble* t) {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  *t = (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecMiniSetStream(void* s) {
  g_stream = (hipStream_t)s;
  return PETSC_SUCCESS;
}

#define ERR(code, msg) PetscErrorSet((code), __func__, (msg))
#define HCHK(expr)                                                      \
  do {                                                                  \
    hipError_t e__ = (expr);                                            \
    if (e__ != hipSuccess) return ERR(PETSC_ERR_LIB, hipGetErrorString(e__)); \
  } while (0)

static inline cd tocd(PetscScalar s) { return cfp::make_cd(s.real(), s.imag()); }

// ------------------------------------------------------------------ Vec
enum { MASK_NONE = 0, MASK_CPU = 1, MASK_GPU = 2, MASK_BOTH = 3 };
static const int kVecMagic = 0x56656331;

struct _p_Vec {
  int magic = kVecMagic;
  PetscInt n = 0;
  bool hip = false;
  cd* d = nullptr;
  cd* h = nullptr;
  bool own_d = false, own_h = false;
  int mask = MASK_NONE;
  int device = 0;
  PetscObjectId id = 0;
  PetscObjectState state = 0;  // bumped by every write access (PetscObjectStateGet)
};

static std::atomic<int64_t> g_object_ids{0};
static inline void touch(Vec v) { ++v->state; }

static PetscErrorCode vcheck(Vec v, const char* f) {
  if (!v || v->magic != kVecMagic) return PetscErrorSet(PETSC_ERR_ARG_NULL, f, "invalid Vec");
  return PETSC_SUCCESS;
}
#define VCHK(v) PetscCall(vcheck((v), __func__))

// wait for the kernels already queued on the Vec stream (no-op for a host vector), so a
// host-timed region that starts here does not include earlier asynchronous work
extern "C" PetscErrorCode VecMiniSynchronize(Vec v) {
  VCHK(v);
  if (v->hip) HCHK(hipStreamSynchronize(g_stream));
  return PETSC_SUCCESS;
}

static PetscErrorCode ensure_host(Vec v) {
  if (!v->h) {
    v->h = (cd*)calloc((size_t)(v->n > 0 ? v->n : 1), sizeof(cd));
    if (!v->h) return ERR(PETSC_ERR_MEM, "host allocation");
    v->own_h = true;
  }
  return PETSC_SUCCESS;
}
// make the host copy current (device -> host if only the device is valid)
static PetscErrorCode sync_to_host(Vec v) {
  PetscCall(ensure_host(v));
  if (v->hip && v->mask == MASK_GPU) {
    HCHK(hipMemcpyAsync(v->h, v->d, sizeof(cd) * (size_t)v->n, hipMemcpyDeviceToHost, g_stream));
    HCHK(hipStreamSynchronize(g_stream));
    v->mask = MASK_BOTH;
  }
  if (v->mask == MASK_NONE) v->mask = v->hip ? MASK_BOTH : MASK_CPU;
  return PETSC_SUCCESS;
}
static PetscErrorCode sync_to_device(Vec v) {
  if (!v->hip) return ERR(PETSC_ERR_ARG_WRONG, "not a device vector");
  if (v->mask == MASK_CPU) {
    HCHK(hipMemcpyAsync(v->d, v->h, sizeof(cd) * (size_t)v->n, hipMemcpyHostToDevice, g_stream));
    v->mask = MASK_BOTH;
  }
  if (v->mask == MASK_NONE) v->mask = MASK_GPU;
  return PETSC_SUCCESS;
}

static PetscErrorCode vec_new(PetscInt n, bool hip, const PetscScalar* devarr, Vec* out) {
  if (!out) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  if (n < 0) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "negative size");
  Vec v = new _p_Vec;
  v->id = ++g_object_ids;
  v->n = n;
  v->hip = hip;
  if (hip) {
    hipGetDevice(&v->device);
    if (devarr) {
      v->d = (cd*)devarr;
    } else {
      hipError_t e = hipMalloc(&v->d, sizeof(cd) * (size_t)(n > 0 ? n : 1));
      if (e != hipSuccess) { delete v; return ERR(PETSC_ERR_MEM, hipGetErrorString(e)); }
      v->own_d = true;
      hipMemsetAsync(v->d, 0, sizeof(cd) * (size_t)n, g_stream);
    }
    v->mask = MASK_GPU;
  } else {
    PetscErrorCode rc = ensure_host(v);
    if (rc) { delete v; return rc; }
    v->mask = MASK_CPU;
  }
  *out = v;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecCreateSeq(MPI_Comm, PetscInt n, Vec* v) { return vec_new(n, false, nullptr, v); }
extern "C" PetscErrorCode VecCreateSeqHIP(MPI_Comm, PetscInt n, Vec* v) { return vec_new(n, true, nullptr, v); }
extern "C" PetscErrorCode VecCreateSeqHIPWithArray(MPI_Comm, PetscInt, PetscInt n, const PetscScalar* a, Vec* v) {
  return vec_new(n, true, a, v);
}
extern "C" PetscErrorCode VecCreateMPI(MPI_Comm, PetscInt nlocal, PetscInt N, Vec* v) {
  // single process: the local part is everything
  PetscInt n = N >= 0 ? N : nlocal;
  if (nlocal >= 0 && N >= 0 && nlocal != N) return ERR(PETSC_ERR_ARG_SIZ, "one process: local size must equal N");
  return vec_new(n, true, nullptr, v);
}
extern "C" PetscErrorCode VecDuplicate(Vec v, Vec* nv) {
  VCHK(v);
  return vec_new(v->n, v->hip, nullptr, nv);
}
extern "C" PetscErrorCode VecDestroy(Vec* pv) {
  if (!pv || !*pv) return PETSC_SUCCESS;
  Vec v = *pv;
  VCHK(v);
  if (v->own_d && v->d) hipFree(v->d);
  if (v->own_h && v->h) free(v->h);
  v->magic = 0;
  delete v;
  *pv = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscObjectStateGet(PetscObject obj, PetscObjectState* state) {
  Vec v = (Vec)obj;
  if (!v || v->magic != kVecMagic) return ERR(PETSC_ERR_ARG_WRONG, "PetscObjectStateGet: Vec objects only");
  if (!state) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  *state = v->state;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscObjectGetId(PetscObject obj, PetscObjectId* id) {
  Vec v = (Vec)obj;
  if (!v || v->magic != kVecMagic) return ERR(PETSC_ERR_ARG_WRONG, "PetscObjectGetId: Vec objects only");
  if (!id) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  *id = v->id;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetType(Vec v, VecType* t) {
  VCHK(v);
  *t = v->hip ? VECSEQHIP : VECSEQ;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetSize(Vec v, PetscInt* n) { VCHK(v); *n = v->n; return PETSC_SUCCESS; }
extern "C" PetscErrorCode VecGetLocalSize(Vec v, PetscInt* n) { VCHK(v); *n = v->n; return PETSC_SUCCESS; }
extern "C" PetscErrorCode VecGetOwnershipRange(Vec v, PetscInt* lo, PetscInt* hi) {
  VCHK(v);
  if (lo) *lo = 0;
  if (hi) *hi = v->n;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecGetArray(Vec v, PetscScalar** a) {
  VCHK(v);
  PetscCall(sync_to_host(v));
  *a = (PetscScalar*)v->h;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecRestoreArray(Vec v, PetscScalar** a) {
  VCHK(v);
  v->mask = MASK_CPU;
  touch(v);
  if (a) *a = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetArrayRead(Vec v, const PetscScalar** a) {
  VCHK(v);
  PetscCall(sync_to_host(v));
  *a = (const PetscScalar*)v->h;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecRestoreArrayRead(Vec v, const PetscScalar** a) {
  VCHK(v);
  if (a) *a = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetArrayWrite(Vec v, PetscScalar** a) {
  VCHK(v);
  PetscCall(ensure_host(v));
  *a = (PetscScalar*)v->h;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecRestoreArrayWrite(Vec v, PetscScalar** a) { return VecRestoreArray(v, a); }

extern "C" PetscErrorCode VecHIPGetArrayRead(Vec v, const PetscScalar** a) {
  VCHK(v);
  PetscCall(sync_to_device(v));
  *a = (const PetscScalar*)v->d;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecHIPRestoreArrayRead(Vec v, const PetscScalar** a) {
  VCHK(v);
  if (a) *a = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecHIPGetArray(Vec v, PetscScalar** a) {
  VCHK(v);
  PetscCall(sync_to_device(v));
  *a = (PetscScalar*)v->d;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecHIPRestoreArray(Vec v, PetscScalar** a) {
  VCHK(v);
  v->mask = MASK_GPU;
  touch(v);
  if (a) *a = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecHIPGetArrayWrite(Vec v, PetscScalar** a) {
  VCHK(v);
  if (!v->hip) return ERR(PETSC_ERR_ARG_WRONG, "not a device vector");
  *a = (PetscScalar*)v->d;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecHIPRestoreArrayWrite(Vec v, PetscScalar** a) { return VecHIPRestoreArray(v, a); }

extern "C" PetscErrorCode VecGetArrayReadAndMemType(Vec v, const PetscScalar** a, PetscMemType* m) {
  VCHK(v);
  if (v->hip) {
    if (m) *m = PETSC_MEMTYPE_HIP;
    return VecHIPGetArrayRead(v, a);
  }
  if (m) *m = PETSC_MEMTYPE_HOST;
  return VecGetArrayRead(v, a);
}
extern "C" PetscErrorCode VecRestoreArrayReadAndMemType(Vec v, const PetscScalar** a) {
  VCHK(v);
  if (a) *a = nullptr;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetArrayWriteAndMemType(Vec v, PetscScalar** a, PetscMemType* m) {
  VCHK(v);
  if (v->hip) {
    if (m) *m = PETSC_MEMTYPE_HIP;
    return VecHIPGetArrayWrite(v, a);
  }
  if (m) *m = PETSC_MEMTYPE_HOST;
  return VecGetArrayWrite(v, a);
}
extern "C" PetscErrorCode VecRestoreArrayWriteAndMemType(Vec v, PetscScalar** a) {
  VCHK(v);
  return v->hip ? VecHIPRestoreArray(v, a) : VecRestoreArray(v, a);
}
extern "C" PetscErrorCode VecGetArrayAndMemType(Vec v, PetscScalar** a, PetscMemType* m) {
  VCHK(v);
  if (v->hip) {
    if (m) *m = PETSC_MEMTYPE_HIP;
    return VecHIPGetArray(v, a);
  }
  if (m) *m = PETSC_MEMTYPE_HOST;
  return VecGetArray(v, a);
}
extern "C" PetscErrorCode VecRestoreArrayAndMemType(Vec v, PetscScalar** a) {
  return VecRestoreArrayWriteAndMemType(v, a);
}

// device pointers for an operation that reads `in` vectors and writes `out` (all HIP), or
// host pointers if every vector is host-resident
static bool all_hip(std::initializer_list<Vec> vs) {
  for (Vec v : vs)
    if (!v->hip) return false;
  return true;
}
static PetscErrorCode same_size(Vec a, Vec b) {
  if (a->n != b->n) return ERR(PETSC_ERR_ARG_SIZ, "vector sizes differ");
  return PETSC_SUCCESS;
}
static PetscErrorCode dev_read(Vec v, const cd** p) {
  PetscCall(sync_to_device(v));
  *p = v->d;
  return PETSC_SUCCESS;
}
static PetscErrorCode dev_rw(Vec v, cd** p) {
  PetscCall(sync_to_device(v));
  v->mask = MASK_GPU;
  touch(v);
  *p = v->d;
  return PETSC_SUCCESS;
}
static PetscErrorCode host_read(Vec v, const cd** p) {
  PetscCall(sync_to_host(v));
  *p = v->h;
  return PETSC_SUCCESS;
}
static PetscErrorCode host_rw(Vec v, cd** p) {
  PetscCall(sync_to_host(v));
  v->mask = MASK_CPU;
  touch(v);
  *p = v->h;
  return PETSC_SUCCESS;
}
#define HIPK(expr) HCHK(expr)

extern "C" PetscErrorCode VecSet(Vec v, PetscScalar a) {
  VCHK(v);
  touch(v);
  if (v->hip) {
    v->mask = MASK_GPU;
    HIPK(cfp::blas_set(v->d, tocd(a), v->n, g_stream));
  } else {
    for (PetscInt i = 0; i < v->n; ++i) v->h[i] = tocd(a);
    v->mask = MASK_CPU;
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecSetValue(Vec v, PetscInt i, PetscScalar val, InsertMode mode) {
  return VecSetValues(v, 1, &i, &val, mode);
}
extern "C" PetscErrorCode VecSetValues(Vec v, PetscInt n, const PetscInt* idx, const PetscScalar* y, InsertMode mode) {
  VCHK(v);
  cd* h;
  PetscCall(host_rw(v, &h));
  for (PetscInt k = 0; k < n; ++k) {
    if (idx[k] < 0) continue;
    if (idx[k] >= v->n) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "index out of range");
    cd val = tocd(y[k]);
    if (mode == ADD_VALUES) val = cfp::make_cd(h[idx[k]].x + val.x, h[idx[k]].y + val.y);
    h[idx[k]] = val;
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetValues(Vec v, PetscInt n, const PetscInt* idx, PetscScalar* y) {
  VCHK(v);
  const cd* h;
  PetscCall(host_read(v, &h));
  for (PetscInt k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= v->n) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "index out of range");
    y[k] = PetscScalar(h[idx[k]].x, h[idx[k]].y);
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecAssemblyBegin(Vec v) { VCHK(v); return PETSC_SUCCESS; }
extern "C" PetscErrorCode VecAssemblyEnd(Vec v) { VCHK(v); return PETSC_SUCCESS; }

extern "C" PetscErrorCode VecCopy(Vec x, Vec y) {
  VCHK(x); VCHK(y);
  PetscCall(same_size(x, y));
  if (x == y) return PETSC_SUCCESS;
  touch(y);
  if (y->hip) {
    cd* yd;
    if (x->hip) {
      const cd* xd;
      PetscCall(dev_read(x, &xd));
      y->mask = MASK_GPU;
      HIPK(hipMemcpyAsync(y->d, xd, sizeof(cd) * (size_t)x->n, hipMemcpyDeviceToDevice, g_stream));
    } else {
      (void)yd;
      HIPK(hipMemcpyAsync(y->d, x->h, sizeof(cd) * (size_t)x->n, hipMemcpyHostToDevice, g_stream));
      HIPK(hipStreamSynchronize(g_stream));
      y->mask = MASK_GPU;
    }
  } else {
    const cd* xh;
    PetscCall(host_read(x, &xh));
    std::memcpy(y->h, xh, sizeof(cd) * (size_t)x->n);
    y->mask = MASK_CPU;
  }
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecScale(Vec x, PetscScalar a) {
  VCHK(x);
  if (x->hip) {
    cd* xd;
    PetscCall(dev_rw(x, &xd));
    HIPK(cfp::launch_scale(xd, tocd(a), x->n, g_stream));
  } else {
    cd* h;
    PetscCall(host_rw(x, &h));
    for (PetscInt i = 0; i < x->n; ++i) {
      std::complex<double> v(h[i].x, h[i].y);
      v *= a;
      h[i] = cfp::make_cd(v.real(), v.imag());
    }
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecShift(Vec x, PetscScalar a) {
  VCHK(x);
  if (x->hip) {
    cd* xd;
    PetscCall(dev_rw(x, &xd));
    HIPK(cfp::blas_shift(xd, tocd(a), x->n, g_stream));
  } else {
    cd* h;
    PetscCall(host_rw(x, &h));
    for (PetscInt i = 0; i < x->n; ++i) h[i] = cfp::make_cd(h[i].x + a.real(), h[i].y + a.imag());
  }
  return PETSC_SUCCESS;
}

template <class DevOp, class HostOp>
static PetscErrorCode binop(Vec out, Vec a, Vec b, DevOp dop, HostOp hop) {
  VCHK(out); VCHK(a);
  if (b) { VCHK(b); PetscCall(same_size(a, b)); }
  PetscCall(same_size(out, a));
  if (all_hip({out, a}) && (!b || b->hip)) {
    const cd *ad, *bd = nullptr;
    PetscCall(dev_read(a, &ad));
    if (b) PetscCall(dev_read(b, &bd));
    cd* od;
    PetscCall(dev_rw(out, &od));
    HIPK(dop(od, ad, bd));
  } else {
    const cd *ah, *bh = nullptr;
    PetscCall(host_read(a, &ah));
    if (b) PetscCall(host_read(b, &bh));
    cd* oh;
    PetscCall(host_rw(out, &oh));
    hop(oh, ah, bh);
    if (out->hip) {
      HIPK(hipMemcpyAsync(out->d, out->h, sizeof(cd) * (size_t)out->n, hipMemcpyHostToDevice, g_stream));
      out->mask = MASK_BOTH;
    }
  }
  return PETSC_SUCCESS;
}

static inline std::complex<double> C(cd v) { return {v.x, v.y}; }
static inline cd D(std::complex<double> v) { return cfp::make_cd(v.real(), v.imag()); }

extern "C" PetscErrorCode VecAXPY(Vec y, PetscScalar a, Vec x) {  // y += a x
  const i64 n = y ? y->n : 0;
  return binop(y, x, nullptr,
               [&](cd* o, const cd* xa, const cd*) { return cfp::blas_axpy(o, tocd(a), xa, n, g_stream); },
               [&](cd* o, const cd* xa, const cd*) { for (i64 i = 0; i < n; ++i) o[i] = D(C(o[i]) + a * C(xa[i])); });
}
extern "C" PetscErrorCode VecAYPX(Vec y, PetscScalar b, Vec x) {  // y = x + b y
  const i64 n = y ? y->n : 0;
  return binop(y, x, nullptr,
               [&](cd* o, const cd* xa, const cd*) { return cfp::blas_aypx(o, tocd(b), xa, n, g_stream); },
               [&](cd* o, const cd* xa, const cd*) { for (i64 i = 0; i < n; ++i) o[i] = D(C(xa[i]) + b * C(o[i])); });
}
extern "C" PetscErrorCode VecWAXPY(Vec w, PetscScalar a, Vec x, Vec y) {  // w = a x + y
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](cd* o, const cd* xa, const cd* yb) { return cfp::blas_waxpy(o, tocd(a), xa, yb, n, g_stream); },
               [&](cd* o, const cd* xa, const cd* yb) { for (i64 i = 0; i < n; ++i) o[i] = D(a * C(xa[i]) + C(yb[i])); });
}
extern "C" PetscErrorCode VecPointwiseDivide(Vec w, Vec x, Vec y) {
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](cd* o, const cd* xa, const cd* yb) { return cfp::launch_pointwise_divide(o, xa, yb, n, g_stream); },
               [&](cd* o, const cd* xa, const cd* yb) {  // PETSc: a zero divisor gives 0 (bvec2.c)
                 for (i64 i = 0; i < n; ++i) o[i] = C(yb[i]) != 0.0 ? D(C(xa[i]) / C(yb[i])) : D(0.0);
               });
}
extern "C" PetscErrorCode VecPointwiseMult(Vec w, Vec x, Vec y) {
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](cd* o, const cd* xa, const cd* yb) { return cfp::blas_pmult(o, xa, yb, n, g_stream); },
               [&](cd* o, const cd* xa, const cd* yb) { for (i64 i = 0; i < n; ++i) o[i] = D(C(xa[i]) * C(yb[i])); });
}

extern "C" PetscErrorCode VecDot(Vec x, Vec y, PetscScalar* val) {  // y^H x
  VCHK(x); VCHK(y);
  PetscCall(same_size(x, y));
  if (x->hip && y->hip) {
    const cd *xd, *yd;
    PetscCall(dev_read(x, &xd));
    PetscCall(dev_read(y, &yd));
    cd r;
    HIPK(cfp::blas_dot(xd, yd, x->n, &r, g_stream));
    *val = PetscScalar(r.x, r.y);
  } else {
    const cd *xh, *yh;
    PetscCall(host_read(x, &xh));
    PetscCall(host_read(y, &yh));
    std::complex<double> s = 0;
    for (i64 i = 0; i < x->n; ++i) s += C(xh[i]) * std::conj(C(yh[i]));
    *val = s;
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecNorm(Vec x, NormType t, PetscReal* val) {
  VCHK(x);
  if (t == NORM_FROBENIUS) t = NORM_2;
  if (x->hip) {
    const cd* xd;
    PetscCall(dev_read(x, &xd));
    HIPK(cfp::blas_norm(xd, x->n, (int)t, val, g_stream));
  } else {
    const cd* h;
    PetscCall(host_read(x, &h));
    double s = 0;
    for (i64 i = 0; i < x->n; ++i) {
      if (t == NORM_2) s += h[i].x * h[i].x + h[i].y * h[i].y;
      else if (t == NORM_1) s += std::fabs(h[i].x) + std::fabs(h[i].y);
      else s = std::fmax(s, std::hypot(h[i].x, h[i].y));
    }
    *val = t == NORM_2 ? std::sqrt(s) : s;
  }
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecMDot(Vec x, PetscInt nv, const Vec y[], PetscScalar val[]) {
  VCHK(x);
  if (nv <= 0) return PETSC_SUCCESS;
  bool dev = x->hip;
  for (PetscInt j = 0; j < nv; ++j) {
    VCHK(y[j]);
    PetscCall(same_size(x, y[j]));
    dev = dev && y[j]->hip;
  }
  if (dev) {
    const cd* xd;
    PetscCall(dev_read(x, &xd));
    std::vector<const cd*> ys((size_t)nv);
    for (PetscInt j = 0; j < nv; ++j) PetscCall(dev_read(y[j], &ys[(size_t)j]));
    std::vector<cd> r((size_t)nv);
    HIPK(cfp::blas_mdot(xd, (int)nv, ys.data(), x->n, r.data(), g_stream));
    for (PetscInt j = 0; j < nv; ++j) val[j] = PetscScalar(r[(size_t)j].x, r[(size_t)j].y);
    return PETSC_SUCCESS;
  }
  for (PetscInt j = 0; j < nv; ++j) PetscCall(VecDot(x, y[j], &val[j]));
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecMAXPY(Vec y, PetscInt nv, const PetscScalar alpha[], Vec x[]) {
  VCHK(y);
  if (nv <= 0) return PETSC_SUCCESS;
  bool dev = y->hip;
  for (PetscInt j = 0; j < nv; ++j) {
    VCHK(x[j]);
    PetscCall(same_size(y, x[j]));
    dev = dev && x[j]->hip;
  }
  if (dev) {
    std::vector<const cd*> xs((size_t)nv);
    std::vector<cd> a((size_t)nv);
    for (PetscInt j = 0; j < nv; ++j) {
      PetscCall(dev_read(x[j], &xs[(size_t)j]));
      a[(size_t)j] = tocd(alpha[j]);
    }
    cd* yd;
    PetscCall(dev_rw(y, &yd));
    HIPK(cfp::blas_maxpy(yd, (int)nv, a.data(), xs.data(), y->n, g_stream));
    return PETSC_SUCCESS;
  }
  for (PetscInt j = 0; j < nv; ++j) PetscCall(VecAXPY(y, alpha[j], x[j]));
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecDuplicateVecs(Vec v, PetscInt m, Vec* V[]) {
  VCHK(v);
  if (!V) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  Vec* arr = (Vec*)calloc((size_t)(m > 0 ? m : 1), sizeof(Vec));
  for (PetscInt j = 0; j < m; ++j) {
    PetscErrorCode rc = VecDuplicate(v, &arr[j]);
    if (rc) {
      for (PetscInt q = 0; q < j; ++q) VecDestroy(&arr[q]);
      free(arr);
      return rc;
    }
  }
  *V = arr;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecDestroyVecs(PetscInt m, Vec* V[]) {
  if (!V || !*V) return PETSC_SUCCESS;
  for (PetscInt j = 0; j < m; ++j) PetscCall(VecDestroy(&(*V)[j]));
  free(*V);
  *V = nullptr;
  return PETSC_SUCCESS;
}

// ------------------------------------------------------------------ Mat
static const int kMatMagic = 0x4d617431;
typedef PetscErrorCode (*MatMultFn)(Mat, Vec, Vec);
typedef PetscErrorCode (*MatDestroyFn)(Mat);

struct _p_Mat {
  int magic = kMatMagic;
  std::string type;
  PetscInt m = 0, n = 0;
  void* ctx = nullptr;
  MatMultFn mult = nullptr, multT = nullptr;
  MatDestroyFn destroy = nullptr;
  // AIJ (device CSR)
  i64 *rowptr = nullptr, *col = nullptr;
  cd* val = nullptr;
  std::vector<i64> h_rowptr, h_col;
  std::vector<cd> h_val;
};

static PetscErrorCode mcheck(Mat A, const char* f) {
  if (!A || A->magic != kMatMagic) return PetscErrorSet(PETSC_ERR_ARG_NULL, f, "invalid Mat");
  return PETSC_SUCCESS;
}
#define MCHK(A) PetscCall(mcheck((A), __func__))

extern "C" PetscErrorCode MatCreateShell(MPI_Comm, PetscInt m, PetscInt n, PetscInt M, PetscInt N, void* ctx, Mat* A) {
  if (!A) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  Mat a = new _p_Mat;
  a->type = MATSHELL;
  a->m = M >= 0 ? M : m;
  a->n = N >= 0 ? N : n;
  a->ctx = ctx;
  *A = a;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatShellSetOperation(Mat A, MatOperation op, void (*f)(void)) {
  MCHK(A);
  if (op == MATOP_MULT) A->mult = (MatMultFn)f;
  else if (op == MATOP_MULT_TRANSPOSE) A->multT = (MatMultFn)f;
  else if (op == MATOP_DESTROY) A->destroy = (MatDestroyFn)f;
  else return ERR(PETSC_ERR_SUP, "operation not supported by the stand-in MATSHELL");
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatShellGetContext(Mat A, void* ctx) {
  MCHK(A);
  if (A->type != MATSHELL) return ERR(PETSC_ERR_ARG_WRONG, "not a MATSHELL");
  *(void**)ctx = A->ctx;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatCreateSeqAIJWithArrays(MPI_Comm, PetscInt m, PetscInt n, PetscInt* i, PetscInt* j,
                                                    PetscScalar* a, Mat* A) {
  if (!A || !i || !j || !a) return ERR(PETSC_ERR_ARG_NULL, "NULL argument");
  Mat M = new _p_Mat;
  M->type = MATSEQAIJ;
  M->m = m;
  M->n = n;
  const i64 nnz = i[m];
  M->h_rowptr.assign(i, i + m + 1);
  M->h_col.assign(j, j + nnz);
  M->h_val.resize((size_t)nnz);
  for (i64 k = 0; k < nnz; ++k) M->h_val[k] = tocd(a[k]);
  *A = M;  // the device copy is made by the first MatMult on HIP vectors
  return PETSC_SUCCESS;
}
// mirror the host CSR into device memory (once; MatShift refreshes the values)
static PetscErrorCode aij_upload(Mat M) {
  if (M->rowptr) return PETSC_SUCCESS;
  const size_t nnz = M->h_col.size();
  hipError_t e = hipMalloc(&M->rowptr, sizeof(i64) * (size_t)(M->m + 1));
  if (e == hipSuccess) e = hipMalloc(&M->col, sizeof(i64) * (nnz > 0 ? nnz : 1));
  if (e == hipSuccess) e = hipMalloc(&M->val, sizeof(cd) * (nnz > 0 ? nnz : 1));
  if (e == hipSuccess) e = hipMemcpy(M->rowptr, M->h_rowptr.data(), sizeof(i64) * (size_t)(M->m + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess && nnz) e = hipMemcpy(M->col, M->h_col.data(), sizeof(i64) * nnz, hipMemcpyHostToDevice);
  if (e == hipSuccess && nnz) e = hipMemcpy(M->val, M->h_val.data(), sizeof(cd) * nnz, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (M->rowptr) hipFree(M->rowptr);
    if (M->col) hipFree(M->col);
    if (M->val) hipFree(M->val);
    M->rowptr = M->col = nullptr;
    M->val = nullptr;
    return ERR(PETSC_ERR_MEM, hipGetErrorString(e));
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetType(Mat A, MatType* t) {
  MCHK(A);
  *t = A->type == MATSEQAIJ ? MATSEQAIJ : MATSHELL;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetSize(Mat A, PetscInt* m, PetscInt* n) {
  MCHK(A);
  if (m) *m = A->m;
  if (n) *n = A->n;
  return PETSC_SUCCESS;
}
static PetscErrorCode aij_mult(Mat A, Vec x, Vec y) {
  if (x->n != A->n || y->n != A->m) return ERR(PETSC_ERR_ARG_SIZ, "MatMult sizes");
  if (x == y) return ERR(PETSC_ERR_ARG_IDN, "x and y must be different vectors");
  if (x->hip && y->hip) {
    PetscCall(aij_upload(A));
    const cd* xd;
    PetscCall(dev_read(x, &xd));
    cd* yd;
    PetscCall(dev_rw(y, &yd));
    HIPK(cfp::blas_csr_spmv(A->m, A->rowptr, A->col, A->val, xd, yd, g_stream));
  } else {
    const cd* xh;
    PetscCall(host_read(x, &xh));
    cd* yh;
    PetscCall(host_rw(y, &yh));
    for (i64 r = 0; r < A->m; ++r) {
      std::complex<double> s = 0;
      for (i64 p = A->h_rowptr[r]; p < A->h_rowptr[r + 1]; ++p) s += C(A->h_val[p]) * C(xh[A->h_col[p]]);
      yh[r] = D(s);
    }
    if (y->hip) {
      HIPK(hipMemcpyAsync(y->d, y->h, sizeof(cd) * (size_t)y->n, hipMemcpyHostToDevice, g_stream));
      y->mask = MASK_BOTH;
    }
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatMult(Mat A, Vec x, Vec y) {
  MCHK(A); VCHK(x); VCHK(y);
  if (A->type == MATSEQAIJ) return aij_mult(A, x, y);
  if (!A->mult) return ERR(PETSC_ERR_SUP, "MatMult not set on this MATSHELL");
  return A->mult(A, x, y);
}
extern "C" PetscErrorCode MatMultTranspose(Mat A, Vec x, Vec y) {
  MCHK(A); VCHK(x); VCHK(y);
  if (A->type == MATSEQAIJ) return ERR(PETSC_ERR_SUP, "MatMultTranspose on AIJ not provided by the stand-in");
  if (!A->multT) return ERR(PETSC_ERR_SUP, "MatMultTranspose not set on this MATSHELL");
  return A->multT(A, x, y);
}
extern "C" PetscErrorCode MatShift(Mat A, PetscScalar a) {
  MCHK(A);
  if (A->type != MATSEQAIJ) return ERR(PETSC_ERR_SUP, "MatShift only for AIJ in the stand-in");
  for (i64 r = 0; r < A->m; ++r) {
    bool found = false;
    for (i64 p = A->h_rowptr[r]; p < A->h_rowptr[r + 1]; ++p)
      if (A->h_col[p] == r) { A->h_val[p] = D(C(A->h_val[p]) + a); found = true; }
    if (!found) return ERR(PETSC_ERR_ARG_WRONGSTATE, "MatShift needs an allocated diagonal");
  }
  if (A->val && !A->h_val.empty())
    HCHK(hipMemcpy(A->val, A->h_val.data(), sizeof(cd) * A->h_val.size(), hipMemcpyHostToDevice));
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatDestroy(Mat* pA) {
  if (!pA || !*pA) return PETSC_SUCCESS;
  Mat A = *pA;
  MCHK(A);
  PetscErrorCode rc = PETSC_SUCCESS;
  if (A->destroy) rc = A->destroy(A);
  if (A->rowptr) hipFree(A->rowptr);
  if (A->col) hipFree(A->col);
  if (A->val) hipFree(A->val);
  A->magic = 0;
  delete A;
  *pA = nullptr;
  return rc;
}
extern "C" PetscErrorCode MatCreateFFT(MPI_Comm comm, PetscInt ndim, const PetscInt dims[], MatType type, Mat* A) {
  if (!type || std::strcmp(type, MATFFTW) != 0)
    return ERR(PETSC_ERR_SUP, "MatCreateFFT: only MATFFTW (served by the HIP plan) is available");
  return MatCreateFFTHIP(comm, ndim, dims, A);
}
extern "C" PetscErrorCode MatCreateVecsFFTW(Mat A, Vec* x, Vec* y, Vec* z) {
  MCHK(A);
  Vec* outs[3] = {x, y, z};
  for (Vec* o : outs)
    if (o) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, A->n, o));
  return PETSC_SUCCESS;
}

// ------------------------------------------------------------------ PC
static const int kPCMagic = 0x50433131;
struct _p_PC {
  int magic = kPCMagic;
  std::string type = "";
  std::string name;
  void* ctx = nullptr;
  PetscErrorCode (*apply)(PC, Vec, Vec) = nullptr;
  PetscErrorCode (*setup)(PC) = nullptr;
  PetscErrorCode (*destroy)(PC) = nullptr;
  bool setupcalled = false;
};
static PetscErrorCode pcheck(PC pc, const char* f) {
  if (!pc || pc->magic != kPCMagic) return PetscErrorSet(PETSC_ERR_ARG_NULL, f, "invalid PC");
  return PETSC_SUCCESS;
}
#define PCCHK(pc) PetscCall(pcheck((pc), __func__))

extern "C" PetscErrorCode PCCreate(MPI_Comm, PC* pc) {
  if (!pc) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  *pc = new _p_PC;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCSetType(PC pc, PCType t) {
  PCCHK(pc);
  if (!t || (std::strcmp(t, PCSHELL) && std::strcmp(t, PCNONE))) return ERR(PETSC_ERR_SUP, "stand-in PC types: shell, none");
  pc->type = t;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCGetType(PC pc, PCType* t) { PCCHK(pc); *t = pc->type.c_str(); return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCShellSetContext(PC pc, void* ctx) { PCCHK(pc); pc->ctx = ctx; return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCShellGetContext(PC pc, void* ctx) {
  PCCHK(pc);
  if (!ctx) return ERR(PETSC_ERR_ARG_NULL, "ctx must point to the caller's context pointer");
  *(void**)ctx = pc->ctx;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCShellSetApply(PC pc, PetscErrorCode (*f)(PC, Vec, Vec)) { PCCHK(pc); pc->apply = f; return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCShellSetSetUp(PC pc, PetscErrorCode (*f)(PC)) { PCCHK(pc); pc->setup = f; return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCShellSetDestroy(PC pc, PetscErrorCode (*f)(PC)) { PCCHK(pc); pc->destroy = f; return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCShellSetName(PC pc, const char* n) { PCCHK(pc); pc->name = n ? n : ""; return PETSC_SUCCESS; }
extern "C" PetscErrorCode PCSetUp(PC pc) {
  PCCHK(pc);
  if (pc->setupcalled) return PETSC_SUCCESS;
  if (pc->type == PCSHELL && pc->setup) PetscCall(pc->setup(pc));
  pc->setupcalled = true;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCApply(PC pc, Vec x, Vec y) {
  PCCHK(pc); VCHK(x); VCHK(y);
  if (x == y) return ERR(PETSC_ERR_ARG_IDN, "x and y must be different vectors");
  PetscCall(PCSetUp(pc));
  if (pc->type == PCNONE || pc->type.empty()) return VecCopy(x, y);
  if (!pc->apply) return ERR(PETSC_ERR_ARG_WRONGSTATE, "PCSHELL has no apply callback");
  return pc->apply(pc, x, y);
}
extern "C" PetscErrorCode PCDestroy(PC* ppc) {
  if (!ppc || !*ppc) return PETSC_SUCCESS;
  PC pc = *ppc;
  PCCHK(pc);
  PetscErrorCode rc = PETSC_SUCCESS;
  if (pc->type == PCSHELL && pc->destroy) rc = pc->destroy(pc);
  pc->magic = 0;
  delete pc;
  *ppc = nullptr;
  return rc;
}

#endif  // CFP_WITH_PETSC
