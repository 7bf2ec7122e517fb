// petsc_mini.cpp -- stand-in for the PETSc subset declared in include/petsc_mini.h.
//
// PETSc is not installed in this image or on the GPU box, so the PCSHELL
// boundary would otherwise be untestable.  This file gives Vec (host VECSEQ and device
// VECSEQHIP with PETSc's offload-mask semantics), Mat (MATSHELL, MATSEQAIJ, the FFT shell)
// and PC (PCSHELL, PCNONE) objects with PETSc's names and argument conventions.  It is
// compiled out when building against a real PETSc (-DCFP_WITH_PETSC).
#ifndef CFP_WITH_PETSC
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <sys/time.h>

#include <cmath>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pcshell_fft3d.h"
#include "../../include/petsc_mini.h"
#include "cfp_blas.h"
#include "cfp_internal.h"
#include "cfp_rccl.h"

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
extern "C" PetscErrorCode VecMiniGetStream(void** s) {
  if (!s) return PetscErrorSet(PETSC_ERR_ARG_NULL, __func__, "NULL output");
  *s = (void*)g_stream;
  return PETSC_SUCCESS;
}

#define ERR(code, msg) PetscErrorSet((code), __func__, (msg))

// ------------------------------------------------------------------ communicators
// handle 0 = PETSC_COMM_WORLD (resolves to g_world), 1 = PETSC_COMM_SELF, >= 2 created ones
struct CommRec {
  bool live = false;
  int size = 1, rank = 0;
  PetscMiniCommOps ops{};
  ncclComm_t nccl = nullptr;
  double* dbuf = nullptr;           // RCCL all-reduce staging (device)
  int64_t dbuf_n = 0;
  void* hsend = nullptr;            // exchange staging (pinned host)
  void* hrecv = nullptr;
  size_t hbytes = 0;
  int refs = 0;                     // FFT matrices (slab plans) built on this communicator
};
static std::mutex g_comm_mu;
static std::vector<CommRec> g_comms(2);
static MPI_Comm g_world = PETSC_COMM_SELF;

static CommRec* comm_rec(MPI_Comm c) {
  if (c == PETSC_COMM_WORLD) c = g_world;
  if (c < 1 || c >= (MPI_Comm)g_comms.size() || (c >= 2 && !g_comms[(size_t)c].live)) return nullptr;
  return &g_comms[(size_t)c];
}
static MPI_Comm comm_resolve(MPI_Comm c) { return c == PETSC_COMM_WORLD ? g_world : c; }

extern "C" int MPI_Comm_size(MPI_Comm c, int* size) {
  CommRec* r = comm_rec(c);
  if (!r || !size) return 1;
  *size = r->size;
  return MPI_SUCCESS;
}
extern "C" int MPI_Comm_rank(MPI_Comm c, int* rank) {
  CommRec* r = comm_rec(c);
  if (!r || !rank) return 1;
  *rank = r->rank;
  return MPI_SUCCESS;
}

static PetscErrorCode comm_new(CommRec rec, MPI_Comm* out) {
  std::lock_guard<std::mutex> g(g_comm_mu);
  rec.live = true;
  for (size_t i = 2; i < g_comms.size(); ++i)
    if (!g_comms[i].live) {
      g_comms[i] = rec;
      *out = (MPI_Comm)i;
      return PETSC_SUCCESS;
    }
  g_comms.push_back(rec);
  *out = (MPI_Comm)(g_comms.size() - 1);
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniCommCreate(int size, int rank, const PetscMiniCommOps* ops, MPI_Comm* comm) {
  if (!comm) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  if (size < 1 || rank < 0 || rank >= size) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "rank / size");
  if (size > 1 && (!ops || !ops->alltoall || !ops->allreduce))
    return ERR(PETSC_ERR_ARG_NULL, "a communicator of several ranks needs alltoall and allreduce");
  CommRec r;
  r.size = size;
  r.rank = rank;
  if (ops) r.ops = *ops;
  return comm_new(r, comm);
}

extern "C" PetscErrorCode PetscMiniCommCreateRCCL(int size, int rank, const char* uid, MPI_Comm* comm) {
  if (!comm || !uid) return ERR(PETSC_ERR_ARG_NULL, "NULL argument");
  if (size < 1 || rank < 0 || rank >= size) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "rank / size");
  CommRec r;
  r.size = size;
  r.rank = rank;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  bool timed_out = false;  // non-blocking creation against a deadline (cfp_rccl.h)
  ncclResult_t nr = cfp::rccl_init_rank(&r.nccl, size, id, rank, cfp::kRcclDefaultTimeoutS, &timed_out);
  if (nr != ncclSuccess) return ERR(PETSC_ERR_LIB, timed_out ? "ncclCommInitRankConfig: timed out" : ncclGetErrorString(nr));
  return comm_new(r, comm);
}

extern "C" PetscErrorCode PetscMiniCommDestroy(MPI_Comm* comm) {
  if (!comm || *comm < 2) return PETSC_SUCCESS;
  std::lock_guard<std::mutex> g(g_comm_mu);
  if (*comm >= (MPI_Comm)g_comms.size()) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  CommRec& r = g_comms[(size_t)*comm];
  if (r.refs > 0)  // a slab plan still sends over it (its ncclComm_t, or the callbacks)
    return ERR(PETSC_ERR_ARG_WRONGSTATE, "communicator still used by FFT matrices: destroy them first");
  if (r.nccl) cfp::rccl_destroy(r.nccl, cfp::kRcclDefaultTimeoutS);
  if (r.dbuf) hipFree(r.dbuf);
  if (r.hsend) hipHostFree(r.hsend);
  if (r.hrecv) hipHostFree(r.hrecv);
  if (g_world == *comm) g_world = PETSC_COMM_SELF;
  r = CommRec();
  *comm = PETSC_COMM_SELF;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniCommRetain(MPI_Comm comm) {
  std::lock_guard<std::mutex> g(g_comm_mu);
  CommRec* r = comm_rec(comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  ++r->refs;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscMiniCommRelease(MPI_Comm comm) {
  std::lock_guard<std::mutex> g(g_comm_mu);
  CommRec* r = comm_rec(comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  if (r->refs > 0) --r->refs;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniSetCommWorld(MPI_Comm comm) {
  comm = comm_resolve(comm);
  if (!comm_rec(comm)) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  g_world = comm;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniCommResolve(MPI_Comm comm, MPI_Comm* out) {
  if (!out) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  *out = comm_resolve(comm);
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniCommGetNCCL(MPI_Comm comm, void** nccl) {
  CommRec* r = comm_rec(comm);
  if (!r || !nccl) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  *nccl = (void*)r->nccl;
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode PetscMiniAllreduce(MPI_Comm comm, double* buf, int64_t count, int op) {
  CommRec* r = comm_rec(comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  if (r->size == 1 || count <= 0) return PETSC_SUCCESS;
  if (r->nccl) {
    if (r->dbuf_n < count) {
      if (r->dbuf) hipFree(r->dbuf);
      r->dbuf = nullptr;
      r->dbuf_n = 0;
      if (hipMalloc(&r->dbuf, sizeof(double) * (size_t)count) != hipSuccess) return ERR(PETSC_ERR_MEM, "allreduce buffer");
      r->dbuf_n = count;
    }
    if (hipMemcpyAsync(r->dbuf, buf, sizeof(double) * (size_t)count, hipMemcpyHostToDevice, g_stream) != hipSuccess)
      return ERR(PETSC_ERR_LIB, "allreduce copy");
    ncclResult_t nr = cfp::rccl_settle(
        r->nccl, ncclAllReduce(r->dbuf, r->dbuf, (size_t)count, ncclDouble, op == PETSCMINI_OP_MAX ? ncclMax : ncclSum,
                               r->nccl, g_stream), cfp::kRcclDefaultTimeoutS);
    if (nr != ncclSuccess) return ERR(PETSC_ERR_LIB, ncclGetErrorString(nr));
    if (hipMemcpyAsync(buf, r->dbuf, sizeof(double) * (size_t)count, hipMemcpyDeviceToHost, g_stream) != hipSuccess ||
        hipStreamSynchronize(g_stream) != hipSuccess)
      return ERR(PETSC_ERR_LIB, "allreduce copy back");
    return PETSC_SUCCESS;
  }
  if (r->ops.allreduce(r->ops.user, buf, count, op)) return ERR(PETSC_ERR_LIB, "allreduce callback failed");
  return PETSC_SUCCESS;
}

// host all-to-all of `per_peer` bytes from every rank to every rank ([size][per_peer] in and
// out): the caller's callback, or RCCL through device staging
static PetscErrorCode comm_alltoall_host(CommRec* r, const void* send, void* recv, size_t per_peer) {
  const size_t total = per_peer * (size_t)r->size;
  if (r->size == 1 || per_peer == 0) {
    std::memcpy(recv, send, total);
    return PETSC_SUCCESS;
  }
  if (!r->nccl) {
    if (r->ops.alltoall(r->ops.user, send, recv, (int64_t)per_peer)) return ERR(PETSC_ERR_LIB, "alltoall callback failed");
    return PETSC_SUCCESS;
  }
  char* d = nullptr;
  if (hipMalloc(&d, 2 * total) != hipSuccess) return ERR(PETSC_ERR_MEM, "alltoall staging");
  PetscErrorCode rc = PETSC_SUCCESS;
  if (hipMemcpyAsync(d, send, total, hipMemcpyHostToDevice, g_stream) != hipSuccess) rc = ERR(PETSC_ERR_LIB, "alltoall copy");
  if (!rc && ncclGroupStart() != ncclSuccess) rc = ERR(PETSC_ERR_LIB, "ncclGroupStart");
  if (!rc) {
    for (int q = 0; q < r->size && !rc; ++q)
      if (ncclSend(d + q * per_peer, per_peer, ncclChar, q, r->nccl, g_stream) != ncclSuccess ||
          ncclRecv(d + total + q * per_peer, per_peer, ncclChar, q, r->nccl, g_stream) != ncclSuccess)
        rc = ERR(PETSC_ERR_LIB, "ncclSend / ncclRecv");
    if (cfp::rccl_settle(r->nccl, ncclGroupEnd(), cfp::kRcclDefaultTimeoutS) != ncclSuccess && !rc)
      rc = ERR(PETSC_ERR_LIB, "ncclGroupEnd");
  }
  if (!rc && (hipMemcpyAsync(recv, d + total, total, hipMemcpyDeviceToHost, g_stream) != hipSuccess ||
              hipStreamSynchronize(g_stream) != hipSuccess))
    rc = ERR(PETSC_ERR_LIB, "alltoall copy back");
  hipFree(d);
  return rc;
}

// one exchange piece of a slab plan (include/circulant_fft_dist.h, cfp_dist_exchange_fn)
extern "C" int PetscMiniCommExchange(void* user, const double* src, double* dst, int64_t chunk, int64_t off,
                                     int64_t count, void* stream) {
  CommRec* r = comm_rec((MPI_Comm)(intptr_t)user);
  if (!r) return PetscErrorSet(PETSC_ERR_ARG_WRONG, __func__, "unknown communicator");
  hipStream_t st = (hipStream_t)stream;
  const cd* s = (const cd*)src + off;
  cd* d = (cd*)dst + off;
  const size_t bytes = sizeof(cd) * (size_t)count, pitch = sizeof(cd) * (size_t)chunk;
  if (r->nccl) {
    if (hipMemcpyAsync(d + r->rank * chunk, s + r->rank * chunk, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return PetscErrorSet(PETSC_ERR_LIB, __func__, "self copy");
    if (ncclGroupStart() != ncclSuccess) return PetscErrorSet(PETSC_ERR_LIB, __func__, "ncclGroupStart");
    for (int q = 0; q < r->size; ++q) {
      if (q == r->rank) continue;
      if (ncclSend(s + q * chunk, 2 * (size_t)count, ncclDouble, q, r->nccl, st) != ncclSuccess ||
          ncclRecv(d + q * chunk, 2 * (size_t)count, ncclDouble, q, r->nccl, st) != ncclSuccess)
        return PetscErrorSet(PETSC_ERR_LIB, __func__, "ncclSend / ncclRecv");
    }
    if (cfp::rccl_settle(r->nccl, ncclGroupEnd(), cfp::kRcclDefaultTimeoutS) != ncclSuccess)
      return PetscErrorSet(PETSC_ERR_LIB, __func__, "ncclGroupEnd");
    return 0;
  }
  // callback communicator: [size][count] pieces through pinned host buffers
  const size_t total = bytes * (size_t)r->size;
  if (r->hbytes < total) {
    if (r->hsend) hipHostFree(r->hsend);
    if (r->hrecv) hipHostFree(r->hrecv);
    r->hsend = r->hrecv = nullptr;
    r->hbytes = 0;
    if (hipHostMalloc(&r->hsend, total) != hipSuccess || hipHostMalloc(&r->hrecv, total) != hipSuccess)
      return PetscErrorSet(PETSC_ERR_MEM, __func__, "pinned staging");
    r->hbytes = total;
  }
  if (hipMemcpy2DAsync(r->hsend, bytes, s, pitch, bytes, (size_t)r->size, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return PetscErrorSet(PETSC_ERR_LIB, __func__, "device to host");
  if (r->size == 1) std::memcpy(r->hrecv, r->hsend, bytes);
  else if (r->ops.alltoall(r->ops.user, r->hsend, r->hrecv, (int64_t)bytes))
    return PetscErrorSet(PETSC_ERR_LIB, __func__, "alltoall callback failed");
  if (hipMemcpy2DAsync(d, pitch, r->hrecv, bytes, bytes, (size_t)r->size, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)  // the staging buffers are reused by the next piece
    return PetscErrorSet(PETSC_ERR_LIB, __func__, "host to device");
  return 0;
}
#define HCHK(expr)                                                      \
  do {                                                                  \
    hipError_t e__ = (expr);                                            \
    if (e__ != hipSuccess) return ERR(PETSC_ERR_LIB, hipGetErrorString(e__)); \
  } while (0)

// Vec / AIJ storage: complex double (cd) or, in the real-scalar build (-DCFP_REAL_SCALAR,
// PetscScalar = double, the reference's !PETSC_USE_COMPLEX branch), double.  Host arithmetic goes
// through std::complex (C / D); with real operands its results are real.
#ifdef CFP_REAL_SCALAR
typedef double VS;
static inline VS tocd(PetscScalar s) { return s; }
static inline std::complex<double> C(VS v) { return {v, 0.0}; }
static inline VS D(std::complex<double> v) { return v.real(); }
static inline PetscScalar to_scalar(double re, double) { return re; }
static inline double re_of(PetscScalar s) { return s; }
static inline double im_of(PetscScalar) { return 0.0; }
static inline hipError_t dev_scale(VS* x, VS a, i64 n, hipStream_t s) { return cfp::blas_scale(x, a, n, s); }
static inline hipError_t dev_pdivide(VS* w, const VS* x, const VS* y, i64 n, hipStream_t s) {
  return cfp::blas_pdivide(w, x, y, n, s);
}
#else
typedef cd VS;
static inline VS tocd(PetscScalar s) { return cfp::make_cd(s.real(), s.imag()); }
static inline std::complex<double> C(VS v) { return {v.x, v.y}; }
static inline VS D(std::complex<double> v) { return cfp::make_cd(v.real(), v.imag()); }
static inline PetscScalar to_scalar(double re, double im) { return PetscScalar(re, im); }
static inline double re_of(PetscScalar s) { return s.real(); }
static inline double im_of(PetscScalar s) { return s.imag(); }
static inline hipError_t dev_scale(VS* x, VS a, i64 n, hipStream_t s) { return cfp::launch_scale(x, a, n, s); }
static inline hipError_t dev_pdivide(VS* w, const VS* x, const VS* y, i64 n, hipStream_t s) {
  return cfp::launch_pointwise_divide(w, x, y, n, s);
}
#endif
static constexpr int kDPS = (int)(sizeof(VS) / sizeof(double));  // doubles per scalar

// ------------------------------------------------------------------ Vec
enum { MASK_NONE = 0, MASK_CPU = 1, MASK_GPU = 2, MASK_BOTH = 3 };
static const int kVecMagic = 0x56656331;

struct _p_Vec {
  int magic = kVecMagic;
  PetscInt n = 0;        // local size
  PetscInt N = 0;        // global size
  PetscInt rstart = 0;   // first global row of this rank
  MPI_Comm comm = PETSC_COMM_SELF;
  int nranks = 1;
  bool hip = false;
  VS* d = nullptr;
  VS* h = nullptr;
  bool own_d = false, own_h = false;
  int mask = MASK_NONE;
  int device = 0;
  PetscObjectId id = 0;
  PetscObjectState state = 0;  // bumped by every write access (PetscObjectStateGet)
  // |x|^2 partials of the last device VecAXPY into this vector (mapped pinned memory), valid while
  // state == nrm_state: a VecNorm(NORM_2) right after it sums them instead of re-reading the
  // vector (PETSc likewise caches norms against the object state)
  double *nrm_h = nullptr, *nrm_hd = nullptr;
  unsigned nrm_nb = 0;
  PetscObjectState nrm_state = -1;
  // VecSetValues entries of rows owned by other ranks, delivered by VecAssemblyBegin/End
  std::vector<PetscInt> st_idx;
  std::vector<VS> st_val;
  std::vector<char> st_add;
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
  if (v->hip) HCHK(cfp::host_wait(g_stream));
  return PETSC_SUCCESS;
}

static PetscErrorCode ensure_host(Vec v) {
  if (!v->h) {
    v->h = (VS*)calloc((size_t)(v->n > 0 ? v->n : 1), sizeof(VS));
    if (!v->h) return ERR(PETSC_ERR_MEM, "host allocation");
    v->own_h = true;
  }
  return PETSC_SUCCESS;
}
// make the host copy current (device -> host if only the device is valid)
static PetscErrorCode sync_to_host(Vec v) {
  PetscCall(ensure_host(v));
  if (v->hip && v->mask == MASK_GPU) {
    HCHK(hipMemcpyAsync(v->h, v->d, sizeof(VS) * (size_t)v->n, hipMemcpyDeviceToHost, g_stream));
    HCHK(hipStreamSynchronize(g_stream));
    v->mask = MASK_BOTH;
  }
  if (v->mask == MASK_NONE) v->mask = v->hip ? MASK_BOTH : MASK_CPU;
  return PETSC_SUCCESS;
}
static PetscErrorCode sync_to_device(Vec v) {
  if (!v->hip) return ERR(PETSC_ERR_ARG_WRONG, "not a device vector");
  if (v->mask == MASK_CPU) {
    HCHK(hipMemcpyAsync(v->d, v->h, sizeof(VS) * (size_t)v->n, hipMemcpyHostToDevice, g_stream));
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
  v->N = n;
  v->hip = hip;
  if (hip) {
    hipGetDevice(&v->device);
    if (devarr) {
      v->d = (VS*)devarr;
    } else {
      hipError_t e = hipMalloc(&v->d, sizeof(VS) * (size_t)(n > 0 ? n : 1));
      if (e != hipSuccess) { delete v; return ERR(PETSC_ERR_MEM, hipGetErrorString(e)); }
      v->own_d = true;
      hipMemsetAsync(v->d, 0, sizeof(VS) * (size_t)n, g_stream);
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
// PETSC_DECIDE rows (PetscSplitOwnership): N / size each, the first N % size ranks one more;
// with every local size given, N and the row start come from one all-reduce of the sizes
static PetscErrorCode mpi_layout(MPI_Comm comm, PetscInt nlocal, PetscInt N, PetscInt* n, PetscInt* Ng, PetscInt* rstart) {
  CommRec* r = comm_rec(comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  if (nlocal < 0 && N < 0) return ERR(PETSC_ERR_ARG_WRONG, "local or global size must be given");
  const int P = r->size, k = r->rank;
  if (nlocal < 0) {
    *n = N / P + (k < N % P ? 1 : 0);
    *Ng = N;
    *rstart = k * (N / P) + (k < N % P ? k : N % P);
    return PETSC_SUCCESS;
  }
  std::vector<double> sizes((size_t)P, 0.0);
  sizes[(size_t)k] = (double)nlocal;
  PetscCall(PetscMiniAllreduce(comm, sizes.data(), P, PETSCMINI_OP_SUM));
  PetscInt tot = 0, start = 0;
  for (int q = 0; q < P; ++q) {
    if (q == k) start = tot;
    tot += (PetscInt)sizes[(size_t)q];
  }
  if (N >= 0 && N != tot) return ERR(PETSC_ERR_ARG_SIZ, "the local sizes do not add up to N");
  *n = nlocal;
  *Ng = tot;
  *rstart = start;
  return PETSC_SUCCESS;
}

static PetscErrorCode vec_mpi(MPI_Comm comm, PetscInt nlocal, PetscInt N, bool hip, Vec* v,
                              const PetscScalar* devarr = nullptr) {
  comm = comm_resolve(comm);
  PetscInt n, Ng, rs;
  PetscCall(mpi_layout(comm, nlocal, N, &n, &Ng, &rs));
  PetscCall(vec_new(n, hip, devarr, v));
  (*v)->N = Ng;
  (*v)->rstart = rs;
  (*v)->comm = comm;
  MPI_Comm_size(comm, &(*v)->nranks);
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecCreateMPI(MPI_Comm comm, PetscInt nlocal, PetscInt N, Vec* v) {
  return vec_mpi(comm, nlocal, N, false, v);
}
extern "C" PetscErrorCode VecCreateMPIHIP(MPI_Comm comm, PetscInt nlocal, PetscInt N, Vec* v) {
  return vec_mpi(comm, nlocal, N, true, v);
}
extern "C" PetscErrorCode VecCreateMPIHIPWithArray(MPI_Comm comm, PetscInt, PetscInt nlocal, PetscInt N,
                                                   const PetscScalar* a, Vec* v) {
  if (!a) return ERR(PETSC_ERR_ARG_NULL, "NULL array");
  return vec_mpi(comm, nlocal, N, true, v, a);
}
extern "C" PetscErrorCode VecGetComm(Vec v, MPI_Comm* comm) {
  VCHK(v);
  *comm = v->comm;
  return PETSC_SUCCESS;
}
static void vec_copy_layout(Vec from, Vec to) {
  to->N = from->N;
  to->rstart = from->rstart;
  to->comm = from->comm;
  to->nranks = from->nranks;
}
extern "C" PetscErrorCode VecDuplicate(Vec v, Vec* nv) {
  VCHK(v);
  PetscCall(vec_new(v->n, v->hip, nullptr, nv));
  vec_copy_layout(v, *nv);
  return PETSC_SUCCESS;
}
// sum (or max) over the Vec's communicator; no-op on one rank
static PetscErrorCode vec_reduce(Vec v, double* buf, int64_t count, int op) {
  if (v->nranks == 1) return PETSC_SUCCESS;
  return PetscMiniAllreduce(v->comm, buf, count, op);
}
extern "C" PetscErrorCode VecDestroy(Vec* pv) {
  if (!pv || !*pv) return PETSC_SUCCESS;
  Vec v = *pv;
  VCHK(v);
  if (v->own_d && v->d) hipFree(v->d);
  if (v->own_h && v->h) free(v->h);
  if (v->nrm_h) hipHostFree(v->nrm_h);
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
  *t = v->nranks > 1 ? (v->hip ? VECMPIHIP : VECMPI) : (v->hip ? VECSEQHIP : VECSEQ);
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetSize(Vec v, PetscInt* n) { VCHK(v); *n = v->N; return PETSC_SUCCESS; }
extern "C" PetscErrorCode VecGetLocalSize(Vec v, PetscInt* n) { VCHK(v); *n = v->n; return PETSC_SUCCESS; }
extern "C" PetscErrorCode VecGetOwnershipRange(Vec v, PetscInt* lo, PetscInt* hi) {
  VCHK(v);
  if (lo) *lo = v->rstart;
  if (hi) *hi = v->rstart + v->n;
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
static PetscErrorCode dev_read(Vec v, const VS** p) {
  PetscCall(sync_to_device(v));
  *p = v->d;
  return PETSC_SUCCESS;
}
static PetscErrorCode dev_rw(Vec v, VS** p) {
  PetscCall(sync_to_device(v));
  v->mask = MASK_GPU;
  touch(v);
  *p = v->d;
  return PETSC_SUCCESS;
}
static PetscErrorCode host_read(Vec v, const VS** p) {
  PetscCall(sync_to_host(v));
  *p = v->h;
  return PETSC_SUCCESS;
}
static PetscErrorCode host_rw(Vec v, VS** p) {
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
  VS* h;
  PetscCall(host_rw(v, &h));
  for (PetscInt k = 0; k < n; ++k) {
    if (idx[k] < 0) continue;
    if (idx[k] >= v->N) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "index out of range");
    const PetscInt i = idx[k] - v->rstart;  // global row -> local
    if (i < 0 || i >= v->n) {  // another rank's row: stashed until VecAssemblyBegin/End
      if (v->st_idx.size() >= ((size_t)1 << 27))
        return ERR(PETSC_ERR_MEM, "VecSetValues: 2^27 off-rank entries stashed without VecAssemblyBegin");
      v->st_idx.push_back(idx[k]);
      v->st_val.push_back(tocd(y[k]));
      v->st_add.push_back(mode == ADD_VALUES);
      continue;
    }
    VS val = tocd(y[k]);
    if (mode == ADD_VALUES) val = D(C(h[i]) + C(val));
    h[i] = val;
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecGetValues(Vec v, PetscInt n, const PetscInt* idx, PetscScalar* y) {
  VCHK(v);
  const VS* h;
  PetscCall(host_read(v, &h));
  for (PetscInt k = 0; k < n; ++k) {
    const PetscInt i = idx[k] - v->rstart;  // local rows only, as PETSc's VecGetValues
    if (i < 0 || i >= v->n) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "index not owned by this rank");
    y[k] = to_scalar(C(h[i]).real(), C(h[i]).imag());
  }
  return PETSC_SUCCESS;
}
// Collective, as in PETSc: every rank's stashed entries travel to their owners (one all-reduce of
// the largest per-peer count, one all-to-all of 32-byte records [row, re, im, add]) and are
// applied there in rank order.  Begin does the whole exchange; End only completes the pair.
extern "C" PetscErrorCode VecAssemblyBegin(Vec v) {
  VCHK(v);
  if (v->nranks == 1) {
    v->st_idx.clear(), v->st_val.clear(), v->st_add.clear();
    return PETSC_SUCCESS;
  }
  CommRec* r = comm_rec(v->comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  const int P = r->size;
  // owner of a global row: the Vec's layout, gathered from every rank's start (one all-reduce)
  std::vector<double> starts((size_t)P, 0.0);
  starts[(size_t)r->rank] = (double)v->rstart;
  PetscCall(PetscMiniAllreduce(v->comm, starts.data(), P, PETSCMINI_OP_SUM));
  const auto owner = [&](PetscInt g) {
    int q = (int)(std::upper_bound(starts.begin(), starts.end(), (double)g) - starts.begin()) - 1;
    return q < 0 ? 0 : q;
  };
  std::vector<std::vector<size_t>> to((size_t)P);
  for (size_t k = 0; k < v->st_idx.size(); ++k) to[(size_t)owner(v->st_idx[k])].push_back(k);
  double mx = 0.0;
  for (const auto& t : to) mx = std::max(mx, (double)t.size());
  PetscCall(PetscMiniAllreduce(v->comm, &mx, 1, PETSCMINI_OP_MAX));
  const size_t M = (size_t)mx;
  if (M) {
    std::vector<double> send((size_t)P * M * 4, -1.0), recv((size_t)P * M * 4);
    for (int q = 0; q < P; ++q)
      for (size_t j = 0; j < to[(size_t)q].size(); ++j) {
        const size_t k = to[(size_t)q][j];
        double* rec = &send[((size_t)q * M + j) * 4];
        rec[0] = (double)v->st_idx[k];  // exact: rows < 2^53
        rec[1] = C(v->st_val[k]).real();
        rec[2] = C(v->st_val[k]).imag();
        rec[3] = v->st_add[k] ? 1.0 : 0.0;
      }
    PetscCall(comm_alltoall_host(r, send.data(), recv.data(), M * 4 * sizeof(double)));
    VS* h;
    PetscCall(host_rw(v, &h));
    for (size_t e = 0; e < (size_t)P * M; ++e) {
      const double* rec = &recv[e * 4];
      if (rec[0] < 0) continue;  // padding
      const PetscInt i = (PetscInt)rec[0] - v->rstart;
      if (i < 0 || i >= v->n) return ERR(PETSC_ERR_PLIB, "stashed entry delivered to the wrong rank");
      const std::complex<double> val(rec[1], rec[2]);
      h[i] = rec[3] != 0.0 ? D(C(h[i]) + val) : D(val);
    }
  }
  v->st_idx.clear(), v->st_val.clear(), v->st_add.clear();
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecAssemblyEnd(Vec v) { VCHK(v); return PETSC_SUCCESS; }

extern "C" PetscErrorCode VecCopy(Vec x, Vec y) {
  VCHK(x); VCHK(y);
  PetscCall(same_size(x, y));
  if (x == y) return PETSC_SUCCESS;
  touch(y);
  if (y->hip) {
    VS* yd;
    if (x->hip) {
      const VS* xd;
      PetscCall(dev_read(x, &xd));
      y->mask = MASK_GPU;
      HIPK(cfp::blas_copy_bytes(y->d, xd, sizeof(VS) * (size_t)x->n, g_stream));
    } else {
      (void)yd;
      HIPK(hipMemcpyAsync(y->d, x->h, sizeof(VS) * (size_t)x->n, hipMemcpyHostToDevice, g_stream));
      HIPK(hipStreamSynchronize(g_stream));
      y->mask = MASK_GPU;
    }
  } else {
    const VS* xh;
    PetscCall(host_read(x, &xh));
    std::memcpy(y->h, xh, sizeof(VS) * (size_t)x->n);
    y->mask = MASK_CPU;
  }
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecScale(Vec x, PetscScalar a) {
  VCHK(x);
  if (x->hip) {
    VS* xd;
    PetscCall(dev_rw(x, &xd));
    HIPK(dev_scale(xd, tocd(a), x->n, g_stream));
  } else {
    VS* h;
    PetscCall(host_rw(x, &h));
    for (PetscInt i = 0; i < x->n; ++i) {
      h[i] = D(C(h[i]) * a);
    }
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecShift(Vec x, PetscScalar a) {
  VCHK(x);
  if (x->hip) {
    VS* xd;
    PetscCall(dev_rw(x, &xd));
    HIPK(cfp::blas_shift(xd, tocd(a), x->n, g_stream));
  } else {
    VS* h;
    PetscCall(host_rw(x, &h));
    for (PetscInt i = 0; i < x->n; ++i) h[i] = D(C(h[i]) + a);
  }
  return PETSC_SUCCESS;
}

template <class DevOp, class HostOp>
static PetscErrorCode binop(Vec out, Vec a, Vec b, DevOp dop, HostOp hop) {
  VCHK(out); VCHK(a);
  if (b) { VCHK(b); PetscCall(same_size(a, b)); }
  PetscCall(same_size(out, a));
  if (all_hip({out, a}) && (!b || b->hip)) {
    const VS *ad, *bd = nullptr;
    PetscCall(dev_read(a, &ad));
    if (b) PetscCall(dev_read(b, &bd));
    VS* od;
    PetscCall(dev_rw(out, &od));
    HIPK(dop(od, ad, bd));
  } else {
    const VS *ah, *bh = nullptr;
    PetscCall(host_read(a, &ah));
    if (b) PetscCall(host_read(b, &bh));
    VS* oh;
    PetscCall(host_rw(out, &oh));
    hop(oh, ah, bh);
    if (out->hip) {
      HIPK(hipMemcpyAsync(out->d, out->h, sizeof(VS) * (size_t)out->n, hipMemcpyHostToDevice, g_stream));
      out->mask = MASK_BOTH;
    }
  }
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecAXPY(Vec y, PetscScalar a, Vec x) {  // y += a x
  const i64 n = y ? y->n : 0;
  // on the device the sweep also leaves |y|^2 partials for a following VecNorm (the time loops'
  // VecAXPY(dU, -1, U); VecNorm(dU): one sweep of dU fewer per step)
  if (y && y->magic == kVecMagic && y->hip && !y->nrm_h) {
    if (hipHostMalloc(&y->nrm_h, sizeof(double) * BLAS_NORM_PARTIALS, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&y->nrm_hd, y->nrm_h, 0) != hipSuccess) {
      if (y->nrm_h) hipHostFree(y->nrm_h);
      y->nrm_h = y->nrm_hd = nullptr;
      (void)hipGetLastError();
    }
  }
  unsigned nb = 0;
  bool dev = false;
  PetscCall(binop(y, x, nullptr,
                  [&](VS* o, const VS* xa, const VS*) {
                    dev = true;
                    if (y->nrm_hd) return cfp::blas_axpy_partials(o, tocd(a), xa, n, y->nrm_hd, &nb, g_stream);
                    return cfp::blas_axpy(o, tocd(a), xa, n, g_stream);
                  },
                  [&](VS* o, const VS* xa, const VS*) { for (i64 i = 0; i < n; ++i) o[i] = D(C(o[i]) + a * C(xa[i])); }));
  y->nrm_nb = dev ? nb : 0;
  y->nrm_state = y->state;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecAYPX(Vec y, PetscScalar b, Vec x) {  // y = x + b y
  const i64 n = y ? y->n : 0;
  return binop(y, x, nullptr,
               [&](VS* o, const VS* xa, const VS*) { return cfp::blas_aypx(o, tocd(b), xa, n, g_stream); },
               [&](VS* o, const VS* xa, const VS*) { for (i64 i = 0; i < n; ++i) o[i] = D(C(xa[i]) + b * C(o[i])); });
}
extern "C" PetscErrorCode VecWAXPY(Vec w, PetscScalar a, Vec x, Vec y) {  // w = a x + y
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](VS* o, const VS* xa, const VS* yb) { return cfp::blas_waxpy(o, tocd(a), xa, yb, n, g_stream); },
               [&](VS* o, const VS* xa, const VS* yb) { for (i64 i = 0; i < n; ++i) o[i] = D(a * C(xa[i]) + C(yb[i])); });
}
extern "C" PetscErrorCode VecPointwiseDivide(Vec w, Vec x, Vec y) {
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](VS* o, const VS* xa, const VS* yb) { return dev_pdivide(o, xa, yb, n, g_stream); },
               [&](VS* o, const VS* xa, const VS* yb) {  // PETSc: a zero divisor gives 0 (bvec2.c)
                 for (i64 i = 0; i < n; ++i) o[i] = C(yb[i]) != 0.0 ? D(C(xa[i]) / C(yb[i])) : D(0.0);
               });
}
extern "C" PetscErrorCode VecPointwiseMult(Vec w, Vec x, Vec y) {
  const i64 n = w ? w->n : 0;
  return binop(w, x, y,
               [&](VS* o, const VS* xa, const VS* yb) { return cfp::blas_pmult(o, xa, yb, n, g_stream); },
               [&](VS* o, const VS* xa, const VS* yb) { for (i64 i = 0; i < n; ++i) o[i] = D(C(xa[i]) * C(yb[i])); });
}

extern "C" PetscErrorCode VecDot(Vec x, Vec y, PetscScalar* val) {  // y^H x
  VCHK(x); VCHK(y);
  PetscCall(same_size(x, y));
  if (x->hip && y->hip) {
    const VS *xd, *yd;
    PetscCall(dev_read(x, &xd));
    PetscCall(dev_read(y, &yd));
    VS r;
    HIPK(cfp::blas_dot(xd, yd, x->n, &r, g_stream));
    *val = to_scalar(C(r).real(), C(r).imag());
  } else {
    const VS *xh, *yh;
    PetscCall(host_read(x, &xh));
    PetscCall(host_read(y, &yh));
    std::complex<double> s = 0;
    for (i64 i = 0; i < x->n; ++i) s += C(xh[i]) * std::conj(C(yh[i]));
    *val = to_scalar(s.real(), s.imag());
  }
  double buf[2] = {re_of(*val), im_of(*val)};
  PetscCall(vec_reduce(x, buf, 2, PETSCMINI_OP_SUM));
  *val = to_scalar(buf[0], buf[1]);
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode VecNorm(Vec x, NormType t, PetscReal* val) {
  VCHK(x);
  if (t == NORM_FROBENIUS) t = NORM_2;
  if (x->hip && t == NORM_2 && x->nrm_nb > 0 && x->nrm_state == x->state) {  // VecAXPY's partials
    HIPK(cfp::host_wait(g_stream));
    double s = 0.0;
    for (unsigned q = 0; q < x->nrm_nb; ++q) s += x->nrm_h[q];
    *val = std::sqrt(s);
  } else if (x->hip) {
    const VS* xd;
    PetscCall(dev_read(x, &xd));
    HIPK(cfp::blas_norm(xd, x->n, (int)t, val, g_stream));
  } else {
    const VS* h;
    PetscCall(host_read(x, &h));
    double s = 0;
    for (i64 i = 0; i < x->n; ++i) {
      const std::complex<double> v = C(h[i]);
      if (t == NORM_2) s += std::norm(v);
      else if (t == NORM_1) s += std::fabs(v.real()) + std::fabs(v.imag());
      else s = std::fmax(s, std::abs(v));
    }
    *val = t == NORM_2 ? std::sqrt(s) : s;
  }
  if (x->nranks > 1) {  // local norms -> the global one
    double v = t == NORM_2 ? (*val) * (*val) : *val;
    PetscCall(vec_reduce(x, &v, 1, t == NORM_INFINITY ? PETSCMINI_OP_MAX : PETSCMINI_OP_SUM));
    *val = t == NORM_2 ? std::sqrt(v) : v;
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
    const VS* xd;
    PetscCall(dev_read(x, &xd));
    std::vector<const VS*> ys((size_t)nv);
    for (PetscInt j = 0; j < nv; ++j) PetscCall(dev_read(y[j], &ys[(size_t)j]));
    std::vector<VS> r((size_t)nv);
    HIPK(cfp::blas_mdot(xd, (int)nv, ys.data(), x->n, r.data(), g_stream));
    PetscCall(vec_reduce(x, (double*)r.data(), kDPS * nv, PETSCMINI_OP_SUM));  // one all-reduce for all nv
    for (PetscInt j = 0; j < nv; ++j) val[j] = to_scalar(C(r[(size_t)j]).real(), C(r[(size_t)j]).imag());
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
    std::vector<const VS*> xs((size_t)nv);
    std::vector<VS> a((size_t)nv);
    for (PetscInt j = 0; j < nv; ++j) {
      PetscCall(dev_read(x[j], &xs[(size_t)j]));
      a[(size_t)j] = tocd(alpha[j]);
    }
    VS* yd;
    PetscCall(dev_rw(y, &yd));
    HIPK(cfp::blas_maxpy(yd, (int)nv, a.data(), xs.data(), y->n, g_stream));
    return PETSC_SUCCESS;
  }
  for (PetscInt j = 0; j < nv; ++j) PetscCall(VecAXPY(y, alpha[j], x[j]));
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecMiniMAXPYNorm(Vec y, PetscInt nv, const PetscScalar alpha[], Vec x[], PetscBool overwrite,
                                            PetscReal* norm) {
  VCHK(y);
  bool dev = y->hip;
  for (PetscInt j = 0; j < nv; ++j) {
    VCHK(x[j]);
    PetscCall(same_size(y, x[j]));
    dev = dev && x[j]->hip;
  }
  if (!dev) {  // host: the unfused operations
    if (overwrite) PetscCall(VecSet(y, 0.0));
    if (nv > 0) PetscCall(VecMAXPY(y, nv, alpha, x));
    if (norm) PetscCall(VecNorm(y, NORM_2, norm));
    return PETSC_SUCCESS;
  }
  std::vector<const VS*> xs((size_t)(nv > 0 ? nv : 1));
  std::vector<VS> a((size_t)(nv > 0 ? nv : 1));
  for (PetscInt j = 0; j < nv; ++j) {
    PetscCall(dev_read(x[j], &xs[(size_t)j]));
    a[(size_t)j] = tocd(alpha[j]);
  }
  VS* yd;
  if (overwrite) {  // no read of y: nothing to bring to the device first
    touch(y);
    y->mask = MASK_GPU;
    yd = y->d;
  } else {
    PetscCall(dev_rw(y, &yd));
  }
  double s2 = 0.0;
  HIPK(cfp::blas_maxpy_norm(yd, (int)nv, a.data(), xs.data(), y->n, overwrite, norm ? &s2 : nullptr, g_stream));
  if (norm) {
    PetscCall(vec_reduce(y, &s2, 1, PETSCMINI_OP_SUM));
    *norm = std::sqrt(s2);
  }
  return PETSC_SUCCESS;
}

// Classical Gram-Schmidt in one call: dots[j] = V[j]^H w, w += sum_j scale[j] dots[j] V[j],
// *norm = |w|.  Device Vecs of one rank, nv <= 32: the coefficients are formed on the device
// between the multi-dot and the MAXPY, so the step waits for the host once (cfp_blas.hip);
// otherwise VecMDot (its all-reduce on several ranks) and VecMiniMAXPYNorm.
extern "C" PetscErrorCode VecMiniMDotMAXPYNorm(Vec w, PetscInt nv, const PetscReal scale[], Vec V[],
                                               PetscScalar dots[], PetscReal* norm) {
  VCHK(w);
  if (nv <= 0) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "nv must be >= 1");
  bool dev = w->hip && w->nranks == 1 && nv <= MV_MAX;
  for (PetscInt j = 0; j < nv; ++j) {
    VCHK(V[j]);
    PetscCall(same_size(w, V[j]));
    dev = dev && V[j]->hip;
  }
  if (!dev) {
    PetscCall(VecMDot(w, nv, V, dots));
    std::vector<PetscScalar> a((size_t)nv);
    for (PetscInt j = 0; j < nv; ++j) a[(size_t)j] = scale[j] * dots[j];
    return VecMiniMAXPYNorm(w, nv, a.data(), V, PETSC_FALSE, norm);
  }
  std::vector<const VS*> ys((size_t)nv);
  for (PetscInt j = 0; j < nv; ++j) PetscCall(dev_read(V[j], &ys[(size_t)j]));
  VS* wd;
  PetscCall(dev_rw(w, &wd));
  std::vector<VS> r((size_t)nv);
  double s2 = 0.0;
  HIPK(cfp::blas_mdot_maxpy_norm(wd, (int)nv, ys.data(), scale, w->n, r.data(), &s2, g_stream));
  for (PetscInt j = 0; j < nv; ++j) dots[j] = to_scalar(C(r[(size_t)j]).real(), C(r[(size_t)j]).imag());
  if (norm) *norm = std::sqrt(s2);
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode VecMiniMAXPYNormDeviceDots(Vec w, PetscInt nv, const PetscReal scale[], Vec V[],
                                                     const double* dots_dev, PetscScalar dots[], PetscReal* norm) {
  VCHK(w);
  if (nv <= 0 || nv > MV_MAX) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "nv must be in 1..32");
  if (!dots_dev || !dots || !scale) return ERR(PETSC_ERR_ARG_NULL, "NULL argument");
#ifdef CFP_REAL_SCALAR
  return ERR(PETSC_ERR_SUP, "VecMiniMAXPYNormDeviceDots: complex scalars only");
#else
  if (!w->hip || w->nranks != 1) return ERR(PETSC_ERR_SUP, "VecMiniMAXPYNormDeviceDots: device Vecs of one rank");
  std::vector<const VS*> ys((size_t)nv);
  for (PetscInt j = 0; j < nv; ++j) {
    VCHK(V[j]);
    PetscCall(same_size(w, V[j]));
    if (!V[j]->hip) return ERR(PETSC_ERR_SUP, "VecMiniMAXPYNormDeviceDots: device Vecs only");
    PetscCall(dev_read(V[j], &ys[(size_t)j]));
  }
  VS* wd;
  PetscCall(dev_rw(w, &wd));
  std::vector<VS> r((size_t)nv);
  double s2 = 0.0;
  HIPK(cfp::blas_maxpy_dc_norm(wd, (int)nv, ys.data(), scale, dots_dev, w->n, r.data(), &s2, g_stream));
  for (PetscInt j = 0; j < nv; ++j) dots[j] = to_scalar(C(r[(size_t)j]).real(), C(r[(size_t)j]).imag());
  if (norm) *norm = std::sqrt(s2);
  return PETSC_SUCCESS;
#endif
}

extern "C" PetscErrorCode PetscMiniProfileBegin(PetscInt max_records) {
  if (max_records < 1 || max_records > (1 << 22)) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "max_records out of range");
  HCHK(cfp::kprof_begin((size_t)max_records));
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscMiniProfileEnd(double ms[4], int64_t launches[4]) {
  if (!ms || !launches) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  long long l[4];
  HCHK(cfp::kprof_end(ms, l));
  for (int k = 0; k < 4; ++k) launches[k] = l[k];
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscMiniDeviceRead(const double* dev, PetscInt n, double* host) {
  if (n <= 0) return PETSC_SUCCESS;
  if (!dev || !host) return ERR(PETSC_ERR_ARG_NULL, "NULL argument");
  HCHK(hipMemcpyAsync(host, dev, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
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
  PetscInt m = 0, n = 0;    // global sizes
  PetscInt lm = 0, ln = 0;  // local sizes
  MPI_Comm comm = PETSC_COMM_SELF;
  void* ctx = nullptr;
  MatMultFn mult = nullptr, multT = nullptr;
  MatDestroyFn destroy = nullptr;
  // AIJ (device CSR)
  i64 *rowptr = nullptr, *col = nullptr;
  VS* val = nullptr;
  std::vector<i64> h_rowptr, h_col;
  std::vector<VS> h_val;
  // AIJ in row-class diagonal form (aij_build_dia), when the matrix has one: no device CSR then
  int dia = -1;  // -1: not tried yet, 0: not representable, 1: built
  cfp::DiaDesc dia_d{};
  unsigned char *dia_cls = nullptr, *dia_mask = nullptr;
  VS* dia_tab = nullptr;
  std::vector<unsigned char> h_cls, h_mask;  // host copies of the classes (PetscMiniMatAIJGetDia)
  i64 xloc_len = -1;                         // row length of the cached x-locality test
  bool xloc = false;
  unsigned char* dia_cls_x = nullptr;        // [xloc_len] when the classes repeat with the row length
  // AIJ in block row-class form (aij_build_bdia) when the row-class form does not fit: B x B blocks
  int bdia = -1;  // -1: not tried yet, 0: not representable, 1: built
  cfp::BDiaDesc bdia_d{};
  unsigned char* bdia_cls = nullptr;
  unsigned short *bdia_mask = nullptr, *bdia_cbase = nullptr;
  unsigned* bdia_bnz = nullptr;
  VS* bdia_tab = nullptr;
  // MatCreateAIJ (r06): entries from MatSetValue(s) wait here until MatAssemblyEnd.  This rank's
  // rows [rstart, rstart + lm); set_*: its own rows' entries, st_*: other ranks' (the stash).
  bool building = false;
  int nranks = 1;
  i64 rstart = 0;
  std::vector<i64> set_r, set_c, st_r, st_c;
  std::vector<VS> set_v, st_v;
  std::vector<char> set_add, st_add;
  // MATMPIAIJ after assembly: the diagonal block (local rows x local columns, a MATSEQAIJ with
  // local indices) and the off-diagonal block over the ghost slots q hM + j (the j-th column this
  // rank needs from rank q); send_idx[q hM + j] = the local row rank q needs from this rank (-1:
  // padding).  hM = the largest per-peer halo of any rank (0: no exchange at all).
  Mat dblk = nullptr;
  std::vector<i64> o_rowptr, o_col;
  std::vector<VS> o_val;
  i64 nghost = 0, hM = 0;
  std::vector<i64> send_idx;
  i64 *d_orowptr = nullptr, *d_ocol = nullptr, *d_send_idx = nullptr;
  VS *d_oval = nullptr, *d_sendbuf = nullptr, *d_recvbuf = nullptr;
  std::vector<VS> h_sendbuf, h_recvbuf;
};

static PetscErrorCode mcheck(Mat A, const char* f) {
  if (!A || A->magic != kMatMagic) return PetscErrorSet(PETSC_ERR_ARG_NULL, f, "invalid Mat");
  return PETSC_SUCCESS;
}
#define MCHK(A) PetscCall(mcheck((A), __func__))

extern "C" PetscErrorCode MatCreateShell(MPI_Comm comm, PetscInt m, PetscInt n, PetscInt M, PetscInt N, void* ctx, Mat* A) {
  if (!A) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  Mat a = new _p_Mat;
  a->type = MATSHELL;
  a->m = M >= 0 ? M : m;
  a->n = N >= 0 ? N : n;
  a->lm = m >= 0 ? m : a->m;
  a->ln = n >= 0 ? n : a->n;
  a->comm = comm_resolve(comm);
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
  M->m = M->lm = m;
  M->n = M->ln = n;
  const i64 nnz = i[m];
  M->h_rowptr.assign(i, i + m + 1);
  M->h_col.assign(j, j + nnz);
  M->h_val.resize((size_t)nnz);
  for (i64 k = 0; k < nnz; ++k) M->h_val[k] = tocd(a[k]);
  *A = M;  // the device copy is made by the first MatMult on HIP vectors
  return PETSC_SUCCESS;
}
// Row-class diagonal form of the host CSR (cfp_blas.h, k_dia_spmv): every nonzero on one of at
// most DIA_MAX diagonals (column - row), each row's entries on distinct diagonals, at most 256
// distinct rows.  A constant-coefficient stencil on a Cartesian grid (the transport operator,
// transport_cartesian.cpp: the interior row plus the border rows) qualifies; a mesh remap or the
// interleaved wave operator does not, and keeps the CSR kernels.
static bool aij_build_dia(Mat M, cfp::DiaDesc* d, std::vector<unsigned char>* cls, std::vector<unsigned char>* masks,
                          std::vector<VS>* tab) {
  const i64 m = M->m;
  if (m <= 0 || M->h_col.empty()) return false;
  std::vector<i64> offs;
  for (i64 r = 0; r < m; ++r)
    for (i64 p = M->h_rowptr[r]; p < M->h_rowptr[r + 1]; ++p) {
      const i64 o = M->h_col[p] - r;
      if (std::find(offs.begin(), offs.end(), o) == offs.end()) {
        if ((int)offs.size() == DIA_MAX) return false;
        offs.push_back(o);
      }
    }
  std::sort(offs.begin(), offs.end());
  const int nd = (int)offs.size();
  cls->assign((size_t)m, 0);
  masks->clear();
  tab->clear();
  std::vector<VS> row((size_t)nd);
  int last = -1;
  for (i64 r = 0; r < m; ++r) {
    unsigned mk = 0;
    for (int k = 0; k < nd; ++k) row[(size_t)k] = D(std::complex<double>(0.0, 0.0));
    for (i64 p = M->h_rowptr[r]; p < M->h_rowptr[r + 1]; ++p) {
      const int k = (int)(std::lower_bound(offs.begin(), offs.end(), M->h_col[p] - r) - offs.begin());
      if (mk & (1u << k)) return false;  // two entries on one diagonal (duplicate column)
      mk |= 1u << k;
      row[(size_t)k] = M->h_val[(size_t)p];
    }
    const auto same = [&](int c) {
      if ((*masks)[(size_t)c] != mk) return false;
      return std::memcmp(&(*tab)[(size_t)c * nd], row.data(), sizeof(VS) * (size_t)nd) == 0;
    };
    int c = (last >= 0 && same(last)) ? last : -1;  // consecutive rows mostly share a class
    for (int q = 0; c < 0 && q < (int)masks->size(); ++q)
      if (same(q)) c = q;
    if (c < 0) {
      if (masks->size() == 256) return false;
      c = (int)masks->size();
      masks->push_back((unsigned char)mk);
      tab->insert(tab->end(), row.begin(), row.end());
    }
    (*cls)[(size_t)r] = (unsigned char)c;
    last = c;
  }
  for (int k = 0; k < nd; ++k) d->off[k] = offs[(size_t)k];
  d->nd = nd;
  d->ncls = (int)masks->size();
  return true;
}

// Block row-class form of the host CSR (cfp_blas.h, k_bdia_spmv), tried when the row-class form
// does not fit: the matrix cut into B x B blocks (B = 2, 3, 4), every nonzero block on one of at
// most BDIA_MAX block diagonals (a 3-D periodic stencil has 13), at most 256 distinct block
// rows, their present blocks within the LDS budget.  The interleaved wave operator
// (wave_system.cpp: d + 1 unknowns per cell, a 2d + 1 cell stencil) qualifies with B = d + 1.  Among the block sizes that fit, the one with the fewest
// multiply-adds per row (nd B) wins; the product is the same up to summation order.
static bool aij_build_bdia_b(Mat M, int B, cfp::BDiaDesc* d, std::vector<unsigned char>* cls,
                             std::vector<unsigned short>* masks, std::vector<unsigned short>* cbase,
                             std::vector<unsigned>* bnz, std::vector<VS>* tab) {
  const i64 m = M->m;
  if (m <= 0 || m % B || M->n != m || M->h_col.empty()) return false;
  const i64 mb = m / B;
  std::vector<i64> offs;
  for (i64 r = 0; r < m; ++r)
    for (i64 p = M->h_rowptr[r]; p < M->h_rowptr[r + 1]; ++p) {
      const i64 o = M->h_col[p] / B - r / B;
      if (std::find(offs.begin(), offs.end(), o) == offs.end()) {
        if ((int)offs.size() == BDIA_MAX) return false;
        offs.push_back(o);
      }
    }
  std::sort(offs.begin(), offs.end());
  const int nd = (int)offs.size(), bs = nd * B * B;
  const size_t per_cls = sizeof(VS) * (size_t)bs;
  const size_t blk_bytes = sizeof(VS) * (size_t)(B * B);
  cls->assign((size_t)mb, 0);
  masks->clear();
  std::vector<VS> dense;  // classes' rows, dense over all nd diagonals (for the comparison)
  std::vector<VS> row((size_t)bs);
  std::unordered_map<uint64_t, std::vector<int>> seen;  // hash of (mask, values) -> classes
  size_t nblk = 0;
  int last = -1;
  for (i64 R = 0; R < mb; ++R) {
    unsigned mk = 0;
    for (int q = 0; q < bs; ++q) row[(size_t)q] = D(std::complex<double>(0.0, 0.0));
    for (int i = 0; i < B; ++i) {
      const i64 r = R * B + i;
      for (i64 p = M->h_rowptr[r]; p < M->h_rowptr[r + 1]; ++p) {
        const i64 c = M->h_col[p];
        const int k = (int)(std::lower_bound(offs.begin(), offs.end(), c / B - R) - offs.begin());
        mk |= 1u << k;
        VS& v = row[(size_t)((k * B + i) * B + (int)(c % B))];
        v = D(C(v) + C(M->h_val[(size_t)p]));  // duplicates add, as the CSR product does
      }
    }
    const auto same = [&](int c) {
      return (*masks)[(size_t)c] == mk && std::memcmp(&dense[(size_t)c * bs], row.data(), per_cls) == 0;
    };
    int c = (last >= 0 && same(last)) ? last : -1;  // consecutive cells mostly share a class
    uint64_t h = 1469598103934665603ull ^ mk;
    if (c < 0) {
      const unsigned char* b = reinterpret_cast<const unsigned char*>(row.data());
      for (size_t q = 0; q < per_cls; ++q) h = (h ^ b[q]) * 1099511628211ull;
      for (int q : seen[h])
        if (same(q)) {
          c = q;
          break;
        }
    }
    if (c < 0) {
      nblk += (size_t)__builtin_popcount(mk);
      if (masks->size() == 256 || nblk * blk_bytes > BDIA_LDS_MAX) return false;
      c = (int)masks->size();
      masks->push_back((unsigned short)mk);
      dense.insert(dense.end(), row.begin(), row.end());
      seen[h].push_back(c);
    }
    (*cls)[(size_t)R] = (unsigned char)c;
    last = c;
  }
  // the table: each class's present blocks in ascending k, with their nonzero and column masks
  cbase->clear();
  bnz->clear();
  tab->clear();
  const VS zero = D(std::complex<double>(0.0, 0.0));
  for (size_t c = 0; c < masks->size(); ++c) {
    cbase->push_back((unsigned short)(tab->size() / (size_t)(B * B)));
    for (int k = 0; k < nd; ++k)
      if (((*masks)[c] >> k) & 1u) {
        const VS* b0 = &dense[c * (size_t)bs + (size_t)k * B * B];
        unsigned nz = 0;
        for (int e = 0; e < B * B; ++e)
          if (std::memcmp(&b0[e], &zero, sizeof(VS)) != 0) nz |= (1u << e) | (1u << (16 + e % B));
        bnz->push_back(nz);
        tab->insert(tab->end(), b0, b0 + B * B);
      }
  }
  for (int k = 0; k < nd; ++k) d->off[k] = offs[(size_t)k];
  d->nd = nd;
  d->ncls = (int)masks->size();
  d->B = B;
  d->nblk = (int)(tab->size() / (size_t)(B * B));
  d->re = 1;
  for (const VS& v : *tab)
    if (C(v).imag() != 0.0) d->re = 0;
  return true;
}
static bool aij_build_bdia(Mat M, cfp::BDiaDesc* d, std::vector<unsigned char>* cls, std::vector<unsigned short>* masks,
                           std::vector<unsigned short>* cbase, std::vector<unsigned>* bnz, std::vector<VS>* tab) {
  bool any = false;
  for (int B = 4; B >= 2; --B) {
    cfp::BDiaDesc dd{};
    std::vector<unsigned char> cc;
    std::vector<unsigned short> mm, bb;
    std::vector<unsigned> zz;
    std::vector<VS> tt;
    if (!aij_build_bdia_b(M, B, &dd, &cc, &mm, &bb, &zz, &tt)) continue;
    if (!any || dd.nd * dd.B < d->nd * d->B) {
      *d = dd;
      cls->swap(cc);
      masks->swap(mm);
      cbase->swap(bb);
      bnz->swap(zz);
      tab->swap(tt);
      any = true;
    }
  }
  return any;
}

static void aij_free_device(Mat M) {
  if (M->rowptr) hipFree(M->rowptr);
  if (M->col) hipFree(M->col);
  if (M->val) hipFree(M->val);
  if (M->dia_cls) hipFree(M->dia_cls);
  if (M->dia_mask) hipFree(M->dia_mask);
  if (M->dia_tab) hipFree(M->dia_tab);
  if (M->dia_cls_x) hipFree(M->dia_cls_x);
  if (M->bdia_cls) hipFree(M->bdia_cls);
  if (M->bdia_mask) hipFree(M->bdia_mask);
  if (M->bdia_tab) hipFree(M->bdia_tab);
  if (M->bdia_cbase) hipFree(M->bdia_cbase);
  if (M->bdia_bnz) hipFree(M->bdia_bnz);
  M->bdia_bnz = nullptr;
  M->bdia_cls = nullptr;
  M->bdia_mask = M->bdia_cbase = nullptr;
  M->bdia_tab = nullptr;
  M->bdia = -1;
  M->dia_cls_x = nullptr;
  M->rowptr = M->col = nullptr;
  M->val = M->dia_tab = nullptr;
  M->dia_cls = M->dia_mask = nullptr;
  M->dia = -1;
  M->h_cls.clear();
  M->h_mask.clear();
  M->xloc_len = -1;
}

// the device copy: the row-class diagonal form when the matrix has one, else the CSR (once;
// MatShift rebuilds it)
static PetscErrorCode aij_upload(Mat M) {
  if (M->rowptr || M->dia == 1 || M->bdia == 1) return PETSC_SUCCESS;
  if (M->dia < 0) {
    std::vector<unsigned char> cls, masks;
    std::vector<VS> tab;
    cfp::DiaDesc d{};
    M->dia = aij_build_dia(M, &d, &cls, &masks, &tab) ? 1 : 0;
    if (M->dia == 1) {
      hipError_t e = hipMalloc(&M->dia_cls, cls.size());
      if (e == hipSuccess) e = hipMalloc(&M->dia_mask, masks.size());
      if (e == hipSuccess) e = hipMalloc(&M->dia_tab, sizeof(VS) * tab.size());
      if (e == hipSuccess) e = hipMemcpy(M->dia_cls, cls.data(), cls.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(M->dia_mask, masks.data(), masks.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(M->dia_tab, tab.data(), sizeof(VS) * tab.size(), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        aij_free_device(M);
        return ERR(PETSC_ERR_MEM, hipGetErrorString(e));
      }
      M->dia_d = d;
      M->h_cls.swap(cls);
      M->h_mask.swap(masks);
      M->xloc_len = -1;
      return PETSC_SUCCESS;
    }
  }
  if (M->bdia < 0) {
    std::vector<unsigned char> cls;
    std::vector<unsigned short> masks, cbase;
    std::vector<unsigned> bnz;
    std::vector<VS> tab;
    cfp::BDiaDesc d{};
    M->bdia = aij_build_bdia(M, &d, &cls, &masks, &cbase, &bnz, &tab) ? 1 : 0;
    if (M->bdia == 1) {
      const size_t mb = sizeof(unsigned short) * masks.size();
      hipError_t e = hipMalloc(&M->bdia_cls, cls.size());
      if (e == hipSuccess) e = hipMalloc(&M->bdia_mask, mb);
      if (e == hipSuccess) e = hipMalloc(&M->bdia_cbase, mb);
      if (e == hipSuccess) e = hipMalloc(&M->bdia_bnz, sizeof(unsigned) * bnz.size());
      if (e == hipSuccess)
        e = hipMemcpy(M->bdia_bnz, bnz.data(), sizeof(unsigned) * bnz.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMalloc(&M->bdia_tab, sizeof(VS) * tab.size());
      if (e == hipSuccess) e = hipMemcpy(M->bdia_cls, cls.data(), cls.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(M->bdia_mask, masks.data(), mb, hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(M->bdia_cbase, cbase.data(), mb, hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(M->bdia_tab, tab.data(), sizeof(VS) * tab.size(), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        aij_free_device(M);
        return ERR(PETSC_ERR_MEM, hipGetErrorString(e));
      }
      M->bdia_d = d;
      return PETSC_SUCCESS;
    }
  }
  const size_t nnz = M->h_col.size();
  hipError_t e = hipMalloc(&M->rowptr, sizeof(i64) * (size_t)(M->m + 1));
  if (e == hipSuccess) e = hipMalloc(&M->col, sizeof(i64) * (nnz > 0 ? nnz : 1));
  if (e == hipSuccess) e = hipMalloc(&M->val, sizeof(VS) * (nnz > 0 ? nnz : 1));
  if (e == hipSuccess) e = hipMemcpy(M->rowptr, M->h_rowptr.data(), sizeof(i64) * (size_t)(M->m + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess && nnz) e = hipMemcpy(M->col, M->h_col.data(), sizeof(i64) * nnz, hipMemcpyHostToDevice);
  if (e == hipSuccess && nnz) e = hipMemcpy(M->val, M->h_val.data(), sizeof(VS) * nnz, hipMemcpyHostToDevice);
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
extern "C" PetscErrorCode PetscMiniMatAIJGetFormat(Mat A, int* format) {
  MCHK(A);
  if (!format) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  if (A->type != MATSEQAIJ) return ERR(PETSC_ERR_ARG_WRONG, "not a MATSEQAIJ");
  *format = A->dia == 1 ? 1 : A->bdia == 1 ? 2 : (A->rowptr ? 0 : -1);
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscMiniMatAIJGetDia(Mat A, PetscInt rowlen, PetscBool* has, PetscBool* x_local,
                                                 PetscMiniDia* dia) {
  MCHK(A);
  if (!has || !x_local || !dia) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  if (rowlen < 1) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "rowlen must be >= 1");
  *has = PETSC_FALSE;
  *x_local = PETSC_FALSE;
  if (A->type != MATSEQAIJ) return PETSC_SUCCESS;
  PetscCall(aij_upload(A));
  if (A->dia != 1) return PETSC_SUCCESS;
  if (A->xloc_len != rowlen) {  // every present entry's column in its row's run of rowlen indices
    // per class the lowest and highest offset present, then one pass over the rows' positions
    const int nc = A->dia_d.ncls;
    std::vector<i64> lo((size_t)nc, 0), hi((size_t)nc, 0);
    for (int c = 0; c < nc; ++c)
      for (int k = 0; k < A->dia_d.nd; ++k)
        if ((A->h_mask[(size_t)c] >> k) & 1u) {
          lo[(size_t)c] = std::min(lo[(size_t)c], A->dia_d.off[k]);
          hi[(size_t)c] = std::max(hi[(size_t)c], A->dia_d.off[k]);
        }
    bool ok = A->m % rowlen == 0 && A->m == A->n;
    const unsigned char* cl = A->h_cls.data();
    for (i64 r0 = 0; ok && r0 < A->m; r0 += rowlen)
      for (i64 q = 0; q < rowlen; ++q) {
        const int c = cl[r0 + q];
        if (q + lo[(size_t)c] < 0 || q + hi[(size_t)c] >= rowlen) { ok = false; break; }
      }
    A->xloc = ok;
    A->xloc_len = rowlen;
    // classes set by the position in the row alone: keep the first row's on the device
    bool per = A->m % rowlen == 0;
    for (i64 r = rowlen; per && r < A->m; ++r) per = cl[r] == cl[r % rowlen];
    if (A->dia_cls_x) hipFree(A->dia_cls_x);
    A->dia_cls_x = nullptr;
    if (per && (hipMalloc(&A->dia_cls_x, (size_t)rowlen) != hipSuccess ||
                hipMemcpy(A->dia_cls_x, cl, (size_t)rowlen, hipMemcpyHostToDevice) != hipSuccess)) {
      if (A->dia_cls_x) hipFree(A->dia_cls_x);
      A->dia_cls_x = nullptr;
      A->xloc_len = -1;
      return ERR(PETSC_ERR_MEM, "row-class table");
    }
  }
  *has = PETSC_TRUE;
  *x_local = A->xloc ? PETSC_TRUE : PETSC_FALSE;
  dia->cls = A->dia_cls;
  dia->mask = A->dia_mask;
  dia->tab = (const PetscScalar*)A->dia_tab;
  for (int k = 0; k < 8; ++k) dia->off[k] = k < A->dia_d.nd ? A->dia_d.off[k] : 0;
  dia->nd = A->dia_d.nd;
  dia->ncls = A->dia_d.ncls;
  dia->cls_x = A->dia_cls_x;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetType(Mat A, MatType* t) {
  MCHK(A);
  *t = A->type == MATSEQAIJ ? MATSEQAIJ : (A->type == MATMPIAIJ ? MATMPIAIJ : MATSHELL);
  return PETSC_SUCCESS;
}

// ------------------------------------------------------------------ MatCreateAIJ
extern "C" PetscErrorCode MatCreateAIJ(MPI_Comm comm, PetscInt m, PetscInt n, PetscInt M, PetscInt N, PetscInt,
                                       const PetscInt[], PetscInt, const PetscInt[], Mat* A) {
  if (!A) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  comm = comm_resolve(comm);
  PetscInt lm, gm, rs, ln, gn, cs;
  PetscCall(mpi_layout(comm, m, M, &lm, &gm, &rs));
  PetscCall(mpi_layout(comm, n, N, &ln, &gn, &cs));
  Mat a = new _p_Mat;
  MPI_Comm_size(comm, &a->nranks);
  a->type = a->nranks > 1 ? MATMPIAIJ : MATSEQAIJ;
  a->m = gm;
  a->n = gn;
  a->lm = lm;
  a->ln = ln;
  a->rstart = rs;
  a->comm = comm;
  a->building = true;
  if (a->nranks > 1 && (gm != gn || rs != cs)) {
    delete a;
    return ERR(PETSC_ERR_SUP, "the stand-in MPIAIJ needs a square matrix with the same row and column layout");
  }
  *A = a;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatSetValues(Mat A, PetscInt m, const PetscInt idxm[], PetscInt n, const PetscInt idxn[],
                                       const PetscScalar v[], InsertMode mode) {
  MCHK(A);
  if (!A->building) return ERR(PETSC_ERR_ARG_WRONGSTATE, "MatSetValues: only on a MatCreateAIJ matrix before MatAssemblyEnd");
  for (PetscInt a = 0; a < m; ++a) {
    const PetscInt i = idxm[a];
    if (i < 0) continue;
    if (i >= A->m) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "MatSetValues: row out of range");
    const bool mine = i >= A->rstart && i < A->rstart + A->lm;
    for (PetscInt b = 0; b < n; ++b) {
      const PetscInt j = idxn[b];
      if (j < 0) continue;
      if (j >= A->n) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "MatSetValues: column out of range");
      auto& R = mine ? A->set_r : A->st_r;
      if (R.size() >= ((size_t)1 << 28)) return ERR(PETSC_ERR_MEM, "MatSetValues: 2^28 entries pending");
      R.push_back(i);
      (mine ? A->set_c : A->st_c).push_back(j);
      (mine ? A->set_v : A->st_v).push_back(tocd(v[a * n + b]));
      (mine ? A->set_add : A->st_add).push_back(mode == ADD_VALUES);
    }
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatSetValue(Mat A, PetscInt i, PetscInt j, PetscScalar v, InsertMode mode) {
  return MatSetValues(A, 1, &i, 1, &j, &v, mode);
}
extern "C" PetscErrorCode MatGetOwnershipRange(Mat A, PetscInt* lo, PetscInt* hi) {
  MCHK(A);
  const PetscInt rs = A->type == MATMPIAIJ || A->building ? A->rstart : 0;
  if (lo) *lo = rs;
  if (hi) *hi = rs + A->lm;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PetscMiniMatMPIAIJGetHalo(Mat A, PetscInt* ghosts, PetscInt* max_per_peer) {
  MCHK(A);
  if (ghosts) *ghosts = A->type == MATMPIAIJ ? A->nghost : 0;
  if (max_per_peer) *max_per_peer = A->type == MATMPIAIJ ? A->hM : 0;
  return PETSC_SUCCESS;
}
// Collective, as PETSc's: the stash travels to the row owners (records [row, col, re, im, add]
// through one all-to-all, padded to the largest per-peer count); then End builds the matrix.
extern "C" PetscErrorCode MatAssemblyBegin(Mat A, MatAssemblyType) {
  MCHK(A);
  if (!A->building) return PETSC_SUCCESS;  // already assembled (PETSc allows re-assembly)
  if (A->nranks == 1) {
    if (!A->st_r.empty()) return ERR(PETSC_ERR_PLIB, "stashed rows on one rank");
    return PETSC_SUCCESS;
  }
  CommRec* r = comm_rec(A->comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  const int P = r->size;
  std::vector<double> starts((size_t)P, 0.0);
  starts[(size_t)r->rank] = (double)A->rstart;
  PetscCall(PetscMiniAllreduce(A->comm, starts.data(), P, PETSCMINI_OP_SUM));
  const auto owner = [&](PetscInt g) {
    int q = (int)(std::upper_bound(starts.begin(), starts.end(), (double)g) - starts.begin()) - 1;
    return q < 0 ? 0 : q;
  };
  std::vector<std::vector<size_t>> to((size_t)P);
  for (size_t k = 0; k < A->st_r.size(); ++k) to[(size_t)owner(A->st_r[k])].push_back(k);
  double mx = 0.0;
  for (const auto& t : to) mx = std::max(mx, (double)t.size());
  PetscCall(PetscMiniAllreduce(A->comm, &mx, 1, PETSCMINI_OP_MAX));
  const size_t Mx = (size_t)mx;
  if (Mx) {
    std::vector<double> send((size_t)P * Mx * 5, -1.0), recv((size_t)P * Mx * 5);
    for (int q = 0; q < P; ++q)
      for (size_t j = 0; j < to[(size_t)q].size(); ++j) {
        const size_t k = to[(size_t)q][j];
        double* rec = &send[((size_t)q * Mx + j) * 5];
        rec[0] = (double)A->st_r[k];  // exact: indices < 2^53
        rec[1] = (double)A->st_c[k];
        rec[2] = C(A->st_v[k]).real();
        rec[3] = C(A->st_v[k]).imag();
        rec[4] = A->st_add[k] ? 1.0 : 0.0;
      }
    PetscCall(comm_alltoall_host(r, send.data(), recv.data(), Mx * 5 * sizeof(double)));
    for (size_t e = 0; e < (size_t)P * Mx; ++e) {
      const double* rec = &recv[e * 5];
      if (rec[0] < 0) continue;  // padding
      const i64 row = (i64)rec[0];
      if (row < A->rstart || row >= A->rstart + A->lm) return ERR(PETSC_ERR_PLIB, "stashed entry delivered to the wrong rank");
      A->set_r.push_back(row);
      A->set_c.push_back((i64)rec[1]);
      A->set_v.push_back(D(std::complex<double>(rec[2], rec[3])));
      A->set_add.push_back(rec[4] != 0.0);
    }
  }
  A->st_r.clear(), A->st_c.clear(), A->st_v.clear(), A->st_add.clear();
  return PETSC_SUCCESS;
}

static void mpiaij_free(Mat A) {
  if (A->dblk) MatDestroy(&A->dblk);
  hipFree(A->d_orowptr);
  hipFree(A->d_ocol);
  hipFree(A->d_oval);
  hipFree(A->d_send_idx);
  hipFree(A->d_sendbuf);
  hipFree(A->d_recvbuf);
  A->d_orowptr = A->d_ocol = A->d_send_idx = nullptr;
  A->d_oval = A->d_sendbuf = A->d_recvbuf = nullptr;
}

// the pending entries of the local rows, folded in order (INSERT sets, ADD adds), as CSR with
// global columns; square matrices get their diagonal stored (MatShift needs it)
static void fold_rows(Mat A, std::vector<i64>* rowptr, std::vector<i64>* col, std::vector<VS>* val) {
  const size_t ne = A->set_r.size();
  std::vector<size_t> ord(ne);
  for (size_t k = 0; k < ne; ++k) ord[k] = k;
  std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
    return A->set_r[a] != A->set_r[b] ? A->set_r[a] < A->set_r[b] : A->set_c[a] < A->set_c[b];
  });
  rowptr->assign((size_t)A->lm + 1, 0);
  col->clear();
  val->clear();
  const bool square = A->m == A->n;
  size_t k = 0;
  for (i64 lr = 0; lr < A->lm; ++lr) {
    const i64 row = A->rstart + lr;
    bool diag = false;
    while (k < ne && A->set_r[ord[k]] == row) {
      const i64 c = A->set_c[ord[k]];
      if (square && !diag && c > row) {  // the diagonal, absent so far: a stored zero
        col->push_back(row);
        val->push_back(D(std::complex<double>(0.0, 0.0)));
        diag = true;
      }
      std::complex<double> acc = 0.0;
      for (; k < ne && A->set_r[ord[k]] == row && A->set_c[ord[k]] == c; ++k)
        acc = A->set_add[ord[k]] ? acc + C(A->set_v[ord[k]]) : C(A->set_v[ord[k]]);
      col->push_back(c);
      val->push_back(D(acc));
      diag = diag || c == row;
    }
    if (square && !diag) {
      col->push_back(row);
      val->push_back(D(std::complex<double>(0.0, 0.0)));
    }
    (*rowptr)[(size_t)lr + 1] = (i64)col->size();
  }
  A->set_r.clear(), A->set_c.clear(), A->set_v.clear(), A->set_add.clear();
  A->set_r.shrink_to_fit(), A->set_c.shrink_to_fit(), A->set_v.shrink_to_fit(), A->set_add.shrink_to_fit();
}

extern "C" PetscErrorCode MatAssemblyEnd(Mat A, MatAssemblyType type) {
  MCHK(A);
  if (!A->building || type == MAT_FLUSH_ASSEMBLY) return PETSC_SUCCESS;
  std::vector<i64> rp, cl;
  std::vector<VS> vl;
  fold_rows(A, &rp, &cl, &vl);
  A->building = false;
  if (A->nranks == 1) {  // MATSEQAIJ: the CSR is the matrix
    A->h_rowptr.swap(rp);
    A->h_col.swap(cl);
    A->h_val.swap(vl);
    return PETSC_SUCCESS;
  }
  CommRec* r = comm_rec(A->comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  const int P = r->size;
  // split: own columns -> the diagonal block (local indices), others -> ghosts
  const i64 c0 = A->rstart, c1 = A->rstart + A->ln;
  std::vector<i64> drp((size_t)A->lm + 1, 0), dcl, orp((size_t)A->lm + 1, 0), ocl_g;
  std::vector<VS> dvl, ovl;
  for (i64 lr = 0; lr < A->lm; ++lr) {
    for (i64 p = rp[(size_t)lr]; p < rp[(size_t)lr + 1]; ++p) {
      const i64 c = cl[(size_t)p];
      if (c >= c0 && c < c1) {
        dcl.push_back(c - c0);
        dvl.push_back(vl[(size_t)p]);
      } else {
        ocl_g.push_back(c);
        ovl.push_back(vl[(size_t)p]);
      }
    }
    drp[(size_t)lr + 1] = (i64)dcl.size();
    orp[(size_t)lr + 1] = (i64)ocl_g.size();
  }
  // ghosts grouped by owner (the column layout equals the row layout)
  std::vector<double> starts((size_t)P, 0.0);
  starts[(size_t)r->rank] = (double)A->rstart;
  PetscCall(PetscMiniAllreduce(A->comm, starts.data(), P, PETSCMINI_OP_SUM));
  const auto owner = [&](i64 g) {
    int q = (int)(std::upper_bound(starts.begin(), starts.end(), (double)g) - starts.begin()) - 1;
    return q < 0 ? 0 : q;
  };
  std::vector<i64> gh(ocl_g);
  std::sort(gh.begin(), gh.end());
  gh.erase(std::unique(gh.begin(), gh.end()), gh.end());
  std::vector<std::vector<i64>> need((size_t)P);
  for (i64 g : gh) need[(size_t)owner(g)].push_back(g);
  double mx = 0.0;
  for (const auto& t : need) mx = std::max(mx, (double)t.size());
  PetscCall(PetscMiniAllreduce(A->comm, &mx, 1, PETSCMINI_OP_MAX));
  const i64 hM = (i64)mx;
  A->nghost = (i64)gh.size();
  A->hM = hM;
  // each owner learns which of its rows every peer needs (one all-to-all of the requests)
  A->send_idx.assign((size_t)P * (size_t)hM, -1);
  if (hM) {
    std::vector<double> rq((size_t)P * hM, -1.0), got((size_t)P * hM);
    for (int q = 0; q < P; ++q)
      for (size_t j = 0; j < need[(size_t)q].size(); ++j) rq[(size_t)q * hM + j] = (double)need[(size_t)q][j];
    PetscCall(comm_alltoall_host(r, rq.data(), got.data(), (size_t)hM * sizeof(double)));
    for (size_t e = 0; e < got.size(); ++e)
      if (got[e] >= 0) {
        const i64 g = (i64)got[e];
        if (g < c0 || g >= c1) return ERR(PETSC_ERR_PLIB, "halo request for a row this rank does not own");
        A->send_idx[e] = g - c0;
      }
  }
  // off-block columns -> ghost slots q hM + j
  std::vector<i64> ocl(ocl_g.size());
  for (size_t p = 0; p < ocl_g.size(); ++p) {
    const i64 g = ocl_g[p];
    const int q = owner(g);
    const auto& nq = need[(size_t)q];
    ocl[p] = (i64)q * hM + (i64)(std::lower_bound(nq.begin(), nq.end(), g) - nq.begin());
  }
  A->o_rowptr.swap(orp);
  A->o_col.swap(ocl);
  A->o_val.swap(ovl);
  mpiaij_free(A);
  PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, A->lm, A->ln, reinterpret_cast<PetscInt*>(drp.data()),
                                      reinterpret_cast<PetscInt*>(dcl.data()),
                                      reinterpret_cast<PetscScalar*>(dvl.data()), &A->dblk));
  return PETSC_SUCCESS;
}

// y = A x on several ranks: the halo (gather the rows peers need, one all-to-all), the diagonal
// block's SpMV into y, then y += the off-diagonal block on the ghosts
// y = B x on the device in the form aij_upload chose
static PetscErrorCode aij_spmv_dev(Mat B, const VS* xd, VS* yd) {
  if (B->dia == 1)
    HIPK(cfp::blas_dia_spmv(B->m, B->dia_d, B->dia_cls, B->dia_mask, B->dia_tab, xd, yd, g_stream));
  else if (B->bdia == 1)
    HIPK(cfp::blas_bdia_spmv(B->m / B->bdia_d.B, B->bdia_d, B->bdia_cls, B->bdia_mask, B->bdia_cbase, B->bdia_bnz,
                             B->bdia_tab, xd, yd, g_stream));
  else
    HIPK(cfp::blas_csr_spmv(B->m, (i64)B->h_col.size(), B->rowptr, B->col, B->val, xd, yd, g_stream));
  return PETSC_SUCCESS;
}

static PetscErrorCode mpiaij_mult(Mat A, Vec x, Vec y) {
  if (x->n != A->ln || y->n != A->lm || x->N != A->n || y->N != A->m) return ERR(PETSC_ERR_ARG_SIZ, "MatMult sizes");
  if (x == y) return ERR(PETSC_ERR_ARG_IDN, "x and y must be different vectors");
  if (x->rstart != A->rstart || y->rstart != A->rstart) return ERR(PETSC_ERR_ARG_WRONG, "MatMult: Vec layout differs from the matrix");
  CommRec* r = comm_rec(A->comm);
  if (!r) return ERR(PETSC_ERR_ARG_WRONG, "unknown communicator");
  const int P = r->size;
  const size_t hl = (size_t)P * (size_t)A->hM;
  const bool dev = x->hip && y->hip;
  if (dev) {
    const VS* xd;
    PetscCall(dev_read(x, &xd));
    VS* yd;
    PetscCall(dev_rw(y, &yd));
    if (hl) {
      if (!A->d_send_idx) {
        HCHK(hipMalloc(&A->d_send_idx, sizeof(i64) * hl));
        HCHK(hipMalloc(&A->d_sendbuf, sizeof(VS) * hl));
        HCHK(hipMalloc(&A->d_recvbuf, sizeof(VS) * hl));
        HCHK(hipMemcpy(A->d_send_idx, A->send_idx.data(), sizeof(i64) * hl, hipMemcpyHostToDevice));
        const size_t no = A->o_col.size();
        HCHK(hipMalloc(&A->d_orowptr, sizeof(i64) * A->o_rowptr.size()));
        HCHK(hipMalloc(&A->d_ocol, sizeof(i64) * (no ? no : 1)));
        HCHK(hipMalloc(&A->d_oval, sizeof(VS) * (no ? no : 1)));
        HCHK(hipMemcpy(A->d_orowptr, A->o_rowptr.data(), sizeof(i64) * A->o_rowptr.size(), hipMemcpyHostToDevice));
        if (no) HCHK(hipMemcpy(A->d_ocol, A->o_col.data(), sizeof(i64) * no, hipMemcpyHostToDevice));
        if (no) HCHK(hipMemcpy(A->d_oval, A->o_val.data(), sizeof(VS) * no, hipMemcpyHostToDevice));
        A->h_sendbuf.resize(hl);
        A->h_recvbuf.resize(hl);
      }
      HIPK(cfp::blas_gather(A->d_sendbuf, xd, A->d_send_idx, (i64)hl, g_stream));
      HCHK(cfp::kprof_copy(A->h_sendbuf.data(), A->d_sendbuf, sizeof(VS) * hl, hipMemcpyDeviceToHost, g_stream));
      HCHK(hipStreamSynchronize(g_stream));
      PetscCall(comm_alltoall_host(r, A->h_sendbuf.data(), A->h_recvbuf.data(), sizeof(VS) * (size_t)A->hM));
      HCHK(cfp::kprof_copy(A->d_recvbuf, A->h_recvbuf.data(), sizeof(VS) * hl, hipMemcpyHostToDevice, g_stream));
    }
    Mat B = A->dblk;
    PetscCall(aij_upload(B));
    PetscCall(aij_spmv_dev(B, xd, yd));
    if (hl && !A->o_col.empty())
      HIPK(cfp::blas_csr_spmv_add(A->lm, A->d_orowptr, A->d_ocol, A->d_oval, A->d_recvbuf, yd, g_stream));
    return PETSC_SUCCESS;
  }
  const VS* xh;
  PetscCall(host_read(x, &xh));
  std::vector<VS> sendb(hl), recvb(hl);
  for (size_t e = 0; e < hl; ++e)
    sendb[e] = A->send_idx[e] >= 0 ? xh[A->send_idx[e]] : D(std::complex<double>(0.0, 0.0));
  if (hl) PetscCall(comm_alltoall_host(r, sendb.data(), recvb.data(), sizeof(VS) * (size_t)A->hM));
  VS* yh;
  PetscCall(host_rw(y, &yh));
  const Mat B = A->dblk;
  for (i64 lr = 0; lr < A->lm; ++lr) {
    std::complex<double> acc = 0.0;
    for (i64 p = B->h_rowptr[lr]; p < B->h_rowptr[lr + 1]; ++p) acc += C(B->h_val[p]) * C(xh[B->h_col[p]]);
    for (i64 p = A->o_rowptr[lr]; p < A->o_rowptr[lr + 1]; ++p) acc += C(A->o_val[p]) * C(recvb[A->o_col[p]]);
    yh[lr] = D(acc);
  }
  if (y->hip) {
    HIPK(hipMemcpyAsync(y->d, y->h, sizeof(VS) * (size_t)y->n, hipMemcpyHostToDevice, g_stream));
    y->mask = MASK_BOTH;
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetSize(Mat A, PetscInt* m, PetscInt* n) {
  MCHK(A);
  if (m) *m = A->m;
  if (n) *n = A->n;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetLocalSize(Mat A, PetscInt* m, PetscInt* n) {
  MCHK(A);
  if (m) *m = A->lm;
  if (n) *n = A->ln;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatGetComm(Mat A, MPI_Comm* comm) {
  MCHK(A);
  *comm = A->comm;
  return PETSC_SUCCESS;
}
static PetscErrorCode aij_mult(Mat A, Vec x, Vec y) {
  if (x->nranks > 1 || y->nranks > 1) return ERR(PETSC_ERR_SUP, "the stand-in AIJ matrix is sequential");
  if (x->n != A->n || y->n != A->m) return ERR(PETSC_ERR_ARG_SIZ, "MatMult sizes");
  if (x == y) return ERR(PETSC_ERR_ARG_IDN, "x and y must be different vectors");
  if (x->hip && y->hip) {
    PetscCall(aij_upload(A));
    const VS* xd;
    PetscCall(dev_read(x, &xd));
    VS* yd;
    PetscCall(dev_rw(y, &yd));
    PetscCall(aij_spmv_dev(A, xd, yd));
  } else {
    const VS* xh;
    PetscCall(host_read(x, &xh));
    VS* yh;
    PetscCall(host_rw(y, &yh));
    for (i64 r = 0; r < A->m; ++r) {
      std::complex<double> s = 0;
      for (i64 p = A->h_rowptr[r]; p < A->h_rowptr[r + 1]; ++p) s += C(A->h_val[p]) * C(xh[A->h_col[p]]);
      yh[r] = D(s);
    }
    if (y->hip) {
      HIPK(hipMemcpyAsync(y->d, y->h, sizeof(VS) * (size_t)y->n, hipMemcpyHostToDevice, g_stream));
      y->mask = MASK_BOTH;
    }
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatMult(Mat A, Vec x, Vec y) {
  MCHK(A); VCHK(x); VCHK(y);
  if (A->building) return ERR(PETSC_ERR_ARG_WRONGSTATE, "MatMult before MatAssemblyEnd");
  if (A->type == MATSEQAIJ) return aij_mult(A, x, y);
  if (A->type == MATMPIAIJ) return mpiaij_mult(A, x, y);
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
  if (A->building) return ERR(PETSC_ERR_ARG_WRONGSTATE, "MatShift before MatAssemblyEnd");
  if (A->type == MATMPIAIJ) return MatShift(A->dblk, a);  // the diagonal lives in the diagonal block
  if (A->type != MATSEQAIJ) return ERR(PETSC_ERR_SUP, "MatShift only for AIJ in the stand-in");
  for (i64 r = 0; r < A->m; ++r) {
    bool found = false;
    for (i64 p = A->h_rowptr[r]; p < A->h_rowptr[r + 1]; ++p)
      if (A->h_col[p] == r) { A->h_val[p] = D(C(A->h_val[p]) + a); found = true; }
    if (!found) return ERR(PETSC_ERR_ARG_WRONGSTATE, "MatShift needs an allocated diagonal");
  }
  if (A->dia == 1 || A->bdia == 1) {  // the classes change with the diagonal: rebuild at the next device MatMult
    HCHK(hipDeviceSynchronize());
    aij_free_device(A);
  } else if (A->val && !A->h_val.empty()) {
    HCHK(hipMemcpy(A->val, A->h_val.data(), sizeof(VS) * A->h_val.size(), hipMemcpyHostToDevice));
  }
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatDestroy(Mat* pA) {
  if (!pA || !*pA) return PETSC_SUCCESS;
  Mat A = *pA;
  MCHK(A);
  PetscErrorCode rc = PETSC_SUCCESS;
  if (A->destroy) rc = A->destroy(A);
  aij_free_device(A);
  mpiaij_free(A);
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
  int P = 1;
  MPI_Comm_size(A->comm, &P);
  // x, z: the input / backward-output side (A's columns); y: the spectrum (A's rows).  Complex
  // scalars: both N; real scalars: N reals and FFTW's r2c half spectrum (pcshell_fft3d.cpp)
  Vec* outs[3] = {x, y, z};
  for (int k = 0; k < 3; ++k) {
    Vec* o = outs[k];
    if (!o) continue;
    const PetscInt nl = k == 1 ? A->lm : A->ln, ng = k == 1 ? A->m : A->n;
    if (P > 1) PetscCall(VecCreateMPIHIP(A->comm, nl, ng, o));  // the matrix' slab rows
    else PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, ng, o));
  }
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
  PetscErrorCode (*applyBA)(PC, PCSide, Vec, Vec, Vec) = nullptr;
  PetscErrorCode (*setup)(PC) = nullptr;
  PetscErrorCode (*destroy)(PC) = nullptr;
  bool setupcalled = false;
  Mat A = nullptr, P = nullptr;        // PCSetOperators (not owned)
  PCMiniApplyDots* dots = nullptr;     // the stand-in KSP's pending dots request
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
extern "C" PetscErrorCode PCSetOperators(PC pc, Mat A, Mat P) {
  PCCHK(pc);
  pc->A = A;
  pc->P = P ? P : A;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCGetOperators(PC pc, Mat* A, Mat* P) {
  PCCHK(pc);
  if (A) *A = pc->A;
  if (P) *P = pc->P;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCShellSetApplyBA(PC pc, PetscErrorCode (*f)(PC, PCSide, Vec, Vec, Vec)) {
  PCCHK(pc);
  pc->applyBA = f;
  return PETSC_SUCCESS;
}
// PETSc's PCApplyBAorAB: the shell's applyBA, else left y = B (A x), right y = A (B x)
extern "C" PetscErrorCode PCApplyBAorAB(PC pc, PCSide side, Vec x, Vec y, Vec work) {
  PCCHK(pc); VCHK(x); VCHK(y); VCHK(work);
  if (x == y) return ERR(PETSC_ERR_ARG_IDN, "x and y must be different vectors");
  if (side != PC_LEFT && side != PC_RIGHT) return ERR(PETSC_ERR_SUP, "stand-in PCApplyBAorAB: left or right side");
  PetscCall(PCSetUp(pc));
  if (pc->type == PCSHELL && pc->applyBA) return pc->applyBA(pc, side, x, y, work);
  if (!pc->A) return ERR(PETSC_ERR_ARG_WRONGSTATE, "PCSetOperators has not been called");
  if (side == PC_LEFT) {
    PetscCall(MatMult(pc->A, x, work));
    return PCApply(pc, work, y);
  }
  PetscCall(PCApply(pc, x, work));
  return MatMult(pc->A, work, y);
}
extern "C" PetscErrorCode PCMiniSetApplyDots(PC pc, PCMiniApplyDots* req) {
  PCCHK(pc);
  if (req) {
    if (req->nv < 1 || req->nv > 8 || !req->out) return ERR(PETSC_ERR_ARG_OUTOFRANGE, "dots request: 1 <= nv <= 8, out set");
    req->done = PETSC_FALSE;
  }
  pc->dots = req;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode PCMiniGetApplyDots(PC pc, PCMiniApplyDots** req) {
  PCCHK(pc);
  if (!req) return ERR(PETSC_ERR_ARG_NULL, "NULL output");
  *req = pc->dots;
  return PETSC_SUCCESS;
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
