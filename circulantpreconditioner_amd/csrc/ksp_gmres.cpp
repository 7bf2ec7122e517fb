// ksp_gmres.cpp -- KSPGMRES of the PETSc stand-in: the Krylov solver the reference's GMRES
// drivers call (tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:120-136,
// KSPSetType(KSPGMRES), KSPSetTolerances(precision, precision, PETSC_DEFAULT, 1000)),
// so the PCSHELL circulant preconditioner can run inside it.
//
// It restates PETSc's GMRES with PETSc's defaults: restart 30, left preconditioning,
// classical Gram-Schmidt without refinement (one VecMDot + one VecMAXPY per iteration),
// the preconditioned residual norm estimated from the rotated Hessenberg right-hand side,
// KSPConvergedDefault (converged when ||r|| <= max(rtol ||r_0||, abstol), diverged when
// ||r|| > dtol ||r_0||), the complex Givens rotations of KSPGMRESUpdateHessenberg, and the
// true residual recomputed at every restart.  Every vector operation is a device kernel
// (cfp_blas.hip); only the (restart+1) x restart Hessenberg lives on the host.
//
// Written against the PETSc API only; compiled out with -DCFP_WITH_PETSC (real PETSc has
// its own KSP).
#ifndef CFP_WITH_PETSC
#include <hip/hip_runtime.h>
#include <sys/time.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/petsc_mini.h"
#include "cfp_internal.h"

namespace {
const int kKSPMagic = 0x4b535031;
typedef std::complex<double> C;
// the Hessenberg algebra runs in complex arithmetic; with real scalars (-DCFP_REAL_SCALAR) its
// results are real and go back as their real parts
#ifdef CFP_REAL_SCALAR
static inline PetscScalar to_ps(C v) { return v.real(); }
#else
static inline PetscScalar to_ps(C v) { return v; }
#endif

double now() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}
}  // namespace

struct _p_KSP {
  int magic = kKSPMagic;
  std::string type = KSPGMRES;
  PetscReal rtol = 1e-5, abstol = 1e-50, dtol = 1e5;
  PetscInt maxits = 10000;
  PetscInt restart = 30;
  PCSide side = PC_LEFT;
  bool guess_nonzero = false;
  Mat A = nullptr, P = nullptr;
  PC pc = nullptr;
  KSPConvergedReason reason = KSP_CONVERGED_ITERATING;
  PetscInt its = 0;
  PetscReal rnorm = 0.0;
  PetscInt pc_calls = 0;
  double pc_seconds = 0.0;
  // PCApply's device time: an event pair around every call on the Vec stream (a device-Vec
  // PCApply is stream-ordered there and returns at once; its time is read at the end of the solve)
  std::vector<hipEvent_t> pc_ev;  // 4 per PCApply: events around it, then the apply's own stamps
  size_t pc_ev_used = 0;
  std::vector<char> pc_stamped;  // per recorded PCApply: the stamps were set (3-sweep apply)
  // work space (sized for the current problem)
  PetscInt n = -1, nvec = 0;
  Vec* V = nullptr;  // restart + 1 basis vectors
  Vec t = nullptr, t2 = nullptr, rhs = nullptr;
  // the dots a shell PC computes inside its apply (PCMiniApplyDots, r06): device results, and
  // whether the basis lives on the device (requests are made only then)
  double* dots_dev = nullptr;
  double *norm_h = nullptr, *norm_hd = nullptr;  // |r|^2 from the apply: pinned host memory (mapped)
  bool dev_basis = false;
  bool fusion = true;  // KSPMiniSetFusion
  PetscInt fused_dots = 0, fused_norms = 0;  // how many Gram-Schmidt dots / norms came from the PC
};

static PetscErrorCode kcheck(KSP k, const char* f) {
  if (!k || k->magic != kKSPMagic) return PetscErrorSet(PETSC_ERR_ARG_NULL, f, "invalid KSP");
  return PETSC_SUCCESS;
}
#define KCHK(k) PetscCall(kcheck((k), __func__))

static void free_events(KSP k) {
  for (auto& e : k->pc_ev) hipEventDestroy(e);
  k->pc_ev.clear();
  k->pc_ev_used = 0;
  k->pc_stamped.clear();
}

static void free_work(KSP k) {
  if (k->dots_dev) hipFree(k->dots_dev);
  if (k->norm_h) hipHostFree(k->norm_h);
  k->dots_dev = nullptr;
  k->norm_h = k->norm_hd = nullptr;
  k->dev_basis = false;
  if (k->V) VecDestroyVecs(k->nvec, &k->V);
  VecDestroy(&k->t);
  VecDestroy(&k->t2);
  VecDestroy(&k->rhs);
  k->n = -1;
  k->nvec = 0;
}

extern "C" PetscErrorCode KSPCreate(MPI_Comm comm, KSP* ksp) {
  if (!ksp) return PetscErrorSet(PETSC_ERR_ARG_NULL, __func__, "NULL output");
  KSP k = new _p_KSP;
  PetscErrorCode rc = PCCreate(comm, &k->pc);
  if (rc) { delete k; return rc; }
  *ksp = k;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPSetType(KSP k, KSPType type) {
  KCHK(k);
  if (!type || (std::strcmp(type, KSPGMRES) && std::strcmp(type, KSPPREONLY)))
    return PetscErrorSet(PETSC_ERR_SUP, __func__, "stand-in KSP types: gmres, preonly");
  k->type = type;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPSetTolerances(KSP k, PetscReal rtol, PetscReal abstol, PetscReal dtol, PetscInt maxits) {
  KCHK(k);
  if (rtol != PETSC_DEFAULT) k->rtol = rtol;
  if (abstol != PETSC_DEFAULT) k->abstol = abstol;
  if (dtol != PETSC_DEFAULT) k->dtol = dtol;
  if (maxits != PETSC_DEFAULT) k->maxits = maxits;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPGMRESSetRestart(KSP k, PetscInt restart) {
  KCHK(k);
  if (restart < 1) return PetscErrorSet(PETSC_ERR_ARG_OUTOFRANGE, __func__, "restart must be >= 1");
  if (restart != k->restart) free_work(k);
  k->restart = restart;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPSetPCSide(KSP k, PCSide side) { KCHK(k); k->side = side; return PETSC_SUCCESS; }
extern "C" PetscErrorCode KSPSetInitialGuessNonzero(KSP k, PetscBool f) {
  KCHK(k);
  k->guess_nonzero = f == PETSC_TRUE;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPGetPC(KSP k, PC* pc) { KCHK(k); *pc = k->pc; return PETSC_SUCCESS; }
extern "C" PetscErrorCode KSPSetOperators(KSP k, Mat A, Mat P) {
  KCHK(k);
  k->A = A;
  k->P = P;
  return PCSetOperators(k->pc, A, P);
}
extern "C" PetscErrorCode KSPSetUp(KSP k) {
  KCHK(k);
  return PCSetUp(k->pc);
}
extern "C" PetscErrorCode KSPGetConvergedReason(KSP k, KSPConvergedReason* r) { KCHK(k); *r = k->reason; return PETSC_SUCCESS; }
extern "C" PetscErrorCode KSPGetIterationNumber(KSP k, PetscInt* its) { KCHK(k); *its = k->its; return PETSC_SUCCESS; }
extern "C" PetscErrorCode KSPGetResidualNorm(KSP k, PetscReal* r) { KCHK(k); *r = k->rnorm; return PETSC_SUCCESS; }
extern "C" PetscErrorCode KSPMiniGetPCApplyStats(KSP k, PetscInt* calls, PetscLogDouble* seconds) {
  KCHK(k);
  if (calls) *calls = k->pc_calls;
  if (seconds) *seconds = k->pc_seconds;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPMiniSetFusion(KSP k, PetscBool on) {
  KCHK(k);
  k->fusion = on == PETSC_TRUE;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPMiniGetFusedCounts(KSP k, PetscInt* dots, PetscInt* norms) {
  KCHK(k);
  if (dots) *dots = k->fused_dots;
  if (norms) *norms = k->fused_norms;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode KSPDestroy(KSP* pk) {
  if (!pk || !*pk) return PETSC_SUCCESS;
  KSP k = *pk;
  KCHK(k);
  free_work(k);
  free_events(k);
  PetscErrorCode rc = PCDestroy(&k->pc);
  k->magic = 0;
  delete k;
  *pk = nullptr;
  return rc;
}

// 64 more PCApply timing events (16 applies); false without a HIP device.  Creating them costs
// ~25 us each, so KSPMiniSetUpWork makes the first batch outside the timed solves.
static bool grow_events(KSP k) {
  for (int i = 0; i < 64; ++i) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
      hipGetLastError();
      return false;
    }
    k->pc_ev.push_back(e);
  }
  return true;
}

extern "C" PetscErrorCode KSPMiniSetUpWork(KSP k, Vec v) {
  KCHK(k);
  PetscInt n;
  PetscCall(VecGetLocalSize(v, &n));
  const PetscInt m = k->restart;
  if (n != k->n || k->nvec != m + 1) {
    free_work(k);
    PetscCall(VecDuplicateVecs(v, m + 1, &k->V));
    k->nvec = m + 1;
    PetscCall(VecDuplicate(v, &k->t));
    PetscCall(VecDuplicate(v, &k->t2));
    PetscCall(VecDuplicate(v, &k->rhs));
    k->n = n;
#ifndef CFP_REAL_SCALAR
    VecType vt;
    PetscCall(VecGetType(v, &vt));
    int P = 1;
    MPI_Comm comm;
    PetscCall(VecGetComm(v, &comm));
    MPI_Comm_size(comm, &P);
    k->dev_basis = P == 1 && std::strcmp(vt, VECSEQHIP) == 0 &&
                   hipMalloc(&k->dots_dev, sizeof(double) * 16) == hipSuccess &&
                   hipHostMalloc(&k->norm_h, sizeof(double) * 16, hipHostMallocMapped | hipHostMallocCoherent) ==
                       hipSuccess &&
                   hipHostGetDevicePointer((void**)&k->norm_hd, k->norm_h, 0) == hipSuccess;
    if (!k->dev_basis) hipGetLastError();
#endif
  }
  if (k->pc_ev.empty()) grow_events(k);  // no device: the applies are timed on the host
  return PETSC_SUCCESS;
}

// one PCApply (ba: PCApplyBAorAB on the left, y = B A x, k->t the scratch), with an optional dots
// request to the shell (PCMiniApplyDots; req->done tells whether the apply computed them)
static PetscErrorCode pc_apply(KSP k, Vec x, Vec y, PCMiniApplyDots* req = nullptr, bool ba = false) {
  if (req) PetscCall(PCMiniSetApplyDots(k->pc, req));
  const auto call = [&]() -> PetscErrorCode {
    const PetscErrorCode rc = ba ? PCApplyBAorAB(k->pc, PC_LEFT, x, y, k->t) : PCApply(k->pc, x, y);
    if (req) PCMiniSetApplyDots(k->pc, nullptr);
    return rc;
  };
  void* st = nullptr;
  PetscCall(VecMiniGetStream(&st));
  bool events = k->pc_ev_used + 4 <= k->pc_ev.size();
  if (!events) events = grow_events(k);
  if (!events) {  // no HIP device (host Vecs on a CPU-only machine): the apply is synchronous
    hipGetLastError();
    const double t0 = now();
    PetscCall(call());
    k->pc_seconds += now() - t0;
    k->pc_calls += 1;
    return PETSC_SUCCESS;
  }
  // recorded in stream order: the first one after the MatMult queued before, the second after
  // the apply (on the same stream, or completed on the host before it returned).  A 3-sweep
  // apply also stamps its own first and last kernel (cfp::g_apply_stamp): the event packets
  // themselves idle the device ~5 us each and read ~35 us high at 256^3 (GMRES).
  const size_t i0 = k->pc_ev_used;
  hipEventRecord(k->pc_ev[i0], (hipStream_t)st);
  cfp::g_apply_stamp = cfp::ApplyStamp{k->pc_ev[i0 + 2], k->pc_ev[i0 + 3], 0};
  const PetscErrorCode rc = call();
  const bool stamped = cfp::g_apply_stamp.hits == 2;
  cfp::g_apply_stamp = cfp::ApplyStamp{};
  PetscCall(rc);
  hipEventRecord(k->pc_ev[i0 + 1], (hipStream_t)st);
  k->pc_ev_used += 4;
  k->pc_stamped.push_back(stamped ? 1 : 0);
  k->pc_calls += 1;
  return PETSC_SUCCESS;
}

// add the recorded PCApply times to pc_seconds (waits for the last event)
static PetscErrorCode pc_collect(KSP k) {
  if (!k->pc_ev_used) return PETSC_SUCCESS;
  if (hipEventSynchronize(k->pc_ev[k->pc_ev_used - 3]) != hipSuccess)  // the last apply's closing event
    return PetscErrorSet(PETSC_ERR_LIB, __func__, "hipEventSynchronize");
  for (size_t a = 0; 4 * a + 3 < k->pc_ev_used; ++a) {
    const size_t i = 4 * a + (k->pc_stamped[a] ? 2 : 0);  // the stamps, else the events around it
    float ms = 0.f;
    hipEventElapsedTime(&ms, k->pc_ev[i], k->pc_ev[i + 1]);
    k->pc_seconds += 1e-3 * (double)ms;
  }
  k->pc_ev_used = 0;
  k->pc_stamped.clear();
  return PETSC_SUCCESS;
}

// KSPConvergedDefault
static void converged(KSP k, PetscReal rnorm0) {
  const PetscReal ttol = std::fmax(k->rtol * rnorm0, k->abstol);
  if (std::isnan(rnorm0) || std::isnan(k->rnorm)) k->reason = KSP_DIVERGED_BREAKDOWN;
  else if (k->rnorm <= ttol) k->reason = k->rnorm < k->abstol ? KSP_CONVERGED_ATOL : KSP_CONVERGED_RTOL;
  else if (k->its > 0 && k->rnorm >= k->dtol * rnorm0) k->reason = KSP_DIVERGED_DTOL;
}

// device pointers of the basis vectors V[0..nv) for a dots request
static PetscErrorCode basis_ptrs(KSP k, PetscInt nv, PCMiniApplyDots* req) {
  req->nv = nv;
  req->out = k->dots_dev;
  for (PetscInt i = 0; i < nv; ++i) {
    const PetscScalar* a;
    PetscCall(VecHIPGetArrayRead(k->V[i], &a));
    req->v[i] = a;
    PetscCall(VecHIPRestoreArrayRead(k->V[i], &a));
  }
  return PETSC_SUCCESS;
}

// preconditioned residual into z (left: z = B (b - A x); right: z = b - A x).  x = 0: left,
// z = B b straight from b (no copy of b); right, z = a copy of b.  *norm = |z| (its square asked
// from the shell's apply on device bases, else VecNorm).
static PetscErrorCode residual(KSP k, Vec b, Vec x, bool x_zero, Vec z, PetscReal* norm) {
  Vec r = k->side == PC_LEFT ? k->t : z;
  if (x_zero && k->side == PC_LEFT) {
    r = b;
  } else if (x_zero) {
    PetscCall(VecCopy(b, r));
  } else {
    PetscCall(MatMult(k->A, x, k->t2));
    PetscCall(VecWAXPY(r, -1.0, k->t2, b));
  }
  PCMiniApplyDots req{};
  bool asked = false;
  if (k->side == PC_LEFT) {
    asked = k->fusion && k->dev_basis && z == k->V[0];
    if (asked) {
      req.nv = 1;
      req.v[0] = nullptr;  // |z|^2, written straight into pinned host memory
      req.out = k->norm_hd;
    }
    PetscCall(pc_apply(k, r, z, asked ? &req : nullptr));
  }
  if (asked && req.done) {
    PetscCall(VecMiniSynchronize(z));
    *norm = std::sqrt(k->norm_h[0]);
    k->fused_norms += 1;
  } else {
    PetscCall(VecNorm(z, NORM_2, norm));
  }
  return PETSC_SUCCESS;
}

// the solve; x_unset: x has not been written yet (a zero initial guess is implied, not stored)
static PetscErrorCode ksp_solve_impl(KSP k, Vec b, Vec x, bool& x_unset) {
  KCHK(k);
  if (!k->A) return PetscErrorSet(PETSC_ERR_ARG_WRONGSTATE, __func__, "KSPSetOperators has not been called");
  PetscCall(PCSetUp(k->pc));
  PetscCall(KSPMiniSetUpWork(k, b));
  const PetscInt m = k->restart;
  k->its = 0;
  k->reason = KSP_CONVERGED_ITERATING;
  k->pc_calls = 0;
  k->pc_seconds = 0.0;
  k->pc_ev_used = 0;
  k->fused_dots = k->fused_norms = 0;
  if (k->type == KSPPREONLY) {
    if (b == x) {  // PCApply needs x != y
      PetscCall(VecCopy(b, k->rhs));
      b = k->rhs;
    }
    PetscCall(pc_apply(k, b, x));
    k->its = 1;
    k->reason = KSP_CONVERGED_ITS;
    return pc_collect(k);
  }
  // KSPSolve(ksp, Un, Un): PETSc copies the right-hand side when b == x.  Here b is read from x
  // until x is first written (the end of the first cycle), and copied only if a restart follows.
  bool b_in_x = b == x;
  // x = 0 initially: not set here; the first solution update overwrites x (VecMiniMAXPYNorm).
  // An error return before that update zeroes x (KSPSolve below), as PETSc's zeroed x would be.
  bool x_zero = !k->guess_nonzero;
  x_unset = x_zero;

  std::vector<C> H((size_t)(m + 1) * m), cc((size_t)m), ss((size_t)m), rs((size_t)m + 1), y((size_t)m);
  auto h = [&](PetscInt i, PetscInt j) -> C& { return H[(size_t)j * (m + 1) + i]; };
  PetscReal rnorm0 = -1.0;
  Vec* V = k->V;
  // The basis is kept unnormalised: v_i = sg[i] u_i with u_i = V[i].  The normalisations are
  // folded into the Gram-Schmidt coefficients (h_ij = sg_i sg_j u_i^H w' for w' = B A u_j, and
  // w'' = w' - sum sg_i^2 (u_i^H w') u_i = w / sg_j), the norm rides in the orthogonalisation
  // sweep, so no VecScale sweep of a basis vector remains.  Same iterates as PETSc's
  // KSPGMRESCycle up to rounding.
  std::vector<double> sg((size_t)m + 1, 1.0);
  const auto renormalise = [&](PetscInt i) -> PetscErrorCode {  // keep |u_i| within range
    if (sg[(size_t)i] > 1e-150 && sg[(size_t)i] < 1e150) return PETSC_SUCCESS;
    PetscCall(VecScale(V[i], sg[(size_t)i]));
    sg[(size_t)i] = 1.0;
    return PETSC_SUCCESS;
  };

  while (true) {
    PetscReal beta;
    PetscCall(residual(k, b, x, x_zero, V[0], &beta));
    x_zero = false;
    k->rnorm = beta;
    if (rnorm0 < 0) rnorm0 = beta;
    converged(k, rnorm0);
    if (k->reason != KSP_CONVERGED_ITERATING) break;
    if (k->its >= k->maxits) { k->reason = KSP_DIVERGED_ITS; break; }
    sg[0] = 1.0 / beta;
    PetscCall(renormalise(0));
    std::fill(rs.begin(), rs.end(), C(0.0));
    rs[0] = beta;
    PetscInt j = 0;
    bool happy = false;
    for (; j < m && k->reason == KSP_CONVERGED_ITERATING && k->its < k->maxits; ++j) {
      // w' = B A u_j (left) or A B u_j (right), written into V[j+1]; w = sg_j w'
      // left: PCApplyBAorAB (a shell may fuse the MatMult into its apply), with the Gram-Schmidt
      // dots u_i^H w' asked from the apply on device bases (at most 4 vectors)
      PCMiniApplyDots req{};
      bool asked = false;
      if (k->side == PC_LEFT) {
        asked = k->fusion && k->dev_basis && j + 1 <= 4;
        if (asked) PetscCall(basis_ptrs(k, j + 1, &req));
        PetscCall(pc_apply(k, V[j], V[j + 1], asked ? &req : nullptr, true));
      } else {
        PetscCall(pc_apply(k, V[j], k->t));
        PetscCall(MatMult(k->A, k->t, V[j + 1]));
      }
      // classical Gram-Schmidt: h_ij = v_i^H w, w -= sum h_ij v_i, and |w|, in two sweeps and
      // one host wait (the MAXPY coefficients -sg_i^2 u_i^H w' are formed on the device)
      std::vector<PetscScalar> hv((size_t)j + 1);
      std::vector<PetscReal> negsq((size_t)j + 1);
      for (PetscInt i = 0; i <= j; ++i) negsq[(size_t)i] = -(sg[(size_t)i] * sg[(size_t)i]);
      PetscReal hn;
      if (asked && req.done) {
        PetscCall(VecMiniMAXPYNormDeviceDots(V[j + 1], j + 1, negsq.data(), V, k->dots_dev, hv.data(), &hn));
        k->fused_dots += 1;
      } else {
        PetscCall(VecMiniMDotMAXPYNorm(V[j + 1], j + 1, negsq.data(), V, hv.data(), &hn));
      }
      for (PetscInt i = 0; i <= j; ++i) h(i, j) = sg[(size_t)i] * sg[(size_t)j] * hv[(size_t)i];
      hn *= sg[(size_t)j];  // |w| = sg_j |w''|
      h(j + 1, j) = hn;
      // happy breakdown test of KSPGMRESCycle: hn < min(hn / |rs_j|, haptol = 1e-30)
      const double hapbnd = std::fmin(hn / std::abs(rs[(size_t)j]), 1e-30);
      happy = hn < hapbnd;
      if (!happy) {
        sg[(size_t)j + 1] = sg[(size_t)j] / hn;  // v_{j+1} = w / hn = (sg_j / hn) w''
        PetscCall(renormalise(j + 1));
      }
      // KSPGMRESUpdateHessenberg: previous rotations, then a new one
      for (PetscInt i = 0; i < j; ++i) {
        const C tt = h(i, j);
        h(i, j) = std::conj(cc[(size_t)i]) * tt + ss[(size_t)i] * h(i + 1, j);
        h(i + 1, j) = cc[(size_t)i] * h(i + 1, j) - ss[(size_t)i] * tt;
      }
      if (!happy) {
        const double tt = std::sqrt(std::norm(h(j, j)) + std::norm(h(j + 1, j)));
        if (tt == 0.0) { k->reason = KSP_DIVERGED_BREAKDOWN; break; }
        cc[(size_t)j] = h(j, j) / tt;
        ss[(size_t)j] = h(j + 1, j) / tt;
        rs[(size_t)j + 1] = -(ss[(size_t)j] * rs[(size_t)j]);
        rs[(size_t)j] = std::conj(cc[(size_t)j]) * rs[(size_t)j];
        h(j, j) = std::conj(cc[(size_t)j]) * h(j, j) + ss[(size_t)j] * h(j + 1, j);
        k->rnorm = std::abs(rs[(size_t)j + 1]);
      } else {  // h(j+1,j) = 0: no new rotation, the residual estimate is exactly zero
        rs[(size_t)j + 1] = 0.0;
        k->rnorm = 0.0;
      }
      k->its += 1;
      converged(k, rnorm0);
      if (happy && k->reason == KSP_CONVERGED_ITERATING) k->reason = KSP_DIVERGED_BREAKDOWN;
      if (k->reason == KSP_CONVERGED_ITERATING && k->its >= k->maxits) k->reason = KSP_DIVERGED_ITS;
      if (k->reason != KSP_CONVERGED_ITERATING || happy) { ++j; break; }
    }
    // back substitution H(0:j, 0:j) y = rs(0:j), then x += V y (left) / x += B V y (right)
    const PetscInt kk = j;
    for (PetscInt i = kk - 1; i >= 0; --i) {
      C s = rs[(size_t)i];
      for (PetscInt q = i + 1; q < kk; ++q) s -= h(i, q) * y[(size_t)q];
      y[(size_t)i] = s / h(i, i);
    }
    // a restart follows: keep b before x (which holds it) is written
    if (b_in_x && k->reason == KSP_CONVERGED_ITERATING) {
      PetscCall(VecCopy(x, k->rhs));
      b = k->rhs;
      b_in_x = false;
    }
    if (kk > 0) {
      std::vector<PetscScalar> yy((size_t)kk);
      for (PetscInt i = 0; i < kk; ++i) yy[(size_t)i] = to_ps(y[(size_t)i] * sg[(size_t)i]);  // v_i = sg_i u_i
      if (k->side == PC_LEFT) {
        PetscCall(VecMiniMAXPYNorm(x, kk, yy.data(), V, x_unset ? PETSC_TRUE : PETSC_FALSE, nullptr));
      } else {
        PetscCall(VecMiniMAXPYNorm(k->t2, kk, yy.data(), V, PETSC_TRUE, nullptr));
        if (x_unset) {
          PetscCall(pc_apply(k, k->t2, x));
        } else {
          PetscCall(pc_apply(k, k->t2, k->t));
          PetscCall(VecAXPY(x, 1.0, k->t));
        }
      }
      x_unset = false;
    }
    if (k->reason != KSP_CONVERGED_ITERATING) break;
  }
  if (x_unset) PetscCall(VecSet(x, 0.0));  // converged before any update (b = 0): x = 0
  x_unset = false;
  return pc_collect(k);
}

extern "C" PetscErrorCode KSPSolve(KSP k, Vec b, Vec x) {
  bool x_unset = false;
  const PetscErrorCode rc = ksp_solve_impl(k, b, x, x_unset);
  // PETSc zeroes x before a zero-guess solve: after an error before the first update x reads 0
  // here too (not the caller's old contents, nor b when b == x); the first error is returned
  if (rc && x_unset) VecSet(x, 0.0);
  return rc;
}
#endif  // CFP_WITH_PETSC
