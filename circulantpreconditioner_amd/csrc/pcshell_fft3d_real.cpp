// pcshell_fft3d_real.cpp -- the PETSc-named boundary of include/pcshell_fft3d.h for a PETSc
// built with real scalars (PetscScalar = double, !PETSC_USE_COMPLEX): the reference's real
// branches of src/FftLinearSolver_3D.c (:6-78 VecPointwiseDivideForRealFFT, :166-190 solve_3D
// with the r2c MATFFTW) and src/PCSHELLFft_3D.cxx (:10-99).  Compiled with -DCFP_REAL_SCALAR
// into libcirculant_fft_real.so, beside the real-scalar stand-in PETSc (petsc_mini.cpp).
//
// Layouts (FFTW's r2c conventions, which a real-scalar MATFFTW uses; third-party semantics):
//   - the grid side of FFT_MAT (b, X, b_cartesien): N = nx ny nz reals, x fastest;
//   - the spectral side (Diag, b_hat, MatMult's output): the half spectrum [nz][ny][nx/2 + 1]
//     of complex values stored as interleaved (re, im) reals, NS = 2 (nx/2 + 1) ny nz reals.
// Arithmetic: the correct real solve X = C^{-1} b = (1/N) c2r( r2c(b) ./ Diag_half ), i.e. the
// complex build's result for real b and real lambda.  The reference's real branch divides only
// the first 2 (size/4 + 1) entries (:54) and scales by 2/size (:186); neither is reproduced
// (parity is against the correct real arithmetic, the oracle's solve of b).
//
// One rank: the register-symbol path runs the real plan (cfp_rplan: r2c rows, half-spectrum
// passes, c2r; 3 sweeps at 128^3 and 256^3) where it supports the grid, else the complex plan on
// b promoted to complex (one extra read and write of N complex values).  An explicit Diag (any
// change to the Diag setup made) takes the complex plan with the Hermitian extension of the
// half-spectrum Diag.
//
// Several ranks (r05; the reference's real branch runs on PETSC_COMM_WORLD
// like the complex one, src/FftLinearSolver_3D.c:6-78,176,186 and src/PCSHELLFft_3D.cxx:34-35):
// the FFT matrix is backed by the complex z-slab plan (include/circulant_fft_dist.h) on b promoted
// to complex.  Every Vec holds its rank's z-planes: the grid side nzl ny nx reals, the spectral
// side FFTW-MPI's non-transposed r2c slab, [nzl][ny][nx/2 + 1] complex.  The half spectrum's
// Hermitian extension would need the X(-kz) planes of another rank, so the c2r side instead
// pads each row locally (cfp_half_spectrum_pad: weight 2 on the paired columns, 0 above nx/2),
// whose real part after the backward transform is the same c2r.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/circulant_fft_real.h"
#include "../../include/pcshell_fft3d.h"
#include "pcshell_common.h"

#if defined(PETSC_USE_COMPLEX)
#error "pcshell_fft3d_real.cpp is the real-scalar boundary: build it with -DCFP_REAL_SCALAR (stand-in) or against a real-scalar PETSc"
#endif

namespace {
using namespace cfp_pc;

extern "C" void cfp_apply_stamp_clear(void);  // cfp_plan.hip (internal)

const int kRFFTMagic = 0x52464654;  // "RFFT"

struct RShell {
  int magic = kRFFTMagic;
  PetscInt dims[3] = {1, 1, 1};  // n_x, n_y, n_z
  PetscInt N = 1, NS = 2;        // grid reals, half-spectrum reals
  // several ranks: the complex slab plan (slab.plan), this rank's z-planes [z0, z0 + nzl) and its
  // grid reals nl / half-spectrum reals nsl (one rank: nl = N, nsl = NS)
  SlabBacking slab;
  int nranks = 1, rank = 0;
  PetscInt z0 = 0, nzl = 1, nl = 1, nsl = 2;
  uint64_t dist_version = 0;  // symbol version of slab.plan (its setter is called here only)
  cfp_plan_t cplan = nullptr;    // complex plan: transforms, explicit Diag, grids cfp_rplan lacks
  cfp_rplan_t rplan = nullptr;   // real plan (NULL where it does not support the grid)
  double* zbuf = nullptr;        // N complex: promoted b / spectrum
  double* fbuf = nullptr;        // N complex: the full (Hermitian-extended) explicit Diag
  bool has_lam = false;
  double lam[3] = {0, 0, 0};
  uint64_t lam_version = 0;   // cplan's symbol version right after lam was set (rplan is valid only then)
  PetscObjectId diag_id = 0;  // the Diag setupFFTPrec3D materialised (id, state, symbol version)
  PetscObjectState diag_state = 0;
  uint64_t diag_version = 0;
  PetscInt solves_own = 0, solves_diag = 0;
};

PetscErrorCode rshell(Mat A, RShell** out) {
  void* ctx = nullptr;
  PetscCall(MatShellGetContext(A, &ctx));
  RShell* s = (RShell*)ctx;
  PetscCheck(s && s->magic == kRFFTMagic, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONG,
             "FFT_MAT is not an FFT matrix made by MatCreateFFT/MatCreateFFTHIP");
  *out = s;
  return PETSC_SUCCESS;
}

PetscErrorCode ensure_bufs(RShell* s, bool full_diag) {
  const size_t bytes = 2 * sizeof(double) * (size_t)s->nl;
  if (!s->zbuf) PetscCheck(hipMalloc(&s->zbuf, bytes) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_MEM, "work buffer");
  if (full_diag && !s->fbuf)
    PetscCheck(hipMalloc(&s->fbuf, bytes) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_MEM, "Diag buffer");
  return PETSC_SUCCESS;
}

// the stream of device-Vec work (stand-in: the Vec stream) and the final wait
struct Stream {
  void* st = nullptr;
  bool wait = true;
  Stream() { device_stream(&st, &wait); }
};

// MatMult: y = r2c(x) (FFTW_FORWARD, unnormalised), the half spectrum
PetscErrorCode rfft_mult(Mat A, Vec x, Vec y) {
  RShell* s;
  PetscCall(rshell(A, &s));
  PetscCall(check_size(x, s->nl, "MatMult: x has the wrong size (n_x n_y n_z reals)"));
  PetscCall(check_size(y, s->nsl, "MatMult: y has the wrong size (2 (n_x/2 + 1) n_y n_z reals)"));
  PetscCall(ensure_bufs(s, s->slab.plan != nullptr));
  DevIn in;
  DevOut out;
  PetscCall(in.get(x, s->nl));
  PetscCall(out.get(y, s->nsl));
  Stream q;
  int rc = cfp_real_to_complex(in.ptr(), s->zbuf, s->nl, q.st);
  double* spec = s->zbuf;
  if (s->slab.plan) {  // natural slab out (FFTW-MPI's non-transposed layout): the half per plane
    if (!rc) rc = cfp_dist_plan_forward(s->slab.plan, s->zbuf, s->fbuf, q.st);
    spec = s->fbuf;
  } else if (!rc) {
    rc = cfp_plan_forward(s->cplan, s->zbuf, s->zbuf, q.st);
  }
  if (!rc) rc = cfp_half_spectrum_extract(spec, out.ptr(), s->dims[0], s->dims[1], s->nzl, q.st);
  if (!rc) rc = cfp_stream_sync(q.st);
  PetscCall(out.put());
  PetscCall(in.put());
  CFPCALL(rc);
  return PETSC_SUCCESS;
}
// MatMultTranspose: x = c2r(y) (FFTW_BACKWARD, unnormalised) of a Hermitian half spectrum
PetscErrorCode rfft_mult_transpose(Mat A, Vec y, Vec x) {
  RShell* s;
  PetscCall(rshell(A, &s));
  PetscCall(check_size(y, s->nsl, "MatMultTranspose: x has the wrong size (2 (n_x/2 + 1) n_y n_z reals)"));
  PetscCall(check_size(x, s->nl, "MatMultTranspose: y has the wrong size (n_x n_y n_z reals)"));
  PetscCall(ensure_bufs(s, s->slab.plan != nullptr));
  DevIn in;
  DevOut out;
  PetscCall(in.get(y, s->nsl));
  PetscCall(out.get(x, s->nl));
  Stream q;
  int rc;
  if (s->slab.plan) {  // row-local padding instead of the extension (its -kz planes live elsewhere)
    rc = cfp_half_spectrum_pad(in.ptr(), nullptr, s->zbuf, s->dims[0], s->dims[1] * s->nzl, q.st);
    if (!rc) rc = cfp_dist_plan_backward(s->slab.plan, s->zbuf, s->fbuf, q.st);
    if (!rc) rc = cfp_complex_real_part(s->fbuf, out.ptr(), s->nl, 1.0, q.st);
  } else {
    rc = cfp_half_spectrum_extend(in.ptr(), s->zbuf, s->dims[0], s->dims[1], s->dims[2], q.st);
    if (!rc) rc = cfp_plan_backward(s->cplan, s->zbuf, s->zbuf, q.st);
    if (!rc) rc = cfp_complex_real_part(s->zbuf, out.ptr(), s->N, 1.0, q.st);
  }
  if (!rc) rc = cfp_stream_sync(q.st);
  PetscCall(out.put());
  PetscCall(in.put());
  CFPCALL(rc);
  return PETSC_SUCCESS;
}
#ifdef CFP_WITH_PETSC
// MatCreateVecsFFTW(A, x, y, z) on the shell: PETSc dispatches it through this composed method
PetscErrorCode rfft_create_vecs(Mat A, Vec* x, Vec* y, Vec* z) {
  if (x) PetscCall(MatCreateVecs(A, x, NULL));
  if (y) PetscCall(MatCreateVecs(A, NULL, y));
  if (z) PetscCall(MatCreateVecs(A, z, NULL));
  return PETSC_SUCCESS;
}
#endif
PetscErrorCode rfft_destroy(Mat A) {
  RShell* s;
  PetscCall(rshell(A, &s));
  if (s->cplan) cfp_plan_destroy(s->cplan);
  if (s->rplan) cfp_rplan_destroy(s->rplan);
  slab_destroy(&s->slab);
  if (s->zbuf) hipFree(s->zbuf);
  if (s->fbuf) hipFree(s->fbuf);
  s->magic = 0;
  delete s;
  return PETSC_SUCCESS;
}

uint64_t cversion(RShell* s) {
  if (s->slab.plan) return s->dist_version;
  uint64_t v = 0;
  cfp_plan_symbol_version(s->cplan, &v);
  return v;
}

PetscErrorCode ensure_transport_symbol(RShell* s, const double lam[3]) {
  if (s->has_lam && cversion(s) == s->lam_version && std::memcmp(s->lam, lam, sizeof(s->lam)) == 0)
    return PETSC_SUCCESS;
  const double l6[6] = {lam[0], 0.0, lam[1], 0.0, lam[2], 0.0};
  if (s->slab.plan) {
    CFPCALL(cfp_dist_plan_set_symbol_transport(s->slab.plan, l6));
    ++s->dist_version;
  } else {
    CFPCALL(cfp_plan_set_symbol_transport(s->cplan, l6));
  }
  if (s->rplan) CFPCALL(cfp_rplan_set_symbol_transport(s->rplan, lam));
  std::memcpy(s->lam, lam, sizeof(s->lam));
  s->has_lam = true;
  s->lam_version = cversion(s);
  return PETSC_SUCCESS;
}

// X = C^{-1} b with the plan's own symbol (own) or the half-spectrum Diag given; b may be X
PetscErrorCode rshell_apply(RShell* s, Vec X, Vec b, bool own, Vec Diag) {
  PetscCall(ensure_bufs(s, !own));
  DevIn bin, din;
  DevOut xout;
  PetscCall(bin.get(b, s->nl));
  if (!own) PetscCall(din.get(Diag, s->nsl));
  PetscCall(xout.get(X, s->nl));
  Stream q;
  int rc;
  if (s->slab.plan) {  // the complex slab plan on the promoted slab; its exchanges are host-driven
    rc = cfp_real_to_complex(bin.ptr(), s->zbuf, s->nl, q.st);
    if (own) {
      if (!rc) rc = cfp_dist_plan_use_diag(s->slab.plan, 0);
      if (!rc) rc = cfp_dist_plan_apply(s->slab.plan, s->zbuf, s->zbuf, q.st);
      if (!rc) rc = cfp_complex_real_part(s->zbuf, xout.ptr(), s->nl, 1.0, q.st);
    } else {  // (1/N) c2r(r2c(b) ./ Diag): forward, divide the half and pad per row, backward
      if (!rc) rc = cfp_dist_plan_forward(s->slab.plan, s->zbuf, s->fbuf, q.st);
      if (!rc) rc = cfp_half_spectrum_pad(nullptr, din.ptr(), s->fbuf, s->dims[0], s->dims[1] * s->nzl, q.st);
      if (!rc) rc = cfp_dist_plan_backward(s->slab.plan, s->fbuf, s->zbuf, q.st);
      if (!rc) rc = cfp_complex_real_part(s->zbuf, xout.ptr(), s->nl, 1.0 / (double)s->N, q.st);
    }
    if (!rc) rc = cfp_stream_sync(q.st);
  } else if (own && s->rplan && cversion(s) == s->lam_version) {  // the real plan: 8-byte grid values end to end
    rc = cfp_rplan_apply(s->rplan, bin.ptr(), xout.ptr(), q.st);
  } else {  // the complex plan on the promoted b, real part out (x is real for a Hermitian symbol)
    rc = cfp_real_to_complex(bin.ptr(), s->zbuf, s->N, q.st);
    if (!rc && own) rc = cfp_plan_apply(s->cplan, s->zbuf, s->zbuf, q.st);
    if (!rc && !own) rc = cfp_half_spectrum_extend(din.ptr(), s->fbuf, s->dims[0], s->dims[1], s->dims[2], q.st);
    if (!rc && !own) rc = cfp_plan_apply_with_diag(s->cplan, s->fbuf, s->zbuf, s->zbuf, q.st);
    if (!rc) rc = cfp_complex_real_part(s->zbuf, xout.ptr(), s->N, 1.0, q.st);
  }
  // staged host sides, and the shared work buffers of the promoted path, need the result now
  if (!rc && (q.wait || bin.tmp || xout.tmp || din.tmp)) rc = cfp_stream_sync(q.st);
  PetscCall(xout.put());
  if (!own) PetscCall(din.put());
  PetscCall(bin.put());
  CFPCALL(rc);
  return PETSC_SUCCESS;
}

PetscErrorCode diag_is_own_symbol(RShell* s, Vec Diag, bool* own) {
  *own = false;
  if (!s->diag_id || s->diag_version != cversion(s)) return PETSC_SUCCESS;
  PetscObjectId id;
  PetscObjectState st;
  PetscCall(PetscObjectGetId((PetscObject)Diag, &id));
  PetscCall(PetscObjectStateGet((PetscObject)Diag, &st));
  *own = id == s->diag_id && st == s->diag_state;
  return PETSC_SUCCESS;
}

// the half-spectrum symbol 1 + sum_d lam_d c_d(k_d) on the host (c_d: the 1-D DFTs of the
// transport columns, from their closed form), planes kz in [z0, z0 + nzl)
std::vector<double> half_symbol(const PetscInt d[3], const double lam[3], PetscInt z0, PetscInt nzl) {
  const PetscInt nx = d[0], ny = d[1], M = nx / 2 + 1;
  std::vector<double> c[3];
  for (int a = 0; a < 3; ++a) {
    c[a].resize(2 * (size_t)d[a]);
    cfp_transport_symbol_1d(d[a], c[a].data());
  }
  std::vector<double> h(2 * (size_t)(M * ny * nzl));
  for (PetscInt kz = z0; kz < z0 + nzl; ++kz)
    for (PetscInt ky = 0; ky < ny; ++ky)
      for (PetscInt kx = 0; kx < M; ++kx) {
        const size_t i = 2 * (size_t)(((kz - z0) * ny + ky) * M + kx);
        h[i] = 1.0 + lam[0] * c[0][2 * kx] + lam[1] * c[1][2 * ky] + lam[2] * c[2][2 * kz];
        h[i + 1] = lam[0] * c[0][2 * kx + 1] + lam[1] * c[1][2 * ky + 1] + lam[2] * c[2][2 * kz + 1];
      }
  return h;
}

struct CtxExtra {
  Mat remapBack = nullptr;
};
std::mutex g_extra_mu;
std::unordered_map<const void*, CtxExtra> g_extra;
Mat ctx_remap_back(const FFTPrecTransportContext* ctx) {
  std::lock_guard<std::mutex> g(g_extra_mu);
  auto it = g_extra.find(ctx);
  return it == g_extra.end() ? nullptr : it->second.remapBack;
}
void ctx_forget(const FFTPrecTransportContext* ctx) {
  std::lock_guard<std::mutex> g(g_extra_mu);
  g_extra.erase(ctx);
}

}  // namespace

extern "C" PetscErrorCode FFTPrecTransportContextSetRemapBack(FFTPrecTransportContext* ctx, Mat remapBack) {
  PetscCheck(ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL context");
  std::lock_guard<std::mutex> g(g_extra_mu);
  if (remapBack) g_extra[ctx].remapBack = remapBack;
  else g_extra.erase(ctx);
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode FFTPrecTransportContextGetRemapBack(const FFTPrecTransportContext* ctx, Mat* remapBack) {
  PetscCheck(ctx && remapBack, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL argument");
  *remapBack = ctx_remap_back(ctx);
  return PETSC_SUCCESS;
}

// MatCreateFFT(comm, ndim, dims, MATFFTW) of a real-scalar PETSc (src/PCSHELLFft_3D.cxx:34-35):
// columns = the N reals of the grid, rows = the half spectrum's NS reals
extern "C" PetscErrorCode MatCreateFFTHIP(MPI_Comm comm, PetscInt ndim, const PetscInt dims[], Mat* A) {
  PetscCheck(ndim >= 1 && ndim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "ndim must be 1, 2 or 3");
  PetscCheck(dims && A, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL argument");
  int nranks = 1, rank = 0;
  PetscCallMPI(MPI_Comm_size(comm, &nranks));
  PetscCallMPI(MPI_Comm_rank(comm, &rank));
  RShell* s = new RShell;
  for (PetscInt d = 0; d < ndim; ++d) s->dims[d] = dims[ndim - 1 - d];  // row-major {n_z, n_y, n_x}
  s->N = s->dims[0] * s->dims[1] * s->dims[2];
  s->NS = 2 * (s->dims[0] / 2 + 1) * s->dims[1] * s->dims[2];
  s->nranks = nranks;
  s->rank = rank;
  s->nzl = s->dims[2];
  s->nl = s->N;
  s->nsl = s->NS;
  int dev = 0;
  hipGetDevice(&dev);
  if (nranks > 1) {  // this rank's z-slab of the complex slab plan (needs nranks | n_z)
    int64_t lay[8];
    int rc = cfp_slab_layout(s->dims[0], s->dims[1], s->dims[2], nranks, rank, lay);
    PetscErrorCode e = rc ? cfp_err(rc, "MatCreateFFTHIP") : slab_create(comm, nranks, rank, s->dims, dev, &s->slab);
    if (e) {
      slab_destroy(&s->slab);
      delete s;
      return e;
    }
    s->nzl = lay[0];
    s->z0 = lay[2];
    s->nl = lay[4];
    s->nsl = 2 * (s->dims[0] / 2 + 1) * s->dims[1] * s->nzl;
  } else {
    int rc = cfp_plan_create(&s->cplan, s->dims[0], s->dims[1], s->dims[2], dev);
    if (rc) {
      delete s;
      return cfp_err(rc, "MatCreateFFTHIP");
    }
    if (cfp_rplan_create(&s->rplan, s->dims[0], s->dims[1], s->dims[2], dev) != CFP_SUCCESS) s->rplan = nullptr;
  }
  PetscCall(MatCreateShell(comm, s->nsl, s->nl, s->NS, s->N, s, A));
  PetscCall(MatShellSetOperation(*A, MATOP_MULT, (void (*)(void))rfft_mult));
  PetscCall(MatShellSetOperation(*A, MATOP_MULT_TRANSPOSE, (void (*)(void))rfft_mult_transpose));
  PetscCall(MatShellSetOperation(*A, MATOP_DESTROY, (void (*)(void))rfft_destroy));
#ifdef CFP_WITH_PETSC
  PetscCall(PetscObjectComposeFunction((PetscObject)*A, "MatCreateVecsFFTW_C", rfft_create_vecs));
#endif
  return PETSC_SUCCESS;
}

// the complex plan behind the real FFT matrix (its symbol setters reach solve_3D's own path)
extern "C" PetscErrorCode MatFFTHIPGetPlan(Mat A, cfp_plan_t* plan) {
  RShell* s;
  PetscCall(rshell(A, &s));
  *plan = s->cplan;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatFFTHIPGetDistPlan(Mat A, struct cfp_dist_plan_s** plan) {
  RShell* s;
  PetscCall(rshell(A, &s));
  *plan = s->slab.plan;
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode MatFFTHIPGetSolveCounts(Mat A, PetscInt* own_symbol, PetscInt* explicit_diag) {
  RShell* s;
  PetscCall(rshell(A, &s));
  if (own_symbol) *own_symbol = s->solves_own;
  if (explicit_diag) *explicit_diag = s->solves_diag;
  return PETSC_SUCCESS;
}
// real-scalar build only: the real plan behind the matrix (NULL where it lacks the grid)
extern "C" PetscErrorCode MatFFTHIPGetRealPlan(Mat A, cfp_rplan_t* plan) {
  RShell* s;
  PetscCall(rshell(A, &s));
  *plan = s->rplan;
  return PETSC_SUCCESS;
}

// build_transport_col, src/FftLinearSolver_3D.c:80-90
extern "C" PetscErrorCode build_transport_col(Vec c, PetscInt size) {
  PetscFunctionBeginUser;
  PetscCall(VecSet(c, 0.0));
  if (size > 1) {
    PetscCall(VecSetValue(c, 0, 1.0, INSERT_VALUES));
    PetscCall(VecSetValue(c, 1, -1.0, INSERT_VALUES));
  }
  PetscCall(VecAssemblyBegin(c));
  PetscCall(VecAssemblyEnd(c));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// build_diag_mat_vec_3D, :136-164, real scalars: the c_d_hat are the 1-D r2c half spectra
// (2 (n_d/2 + 1) reals, a 1-D real MATFFTW's MatMult of build_transport_col), Diag the 3-D half
// spectrum; the mirrored halves of c_y, c_z come from c(n - k) = conj c(k).
extern "C" PetscErrorCode build_diag_mat_vec_3D(Vec Diag, Vec cx, Vec cy, Vec cz, PetscInt nx, PetscInt ny,
                                                PetscInt nz, PetscScalar lx, PetscScalar ly, PetscScalar lz) {
  PetscFunctionBeginUser;
  const PetscInt M = nx / 2 + 1;
  // a distributed Diag holds its rank's whole z-planes of the half spectrum
  PetscInt Ng, nloc, lo;
  PetscCall(VecGetSize(Diag, &Ng));
  PetscCall(VecGetLocalSize(Diag, &nloc));
  PetscCall(VecGetOwnershipRange(Diag, &lo, NULL));
  PetscCheck(Ng == 2 * M * ny * nz, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ,
             "build_diag_mat_vec_3D: Diag size != 2 (n_x/2 + 1) n_y n_z");
  PetscCheck(lo % (2 * M * ny) == 0 && nloc % (2 * M * ny) == 0, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ,
             "build_diag_mat_vec_3D: a distributed Diag must hold whole z-planes");
  const PetscInt z0 = lo / (2 * M * ny), nzl = nloc / (2 * M * ny);
  PetscCall(check_size(cx, 2 * (nx / 2 + 1), "build_diag_mat_vec_3D: c_x_hat size != 2 (n_x/2 + 1)"));
  PetscCall(check_size(cy, 2 * (ny / 2 + 1), "build_diag_mat_vec_3D: c_y_hat size != 2 (n_y/2 + 1)"));
  PetscCall(check_size(cz, 2 * (nz / 2 + 1), "build_diag_mat_vec_3D: c_z_hat size != 2 (n_z/2 + 1)"));
  const PetscScalar *ax, *ay, *az;
  PetscCall(VecGetArrayRead(cx, &ax));
  PetscCall(VecGetArrayRead(cy, &ay));
  PetscCall(VecGetArrayRead(cz, &az));
  const auto full = [](const PetscScalar* c, PetscInt n, PetscInt k) {
    return k <= n / 2 ? std::complex<double>(c[2 * k], c[2 * k + 1])
                      : std::complex<double>(c[2 * (n - k)], -c[2 * (n - k) + 1]);
  };
  PetscScalar* d;
  PetscCall(VecGetArrayWrite(Diag, &d));
  for (PetscInt kz = z0; kz < z0 + nzl; ++kz)
    for (PetscInt ky = 0; ky < ny; ++ky)
      for (PetscInt kx = 0; kx < M; ++kx) {
        const std::complex<double> v = 1.0 + lx * full(ax, nx, kx) + ly * full(ay, ny, ky) + lz * full(az, nz, kz);
        const size_t i = 2 * (size_t)(((kz - z0) * ny + ky) * M + kx);
        d[i] = v.real();
        d[i + 1] = v.imag();
      }
  PetscCall(VecRestoreArrayWrite(Diag, &d));
  PetscCall(VecRestoreArrayRead(cz, &az));
  PetscCall(VecRestoreArrayRead(cy, &ay));
  PetscCall(VecRestoreArrayRead(cx, &ax));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// solve_3D, :166-190 (real scalars): X = (1/size) c2r( r2c(b) ./ Diag ) -- the correct real
// solve (see the file header for the reference's loop bound and 2/size); b_hat is untouched.
extern "C" PetscErrorCode solve_3D(Mat FFT_MAT, Vec X, Vec Diag, Vec b, Vec b_hat, PetscInt size) {
  PetscFunctionBeginUser;
  (void)b_hat;
  RShell* s;
  PetscCall(rshell(FFT_MAT, &s));
  PetscCheck(size == s->N, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ, "solve_3D: size != number of grid cells of FFT_MAT");
  PetscCall(check_size(X, s->nl, "solve_3D: X has the wrong size"));
  PetscCall(check_size(b, s->nl, "solve_3D: b has the wrong size"));
  PetscCall(check_size(Diag, s->nsl, "solve_3D: Diag has the wrong size (2 (n_x/2 + 1) n_y n_z reals)"));
  bool own = false;
  PetscCall(diag_is_own_symbol(s, Diag, &own));
  if (s->slab.plan) {  // every rank takes the same path (the apply holds collectives)
    double f = own ? 0.0 : 1.0;
    PetscCall(comm_max(s->slab.comm, s->nranks, &f, 1));
    own = f == 0.0;
  }
  ++(own ? s->solves_own : s->solves_diag);
  PetscCall(rshell_apply(s, X, b, own, Diag));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// FftTransportSolver, :218-264 (the symbol of real lambdas, cached; FFT_MAT survives)
extern "C" PetscErrorCode FftTransportSolver(PetscInt nx, PetscInt ny, PetscInt nz, PetscScalar lx, PetscScalar ly,
                                             PetscScalar lz, Vec X, Vec b, Mat FFT_MAT) {
  PetscFunctionBeginUser;
  RShell* s;
  PetscCall(rshell(FFT_MAT, &s));
  PetscCheck(s->dims[0] == nx && s->dims[1] == ny && s->dims[2] == nz, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ,
             "FftTransportSolver: grid dims do not match FFT_MAT");
  const double lam[3] = {lx, ly, lz};
  PetscCall(ensure_transport_symbol(s, lam));
  PetscCall(check_size(X, s->nl, "FftTransportSolver: X has the wrong size"));
  PetscCall(check_size(b, s->nl, "FftTransportSolver: b has the wrong size"));
  PetscCall(rshell_apply(s, X, b, true, nullptr));
  PetscFunctionReturn(PETSC_SUCCESS);
}
// :266-281
extern "C" PetscErrorCode Fft3DTransportSolver(PetscInt nx, PetscInt ny, PetscInt nz, PetscScalar ax, PetscScalar ay,
                                               PetscScalar az, PetscScalar dt, PetscScalar dx, PetscScalar dy,
                                               PetscScalar dz, Vec X, Vec b, Mat FFT_MAT) {
  PetscFunctionBeginUser;
  PetscCall(FftTransportSolver(nx, ny, nz, ax * dt / dx, ay * dt / dy, az * dt / dz, X, b, FFT_MAT));
  PetscFunctionReturn(PETSC_SUCCESS);
}
// :283-290
extern "C" PetscErrorCode Fft2DTransportSolver(PetscInt nx, PetscInt ny, PetscScalar ax, PetscScalar ay,
                                               PetscScalar dt, PetscScalar dx, PetscScalar dy, Vec X, Vec b,
                                               Mat FFT_MAT) {
  PetscFunctionBeginUser;
  PetscCall(Fft3DTransportSolver(nx, ny, 1, ax, ay, 0.0, dt, dx, dy, 1.0, X, b, FFT_MAT));
  PetscFunctionReturn(PETSC_SUCCESS);
}
// :292-301
extern "C" PetscErrorCode Fft1DTransportSolver(PetscInt nx, PetscScalar ax, PetscScalar dt, PetscScalar dx, Vec X,
                                               Vec b, Mat FFT_MAT) {
  PetscFunctionBeginUser;
  PetscCall(Fft3DTransportSolver(nx, 1, 1, ax, 0.0, 0.0, dt, dx, 1.0, 1.0, X, b, FFT_MAT));
  PetscFunctionReturn(PETSC_SUCCESS);
}
// :303-312 (context by value, as the reference)
extern "C" PetscErrorCode PetscFft3DTransportSolver(struct StructuredTransportContext c, Vec b, Vec x) {
  PetscFunctionBeginUser;
  PetscCall(Fft3DTransportSolver(c.n_x, c.n_y, c.n_z, c.a_x, c.a_y, c.a_z, c.dt, c.delta_x, c.delta_y, c.delta_z, x,
                                 b, c.FFT_MAT));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// applyFFT3DPrecTransport, src/PCSHELLFft_3D.cxx:10-24
extern "C" PetscErrorCode applyFFT3DPrecTransport(PC pc, Vec b, Vec x) {
  PetscFunctionBeginUser;
  FFTPrecTransportContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  PetscCheck(ctx && ctx->FFT_MAT && ctx->Diag, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONGSTATE,
             "applyFFT3DPrecTransport: setupFFTPrec3D has not run");
  const PetscInt N = ctx->n_x * ctx->n_y * ctx->n_z;
  cfp_apply_stamp_clear();  // the stand-in KSP times this apply by its events (not a 3-sweep-only apply)
  Vec src = b;
  if (ctx->intersectionMatrix) {  // mesh -> Cartesian remap (identity when NULL)
    PetscCall(MatMult(ctx->intersectionMatrix, b, ctx->b_cartesien));
    src = ctx->b_cartesien;
  }
  if (Mat back = ctx_remap_back(ctx)) {
    if (src != ctx->b_cartesien) PetscCall(VecCopy(src, ctx->b_cartesien));
    PetscCall(solve_3D(ctx->FFT_MAT, ctx->b_cartesien, ctx->Diag, ctx->b_cartesien, ctx->b_hat, N));
    PetscCall(MatMult(back, ctx->b_cartesien, x));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  PetscCall(solve_3D(ctx->FFT_MAT, x, ctx->Diag, src, ctx->b_hat, N));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// PCShellSetApplyBA callback (include/pcshell_fft3d.h): real scalars have no fused form, so this is
// PETSc's PCApplyBAorAB without an applyBA -- MatMult with the PC's operator, then the apply
extern "C" PetscErrorCode applyFFT3DPrecTransportBA(PC pc, PCSide side, Vec x, Vec y, Vec work) {
  PetscFunctionBeginUser;
  Mat A = nullptr;
  PetscCall(PCGetOperators(pc, &A, NULL));
  PetscCheck(A, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONGSTATE, "applyFFT3DPrecTransportBA: the PC has no operator");
  if (side == PC_LEFT) {
    PetscCall(MatMult(A, x, work));
    PetscCall(applyFFT3DPrecTransport(pc, work, y));
  } else {
    PetscCheck(side == PC_RIGHT, PETSC_COMM_SELF, PETSC_ERR_SUP, "applyFFT3DPrecTransportBA: left or right preconditioning");
    PetscCall(applyFFT3DPrecTransport(pc, x, work));
    PetscCall(MatMult(A, work, y));
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

// setupFFTPrec3D, :26-84 (real scalars: Diag and b_hat are half spectra, b_cartesien N reals)
extern "C" PetscErrorCode setupFFTPrec3D(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecTransportContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  PetscCheck(ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "setupFFTPrec3D: no context attached to the PC");
  PetscCheck(ctx->n_x >= 1 && ctx->n_y >= 1 && ctx->n_z >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE,
             "setupFFTPrec3D: n_x, n_y, n_z must be >= 1");
  const PetscInt dims[3] = {ctx->n_z, ctx->n_y, ctx->n_x};
  PetscCall(MatCreateFFTHIP(PETSC_COMM_WORLD, 3, dims, &ctx->FFT_MAT));
  PetscCall(MatCreateVecsFFTW(ctx->FFT_MAT, NULL, &ctx->Diag, NULL));
  PetscCall(MatCreateVecsFFTW(ctx->FFT_MAT, &ctx->b_cartesien, &ctx->b_hat, NULL));
  RShell* s;
  PetscCall(rshell(ctx->FFT_MAT, &s));
  const double lam[3] = {ctx->lambda_x, ctx->lambda_y, ctx->lambda_z};
  PetscCall(ensure_transport_symbol(s, lam));
  const std::vector<double> h = half_symbol(s->dims, lam, s->z0, s->nzl);
  PetscScalar* d;
  PetscCall(VecGetArrayWrite(ctx->Diag, &d));
  std::memcpy(d, h.data(), sizeof(double) * h.size());
  PetscCall(VecRestoreArrayWrite(ctx->Diag, &d));
  PetscCall(PetscObjectGetId((PetscObject)ctx->Diag, &s->diag_id));
  PetscCall(PetscObjectStateGet((PetscObject)ctx->Diag, &s->diag_state));
  s->diag_version = cversion(s);
  PetscFunctionReturn(PETSC_SUCCESS);
}

// destroyFFTPrec3D, :86-99
extern "C" PetscErrorCode destroyFFTPrec3D(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecTransportContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  if (!ctx) PetscFunctionReturn(PETSC_SUCCESS);
  PetscCall(VecDestroy(&ctx->Diag));
  PetscCall(VecDestroy(&ctx->b_cartesien));
  PetscCall(VecDestroy(&ctx->b_hat));
  PetscCall(MatDestroy(&ctx->FFT_MAT));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// getFFTPrec3DContext, :101-151 (fills the caller's ctx; lambda formula kept as the reference's)
extern "C" PetscErrorCode getFFTPrec3DContext(PetscInt ndim, PetscScalar dt, PetscInt nbCells, PetscScalar a_x,
                                              PetscScalar a_y, PetscScalar a_z, PetscScalar Xmin, PetscScalar Ymin,
                                              PetscScalar Zmin, PetscScalar Xmax, PetscScalar Ymax, PetscScalar Zmax,
                                              FFTPrecTransportContext* ctx) {
  PetscFunctionBeginUser;
  PetscCheck(ndim > 0 && ndim < 4, PETSC_COMM_WORLD, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  PetscCheck(ctx, PETSC_COMM_WORLD, PETSC_ERR_ARG_NULL, "getFFTPrec3DContext: ctx is NULL");
  PetscInt nx = nbCells, ny = 1, nz = 1;
  if (ndim == 3) nx = ny = nz = (PetscInt)std::floor(std::cbrt((double)nbCells));
  else if (ndim == 2) nx = ny = (PetscInt)std::floor(std::sqrt((double)nbCells));
  std::memset((void*)ctx, 0, sizeof(*ctx));
  ctx_forget(ctx);
  ctx->spaceDim = ndim;
  ctx->n_x = nx;
  ctx->n_y = ny;
  ctx->n_z = nz;
  ctx->lambda_x = a_x * dt * (Xmax - Xmin) / (double)nx;
  ctx->lambda_y = a_y * dt * (Ymax - Ymin) / (double)ny;
  ctx->lambda_z = a_z * dt * (Zmax - Zmin) / (double)nz;
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" FFTPrecTransportContext* FFTPrecTransportContextLast(void) {
  static FFTPrecTransportContext last{};
  return &last;
}

extern "C" PetscErrorCode FFTPrecTransportContextCreate(FFTPrecTransportContext** ctx) {
  PetscCheck(ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL output");
  *ctx = new FFTPrecTransportContext;
  std::memset((void*)*ctx, 0, sizeof(**ctx));
  return PETSC_SUCCESS;
}
extern "C" PetscErrorCode FFTPrecTransportContextDestroy(FFTPrecTransportContext** ctx) {
  if (ctx && *ctx) {
    ctx_forget(*ctx);
    delete *ctx;
    *ctx = nullptr;
  }
  return PETSC_SUCCESS;
}
