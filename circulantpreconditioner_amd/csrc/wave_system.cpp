// wave_system.cpp -- the wave-system operator on a Cartesian grid, the block-circulant PCSHELL
// and the implicit GMRES time loop (include/wave_system.h).
//
//   cfp_wave_csr                    computeDivergenceMatrix + jacobianMatrices,
//                                   src/WaveSystem.cxx:92-176
//   initial_conditions_shock_wave   src/WaveSystem.cxx:25-76
//   WaveSystemGMRES                 WaveSystem_impl_seq, tests/WaveSystem_SphericalExplosion_
//                                   impl_seq.cxx:11-150 (GMRES rtol = abstol = 1e-5, 1000 its),
//                                   with the block-circulant PCSHELL in place of PCILU
#ifndef CFP_WITH_PETSC
#include <sys/time.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/transport_equation.h"
#include "../../include/wave_system.h"
#include "pcshell_common.h"

using namespace cfp_pc;

namespace {
const int kC = 4;  // most unknowns per cell (3-D: pressure, 3 momentum components)

double wall() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

// jacobianMatrices(normal = s e_d, coeff = kappa): (A(n) - |A(n)|) kappa / 2,
// A(n) = [[0, c0^2 n^T], [n, 0]], |A(n)| = diag(c0, c0 n n^T)   (src/WaveSystem.cxx:92-107)
void jacobian_minus(int d, int s, double kappa, double c0, double Am[kC][kC]) {
  for (int r = 0; r < kC; ++r)
    for (int c = 0; c < kC; ++c) Am[r][c] = 0.0;
  const double h = 0.5 * kappa;
  Am[0][0] = -h * c0;
  Am[0][1 + d] = h * c0 * c0 * s;
  Am[1 + d][0] = h * s;
  Am[1 + d][1 + d] = -h * c0;
}

struct Entry {
  int64_t col;
  double val;
};
}  // namespace

extern "C" int cfp_wave_csr_dim(int64_t nx, int64_t ny, int64_t nz, int dim, const double h[3], double dt, double c0,
                                int bc, double shift, int64_t* rowptr, int64_t* col, double* val, int64_t* nnz) {
  if (!h || !rowptr || !col || !val || !nnz) return CFP_ERR_ARG_NULL;
  if (nx < 1 || ny < 1 || nz < 1 || h[0] <= 0 || h[1] <= 0 || h[2] <= 0 || !(c0 > 0)) return CFP_ERR_ARG_OUTOFRANGE;
  if (bc != CFP_WAVE_BC_WALL && bc != CFP_WAVE_BC_PERIODIC && bc != CFP_WAVE_BC_NEUMANN) return CFP_ERR_ARG_OUTOFRANGE;
  if (dim < 1 || dim > 3) return CFP_ERR_ARG_OUTOFRANGE;
  if ((dim < 3 && nz != 1) || (dim < 2 && ny != 1)) return CFP_ERR_ARG_SIZ;
  const int C = dim + 1;  // nbComp (src/WaveSystem.cxx:113)
  const int64_t n[3] = {nx, ny, nz};
  int64_t p = 0;
  rowptr[0] = 0;
  // one cell at a time: its (at most 2 dim + 1) coupled cells and their C x C blocks
  std::vector<Entry> row[kC];
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j)
      for (int64_t i = 0; i < nx; ++i) {
        const int64_t cell = i + nx * (j + ny * k);
        const int64_t idx[3] = {i, j, k};
        double self[kC][kC];
        for (int r = 0; r < kC; ++r)
          for (int c = 0; c < kC; ++c) self[r][c] = r == c ? shift : 0.0;
        for (int r = 0; r < kC; ++r) row[r].clear();
        for (int d = 0; d < dim; ++d) {  // a dim-D mesh has faces along its dim axes only
          const double kappa = dt / h[d];  // dt |F| / |C|
          for (int s = -1; s <= 1; s += 2) {
            double Am[kC][kC];
            jacobian_minus(d, s, kappa, c0, Am);
            const bool border = s < 0 ? idx[d] == 0 : idx[d] == n[d] - 1;
            int64_t other = -1;
            if (!border) {
              other = cell + s * (d == 0 ? 1 : (d == 1 ? nx : nx * ny));
            } else if (bc == CFP_WAVE_BC_PERIODIC) {
              const int64_t wrap = s < 0 ? n[d] - 1 : 0;
              int64_t o[3] = {i, j, k};
              o[d] = wrap;
              other = o[0] + nx * (o[1] + ny * o[2]);
            } else if (bc == CFP_WAVE_BC_WALL) {
              // -Am (2 v v^T), v = (0, n): only column 1+d is hit (src/WaveSystem.cxx:148-155)
              for (int r = 0; r < C; ++r) self[r][1 + d] -= 2.0 * Am[r][1 + d];
              continue;
            } else {
              continue;  // Neumann: nothing
            }
            for (int r = 0; r < C; ++r)
              for (int c = 0; c < C; ++c) {
                if (Am[r][c] == 0.0) continue;
                row[r].push_back({other * C + c, Am[r][c]});  // addValue(j, other, Am)
                self[r][c] -= Am[r][c];                         // addValue(j, j, -Am)
              }
          }
        }
        for (int r = 0; r < C; ++r) {
          for (int c = 0; c < C; ++c)
            if (self[r][c] != 0.0 || c == r) row[r].push_back({cell * C + c, self[r][c]});
          std::vector<Entry>& e = row[r];
          std::sort(e.begin(), e.end(), [](const Entry& a, const Entry& b) { return a.col < b.col; });
          // merge duplicates (periodic wrap on a 1- or 2-cell axis), keep the diagonal
          int64_t start = p;
          for (size_t q = 0; q < e.size(); ++q) {
            if (p > start && col[p - 1] == e[q].col) {
              val[2 * (p - 1)] += e[q].val;
            } else {
              col[p] = e[q].col;
              val[2 * p] = e[q].val;
              val[2 * p + 1] = 0.0;
              ++p;
            }
          }
          // drop exact zeros except the diagonal
          int64_t w = start;
          for (int64_t q = start; q < p; ++q) {
            if (val[2 * q] != 0.0 || col[q] == cell * C + r) {
              col[w] = col[q];
              val[2 * w] = val[2 * q];
              val[2 * w + 1] = 0.0;
              ++w;
            }
          }
          p = w;
          rowptr[cell * C + r + 1] = p;
        }
      }
  *nnz = p;
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_csr(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, double c0, int bc,
                            double shift, int64_t* rowptr, int64_t* col, double* val, int64_t* nnz) {
  return cfp_wave_csr_dim(nx, ny, nz, 3, h, dt, c0, bc, shift, rowptr, col, val, nnz);
}

extern "C" PetscErrorCode computeDivergenceMatrixWaveCartesianDim(PetscInt nx, PetscInt ny, PetscInt nz, PetscInt dim,
                                                                  const PetscReal h[3], PetscReal dt, PetscReal c0,
                                                                  PetscInt bc, Mat* A) {
  PetscFunctionBeginUser;
  PetscCheck(A && h, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "computeDivergenceMatrixWaveCartesian: NULL argument");
  PetscCheck(nx >= 1 && ny >= 1 && nz >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  PetscCheck(dim >= 1 && dim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  const int C = (int)dim + 1;
  const int64_t M = C * nx * ny * nz;
  const int64_t room = (int64_t)C * C * (2 * dim + 1);
  std::vector<int64_t> rowptr((size_t)M + 1), col((size_t)(nx * ny * nz * room));
  std::vector<PetscScalar> val((size_t)(nx * ny * nz * room));
  int64_t nnz = 0;
  const int rc = cfp_wave_csr_dim(nx, ny, nz, (int)dim, h, dt, c0, (int)bc, 0.0, rowptr.data(), col.data(),
                                  reinterpret_cast<double*>(val.data()), &nnz);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, "computeDivergenceMatrixWaveCartesian: bad arguments");
  PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, M, M, rowptr.data(), col.data(), val.data(), A));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode computeDivergenceMatrixWaveCartesian(PetscInt nx, PetscInt ny, PetscInt nz,
                                                               const PetscReal h[3], PetscReal dt, PetscReal c0,
                                                               PetscInt bc, Mat* A) {
  return computeDivergenceMatrixWaveCartesianDim(nx, ny, nz, 3, h, dt, c0, bc, A);
}

extern "C" PetscErrorCode initial_conditions_shock_wave(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal xmin[3],
                                                        const PetscReal xmax[3], Vec U) {
  PetscFunctionBeginUser;
  PetscCheck(xmin && xmax, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL domain bounds");
  PetscInt n;
  PetscCall(VecGetLocalSize(U, &n));
  const PetscInt N = nx * ny * nz;
  PetscCheck(N >= 1 && n % N == 0 && n / N >= 2 && n / N <= kC, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ,
             "U size is not (dim+1)*nx*ny*nz with dim = 1, 2 or 3");
  const int C = (int)(n / N), dim = C - 1;  // nbComp = dim + 1
  const double hx = (xmax[0] - xmin[0]) / (double)nx, hy = (xmax[1] - xmin[1]) / (double)ny,
               hz = (xmax[2] - xmin[2]) / (double)nz;
  const double cx = (xmin[0] + xmax[0]) / 2, cy = (xmin[1] + xmax[1]) / 2, cz = (xmin[2] + xmax[2]) / 2;
  PetscScalar* u;
  PetscCall(VecGetArrayWrite(U, &u));
  for (PetscInt k = 0; k < nz; ++k)
    for (PetscInt j = 0; j < ny; ++j)
      for (PetscInt i = 0; i < nx; ++i) {
        const double x = xmin[0] + (i + 0.5) * hx, y = xmin[1] + (j + 0.5) * hy, z = xmin[2] + (k + 0.5) * hz;
        // src/WaveSystem.cxx:48-61: y enters r for dim > 1, z for dim == 3 (a single cell
        // layer's centre is the domain centre, so a 3-D grid with n = 1 adds 0)
        double r2 = (x - cx) * (x - cx);
        if (dim > 1 && ny > 1) r2 += (y - cy) * (y - cy);
        if (dim == 3 && nz > 1) r2 += (z - cz) * (z - cz);
        const int64_t c = C * (i + nx * (j + ny * k));
        u[c] = std::sqrt(r2) < 0.3 ? 155e5 : 70e5;
        for (int d = 1; d < C; ++d) u[c + d] = 0.0;  // rho0 * velocity, velocity = 0
      }
  PetscCall(VecRestoreArrayWrite(U, &u));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// ------------------------------------------------------------------ PCSHELL
extern "C" PetscErrorCode setupFFTPrec3DWave(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  PetscCheck(ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "setupFFTPrec3DWave: no context attached to the PC");
  PetscCheck(ctx->n_x >= 1 && ctx->n_y >= 1 && ctx->n_z >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE,
             "setupFFTPrec3DWave: n_x, n_y, n_z must be >= 1");
  int dev = 0;
  PetscCheck(hipGetDevice(&dev) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_LIB, "no HIP device");
  if (ctx->plan) CFPCALL(cfp_wave_plan_destroy(ctx->plan));
  ctx->plan = nullptr;
  const int dim = ctx->dim ? (int)ctx->dim : 3;
  CFPCALL(cfp_wave_plan_create_dim(&ctx->plan, ctx->n_x, ctx->n_y, ctx->n_z, dim, dev));
  const double kappa[3] = {ctx->kappa_x, ctx->kappa_y, ctx->kappa_z};
  CFPCALL(cfp_wave_plan_set_symbol(ctx->plan, kappa, ctx->c0));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode applyFFT3DPrecWave(PC pc, Vec b, Vec x) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  PetscCheck(ctx && ctx->plan, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONGSTATE, "applyFFT3DPrecWave: setup has not run");
  const PetscInt M = ((ctx->dim ? ctx->dim : 3) + 1) * ctx->n_x * ctx->n_y * ctx->n_z;
  PetscCall(check_size(b, M, "applyFFT3DPrecWave: b has the wrong size"));
  PetscCall(check_size(x, M, "applyFFT3DPrecWave: x has the wrong size"));
  DevIn in;
  DevOut out;
  PetscCall(in.get(b, M));
  PetscCall(out.get(x, M));
  // device Vecs: ordered on the Vec stream without a host round trip (cfp_pc::device_stream);
  // a staged host Vec is waited for (its buffers are copied back / freed below)
  void* st = nullptr;
  bool wait = true;
  if (!in.tmp && !out.tmp) device_stream(&st, &wait);
  int rc = cfp_wave_plan_apply(ctx->plan, in.ptr(), out.ptr(), st);
  if (rc == CFP_SUCCESS && (wait || in.tmp || out.tmp)) rc = cfp_stream_sync(st);
  PetscCall(out.put());
  PetscCall(in.put());
  CFPCALL(rc);
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode destroyFFTPrec3DWave(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  if (ctx && ctx->plan) {
    CFPCALL(cfp_wave_plan_destroy(ctx->plan));
    ctx->plan = nullptr;
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

// ------------------------------------------------------------------ time loop
extern "C" void cfp_wave_config_default(cfp_wave_config* cfg, int64_t n) {
  if (!cfg) return;
  std::memset((void*)cfg, 0, sizeof(*cfg));
  cfg->nx = cfg->ny = cfg->nz = n;
  for (int d = 0; d < 3; ++d) {
    cfg->xmin[d] = -0.5;
    cfg->xmax[d] = 0.5;
  }
  cfg->c0 = 700.0;
  cfg->cfl = 1.0e3 / 3.0;
  cfg->tmax = 0.05;
  cfg->ntmax = 2000000;
  cfg->precision = 1e-5;
  cfg->max_its = 1000;
  cfg->restart = 30;
  cfg->pc = CFP_WAVE_PC_FFT;
  cfg->bc = CFP_WAVE_BC_WALL;
  cfg->pc_side = PC_LEFT;
  cfg->on_device = 1;
  cfg->dim = 3;
}

extern "C" void cfp_wave_config_default_dim(cfp_wave_config* cfg, int64_t n, int dim) {
  if (!cfg) return;
  cfp_wave_config_default(cfg, n);
  if (dim < 1 || dim > 3) return;
  cfg->dim = dim;
  if (dim < 3) cfg->nz = 1;
  if (dim < 2) cfg->ny = 1;
  cfg->cfl = 1.0e3 / (double)dim;  // main: cfl = 1e3 / getSpaceDimension()
}

extern "C" PetscErrorCode WaveSystemGMRES(const cfp_wave_config* cfg, cfp_wave_result* res, double* U_out) {
  PetscFunctionBeginUser;
  PetscCheck(cfg && res, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "WaveSystemGMRES: NULL argument");
  PetscCheck(cfg->pc == CFP_WAVE_PC_NONE || cfg->on_device, PETSC_COMM_SELF, PETSC_ERR_SUP,
             "the block-circulant preconditioner runs on HIP vectors only");
  std::memset((void*)res, 0, sizeof(*res));
  const double t_setup = wall();
  const int dim = cfg->dim ? cfg->dim : 3;
  PetscCheck(dim >= 1 && dim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  const PetscInt nx = cfg->nx, ny = cfg->ny, nz = cfg->nz, M = (dim + 1) * nx * ny * nz;
  const double h[3] = {(cfg->xmax[0] - cfg->xmin[0]) / (double)nx, (cfg->xmax[1] - cfg->xmin[1]) / (double)ny,
                       (cfg->xmax[2] - cfg->xmin[2]) / (double)nz};
  // dt = cfl * minRatioVolSurf / c0 (impl_seq.cxx:18,73): cell measure over its faces' measure
  const double dt = cfg->cfl * cfp_cartesian_min_ratio_vol_surf(dim, h) / cfg->c0;
  res->dt = dt;
  for (int d = 0; d < 3; ++d) res->kappa[d] = d < dim ? dt / h[d] : 0.0;

  Vec Un, dUn;
  if (cfg->on_device) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, M, &Un));
  else PetscCall(VecCreateSeq(PETSC_COMM_SELF, M, &Un));
  PetscCall(VecDuplicate(Un, &dUn));
  PetscCall(initial_conditions_shock_wave(nx, ny, nz, cfg->xmin, cfg->xmax, Un));
  Mat A;
  PetscCall(computeDivergenceMatrixWaveCartesianDim(nx, ny, nz, dim, h, dt, cfg->c0, cfg->bc, &A));
  PetscCall(MatShift(A, 1.0));  // :86

  KSP ksp;
  PC pc;
  PetscCall(KSPCreate(PETSC_COMM_WORLD, &ksp));
  PetscCall(KSPSetType(ksp, KSPGMRES));
  PetscCall(KSPSetTolerances(ksp, cfg->precision, cfg->precision, PETSC_DEFAULT, cfg->max_its));
  PetscCall(KSPGMRESSetRestart(ksp, cfg->restart > 0 ? cfg->restart : 30));
  PetscCall(KSPSetPCSide(ksp, (PCSide)cfg->pc_side));
  PetscCall(KSPGetPC(ksp, &pc));
  FFTPrecWaveContext ctx;
  std::memset((void*)&ctx, 0, sizeof(ctx));
  if (cfg->pc == CFP_WAVE_PC_FFT) {
    ctx.n_x = nx;
    ctx.n_y = ny;
    ctx.n_z = nz;
    ctx.kappa_x = res->kappa[0];
    ctx.kappa_y = res->kappa[1];
    ctx.kappa_z = res->kappa[2];
    ctx.c0 = cfg->c0;
    ctx.dim = dim;
    PetscCall(PCSetType(pc, PCSHELL));
    PetscCall(PCShellSetContext(pc, &ctx));
    PetscCall(PCShellSetSetUp(pc, setupFFTPrec3DWave));
    PetscCall(PCShellSetApply(pc, applyFFT3DPrecWave));
    PetscCall(PCShellSetDestroy(pc, destroyFFTPrec3DWave));
    PetscCall(PCShellSetName(pc, "block-circulant FFT (HIP)"));
  } else {
    PetscCall(PCSetType(pc, PCNONE));
  }
  PetscCall(KSPSetOperators(ksp, A, A));
  PetscCall(KSPSetUp(ksp));
  PetscCall(KSPMiniSetUpWork(ksp, Un));
  PetscCall(MatMult(A, Un, dUn));  // device copy of A made outside the timed solves
  if (cfg->on_device)
    PetscCheck(cfp_stream_sync(nullptr) == CFP_SUCCESS, PETSC_COMM_SELF, PETSC_ERR_LIB, "stream sync failed");
  res->setup_seconds = wall() - t_setup;

  int64_t it = 0;
  double time = 0.0;
  bool stationary = false;
  res->all_converged = 1;
  res->min_step_its = -1;
  while (it < cfg->ntmax && time <= cfg->tmax && !stationary) {  // :95
    PetscCall(VecCopy(Un, dUn));
    const double v = wall();
    PetscCall(KSPSolve(ksp, Un, Un));
    const double w = wall();
    PetscCall(VecAXPY(dUn, -1.0, Un));
    time += dt;
    it += 1;
    PetscReal norm;
    PetscCall(VecNorm(dUn, NORM_2, &norm));
    stationary = norm < cfg->precision;
    KSPConvergedReason reason;
    PetscInt its;
    PetscReal residu;
    PetscCall(KSPGetConvergedReason(ksp, &reason));
    PetscCall(KSPGetIterationNumber(ksp, &its));
    PetscCall(KSPGetResidualNorm(ksp, &residu));
    PetscInt calls;
    PetscLogDouble pcs;
    PetscCall(KSPMiniGetPCApplyStats(ksp, &calls, &pcs));
    res->solve_seconds += w - v;
    res->pc_seconds += pcs;
    res->pc_calls += calls;
    res->total_its += its;
    res->max_step_its = std::max<int64_t>(res->max_step_its, its);
    res->min_step_its = res->min_step_its < 0 ? its : std::min<int64_t>(res->min_step_its, its);
    res->last_reason = (int)reason;
    res->last_residual = residu;
    res->last_norm_dU = norm;
    if (reason != KSP_CONVERGED_RTOL && reason != KSP_CONVERGED_ATOL) res->all_converged = 0;
  }
  res->steps = it;
  res->time = time;
  if (U_out) {
    const PetscScalar* u;
    PetscCall(VecGetArrayRead(Un, &u));
    std::memcpy(U_out, (const void*)u, sizeof(double) * 2 * (size_t)M);
    PetscCall(VecRestoreArrayRead(Un, &u));
  }
  PetscCall(KSPDestroy(&ksp));
  PetscCall(MatDestroy(&A));
  PetscCall(VecDestroy(&Un));
  PetscCall(VecDestroy(&dUn));
  PetscFunctionReturn(PETSC_SUCCESS);
}
#endif  // CFP_WITH_PETSC
