// transport_cartesian.cpp -- implicit upwind transport operator on a Cartesian grid and the
// GMRES time loop of the reference's transport driver, with the circulant FFT PCSHELL wired
// into the KSP.
//
//   cfp_transport_csr                  computeDivergenceMatrix, src/TransportEquation.cxx:75-133
//   initial_conditions_shock_cartesian initial_conditions_shock, src/TransportEquation.cxx:25-73
//   TransportEquationGMRES             TransportEquation_impl_mpi,
//                                      tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:13-189,
//                                      plus the PCSHELL registration ToDo.md:1 asks for
//
// The operator is assembled on the host once (a 7-point CSR), handed to the stand-in AIJ
// (device SpMV), shifted by 1 (MatShift(A,1), :117) and solved with KSPGMRES each step.
#ifndef CFP_WITH_PETSC
#include <sys/time.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/pcshell_fft3d.h"
#include "../../include/transport_equation.h"

namespace {
double wall() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}
}  // namespace

// One row per cell; the six faces of cell (i,j,k) in the order -x,+x,-y,+y,-z,+z with outward
// normals; un = n . a.  Interior face: un > 0 adds dt |F|/|C| un to the diagonal (:109-110);
// otherwise the neighbour column gets -dt |F|/|C| un (reference sign, :111-112) or
// +dt |F|/|C| un (fixed sign).  Border faces add nothing (Neumann, :114-129).
// rows [r0, r1) of the operator: rowptr[c - r0], global columns
static int transport_csr_rows(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, const double a[3],
                              int sign_mode, double shift, int64_t r0, int64_t r1, int64_t* rowptr, int64_t* col,
                              double* val, int64_t* nnz) {
  if (!h || !a || !rowptr || !col || !val || !nnz) return CFP_ERR_ARG_NULL;
  if (nx < 1 || ny < 1 || nz < 1 || h[0] <= 0 || h[1] <= 0 || h[2] <= 0) return CFP_ERR_ARG_OUTOFRANGE;
  if (sign_mode != CFP_UPWIND_REFERENCE && sign_mode != CFP_UPWIND_FIXED) return CFP_ERR_ARG_OUTOFRANGE;
  if (r0 < 0 || r1 < r0 || r1 > nx * ny * nz) return CFP_ERR_ARG_OUTOFRANGE;
  const int64_t n[3] = {nx, ny, nz};
  const int64_t stride[3] = {1, nx, nx * ny};
  const double sgn = sign_mode == CFP_UPWIND_REFERENCE ? -1.0 : 1.0;
  int64_t p = 0;
  rowptr[0] = 0;
  for (int64_t c = r0; c < r1; ++c) {
        const int64_t i = c % nx, j = (c / nx) % ny, k = c / (nx * ny);
        const int64_t idx[3] = {i, j, k};
        double diag = shift;
        double off[6] = {0, 0, 0, 0, 0, 0};  // neighbour coefficients: -x,+x,-y,+y,-z,+z
        bool has[6] = {false, false, false, false, false, false};
        for (int d = 0; d < 3; ++d) {
          const double coef = dt / h[d];  // dt |F| / |C|
          for (int s = 0; s < 2; ++s) {   // s = 0: face -d (normal -e_d), s = 1: face +d
            const bool border = s == 0 ? idx[d] == 0 : idx[d] == n[d] - 1;
            if (border) continue;
            const double un = s == 0 ? -a[d] : a[d];
            if (un > 0) {
              diag += coef * un;
            } else {
              off[2 * d + s] += sgn * coef * un;
              has[2 * d + s] = true;
            }
          }
        }
        // ascending columns: -z, -y, -x, diag, +x, +y, +z
        const int order[6] = {4, 2, 0, 1, 3, 5};
        for (int q = 0; q < 3; ++q) {
          const int f = order[q];
          if (has[f] && off[f] != 0.0) {
            col[p] = c - stride[f / 2];
            val[2 * p] = off[f];
            val[2 * p + 1] = 0.0;
            ++p;
          }
        }
        col[p] = c;
        val[2 * p] = diag;
        val[2 * p + 1] = 0.0;
        ++p;
        for (int q = 3; q < 6; ++q) {
          const int f = order[q];
          if (has[f] && off[f] != 0.0) {
            col[p] = c + stride[f / 2];
            val[2 * p] = off[f];
            val[2 * p + 1] = 0.0;
            ++p;
          }
        }
        rowptr[c - r0 + 1] = p;
  }
  *nnz = p;
  return CFP_SUCCESS;
}

extern "C" int cfp_transport_csr(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, const double a[3],
                                 int sign_mode, double shift, int64_t* rowptr, int64_t* col, double* val,
                                 int64_t* nnz) {
  return transport_csr_rows(nx, ny, nz, h, dt, a, sign_mode, shift, 0, nx * ny * nz, rowptr, col, val, nnz);
}

extern "C" double cfp_cartesian_min_ratio_vol_surf(int dim, const double h[3]) {
  if (dim <= 1) return h[0] / 2.0;
  if (dim == 2) return h[0] * h[1] / (2.0 * (h[0] + h[1]));
  return h[0] * h[1] * h[2] / (2.0 * (h[0] * h[1] + h[1] * h[2] + h[2] * h[0]));
}

extern "C" PetscErrorCode computeDivergenceMatrixCartesian(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal h[3],
                                                           PetscReal dt, const PetscReal a[3], PetscInt sign_mode,
                                                           Mat* A) {
  PetscFunctionBeginUser;
  PetscCheck(A && h && a, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "computeDivergenceMatrixCartesian: NULL argument");
  PetscCheck(nx >= 1 && ny >= 1 && nz >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const int64_t N = nx * ny * nz;
  std::vector<int64_t> rowptr((size_t)N + 1), col((size_t)(7 * N));
  std::vector<PetscScalar> val((size_t)(7 * N));
  int64_t nnz = 0;
  const int rc = cfp_transport_csr(nx, ny, nz, h, dt, a, (int)sign_mode, 0.0, rowptr.data(), col.data(),
                                   reinterpret_cast<double*>(val.data()), &nnz);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, "computeDivergenceMatrixCartesian: bad arguments");
  PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, N, N, rowptr.data(), col.data(), val.data(), A));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// computeDivergenceMatrix on a communicator (the reference's MatCreateAIJ on PETSC_COMM_WORLD,
// tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:82-84): every rank sets its own rows
// (PETSC_DECIDE blocks = whole z-planes when the size divides n_z) and assembles
extern "C" PetscErrorCode computeDivergenceMatrixCartesianAIJ(MPI_Comm comm, PetscInt nx, PetscInt ny, PetscInt nz,
                                                              const PetscReal h[3], PetscReal dt, const PetscReal a[3],
                                                              PetscInt sign_mode, Mat* A) {
  PetscFunctionBeginUser;
  PetscCheck(A && h && a, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "computeDivergenceMatrixCartesianAIJ: NULL argument");
  PetscCheck(nx >= 1 && ny >= 1 && nz >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const int64_t N = nx * ny * nz;
  PetscCall(MatCreateAIJ(comm, PETSC_DECIDE, PETSC_DECIDE, N, N, 7, NULL, 6, NULL, A));
  PetscInt lo, hi;
  PetscCall(MatGetOwnershipRange(*A, &lo, &hi));
  const int64_t m = hi - lo;
  std::vector<int64_t> rowptr((size_t)m + 1), col((size_t)(7 * (m > 0 ? m : 1)));
  std::vector<PetscScalar> val((size_t)(7 * (m > 0 ? m : 1)));
  int64_t nnz = 0;
  const int rc = transport_csr_rows(nx, ny, nz, h, dt, a, (int)sign_mode, 0.0, lo, hi, rowptr.data(), col.data(),
                                    reinterpret_cast<double*>(val.data()), &nnz);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, "computeDivergenceMatrixCartesianAIJ: bad arguments");
  for (int64_t r = 0; r < m; ++r) {
    const PetscInt row = lo + r, k = rowptr[(size_t)r + 1] - rowptr[(size_t)r];
    PetscCall(MatSetValues(*A, 1, &row, k, col.data() + rowptr[(size_t)r], val.data() + rowptr[(size_t)r], ADD_VALUES));
  }
  PetscCall(MatAssemblyBegin(*A, MAT_FINAL_ASSEMBLY));
  PetscCall(MatAssemblyEnd(*A, MAT_FINAL_ASSEMBLY));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode initial_conditions_shock_cartesian(PetscInt nx, PetscInt ny, PetscInt nz,
                                                             const PetscReal xmin[3], const PetscReal xmax[3], Vec U) {
  PetscFunctionBeginUser;
  PetscCheck(xmin && xmax, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL domain bounds");
  PetscInt n, Ng, lo;
  PetscCall(VecGetLocalSize(U, &n));
  PetscCall(VecGetSize(U, &Ng));
  PetscCall(VecGetOwnershipRange(U, &lo, NULL));
  PetscCheck(Ng == nx * ny * nz, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ, "U size differs from nx*ny*nz");
  const double hx = (xmax[0] - xmin[0]) / (double)nx, hy = (xmax[1] - xmin[1]) / (double)ny,
               hz = (xmax[2] - xmin[2]) / (double)nz;
  const double cx = (xmin[0] + xmax[0]) / 2, cy = (xmin[1] + xmax[1]) / 2, cz = (xmin[2] + xmax[2]) / 2;
  const double rmax = 0.3;
  PetscScalar* u;
  PetscCall(VecGetArrayWrite(U, &u));
  for (PetscInt c = lo; c < lo + n; ++c) {  // this rank's cells
    const PetscInt i = c % nx, j = (c / nx) % ny, k = c / (nx * ny);
    const double x = xmin[0] + (i + 0.5) * hx, y = xmin[1] + (j + 0.5) * hy, z = xmin[2] + (k + 0.5) * hz;
    double r2 = (x - cx) * (x - cx);
    if (ny > 1) r2 += (y - cy) * (y - cy);
    if (nz > 1) r2 += (z - cz) * (z - cz);
    u[c - lo] = std::sqrt(r2) < rmax ? 650.0 : 600.0;
  }
  PetscCall(VecRestoreArrayWrite(U, &u));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" void cfp_transport_config_default(cfp_transport_config* cfg, int64_t n) {
  if (!cfg) return;
  std::memset((void*)cfg, 0, sizeof(*cfg));
  cfg->nx = cfg->ny = cfg->nz = n;
  for (int d = 0; d < 3; ++d) {
    cfg->xmin[d] = -0.5;
    cfg->xmax[d] = 0.5;
  }
  cfg->a[0] = 1.0;
  cfg->cfl = 1.0e3 / 3.0;
  cfg->tmax = 0.05;
  cfg->ntmax = 2000000;
  cfg->precision = 1e-5;
  cfg->max_its = 1000;
  cfg->restart = 30;
  cfg->pc = CFP_TRANSPORT_PC_FFT;
  cfg->sign_mode = CFP_UPWIND_REFERENCE;
  cfg->lambda_mode = CFP_LAMBDA_MATCHED;
  cfg->pc_side = PC_LEFT;
  cfg->on_device = 1;
  cfg->fuse = 1;
  cfg->profile = 0;
}

// TransportEquation_impl_mpi (one rank): the time loop of implicit upwind steps
// (I + dt A) U^{n+1} = U^n solved by GMRES, KSPSolve(ksp, Un, Un) as at :136.
extern "C" PetscErrorCode TransportEquationGMRES(const cfp_transport_config* cfg, cfp_transport_result* res,
                                                 double* U_out) {
  PetscFunctionBeginUser;
  PetscCheck(cfg && res, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "TransportEquationGMRES: NULL argument");
  PetscCheck(cfg->pc == CFP_TRANSPORT_PC_NONE || cfg->on_device, PETSC_COMM_SELF, PETSC_ERR_SUP,
             "the FFT preconditioner runs on HIP vectors only");
  std::memset((void*)res, 0, sizeof(*res));
  const double t_setup = wall();
  const PetscInt nx = cfg->nx, ny = cfg->ny, nz = cfg->nz, N = nx * ny * nz;
  const int dim = nz > 1 ? 3 : (ny > 1 ? 2 : 1);
  const double h[3] = {(cfg->xmax[0] - cfg->xmin[0]) / (double)nx, (cfg->xmax[1] - cfg->xmin[1]) / (double)ny,
                       (cfg->xmax[2] - cfg->xmin[2]) / (double)nz};
  const double anorm = std::sqrt(cfg->a[0] * cfg->a[0] + cfg->a[1] * cfg->a[1] + cfg->a[2] * cfg->a[2]);
  PetscCheck(anorm > 0, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "transport velocity is zero");
  const double dt = cfg->cfl * cfp_cartesian_min_ratio_vol_surf(dim, h) / anorm;  // :54
  res->dt = dt;

  // one rank: sequential Vecs and AIJ; several (PETSC_COMM_WORLD of PetscMiniSetCommWorld): the
  // reference's VecCreateMPI / MatCreateAIJ on PETSC_COMM_WORLD with PETSC_DECIDE rows (:59-84)
  int P = 1;
  PetscCallMPI(MPI_Comm_size(PETSC_COMM_WORLD, &P));
  Vec Un, dUn;
  if (P > 1 && cfg->on_device) PetscCall(VecCreateMPIHIP(PETSC_COMM_WORLD, PETSC_DECIDE, N, &Un));
  else if (P > 1) PetscCall(VecCreateMPI(PETSC_COMM_WORLD, PETSC_DECIDE, N, &Un));
  else if (cfg->on_device) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, N, &Un));
  else PetscCall(VecCreateSeq(PETSC_COMM_SELF, N, &Un));
  PetscCall(VecDuplicate(Un, &dUn));
  PetscCall(initial_conditions_shock_cartesian(nx, ny, nz, cfg->xmin, cfg->xmax, Un));
  PetscInt lo, nloc;
  PetscCall(VecGetOwnershipRange(Un, &lo, NULL));
  PetscCall(VecGetLocalSize(Un, &nloc));
  res->rstart = lo;
  res->nlocal = nloc;

  Mat A;
  if (P > 1) PetscCall(computeDivergenceMatrixCartesianAIJ(PETSC_COMM_WORLD, nx, ny, nz, h, dt, cfg->a, cfg->sign_mode, &A));
  else PetscCall(computeDivergenceMatrixCartesian(nx, ny, nz, h, dt, cfg->a, cfg->sign_mode, &A));
  PetscCall(MatShift(A, 1.0));  // :117

  KSP ksp;
  PC pc;
  PetscCall(KSPCreate(PETSC_COMM_WORLD, &ksp));
  PetscCall(KSPSetType(ksp, KSPGMRES));
  PetscCall(KSPSetTolerances(ksp, cfg->precision, cfg->precision, PETSC_DEFAULT, cfg->max_its));
  PetscCall(KSPGMRESSetRestart(ksp, cfg->restart > 0 ? cfg->restart : 30));
  PetscCall(KSPSetPCSide(ksp, (PCSide)cfg->pc_side));
  PetscCall(KSPMiniSetFusion(ksp, cfg->fuse ? PETSC_TRUE : PETSC_FALSE));
  PetscCall(KSPGetPC(ksp, &pc));
  FFTPrecTransportContext ctx;
  std::memset((void*)&ctx, 0, sizeof(ctx));
  if (cfg->pc == CFP_TRANSPORT_PC_FFT) {
    // the wiring ToDo.md:1 asks for: context factory, then the three PCSHELL callbacks
    PetscCall(getFFTPrec3DContext(3, dt, N, cfg->a[0], cfg->a[1], cfg->a[2], cfg->xmin[0], cfg->xmin[1],
                                  cfg->xmin[2], cfg->xmax[0], cfg->xmax[1], cfg->xmax[2], &ctx));
    // the factory assumes a cube (n = cbrt(nbCells)); a box grid keeps its own sizes
    ctx.n_x = nx;
    ctx.n_y = ny;
    ctx.n_z = nz;
    if (cfg->lambda_mode == CFP_LAMBDA_MATCHED) {
      ctx.lambda_x = cfg->a[0] * dt / h[0];
      ctx.lambda_y = cfg->a[1] * dt / h[1];
      ctx.lambda_z = cfg->a[2] * dt / h[2];
    }
    PetscCall(PCSetType(pc, PCSHELL));
    PetscCall(PCShellSetContext(pc, &ctx));
    PetscCall(PCShellSetSetUp(pc, setupFFTPrec3D));
    PetscCall(PCShellSetApply(pc, applyFFT3DPrecTransport));
    if (cfg->fuse) PetscCall(PCShellSetApplyBA(pc, applyFFT3DPrecTransportBA));
    PetscCall(PCShellSetDestroy(pc, destroyFFTPrec3D));
    PetscCall(PCShellSetName(pc, "circulant FFT (HIP)"));
    res->lambda[0] = ctx.lambda_x.real();
    res->lambda[1] = ctx.lambda_y.real();
    res->lambda[2] = ctx.lambda_z.real();
  } else {
    PetscCall(PCSetType(pc, PCNONE));
  }
  PetscCall(KSPSetOperators(ksp, A, A));
  PetscCall(KSPSetUp(ksp));
  // allocate the Krylov basis and make the device copy of A now, so the timed solves hold
  // only the solver's own work (PETSc would do both inside the first KSPSolve)
  PetscCall(KSPMiniSetUpWork(ksp, Un));
  PetscCall(MatMult(A, Un, dUn));
  if (cfg->on_device)
    PetscCheck(cfp_stream_sync(nullptr) == CFP_SUCCESS, PETSC_COMM_SELF, PETSC_ERR_LIB, "stream sync failed");
  res->setup_seconds = wall() - t_setup;

  int64_t it = 0;
  double time = 0.0;
  bool stationary = false;
  res->all_converged = 1;
  res->min_step_its = -1;
  if (cfg->profile) PetscCall(PetscMiniProfileBegin(1 << 16));
  const double t_loop = wall();
  while (it < cfg->ntmax && time <= cfg->tmax && !stationary) {  // :131
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
    if (reason != KSP_CONVERGED_RTOL && reason != KSP_CONVERGED_ATOL) res->all_converged = 0;  // :166
    PetscInt fd, fn;
    PetscCall(KSPMiniGetFusedCounts(ksp, &fd, &fn));
    res->fused_dots += fd;
    res->fused_norms += fn;
  }
  res->loop_seconds = wall() - t_loop;
  if (cfg->profile) {
    PetscCall(PetscMiniProfileEnd(res->dev_ms, res->dev_launches));
    res->dev_ms[0] = 1e3 * res->pc_seconds;
    res->dev_launches[0] = res->pc_calls;
  }
  res->steps = it;
  res->time = time;
  if (U_out) {  // this rank's rows (all of them on one rank)
    const PetscScalar* u;
    PetscCall(VecGetArrayRead(Un, &u));
    std::memcpy(U_out, (const void*)u, sizeof(double) * 2 * (size_t)nloc);
    PetscCall(VecRestoreArrayRead(Un, &u));
  }
  PetscCall(KSPDestroy(&ksp));  // destroys the PC, whose destroy callback frees setup's objects
  PetscCall(MatDestroy(&A));
  PetscCall(VecDestroy(&Un));
  PetscCall(VecDestroy(&dUn));
  PetscFunctionReturn(PETSC_SUCCESS);
}
// TransportEquationFFT_impl_mpi, tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:20-150:
// the direct-solver loop.  The FFT matrix is made once (:97-99) and reused every step (the
// reference's Fft3DSolver destroys it after the first step, App. A item 6; here it survives).
extern "C" PetscErrorCode TransportEquationFFTDirect(const cfp_transport_config* cfg, cfp_transport_result* res,
                                                     double* U_out) {
  PetscFunctionBeginUser;
  PetscCheck(cfg && res, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "TransportEquationFFTDirect: NULL argument");
  std::memset((void*)res, 0, sizeof(*res));
  const double t_setup = wall();
  const PetscInt nx = cfg->nx, ny = cfg->ny, nz = cfg->nz, N = nx * ny * nz;
  PetscCheck(nx >= 1 && ny >= 1 && nz >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const int dim = nz > 1 ? 3 : (ny > 1 ? 2 : 1);
  const double h[3] = {(cfg->xmax[0] - cfg->xmin[0]) / (double)nx, (cfg->xmax[1] - cfg->xmin[1]) / (double)ny,
                       (cfg->xmax[2] - cfg->xmin[2]) / (double)nz};
  // the velocity has dim components in the reference (Vector(getSpaceDimension())): the others are 0
  const double a[3] = {cfg->a[0], dim > 1 ? cfg->a[1] : 0.0, dim > 2 ? cfg->a[2] : 0.0};
  const double anorm = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  PetscCheck(anorm > 0, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "transport velocity is zero");
  const double dt = cfg->cfl * cfp_cartesian_min_ratio_vol_surf(dim, h) / anorm;  // :44-45
  res->dt = dt;
  for (int d = 0; d < 3; ++d) res->lambda[d] = a[d] * dt / h[d];

  Vec Un, dUn;
  if (cfg->on_device) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, N, &Un));
  else PetscCall(VecCreateSeq(PETSC_COMM_SELF, N, &Un));
  PetscCall(VecDuplicate(Un, &dUn));
  PetscCall(initial_conditions_shock_cartesian(nx, ny, nz, cfg->xmin, cfg->xmax, Un));

  Mat FFT_MAT;
  const PetscInt dims[3] = {nz, ny, nx};
  PetscCall(MatCreateFFT(PETSC_COMM_WORLD, 3, dims, MATFFTW, &FFT_MAT));  // :97-99
  struct StructuredTransportContext ctx = {nx, ny, nz, a[0], a[1], a[2], dt, h[0], h[1], h[2], FFT_MAT};  // :100
  res->setup_seconds = wall() - t_setup;

  int64_t it = 0;
  double time = 0.0;
  bool stationary = false;
  res->all_converged = 1;
  while (it < cfg->ntmax && time <= cfg->tmax && !stationary) {  // :106
    PetscCall(VecCopy(Un, dUn));
    // the copy above is queued on the Vec stream (PETSc's host VecCopy returns when done): drain
    // it, so that the clock brackets the solve only, as the reference's PetscTime pair (:110-112)
    PetscCall(VecMiniSynchronize(dUn));
    const double v = wall();
    PetscCall(PetscFft3DTransportSolver(ctx, Un, Un));  // :111
    PetscCall(VecMiniSynchronize(Un));  // a device-Vec solve is stream-ordered: time it to completion
    const double w = wall();
    PetscCall(VecAXPY(dUn, -1.0, Un));
    time += dt;
    it += 1;
    PetscReal norm;
    PetscCall(VecNorm(dUn, NORM_2, &norm));
    stationary = norm < cfg->precision;
    res->solve_seconds += w - v;
    res->pc_calls += 1;
    res->last_norm_dU = norm;
  }
  res->steps = it;
  res->time = time;
  if (U_out) {
    const PetscScalar* u;
    PetscCall(VecGetArrayRead(Un, &u));
    std::memcpy(U_out, (const void*)u, sizeof(double) * 2 * (size_t)N);
    PetscCall(VecRestoreArrayRead(Un, &u));
  }
  PetscCall(MatDestroy(&FFT_MAT));
  PetscCall(VecDestroy(&Un));
  PetscCall(VecDestroy(&dUn));
  PetscFunctionReturn(PETSC_SUCCESS);
}
#endif  // CFP_WITH_PETSC
