/*
 * wave_system.h -- the (d+1)-block-circulant preconditioner of the linear wave system and the
 * implicit GMRES time loop it plugs into (BASELINE config 4).
 *
 * The reference assembles the implicit upwind wave-system matrix
 *   src/WaveSystem.cxx:92-107   jacobianMatrices(normal, coeff) = (A(n) - |A(n)|) coeff / 2
 *   src/WaveSystem.cxx:109-176  computeDivergenceMatrix(Mesh, Mat*, dt)  (wall / periodic /
 *                               Neumann faces)
 *   src/WaveSystem.cxx:25-76    initial_conditions_shock (pressure 155e5 inside r < 0.3, else
 *                               70e5; velocity 0)
 * and solves it with GMRES + ILU/BJACOBI (tests/WaveSystem_SphericalExplosion_impl_seq.cxx:
 * 11-150, _impl_mpi.cxx).  It has no FFT preconditioner for it (ToDo.md:10 asks for one): the
 * periodic operator is block-circulant with 4x4 blocks (d = 3: pressure, 3 momentum
 * components, interleaved idx = cell*4 + comp as the reference's Un layout, :57-68), and this
 * library inverts it exactly with 5 HBM sweeps, like the scalar plan.
 *
 * Symbol (theta_d = 2 pi k_d / n_d, kappa_d = dt / h_d, c0 = 700, src/WaveSystem.hxx:17):
 *   S = I + sum_d kappa_d sum_{s=+-1} A^-(s e_d) (e^{i s theta_d} - 1),
 *   A^-(n) = (A(n) - |A(n)|) / 2,  A(n) = [[0, c0^2 n^T], [n, 0]],  |A(n)| = diag(c0, c0 n n^T).
 */
#ifndef CFP_WAVE_SYSTEM_H
#define CFP_WAVE_SYSTEM_H

#include <stdint.h>

#include "petsc_mini.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- the block-circulant plan (C ABI, device pointers, dim + 1 interleaved components) */
typedef struct cfp_wave_plan_s *cfp_wave_plan_t;
/* dim = 1, 2 or 3 (nbComp = dim + 1 unknowns per cell, src/WaveSystem.cxx:112-113); the axes
 * above dim must have n = 1.  The reference mains default to dim = 2 (a 50 x 50 square,
 * tests/WaveSystem_SphericalExplosion_impl_seq.cxx:182-197). */
int cfp_wave_plan_create_dim(cfp_wave_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int dim, int device);
/* dim = 3 */
int cfp_wave_plan_create(cfp_wave_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int device);
int cfp_wave_plan_destroy(cfp_wave_plan_t plan);
/* kappa[d] = dt / h_d, c0 = sound speed */
int cfp_wave_plan_set_symbol(cfp_wave_plan_t plan, const double kappa[3], double c0);
/* x = S^{-1} b on the periodic grid (b, x: (dim+1)*nx*ny*nz complex doubles; x may alias b) */
int cfp_wave_plan_apply(cfp_wave_plan_t plan, const double *b, double *x, void *stream);
/* x = S^{-1} b and dots[2 j], dots[2 j + 1] = Re, Im of v[j]^H x for j < nv <= 8 (v[j] NULL or x:
 * |x|^2); dots is a device array of 2 nv doubles, written on `stream`.  On the 3-sweep schedule
 * (3-D 128^3) and nv <= 4 the dots ride in the last sweep's stores (*fused = 1: the Gram-Schmidt
 * dots of the stand-in GMRES, PCMiniApplyDots); otherwise one multi-dot sweep follows the apply
 * (*fused = 0). */
int cfp_wave_plan_apply_dots(cfp_wave_plan_t plan, const double *b, double *x, void *stream, int nv,
                             const double *const *v, double *dots, int *fused);
/* unnormalised forward / backward 3-D DFT of each component (tests and tools) */
int cfp_wave_plan_forward(cfp_wave_plan_t plan, const double *in, double *out, void *stream);
int cfp_wave_plan_backward(cfp_wave_plan_t plan, const double *in, double *out, void *stream);
/* CFP_SCHEDULE_AUTO (default: the 3-sweep apply on a 3-D 128^3 grid, else 5 sweeps),
   CFP_SCHEDULE_FIVE_PASS, or CFP_SCHEDULE_THREE_PASS (3-D 128^3 only; CFP_ERR_SUP otherwise) */
int cfp_wave_plan_set_schedule(cfp_wave_plan_t plan, int schedule);
int cfp_wave_plan_num_passes(cfp_wave_plan_t plan, int *passes);
int cfp_wave_plan_time_passes(cfp_wave_plan_t plan, const double *b, double *x, int iters, double *ms_out,
                              void *stream);

/* ---- host assembly of the wave-system operator */
enum { CFP_WAVE_BC_WALL = 0, CFP_WAVE_BC_PERIODIC = 1, CFP_WAVE_BC_NEUMANN = 2 };
/* CSR of shift*I + computeDivergenceMatrix (src/WaveSystem.cxx:109-176) on an nx*ny*nz
 * Cartesian grid, 4 unknowns per cell.  rowptr: 4n+1 entries; col/val room for 4n*28
 * entries (val interleaved re,im).  Entries that are exactly zero are not stored; every row
 * keeps its diagonal; columns ascend. */
int cfp_wave_csr(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, double c0, int bc, double shift,
                 int64_t *rowptr, int64_t *col, double *val, int64_t *nnz);
/* the same for a dim-dimensional mesh (dim + 1 unknowns per cell, faces only along the first
 * dim axes; the axes above dim must have n = 1).  rowptr: (dim+1)n+1 entries, col/val room for
 * (dim+1)^2 (2 dim + 1) n entries. */
int cfp_wave_csr_dim(int64_t nx, int64_t ny, int64_t nz, int dim, const double h[3], double dt, double c0, int bc,
                     double shift, int64_t *rowptr, int64_t *col, double *val, int64_t *nnz);

/* ---- PETSc-level entry points */
PetscErrorCode computeDivergenceMatrixWaveCartesian(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal h[3],
                                                    PetscReal dt, PetscReal c0, PetscInt bc, Mat *A);
PetscErrorCode computeDivergenceMatrixWaveCartesianDim(PetscInt nx, PetscInt ny, PetscInt nz, PetscInt dim,
                                                       const PetscReal h[3], PetscReal dt, PetscReal c0, PetscInt bc,
                                                       Mat *A);
/* the same as a MatCreateAIJ on comm, each rank setting its own PETSC_DECIDE rows */
PetscErrorCode computeDivergenceMatrixWaveCartesianAIJ(MPI_Comm comm, PetscInt nx, PetscInt ny, PetscInt nz,
                                                       PetscInt dim, const PetscReal h[3], PetscReal dt, PetscReal c0,
                                                       PetscInt bc, Mat *A);
/* pressure 155e5 where |centre - domain centre| < 0.3 else 70e5, momentum 0.  U holds
 * (dim+1)*N values; dim is read from its size (src/WaveSystem.cxx:25-76). */
PetscErrorCode initial_conditions_shock_wave(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal xmin[3],
                                             const PetscReal xmax[3], Vec U);

/* PCSHELL of the block-circulant preconditioner (new capability; same registration pattern
 * as applyFFT3DPrecTransport: PCShellSetContext(pc, &ctx), SetSetUp/SetApply/SetDestroy).
 * With PETSC_COMM_WORLD of P > 1 ranks, setup builds the z-slab plan instead of `plan` and b / x
 * are this rank's PETSC_DECIDE rows: a 3-D grid needs P | n_z, a 2-D grid (n_z = 1) P | n_y
 * (whole planes / rows of cells per rank); other shapes return PETSC_ERR_SUP. */
struct FFTPrecWaveContext {
  PetscInt n_x, n_y, n_z;
  PetscReal kappa_x, kappa_y, kappa_z; /* dt / h_d */
  PetscReal c0;
  cfp_wave_plan_t plan; /* created by setup, destroyed by destroy */
  PetscInt dim;         /* 1, 2 or 3; 0 = 3 */
};
typedef struct FFTPrecWaveContext FFTPrecWaveContext;
PetscErrorCode applyFFT3DPrecWave(PC pc, Vec b, Vec x);
PetscErrorCode setupFFTPrec3DWave(PC pc);
PetscErrorCode destroyFFTPrec3DWave(PC pc);

/* ---- the implicit wave-system time loop (WaveSystem_impl_seq/mpi) */
enum { CFP_WAVE_PC_NONE = 0, CFP_WAVE_PC_FFT = 1 };
typedef struct {
  int64_t nx, ny, nz;
  double xmin[3], xmax[3];
  double c0;          /* 700 (src/WaveSystem.hxx:17) */
  double cfl;         /* reference main: 1e3 / dim */
  double tmax;        /* 0.05 */
  int64_t ntmax;
  double precision;   /* rtol = abstol = stationarity threshold: 1e-5 (src/WaveSystem.hxx:19) */
  int64_t max_its;    /* 1000 */
  int64_t restart;    /* 30 */
  int pc;             /* CFP_WAVE_PC_* */
  int bc;             /* CFP_WAVE_BC_*: wall as the reference mains set up */
  int pc_side;        /* PC_LEFT / PC_RIGHT */
  int on_device;
  int dim;            /* mesh dimension 1, 2 or 3 (nbComp = dim + 1); 0 = 3 */
  int profile;        /* 1: stamp every kernel of the time loop (PetscMiniProfileBegin): dev_ms below */
  int fuse;           /* 1 (default): the KSP asks the block PCSHELL for the Gram-Schmidt dots
                         (KSPMiniSetFusion; they ride in the 3-sweep apply); 0: separate sweeps */
} cfp_wave_config;

/* same layout as cfp_transport_result (transport_equation.h); lambda[] holds kappa */
typedef struct {
  int64_t steps;
  double dt, time;
  int64_t total_its, max_step_its, min_step_its;
  int last_reason;
  int all_converged;
  double last_residual, last_norm_dU;
  double solve_seconds, pc_seconds;
  int64_t pc_calls;
  double setup_seconds;
  double kappa[3];
  int64_t rstart, nlocal; /* this rank's rows of Un (U_out holds nlocal values): 0, (dim+1)N on one rank */
  double loop_seconds;    /* wall time of the time loop */
  double dev_ms[4];       /* profile = 1: device ms of the loop by kind: PCApply, MatMult, vector kernels, copies */
  int64_t dev_launches[4];
  int64_t fused_dots, fused_norms; /* Gram-Schmidt dots / residual norms computed inside the PCSHELL apply */
} cfp_wave_result;

void cfp_wave_config_default(cfp_wave_config *cfg, int64_t n);
/* the reference main's defaults for a dim-dimensional square / cube of n cells a side
 * (cfl = 1e3 / dim, tests/WaveSystem_SphericalExplosion_impl_seq.cxx:212) */
void cfp_wave_config_default_dim(cfp_wave_config *cfg, int64_t n, int dim);
/* U_out: optional final field, complex (interleaved re,im): this rank's res->nlocal rows from
 * res->rstart ((dim+1)N on one rank).  With PETSC_COMM_WORLD of several ranks the loop runs on
 * all of them (VecCreateMPI, MatCreateAIJ, KSP on PETSC_COMM_WORLD as
 * tests/WaveSystem_SphericalExplosion_impl_mpi.cxx; the block-circulant PCSHELL on the z-slab
 * plan: 3-D grids with the rank count dividing n_z, 2-D grids with it dividing n_y) */
PetscErrorCode WaveSystemGMRES(const cfp_wave_config *cfg, cfp_wave_result *res, double *U_out);

#ifdef __cplusplus
}
#endif
#endif /* CFP_WAVE_SYSTEM_H */
