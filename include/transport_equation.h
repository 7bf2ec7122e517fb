/*
 * transport_equation.h -- the implicit upwind transport operator and the GMRES time loop
 * that the circulant preconditioner is meant to plug into.
 *
 * Reference interface each entry point replaces:
 *   src/TransportEquation2.hxx:17        initial_conditions_shock(Mesh, Field&)
 *   src/TransportEquation2.hxx:19        computeDivergenceMatrix(Mesh, Mat*, dt, Vector)
 *   tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:13-189
 *                                        TransportEquation_impl_mpi (GMRES time loop; the
 *                                        PCSHELL wiring is the one ToDo.md:1 asks for)
 * The reference takes a SOLVERLAB Mesh; SOLVERLAB is absent here, so the Cartesian mesh
 * Mesh(xmin,xmax,nx, ymin,ymax,ny, zmin,zmax,nz) is passed as its numbers.  Cell
 * c = i + nx (j + ny k) (x fastest), centre xmin + (i + 1/2) h_x, |F|/|C| = 1/h_d.
 */
#ifndef CFP_TRANSPORT_EQUATION_H
#define CFP_TRANSPORT_EQUATION_H

#include <stdint.h>

#include "petsc_mini.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Sign of the inflow (un < 0) coefficient.
 * CFP_UPWIND_REFERENCE: A(j, nb) += -dt |F|/|C| un, as src/TransportEquation.cxx:112 does
 *                       (this is the wrong sign);
 * CFP_UPWIND_FIXED:     A(j, nb) += +dt |F|/|C| un, the conservative upwind scheme whose
 *                       periodic version is the circulant the preconditioner inverts. */
enum { CFP_UPWIND_REFERENCE = 0, CFP_UPWIND_FIXED = 1 };

/* Host-only CSR of  shift * I + computeDivergenceMatrix  on an nx*ny*nz Cartesian grid.
 * Border faces are skipped (Neumann, src/TransportEquation.cxx:116-129); every row stores
 * its diagonal (so MatShift never meets a missing one); entries that are exactly zero are
 * not stored; columns ascend in each row.  rowptr has n+1 entries, col/val room for 7n
 * (val: interleaved re,im doubles).  *nnz receives the entry count.
 * Returns 0, CFP_ERR_ARG_NULL or CFP_ERR_ARG_OUTOFRANGE (circulant_fft.h numbering). */
int cfp_transport_csr(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, const double a[3],
                      int sign_mode, double shift, int64_t *rowptr, int64_t *col, double *val, int64_t *nnz);

/* min over cells of |C| / sum|F| for the Cartesian cell (SOLVERLAB Mesh::minRatioVolSurf):
 * h_x h_y h_z / (2 (h_x h_y + h_y h_z + h_z h_x)) in 3-D. */
double cfp_cartesian_min_ratio_vol_surf(int dim, const double h[3]);

/* ---- PETSc-level (stand-in) entry points */
/* computeDivergenceMatrix on the Cartesian grid into a new MATSEQAIJ *A (no MatShift). */
PetscErrorCode computeDivergenceMatrixCartesian(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal h[3],
                                                PetscReal dt, const PetscReal a[3], PetscInt sign_mode, Mat *A);
/* initial_conditions_shock: 650 where |centre - domain centre| < 0.3, else 600. */
PetscErrorCode initial_conditions_shock_cartesian(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal xmin[3],
                                                  const PetscReal xmax[3], Vec U);

/* computeDivergenceMatrix on a communicator: MatCreateAIJ(comm, PETSC_DECIDE rows), each rank
 * setting its own rows with MatSetValues, then MatAssemblyBegin/End (no MatShift) */
PetscErrorCode computeDivergenceMatrixCartesianAIJ(MPI_Comm comm, PetscInt nx, PetscInt ny, PetscInt nz,
                                                   const PetscReal h[3], PetscReal dt, const PetscReal a[3],
                                                   PetscInt sign_mode, Mat *A);

/* ---- the implicit transport time loop with GMRES (TransportEquation_impl_mpi) */
enum { CFP_TRANSPORT_PC_NONE = 0, CFP_TRANSPORT_PC_FFT = 1 };
/* lambda of the FFT preconditioner: REFERENCE = getFFTPrec3DContext's a dt (max-min)/n
 * (src/PCSHELLFft_3D.cxx:146-148); MATCHED = a dt / h, the symbol of the operator. */
enum { CFP_LAMBDA_REFERENCE = 0, CFP_LAMBDA_MATCHED = 1 };

typedef struct {
  int64_t nx, ny, nz;
  double xmin[3], xmax[3];
  double a[3];        /* transport velocity (reference main: (1,0,0)) */
  double cfl;         /* reference main: 1e3 / dim */
  double tmax;        /* reference main: 0.05 */
  int64_t ntmax;      /* time steps cap */
  double precision;   /* rtol = abstol = precision, stationarity threshold (1e-5) */
  int64_t max_its;    /* KSP max iterations (1000) */
  int64_t restart;    /* GMRES restart (30) */
  int pc;             /* CFP_TRANSPORT_PC_* */
  int sign_mode;      /* CFP_UPWIND_* */
  int lambda_mode;    /* CFP_LAMBDA_* */
  int pc_side;        /* PC_LEFT (0) / PC_RIGHT (1) */
  int on_device;      /* 1: HIP Vecs (VecCreateSeqHIP), 0: host Vecs (PCNONE only) */
  int fuse;           /* 1 (default): the fused Krylov step -- PCShellSetApplyBA(pc,
                       * applyFFT3DPrecTransportBA) and the KSP's dots asked from the apply;
                       * 0: MatMult + PCApply + VecMDot as separate sweeps (KSPMiniSetFusion) */
  int profile;        /* 1: device time of the loop's kernels by kind (res->dev_ms, PetscMiniProfile*) */
} cfp_transport_config;

typedef struct {
  int64_t steps;          /* time steps taken */
  double dt, time;
  int64_t total_its;      /* sum of KSP iterations over the steps */
  int64_t max_step_its;
  int64_t min_step_its;
  int last_reason;        /* KSPConvergedReason of the last solve */
  int all_converged;      /* every solve ended with reason 2 or 3 (the driver's test) */
  double last_residual;
  double last_norm_dU;
  double solve_seconds;   /* wall time inside KSPSolve, summed */
  double pc_seconds;      /* host wall time inside PCApply, summed */
  int64_t pc_calls;
  double setup_seconds;   /* assembly + PC setup */
  double lambda[3];
  double loop_seconds;    /* wall time of the whole time loop (solves + the loop's own Vec work) */
  /* cfg->profile: device ms over the loop -- [0] PCApply (the KSP's stamps or events; with the
   * fused applyBA it includes the MatMult), [1] MatMult kernels, [2] vector kernels (BLAS-1 and
   * reductions), [3] copies */
  double dev_ms[4];
  int64_t dev_launches[4];
  int64_t fused_dots;     /* Gram-Schmidt steps whose dots came from the PC apply (summed) */
  int64_t fused_norms;    /* residual norms that came from the PC apply (summed) */
  int64_t rstart, nlocal; /* this rank's rows (U_out holds nlocal values): 0, N on one rank */
} cfp_transport_result;

/* fill cfg with the reference main's defaults for an n^3 grid on [-0.5,0.5]^3 */
void cfp_transport_config_default(cfp_transport_config *cfg, int64_t n);
/* run the loop; if U_out != NULL this rank's part of the final field is copied there (interleaved
 * re,im, res->nlocal values from row res->rstart; the whole field, N values, on one rank).  With
 * PETSC_COMM_WORLD of several ranks (PetscMiniSetCommWorld) the loop runs on all of them as the
 * reference's does (VecCreateMPI, MatCreateAIJ, KSP on PETSC_COMM_WORLD; the FFT PCSHELL on the
 * z-slab plan): every rank calls it with the same cfg. */
PetscErrorCode TransportEquationGMRES(const cfp_transport_config *cfg, cfp_transport_result *res, double *U_out);

/* ---- the direct-solver time loop (TransportEquationFFT_impl_mpi,
 * tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:20-150): each implicit step is one
 * PetscFft3DTransportSolver(ctx, Un, Un) with StructuredTransportContext {n, a, dt, delta}
 * (:97-111), i.e. lambda_d = a_d dt / delta_d; dt = cfl minRatioVolSurf / |a| (:45); the loop
 * runs while it < ntmax, time <= tmax and ||U^{n+1} - U^n|| >= precision (:106-118).
 * cfg fields used: nx, ny, nz (the reference's argv; ny = nz = 1 in 1-D, nz = 1 in 2-D: its
 * uninitialised ny / nz), xmin, xmax, a, cfl (reference main: 1e3 / dim),
 * tmax, ntmax, precision, on_device.  res: steps, dt, time, last_norm_dU, solve_seconds (sum of
 * the per-step solve times the reference prints as "solve cpu time", :121). */
PetscErrorCode TransportEquationFFTDirect(const cfp_transport_config *cfg, cfp_transport_result *res, double *U_out);

#ifdef __cplusplus
}
#endif
#endif /* CFP_TRANSPORT_EQUATION_H */
