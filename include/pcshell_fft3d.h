/*
 * pcshell_fft3d.h -- the reference's PETSc-facing interface of the circulant FFT
 * preconditioner, re-implemented on the MI355X plan (libcirculant_fft.so).
 *
 * Same names, argument order and meaning as the reference headers:
 *   src/PCSHELLFft_3D.hxx:8-45    FFTPrecTransportContext, applyFFT3DPrecTransport,
 *                                 setupFFTPrec3D, destroyFFTPrec3D, getFFTPrec3DContext
 *   src/FftLinearSolver_3D.h:7-43 StructuredTransportContext, Fft{3,2,1}DTransportSolver,
 *                                 PetscFft3DTransportSolver, FftTransportSolver, solve_3D,
 *                                 build_diag_mat_vec_3D, build_transport_col
 * Registration by the caller, unchanged from PETSc practice:
 *   PCSetType(pc, PCSHELL); PCShellSetContext(pc, &ctx);
 *   PCShellSetSetUp(pc, setupFFTPrec3D); PCShellSetApply(pc, applyFFT3DPrecTransport);
 *   PCShellSetDestroy(pc, destroyFFTPrec3D);
 *
 * Documented differences (each fixes a reference defect):
 *   - getFFTPrec3DContext's last argument is the context to fill (the reference takes a
 *     SOLVERLAB `Mesh` by value and writes through an uninitialised pointer, item 2); the
 *     reference's 13-argument Mesh form is kept for C++ callers and fills a library slot;
 *   - the callbacks fetch the context with PCShellGetContext(pc, &ctx) (item 2);
 *   - a NULL intersectionMatrix means the identity (Cartesian mesh; the reference never
 *     creates it, item 2);
 *   - FftTransportSolver/Fft3DSolver do not destroy the caller's FFT_MAT (item 6) and cache
 *     the symbol between calls with equal lambdas (item 9);
 *   - none in the context's layout: FFTPrecTransportContext is the reference's 12 members in
 *     the reference's order (src/PCSHELLFft_3D.hxx:8-21), so a translation unit compiled
 *     against the reference header links against this library.  What this build adds per
 *     context -- the Cartesian -> mesh `remapBack` (include/mesh_unstructured.h) -- lives in a
 *     side table keyed by the context's address (FFTPrecTransportContextSetRemapBack), and
 *     the HIP plan is reached through the FFT matrix (MatFFTHIPGetPlan(ctx->FFT_MAT, ...)).
 *     (PetscInt is 64-bit in the stand-in PETSc, as a --with-64-bit-indices build.)
 */
#ifndef CFP_PCSHELL_FFT3D_H
#define CFP_PCSHELL_FFT3D_H

#include "petsc_mini.h"
#include "circulant_fft.h"

#ifdef __cplusplus
extern "C" {
#endif

struct FFTPrecTransportContext {
  PetscInt spaceDim;
  PetscInt n_x;
  PetscInt n_y;
  PetscInt n_z;
  PetscScalar lambda_x;
  PetscScalar lambda_y;
  PetscScalar lambda_z;
  Mat FFT_MAT;
  Mat intersectionMatrix;
  Vec Diag;
  Vec b_hat;
  Vec b_cartesien;
};
typedef struct FFTPrecTransportContext FFTPrecTransportContext;

struct StructuredTransportContext {
  PetscInt n_x;
  PetscInt n_y;
  PetscInt n_z;
  PetscScalar a_x;
  PetscScalar a_y;
  PetscScalar a_z;
  PetscScalar dt;
  PetscScalar delta_x;
  PetscScalar delta_y;
  PetscScalar delta_z;
  Mat FFT_MAT;
};

/* ---- PCSHELL callbacks (src/PCSHELLFft_3D.hxx:23-25) */
PetscErrorCode applyFFT3DPrecTransport(PC pc, Vec b, Vec x);
PetscErrorCode setupFFTPrec3D(PC pc);
PetscErrorCode destroyFFTPrec3D(PC pc);
/* Not in the reference (an addition for its GMRES caller, tests/TransportEquation_SphericalExplosion_
 * impl_mpi.cxx:120-136): the PCShellSetApplyBA callback, y = B A x (left) / A B x (right) with the
 * PC's operator.  On one rank with the stand-in AIJ it forms A x inside the apply's first sweep
 * (no MatMult sweep); otherwise it is MatMult + applyFFT3DPrecTransport, what PETSc's
 * PCApplyBAorAB does for a shell without one.  Register it with
 * PCShellSetApplyBA(pc, applyFFT3DPrecTransportBA) beside PCShellSetApply. */
PetscErrorCode applyFFT3DPrecTransportBA(PC pc, PCSide side, Vec x, Vec y, Vec work);
/* src/PCSHELLFft_3D.hxx:27-41 (Mesh srcMesh -> FFTPrecTransportContext *ctx, see above):
 * n_d = floor(cbrt(nbCells)) (3-D), floor(sqrt) (2-D), nbCells (1-D);
 * lambda_d = a_d * dt * (max_d - min_d) / n_d (src/PCSHELLFft_3D.cxx:146-148, kept as is) */
PetscErrorCode getFFTPrec3DContext(PetscInt ndim, PetscScalar dt, PetscInt nbCells, PetscScalar a_x, PetscScalar a_y,
                                   PetscScalar a_z, PetscScalar Xmin, PetscScalar Ymin, PetscScalar Zmin,
                                   PetscScalar Xmax, PetscScalar Ymax, PetscScalar Zmax,
                                   FFTPrecTransportContext *ctx);

/* ---- direct solver (src/FftLinearSolver_3D.h:21-43) */
PetscErrorCode Fft3DTransportSolver(PetscInt n_x, PetscInt n_y, PetscInt n_z, PetscScalar a_x, PetscScalar a_y,
                                    PetscScalar a_z, PetscScalar dt, PetscScalar delta_x, PetscScalar delta_y,
                                    PetscScalar delta_z, Vec X, Vec b, Mat FFT_MAT);
PetscErrorCode Fft2DTransportSolver(PetscInt n_x, PetscInt n_y, PetscScalar a_x, PetscScalar a_y, PetscScalar dt,
                                    PetscScalar delta_x, PetscScalar delta_y, Vec X, Vec b, Mat FFT_MAT);
PetscErrorCode Fft1DTransportSolver(PetscInt n_x, PetscScalar a_x, PetscScalar dt, PetscScalar delta_x, Vec X, Vec b,
                                    Mat FFT_MAT);
PetscErrorCode PetscFft3DTransportSolver(struct StructuredTransportContext customCtx, Vec b, Vec x);
PetscErrorCode FftTransportSolver(PetscInt n_x, PetscInt n_y, PetscInt n_z, PetscScalar lambda_x,
                                  PetscScalar lambda_y, PetscScalar lambda_z, Vec X, Vec b, Mat FFT_MAT);
/* X = (1/size) F^T(F(b) ./ Diag) as one fused apply.  Difference from the reference
 * (src/FftLinearSolver_3D.c:170-176): b_hat, the reference's scratch vector, is neither read nor
 * written -- after the call it does NOT hold F(b) ./ Diag, in the complex and the real-scalar
 * build alike (a caller that wants the divided spectrum calls MatMult and VecPointwiseDivide).
 * Real scalars: Diag, b_hat are half spectra; X is the correct real solve (not the reference's
 * 2 (size/4 + 1)-entry divide and 2/size scale); several ranks work in both builds. */
PetscErrorCode solve_3D(Mat FFT_MAT, Vec X, Vec Diag, Vec b, Vec b_hat, PetscInt size);
PetscErrorCode build_diag_mat_vec_3D(Vec Diag, Vec c_x_hat, Vec c_y_hat, Vec c_z_hat, PetscInt n_x, PetscInt n_y,
                                     PetscInt n_z, PetscScalar lambda_x, PetscScalar lambda_y, PetscScalar lambda_z);
PetscErrorCode build_transport_col(Vec c, PetscInt size);

/* ---- helpers that are not in the reference */
/* FFT matrix backed by the HIP plan (what MatCreateFFT(.., MATFFTW, ..) returns here) */
PetscErrorCode MatCreateFFTHIP(MPI_Comm comm, PetscInt ndim, const PetscInt dims[], Mat *A);
/* the plan behind an FFT matrix made by MatCreateFFT/MatCreateFFTHIP (NULL otherwise) */
PetscErrorCode MatFFTHIPGetPlan(Mat A, cfp_plan_t *plan);
/* the z-slab plan behind an FFT matrix made on a communicator of several ranks (NULL on one) */
PetscErrorCode MatFFTHIPGetDistPlan(Mat A, struct cfp_dist_plan_s **plan);
/* How many solve_3D calls on this FFT matrix divided by the plan's own symbol in registers
 * (Diag untouched since setupFFTPrec3D materialised it: same object id and PetscObjectState,
 * symbol unchanged) and how many streamed the Diag they were given. */
PetscErrorCode MatFFTHIPGetSolveCounts(Mat A, PetscInt *own_symbol, PetscInt *explicit_diag);
/* Side table of this build's per-context additions (not in the struct, see above).
 * remapBack: Cartesian -> mesh remap applied to the solve's result (NULL, the default: x stays
 * on the Cartesian grid, as the reference's apply leaves it).  The Mat stays the caller's.
 * getFFTPrec3DContext and FFTPrecTransportContextDestroy clear the entry of their ctx. */
PetscErrorCode FFTPrecTransportContextSetRemapBack(FFTPrecTransportContext *ctx, Mat remapBack);
PetscErrorCode FFTPrecTransportContextGetRemapBack(const FFTPrecTransportContext *ctx, Mat *remapBack);
PetscErrorCode FFTPrecTransportContextCreate(FFTPrecTransportContext **ctx);
PetscErrorCode FFTPrecTransportContextDestroy(FFTPrecTransportContext **ctx);
/* the library's context slot that the 13-argument C++ form below fills */
FFTPrecTransportContext *FFTPrecTransportContextLast(void);

#ifdef __cplusplus
}

#include <cstddef>
#include <type_traits>

/* The reference's own 13-argument form, `Mesh srcMesh` by value (src/PCSHELLFft_3D.hxx:27-41),
 * so a reference caller compiles unchanged against this header.  The mesh is not read (the
 * reference does not read it either, src/PCSHELLFft_3D.cxx:101-151); the context lands in the
 * library slot FFTPrecTransportContextLast(), where a caller can pick it up -- the reference
 * writes it through an uninitialised pointer and loses it.  A call
 * whose last argument is an FFTPrecTransportContext * resolves to the C function above; the
 * template takes class types only, so NULL / 0 / nullptr there still reach the C function and its
 * PETSC_ERR_ARG_NULL check.  The slot is one process-wide object (not thread-safe; each call
 * overwrites it). */
template <class MeshT, typename std::enable_if<!std::is_pointer<MeshT>::value && !std::is_integral<MeshT>::value &&
                                                   !std::is_same<MeshT, std::nullptr_t>::value,
                                               int>::type = 0>
inline PetscErrorCode getFFTPrec3DContext(PetscInt ndim, PetscScalar dt, PetscInt nbCells, PetscScalar a_x,
                                          PetscScalar a_y, PetscScalar a_z, PetscScalar Xmin, PetscScalar Ymin,
                                          PetscScalar Zmin, PetscScalar Xmax, PetscScalar Ymax, PetscScalar Zmax,
                                          MeshT srcMesh) {
  (void)srcMesh;
  return getFFTPrec3DContext(ndim, dt, nbCells, a_x, a_y, a_z, Xmin, Ymin, Zmin, Xmax, Ymax, Zmax,
                             FFTPrecTransportContextLast());
}
#endif
#endif /* CFP_PCSHELL_FFT3D_H */
