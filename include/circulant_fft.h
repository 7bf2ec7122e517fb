/*
 * circulant_fft.h -- C ABI of the MI355X-native circulant FFT preconditioner (libcirculant_fft.so).
 *
 * This is the plan-level boundary.  Every pointer argument named `*_dev` is a device
 * pointer (hipMalloc'd, HBM-resident); complex values are interleaved (re, im) doubles;
 * grids are x-fastest, i = ix + nx*(iy + ny*iz) -- the row-major {nz, ny, nx} layout of the
 * reference's MatCreateFFT(..., dims = {n_z, n_y, n_x}) (src/PCSHELLFft_3D.cxx:34-35).
 * `stream` is a hipStream_t (NULL = default stream).  Calls that take a stream only
 * enqueue work (stream-ordered, like any HIP library call); cfp_stream_sync() waits.
 *
 * Return values are error codes numerically equal to PETSc's (petscerror.h): 0 =
 * PETSC_SUCCESS, so a PETSc caller may PetscCall() them directly.  cfp_last_error()
 * returns a message for the calling thread's last failure.
 *
 * What each entry replaces in the reference (/root/reference):
 *   cfp_plan_create + cfp_plan_set_symbol_*      setupFFTPrec3D            src/PCSHELLFft_3D.cxx:26-84
 *                                                (MatCreateFFT + Diag build, src/FftLinearSolver_3D.c:136-164)
 *   cfp_plan_apply                               solve_3D (complex build)  src/FftLinearSolver_3D.c:166-190
 *                                                (the arithmetic of applyFFT3DPrecTransport, src/PCSHELLFft_3D.cxx:10-24)
 *   cfp_plan_apply_with_diag                     solve_3D with a caller-owned Diag Vec  :166-190
 *   cfp_plan_forward / cfp_plan_backward         MatMult / MatMultTranspose on MATFFTW (:170, :180)
 *   cfp_pointwise_divide / cfp_scale             VecPointwiseDivide (:174) / VecScale (:184)
 *   cfp_build_diag_3d                            build_diag_mat_vec_3D      :136-164
 *   cfp_transport_symbol_1d                      build_transport_col + 1-D MatMult (:80-90, :235-249)
 *   cfp_plan_destroy                             destroyFFTPrec3D           src/PCSHELLFft_3D.cxx:86-99
 * The PETSc-typed PCSHELL callbacks themselves are declared in pcshell_fft3d.h.
 */
#ifndef CIRCULANT_FFT_H
#define CIRCULANT_FFT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (values of petscerror.h) */
#define CFP_SUCCESS 0
#define CFP_ERR_MEM 55         /* PETSC_ERR_MEM */
#define CFP_ERR_SUP 56         /* PETSC_ERR_SUP: unsupported size / layout */
#define CFP_ERR_ARG_SIZ 60     /* PETSC_ERR_ARG_SIZ */
#define CFP_ERR_ARG_WRONG 62   /* PETSC_ERR_ARG_WRONG */
#define CFP_ERR_ARG_OUTOFRANGE 63 /* PETSC_ERR_ARG_OUTOFRANGE */
#define CFP_ERR_ARG_WRONGSTATE 73 /* PETSC_ERR_ARG_WRONGSTATE (no symbol set yet) */
#define CFP_ERR_LIB 76         /* PETSC_ERR_LIB: HIP / RCCL runtime failure */
#define CFP_ERR_ARG_NULL 85    /* PETSC_ERR_ARG_NULL */

typedef struct cfp_plan_s *cfp_plan_t;

/* ---- version / diagnostics */
const char *cfp_version(void);
const char *cfp_last_error(void);
int cfp_device_count(int *count);
int cfp_stream_sync(void *stream);
/* Device-to-device copy of `bytes` on `stream` with the library's copy kernel (16-byte lanes,
 * non-temporal stores; the stand-in VecCopy uses it).  Unaligned or non-multiple-of-16 sizes go
 * through hipMemcpyAsync.  bench.py times it as the box's copy rate beside the roofline. */
int cfp_device_copy(void *dst, const void *src, size_t bytes, void *stream);

/* ---- single-GPU plan: n_x, n_y, n_z >= 1; `device` = HIP ordinal.  Axes up to 4096 take one
 * pass each (powers of two 16..1024 register-resident, others LDS mixed-radix); a longer axis
 * must be a product n1 n2 of two factors <= 4096 (four-step: two passes, spectrum kept in
 * four-step order) -- for such plans cfp_plan_forward/backward and an explicit Diag
 * (cfp_plan_set_diag, cfp_plan_apply_with_diag) return CFP_ERR_SUP; the symbol applies work. */
int cfp_plan_create(cfp_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int device);
int cfp_plan_destroy(cfp_plan_t plan);

/* Transport symbol in closed form: Diag[k] = 1 + sum_d lambda_d (1 - e^{-2 pi i k_d / n_d}),
 * lam = {lx.re, lx.im, ly.re, ly.im, lz.re, lz.im}.  Axes with n_d == 1 contribute 0
 * (build_transport_col leaves a size-1 column zero, src/FftLinearSolver_3D.c:83). */
int cfp_plan_set_symbol_transport(cfp_plan_t plan, const double lam[6]);
/* Separable symbol from caller-given 1-D eigenvalue vectors (host arrays of n_x, n_y, n_z
 * complex values, e.g. the 1-D DFTs of arbitrary circulant columns):
 * Diag = 1 + lx*tile(cx_hat) + ly*repeat(tile(cy_hat)) + lz*repeat(cz_hat)   (:136-164). */
int cfp_plan_set_symbol_separable(cfp_plan_t plan, const double *cx_hat, const double *cy_hat,
                                  const double *cz_hat, const double lam[6]);
/* General symbol: an explicit Diag vector of N complex values (copied into the plan).
 * diag_is_device != 0 means `diag` is a device pointer. */
int cfp_plan_set_diag(cfp_plan_t plan, const double *diag, int diag_is_device);
/* Counter bumped by every symbol setter above (set_symbol_*, set_diag), whoever calls it: a
 * caller that cached "the plan holds the symbol I set" compares versions instead. */
int cfp_plan_symbol_version(cfp_plan_t plan, uint64_t *version);
/* Materialise the plan's current symbol as a full Diag vector (device). */
int cfp_plan_get_diag(cfp_plan_t plan, double *diag_dev, void *stream);

/* x = (1/N) * IDFT3( DFT3(b) ./ Diag ): one PCApply / one direct solve.
 * b_dev may alias x_dev (the direct solver passes Un, Un). */
int cfp_plan_apply(cfp_plan_t plan, const double *b_dev, double *x_dev, void *stream);
/* Same with a caller-owned Diag vector (device), as solve_3D(FFT_MAT, X, Diag, b, b_hat, size). */
int cfp_plan_apply_with_diag(cfp_plan_t plan, const double *diag_dev, const double *b_dev, double *x_dev,
                             void *stream);
/* Host-buffer variant (PCIe-inclusive): stages b through the plan's device buffers. Synchronous. */
int cfp_plan_apply_host(cfp_plan_t plan, const double *b_host, double *x_host);
/* Same with a caller-owned device Diag (solve_3D on host Vecs with an explicit Diag). */
int cfp_plan_apply_with_diag_host(cfp_plan_t plan, const double *diag_dev, const double *b_host, double *x_host);

/* ---- the Krylov step around a PCApply, fused into the apply's sweeps (not in the reference; the
 * stand-in GMRES's MatMult -> PCApply -> VecMDot chain of tests/TransportEquation_SphericalExplosion_
 * impl_mpi.cxx:120-136, PETSc's KSP_PCApplyBAorAB followed by KSPGMRESClassicalGramSchmidt's VecMDot).
 *
 * pre: the apply reads y = A b instead of b, A in row-class diagonal form (the stand-in AIJ's
 *   k_dia_spmv layout): row r has class cls[r] < ncls; class c has the entries tab[c nd + k]
 *   (complex) on the diagonals off[k] (column - row, ascending) whose bit k is set in mask[c].
 *   x_local != 0 asserts that every present entry stays inside the row's x-line (column and row
 *   in one run of n_x consecutive indices).
 * post: after the apply, out[2 j], out[2 j + 1] = (re, im) of v[j]^H x for j < nv (v[j] == NULL:
 *   x itself, so out[2 j] = |x|^2); out is a device array of 2 nv doubles, written on `stream`.
 * fused (output): 1 when both ran inside the apply's own sweeps (the 256^3 3-sweep schedule: P1
 *   streams b once and forms A b in registers when the stencil is x-local with diagonals in
 *   {-1, 0, +1} and ncls <= 16; P3 reads the v[j] beside its stores, nv <= 4), 0 when they ran
 *   as separate kernels around a plain apply (same results up to rounding).  b must not alias x
 *   when pre is given. */
typedef struct {
  const unsigned char *cls;   /* [N] device */
  const unsigned char *mask;  /* [ncls] device */
  const double *tab;          /* [ncls * nd] complex, device */
  int64_t off[8];
  int nd, ncls, x_local;
  const unsigned char *cls_x; /* optional [n_x] device: cls[r] = cls_x[r mod n_x] for every row
                               * (classes set by x alone, as an operator coupling along x only);
                               * the fused P1 then reads one byte per column instead of N */
} cfp_stencil_t;
typedef struct {
  const cfp_stencil_t *pre; /* NULL: none */
  int post_nv;              /* 0: none; at most 8 */
  const double *post_v[8];
  double *post_out;
  int fused;
} cfp_apply_ex_t;
int cfp_plan_apply_ex(cfp_plan_t plan, const double *b_dev, double *x_dev, void *stream, cfp_apply_ex_t *ex);
/* *fusable = 1 when cfp_plan_apply_ex with this stencil (NULL: none) and post_nv dots would run
 * them inside the apply (ex->fused = 1); a caller for which the separate kernels are no gain (they
 * are what it would launch itself) asks first. */
int cfp_plan_apply_ex_fusable(cfp_plan_t plan, const cfp_stencil_t *pre, int post_nv, int *fusable);

/* Unnormalised 3-D transforms: forward (e^{-}, MatMult) and backward (e^{+}, MatMultTranspose). */
int cfp_plan_forward(cfp_plan_t plan, const double *in_dev, double *out_dev, void *stream);
int cfp_plan_backward(cfp_plan_t plan, const double *in_dev, double *out_dev, void *stream);

/* Schedule option: > 0 runs the x and y passes of 3-D grids alternately over blocks of
 * `chunk_planes` z-planes (Infinity-Cache-resident hand-off between the two passes);
 * 0 (default) = one launch per axis pass. */
int cfp_plan_set_chunking(cfp_plan_t plan, int64_t chunk_planes);

/* HIP-graph replay of cfp_plan_apply (off by default).  On: the first apply of a (b, x) pair
 * runs eagerly and captures its launches into a graph; later applies of the same pair launch
 * that graph into the caller's stream (one host call instead of 3-5 kernel launches, for the
 * launch-bound small grids inside GMRES).  Up to 64 pairs are kept; every setter that changes
 * buffers or the schedule drops them.  Values written into the plan's symbol / Diag are seen;
 * profiling applies (cfp_plan_profile_begin) run eagerly.  Measured on MI355X / ROCm 7 it is
 * ~6 us SLOWER per host-synchronous apply than the direct launches at every grid from 32^3 to
 * 256^3 (profiles/r02z_graph_timing.txt), so it stays off by default. */
int cfp_plan_set_graph(cfp_plan_t plan, int on);

/* Apply schedule.  FIVE_PASS: x, y fwd, z fused with the symbol, y, x inv.
 * FIVE_PASS_YFUSED: x, z fwd, y fused, z, x inv.  AUTO (default): THREE_PASS on 256^3 plans
 * (separable symbol, no chunking), YFUSED when ny, nz >= 512, else FIVE_PASS.  THREE_PASS
 * (128^3 and 256^3 plans only, CFP_ERR_SUP
 * otherwise; an explicit Diag still takes 5 passes): x + first y stage | last y stage + z +
 * symbol + inverses | inverse of the first, 96 N bytes instead of 160 N.
 * PLANE (n_x = n_y in {32, 64, 100, 128}, n_z > 1; CFP_ERR_SUP otherwise; AUTO picks it for
 * n_x = n_y = 100 when THREE_PASS does not apply, 64 and 32): x + y DFTs of whole z-planes | z fused with
 * the symbol | inverse planes, 3 launches instead of 5 (any symbol, explicit Diag included). */
#define CFP_SCHEDULE_AUTO 0
#define CFP_SCHEDULE_FIVE_PASS 1
#define CFP_SCHEDULE_THREE_PASS 2
#define CFP_SCHEDULE_FIVE_PASS_YFUSED 3
#define CFP_SCHEDULE_PLANE 4
int cfp_plan_set_schedule(cfp_plan_t plan, int schedule);
/* Kernel shape of the 3-sweep schedule at 256^3, for tests and measurements (0, 0 = the
 * measured default; the shape never changes the result beyond rounding).  n1: the y split
 * ny = n1 * (256 / n1), 0 (default), 32 or 64.  mid: the middle kernel, 0 (default = SWAP64_PF),
 * CFP_TP_MID_LANE64 (y2 DFT across lanes, 64-column tile), CFP_TP_MID_LANE32 (32-column tile) or
 * CFP_TP_MID_SWAP64 (y2 DFT on v_permlane32/16_swap register transposes, 64-column tile;
 * 256^3 only, 128^3 keeps its default).  Other values: CFP_ERR_ARG_OUTOFRANGE. */
#define CFP_TP_MID_DEFAULT 0
#define CFP_TP_MID_LANE64 1
#define CFP_TP_MID_LANE32 2
#define CFP_TP_MID_SWAP64 3
#define CFP_TP_MID_SWAP64_PF 4 /* SWAP64 + LDS-DMA prefetch of half the next unit */
int cfp_plan_set_three_pass_shape(cfp_plan_t plan, int n1, int mid);

/* Introspection: number of kernel launches of one apply, and per-launch timing.
 * cfp_plan_time_passes runs `iters` applies and writes the mean duration (ms) of each of the
 * apply's launches into ms_out[0..passes) (HIP events on `stream`). */
int cfp_plan_num_passes(cfp_plan_t plan, int *passes);
int cfp_plan_pass_info(cfp_plan_t plan, int pass, int *axis, int *n, int64_t *ncols, int *mode, int *fast);
int cfp_plan_time_passes(cfp_plan_t plan, const double *b_dev, double *x_dev, int iters, double *ms_out,
                         void *stream);
/* Profiling mode: every `every`-th following call of cfp_plan_apply (the first, then every-th
 * after it; at most max_applies of them) records one HIP event per launch on its stream -- the
 * caller's own timed applies, no extra launches.  Sampling keeps the events' cost (a few us
 * per apply) out of the caller's throughput.  _profile_end synchronises on the last event and
 * writes the mean duration (ms) of each launch (cfp_plan_num_passes entries) and the number
 * of applies recorded. */
int cfp_plan_profile_begin(cfp_plan_t plan, int max_applies, int every);
int cfp_plan_profile_end(cfp_plan_t plan, double *ms_out, int *applies);

/* ---- vector kernels (device arrays of n complex values) */
int cfp_pointwise_divide(double *w_dev, const double *x_dev, const double *y_dev, int64_t n, void *stream);
int cfp_scale(double *x_dev, double alpha_re, double alpha_im, int64_t n, void *stream);
/* synthetic input of SURVEY.md §8d: element i gets U[-1,1)^2 from SplitMix64(seed ^ 2(i+offset)),
 * SplitMix64(seed ^ 2(i+offset)+1) */
int cfp_fill_uniform(double *x_dev, int64_t n, uint64_t seed, int64_t offset, void *stream);
/* build_diag_mat_vec_3D on device from three device 1-D vectors */
int cfp_build_diag_3d(double *diag_dev, const double *cx_hat_dev, const double *cy_hat_dev,
                      const double *cz_hat_dev, int64_t nx, int64_t ny, int64_t nz, const double lam[6],
                      void *stream);
/* host: out[k] = DFT(1, -1, 0, ...)[k] = 1 - e^{-2 pi i k/n} (0 for n == 1), n complex values */
int cfp_transport_symbol_1d(int64_t n, double *out_host);

#ifdef __cplusplus
}
#endif
#endif /* CIRCULANT_FFT_H */
