/*
 * circulant_fft_real.h -- real-data variant of the circulant apply.
 *
 * The reference's real-scalar branch of solve_3D (src/FftLinearSolver_3D.c:6-78, 166-190:
 * MATFFTW r2c, VecPointwiseDivideForRealFFT on the half spectrum, c2r, VecScale(X, 2./size))
 * for a PETSc built with real scalars.  For real b and a real transport symbol
 * (lambda_d real, so Diag(-k) = conj(Diag(k))) the solution x is real and only half of the
 * spectrum is needed: this plan reads and writes real arrays (8 bytes per cell) and moves
 * ~80 N bytes per apply instead of the complex plan's 160 N.
 *
 * Schedule: r2c along x (each real row is read as nx/2 complex values, FFT of length nx/2,
 * even/odd split with the mirror bin from the partner lane), the y and z passes of the
 * complex plan over the nx/2 x ny x nz half spectrum (+ the Nyquist column kx = nx/2 as its own
 * 1 x ny x nz grid), z fused with the symbol, inverse y, then c2r along x with the 1/N scale.
 * Requires nx even with nx/2 in {16, 32, ..., 512} and ny * nz > 1.
 *
 * At 256^3 the default is a 3-sweep schedule (cfp_three_pass.hip): r2c rows + the 32-point y1
 * DFT of a four-step y split | y2 + z + divide + inverse on the half spectrum | y1 inverse + c2r
 * rows, ~32 N bytes per apply.
 */
#ifndef CFP_CIRCULANT_FFT_REAL_H
#define CFP_CIRCULANT_FFT_REAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfp_rplan_s *cfp_rplan_t;
int cfp_rplan_create(cfp_rplan_t *plan, int64_t nx, int64_t ny, int64_t nz, int device);
int cfp_rplan_destroy(cfp_rplan_t plan);
/* real lambda_x, lambda_y, lambda_z of the transport symbol 1 + sum_d lambda_d (1 - e^{-i theta_d}) */
int cfp_rplan_set_symbol_transport(cfp_rplan_t plan, const double lam[3]);
/* x = C^{-1} b for real b (nx*ny*nz doubles on the device); x may alias b */
int cfp_rplan_apply(cfp_rplan_t plan, const double *b, double *x, void *stream);
/* schedule: CFP_RSCHEDULE_AUTO (3 sweeps at 128^3 and 256^3, else r2c + 3 half-spectrum passes + c2r),
 * CFP_RSCHEDULE_FIVE (always the latter) or CFP_RSCHEDULE_THREE (128^3 and 256^3 only, else CFP_ERR_SUP) */
#define CFP_RSCHEDULE_AUTO 0
#define CFP_RSCHEDULE_FIVE 1
#define CFP_RSCHEDULE_THREE 2
/* the 3-sweep schedule with the row sweeps' FFT exchanges behind workgroup barriers instead of
 * wave-local (the r04 kernels before r04ab; A/B); 128^3 and 256^3 only */
#define CFP_RSCHEDULE_THREE_ALT 3
int cfp_rplan_set_schedule(cfp_rplan_t plan, int schedule);
/* *three = 1 when the next apply runs the 3-sweep schedule */
int cfp_rplan_schedule(cfp_rplan_t plan, int *three);
/* launches of one apply and their mean duration (ms) over `iters` applies */
int cfp_rplan_num_passes(cfp_rplan_t plan, int *passes);
int cfp_rplan_time_passes(cfp_rplan_t plan, const double *b, double *x, int iters, double *ms_out, void *stream);

/* Layout conversions of the real-scalar PETSc boundary (include/pcshell_fft3d.h built with
 * -DCFP_REAL_SCALAR), device arrays, stream-ordered:
 *   cfp_real_to_complex       z[i] = (x[i], 0), n values
 *   cfp_complex_real_part     x[i] = scale * Re z[i]
 *   cfp_half_spectrum_extract half = the [nz][ny][nx/2 + 1] complex r2c half spectrum (FFTW's
 *                             r2c output layout, a real-scalar MATFFTW's MatMult) of the full
 *                             [nz][ny][nx] spectrum
 *   cfp_half_spectrum_extend  the full spectrum from the half by Hermitian symmetry,
 *                             X(kx, ky, kz) = conj X(nx - kx, -ky, -kz) for kx > nx/2
 *   cfp_half_spectrum_pad     rows of nx: Z(kx) = w(kx) S(kx) / D(kx) for kx <= nx/2 (w = 1 at
 *                             kx = 0 and, nx even, kx = nx/2; else 2), 0 above; S = half
 *                             ([rows][nx/2 + 1]) or, half == NULL, full in place; D = diag (half
 *                             layout; 0 where D = 0) or 1 when NULL.  Re IDFT(Z) is the c2r of
 *                             the half spectrum, row-local (no -kz mirror from another z-slab). */
int cfp_real_to_complex(const double *x, double *z, int64_t n, void *stream);
int cfp_complex_real_part(const double *z, double *x, int64_t n, double scale, void *stream);
int cfp_half_spectrum_extract(const double *full, double *half, int64_t nx, int64_t ny, int64_t nz, void *stream);
int cfp_half_spectrum_extend(const double *half, double *full, int64_t nx, int64_t ny, int64_t nz, void *stream);
int cfp_half_spectrum_pad(const double *half, const double *diag, double *full, int64_t nx, int64_t rows,
                          void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CFP_CIRCULANT_FFT_REAL_H */
