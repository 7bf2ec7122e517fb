/*
 * cfp_oracle.c -- CPU restatement of the reference circulant FFT solver.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path (circulantpreconditioner_amd/).  Only tests/, the smoke() entry
 * of __graft_entry__.py and the cpu_baseline leg of bench.py may load it.  The
 * product never links, calls or falls back to it.
 *
 * What it restates (all citations into /root/reference):
 *   build_transport_col            src/FftLinearSolver_3D.c:80-90
 *   vec_kronecker_product_identity_left/right   :92-134
 *   build_diag_mat_vec_3D          :136-164
 *   solve_3D (complex build)       :166-190   FFT -> divide -> IFFT -> 1/N
 *   MatMult / MatMultTranspose on MATFFTW (third-party FFTW semantics):
 *       unnormalised DFT over row-major dims {n_z, n_y, n_x} (x fastest),
 *       forward kernel e^{-2 pi i jk/n}, transpose/backward e^{+...}
 *       (src/PCSHELLFft_3D.cxx:34-35, tests/FFTDirectSolver/testFftSolver_3D.py:38-52)
 *   the circulant operator C = I + sum_d lambda_d (I - S_d)
 *       tests/FFTDirectSolver/testFftSolver_3D.py:12-24 (build_C_3D), applied
 *       matrix-free as a stencil.
 *
 * The FFT is a plain recursive mixed-radix decimation-in-time transform valid
 * for any n (generic O(p^2) butterflies for each prime factor p), twiddles from
 * long-double sin/cos.  FFTW itself is not present in this image; parity of
 * this restatement is pinned by tests/golden/ (fixtures generated from the
 * reference's own Python oracle functions, tests/golden/make_golden.py).
 *
 * Data: complex double, interleaved (re, im), i = ix + nx*(iy + ny*iz).
 */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef double complex cplx;
typedef int64_t i64;

static int g_threads = 1;

void oracle_set_threads(int n) { g_threads = n > 0 ? n : 1; }
int oracle_get_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------------------- 1-D FFT */

static i64 smallest_factor(i64 n) {
    if (n % 4 == 0) return 4;
    if (n % 2 == 0) return 2;
    for (i64 p = 3; p * p <= n; p += 2)
        if (n % p == 0) return p;
    return n;
}

/* table[k] = exp(sign * 2 pi i k / N), k in [0, N) */
static cplx *make_table(i64 N, int sign) {
    cplx *t = (cplx *)malloc(sizeof(cplx) * (size_t)(N > 0 ? N : 1));
    for (i64 k = 0; k < N; ++k) {
        long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)N;
        t[k] = (double)cosl(a) + (double)(sign * sinl(a)) * I;
    }
    return t;
}

/* out[0..n) = DFT_n(in[0], in[is], ...), W_n^j = tw[(j * ts) % N] */
static void fft_rec(i64 n, const cplx *in, i64 is, cplx *out, const cplx *tw, i64 ts, i64 N, cplx *scratch) {
    if (n == 1) { out[0] = in[0]; return; }
    i64 p = smallest_factor(n), m = n / p;
    for (i64 r = 0; r < p; ++r)
        fft_rec(m, in + r * is, is * p, out + r * m, tw, ts * p, N, scratch);
    /* butterflies: X[k + q m] = sum_r W_n^{r k} Y_r[k] W_p^{r q} */
    for (i64 k = 0; k < m; ++k) {
        for (i64 r = 0; r < p; ++r)
            scratch[r] = out[r * m + k] * tw[((r * k) % n) * ts % N];
        for (i64 q = 0; q < p; ++q) {
            cplx acc = 0;
            for (i64 r = 0; r < p; ++r)
                acc += scratch[r] * tw[(((r * q) % p) * m) * ts % N];
            out[q * m + k] = acc;
        }
    }
}

/* In-place 1-D DFT of a strided line (unnormalised). */
static void dft_line(i64 n, cplx *data, i64 stride, const cplx *tw, cplx *buf, cplx *out, cplx *scratch) {
    for (i64 k = 0; k < n; ++k) buf[k] = data[k * stride];
    fft_rec(n, buf, 1, out, tw, 1, n, scratch);
    for (i64 k = 0; k < n; ++k) data[k * stride] = out[k];
}

/* Public 1-D transform: out = DFT(in), sign -1 forward / +1 backward. */
void oracle_dft1d(i64 n, int sign, const double *in, double *out) {
    cplx *tw = make_table(n, sign);
    cplx *buf = (cplx *)malloc(sizeof(cplx) * (size_t)n);
    cplx *scratch = (cplx *)malloc(sizeof(cplx) * (size_t)n);
    memcpy(buf, in, sizeof(cplx) * (size_t)n);
    fft_rec(n, buf, 1, (cplx *)out, tw, 1, n, scratch);
    free(tw); free(buf); free(scratch);
}

/* Unnormalised 3-D DFT over dims {nz, ny, nx} (MatMult on MATFFTW for sign=-1,
 * MatMultTranspose for sign=+1).  in may alias out. */
void oracle_fft3d(i64 nx, i64 ny, i64 nz, int sign, const double *in, double *out) {
    i64 N = nx * ny * nz;
    cplx *d = (cplx *)out;
    if ((const double *)in != out) memcpy(out, in, sizeof(cplx) * (size_t)N);
    i64 dims[3] = {nx, ny, nz};
    i64 strides[3] = {1, nx, nx * ny};
    for (int ax = 0; ax < 3; ++ax) {
        i64 n = dims[ax], s = strides[ax];
        if (n == 1) continue;
        cplx *tw = make_table(n, sign);
        i64 nlines = N / n;
#pragma omp parallel num_threads(g_threads)
        {
            cplx *buf = (cplx *)malloc(sizeof(cplx) * (size_t)n);
            cplx *o = (cplx *)malloc(sizeof(cplx) * (size_t)n);
            cplx *scratch = (cplx *)malloc(sizeof(cplx) * (size_t)n);
#pragma omp for schedule(static)
            for (i64 l = 0; l < nlines; ++l) {
                /* line l -> base offset: lines enumerate all indices with the axis coordinate 0 */
                i64 lo = l % s, hi = l / s;
                i64 base = lo + hi * s * n;
                dft_line(n, d + base, s, tw, buf, o, scratch);
            }
            free(buf); free(o); free(scratch);
        }
        free(tw);
    }
}

/* --------------------------------------------------- Diag construction */

/* build_transport_col, src/FftLinearSolver_3D.c:80-90: c = (1, -1, 0, ...) if size > 1, else 0 */
void oracle_build_transport_col(i64 n, double *c) {
    memset(c, 0, sizeof(cplx) * (size_t)n);
    if (n > 1) { c[0] = 1.0; c[2] = -1.0; }
}

/* vec_kronecker_product_identity_left, :92-112: res[j*c_size + i] = lambda*c[i] */
void oracle_kron_left(const double *c, double *res, i64 c_size, i64 id_size, double lre, double lim) {
    const cplx *cc = (const cplx *)c;
    cplx *r = (cplx *)res;
    cplx lam = lre + lim * I;
    for (i64 i = 0; i < c_size; ++i) {
        cplx cur = cc[i] * lam;
        for (i64 j = 0; j < id_size; ++j) r[j * c_size + i] = cur;
    }
}

/* vec_kronecker_product_identity_right, :114-134: res[i*id_size + j] = lambda*c[i] */
void oracle_kron_right(const double *c, double *res, i64 c_size, i64 id_size, double lre, double lim) {
    const cplx *cc = (const cplx *)c;
    cplx *r = (cplx *)res;
    cplx lam = lre + lim * I;
    for (i64 i = 0; i < c_size; ++i) {
        cplx cur = cc[i] * lam;
        for (i64 j = 0; j < id_size; ++j) r[i * id_size + j] = cur;
    }
}

/* build_diag_mat_vec_3D, :136-164:
 *   Diag = ((kpi_x + kpi_y) + kpi_z) + 1  with
 *   kpi_x = kron_left(cx_hat, nx, ny*nz, lx)
 *   kpi_y = kron_right(kron_left(cy_hat, ny, nz, ly), ny*nz, nx, 1)
 *   kpi_z = kron_right(cz_hat, nz, nx*ny, lz)
 * (the sum vector starts from a VecDuplicate, i.e. zero, then three AXPYs and a shift). */
void oracle_build_diag_3d(double *diag, const double *cx_hat, const double *cy_hat, const double *cz_hat,
                          i64 nx, i64 ny, i64 nz, const double *lam /* 6 doubles: lx re,im, ly, lz */) {
    i64 N = nx * ny * nz;
    cplx *kx = (cplx *)malloc(sizeof(cplx) * (size_t)N);
    cplx *ky = (cplx *)malloc(sizeof(cplx) * (size_t)N);
    cplx *kyi = (cplx *)malloc(sizeof(cplx) * (size_t)(ny * nz));
    cplx *kz = (cplx *)malloc(sizeof(cplx) * (size_t)N);
    oracle_kron_left(cx_hat, (double *)kx, nx, ny * nz, lam[0], lam[1]);
    oracle_kron_left(cy_hat, (double *)kyi, ny, nz, lam[2], lam[3]);
    oracle_kron_right((double *)kyi, (double *)ky, ny * nz, nx, 1.0, 0.0);
    oracle_kron_right(cz_hat, (double *)kz, nz, nx * ny, lam[4], lam[5]);
    cplx *d = (cplx *)diag;
    for (i64 i = 0; i < N; ++i) {
        cplx s = 0;
        s += kx[i];
        s += ky[i];
        s += kz[i];
        d[i] = s + 1.0;
    }
    free(kx); free(ky); free(kyi); free(kz);
}

/* The setup chain of FftTransportSolver (:218-249) / setupFFTPrec3D
 * (src/PCSHELLFft_3D.cxx:39-69): transport columns -> 1-D forward DFT -> Diag. */
void oracle_build_diag_transport(i64 nx, i64 ny, i64 nz, const double *lam, double *diag) {
    i64 n[3] = {nx, ny, nz};
    double *col[3], *hat[3];
    for (int a = 0; a < 3; ++a) {
        col[a] = (double *)malloc(sizeof(cplx) * (size_t)n[a]);
        hat[a] = (double *)malloc(sizeof(cplx) * (size_t)n[a]);
        oracle_build_transport_col(n[a], col[a]);
        oracle_dft1d(n[a], -1, col[a], hat[a]);
    }
    oracle_build_diag_3d(diag, hat[0], hat[1], hat[2], nx, ny, nz, lam);
    for (int a = 0; a < 3; ++a) { free(col[a]); free(hat[a]); }
}

/* ------------------------------------------------------------- solve_3D */

/* solve_3D, src/FftLinearSolver_3D.c:166-190 (complex build):
 *   b_hat = F b ; b_hat ./= Diag ; X = F^T b_hat ; X *= 1/size */
void oracle_solve_3d(i64 nx, i64 ny, i64 nz, const double *diag, const double *b, double *x) {
    i64 N = nx * ny * nz;
    cplx *bh = (cplx *)malloc(sizeof(cplx) * (size_t)N);
    oracle_fft3d(nx, ny, nz, -1, b, (double *)bh);
    const cplx *d = (const cplx *)diag;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (i64 i = 0; i < N; ++i) bh[i] = d[i] != 0 ? bh[i] / d[i] : 0;  /* PETSc VecPointwiseDivide: y = 0 -> 0 */
    oracle_fft3d(nx, ny, nz, +1, (double *)bh, x);
    cplx *xx = (cplx *)x;
    double s = 1. / (double)N;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (i64 i = 0; i < N; ++i) xx[i] = xx[i] * s;
    free(bh);
}

/* ---------------------------------------------------- operator C (stencil) */

/* y = C x with C = I + lx (I - Sx) + ly (I - Sy) + lz (I - Sz), (S_d u)[i] = u[i - e_d mod n_d]:
 * the matrix of testFftSolver_3D.py:12-24 (circulant column (1,-1,0,..) per axis).
 * Axes with n_d == 1 contribute nothing (column is zero, :83). */
void oracle_apply_circulant(i64 nx, i64 ny, i64 nz, const double *lam, const double *x, double *y) {
    const cplx *u = (const cplx *)x;
    cplx *v = (cplx *)y;
    cplx lx = lam[0] + lam[1] * I, ly = lam[2] + lam[3] * I, lz = lam[4] + lam[5] * I;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (i64 iz = 0; iz < nz; ++iz)
        for (i64 iy = 0; iy < ny; ++iy)
            for (i64 ix = 0; ix < nx; ++ix) {
                i64 i = ix + nx * (iy + ny * iz);
                cplx c = u[i];
                cplx acc = c;
                if (nx > 1) acc += lx * (c - u[(ix + nx - 1) % nx + nx * (iy + ny * iz)]);
                if (ny > 1) acc += ly * (c - u[ix + nx * ((iy + ny - 1) % ny + ny * iz)]);
                if (nz > 1) acc += lz * (c - u[ix + nx * (iy + ny * ((iz + nz - 1) % nz))]);
                v[i] = acc;
            }
}

/* Counter-based synthetic input: element i of the grid gets
 * Re, Im = U[-1,1) from SplitMix64(seed ^ (2i)), SplitMix64(seed ^ (2i+1)).
 * The HIP library has its own generator with the same definition; tests compare them. */
static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
void oracle_fill_uniform(i64 n, uint64_t seed, i64 offset, double *out) {
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (i64 i = 0; i < n; ++i) {
        uint64_t g = (uint64_t)(i + offset);
        uint64_t a = splitmix64(seed ^ (2 * g)), b = splitmix64(seed ^ (2 * g + 1));
        out[2 * i] = (double)(a >> 11) * 0x1.0p-52 - 1.0;
        out[2 * i + 1] = (double)(b >> 11) * 0x1.0p-52 - 1.0;
    }
}
