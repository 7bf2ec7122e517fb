// cfp_blas.hip -- device vector kernels (complex double) behind the PETSc-compatible Vec/Mat
// layer: axpy-family updates, PETSc-convention dot / norms, CSR SpMV.  These carry the
// GMRES harness, not the FFT hot path.
#include "cfp_blas.h"

namespace cfp {

#define BLAS_THREADS 256
#define RED_BLOCKS 1024

__device__ __forceinline__ cd bcadd(cd a, cd b) { return make_cd(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd bcmul(cd a, cd b) { return make_cd(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

static unsigned nblocks(i64 n) {
  i64 b = (n + BLAS_THREADS - 1) / BLAS_THREADS;
  if (b > 16384) b = 16384;
  return (unsigned)(b < 1 ? 1 : b);
}

#define GRID_LOOP(i, n) for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (i64)gridDim.x * blockDim.x)

__global__ void k_set(cd* x, cd a, i64 n) { GRID_LOOP(i, n) x[i] = a; }
__global__ void k_shift(cd* x, cd a, i64 n) { GRID_LOOP(i, n) x[i] = bcadd(x[i], a); }
__global__ void k_copy(cd* y, const cd* x, i64 n) { GRID_LOOP(i, n) y[i] = x[i]; }
// y = y + a x
__global__ void k_axpy(cd* y, cd a, const cd* x, i64 n) { GRID_LOOP(i, n) y[i] = bcadd(y[i], bcmul(a, x[i])); }
// y = x + b y
__global__ void k_aypx(cd* y, cd b, const cd* x, i64 n) { GRID_LOOP(i, n) y[i] = bcadd(x[i], bcmul(b, y[i])); }
// w = a x + y
__global__ void k_waxpy(cd* w, cd a, const cd* x, const cd* y, i64 n) {
  GRID_LOOP(i, n) w[i] = bcadd(bcmul(a, x[i]), y[i]);
}
__global__ void k_pmult(cd* w, const cd* x, const cd* y, i64 n) { GRID_LOOP(i, n) w[i] = bcmul(x[i], y[i]); }
// y += sum_j a_j x_j  (the GMRES basis update, up to MV_MAX vectors per launch)
__global__ void k_maxpy(cd* y, int k, MVCoef a, MVPtrs xs, i64 n) {
  GRID_LOOP(i, n) {
    cd acc = y[i];
    for (int j = 0; j < k; ++j) acc = bcadd(acc, bcmul(a.a[j], xs.p[j][i]));
    y[i] = acc;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// kind: 0 = dot y^H x (re, im), 1 = sum |x|^2, 2 = sum |re|+|im|, 3 = max |x|
__global__ void k_reduce(const cd* x, const cd* y, i64 n, int kind, double* partial) {
  __shared__ double s0[BLAS_THREADS / 64], s1[BLAS_THREADS / 64];
  double a = 0.0, b = 0.0;
  GRID_LOOP(i, n) {
    const cd u = x[i];
    if (kind == 0) {
      const cd v = y[i];  // u * conj(v)
      a += u.x * v.x + u.y * v.y;
      b += u.y * v.x - u.x * v.y;
    } else if (kind == 1) {
      a += u.x * u.x + u.y * u.y;
    } else if (kind == 2) {
      a += fabs(u.x) + fabs(u.y);
    } else {
      a = fmax(a, hypot(u.x, u.y));
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (kind == 3) a = wave_max(a);
  else { a = wave_sum(a); b = wave_sum(b); }
  if (lane == 0) { s0[w] = a; s1[w] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = s0[0], tb = s1[0];
    for (int k = 1; k < BLAS_THREADS / 64; ++k) {
      if (kind == 3) ta = fmax(ta, s0[k]);
      else { ta += s0[k]; tb += s1[k]; }
    }
    partial[2 * blockIdx.x] = ta;
    partial[2 * blockIdx.x + 1] = tb;
  }
}

// several dots against one vector, PETSc VecMDot(x, k, y[], val): val_j = y_j^H x.
// One sweep of x per launch; up to MDOT_K accumulators per thread.
#define MDOT_K 8
__global__ void k_mdot(const cd* x, int k, MVPtrs ys, i64 n, double* partial) {
  __shared__ double sm[2 * MDOT_K][BLAS_THREADS / 64];
  double a[MDOT_K], b[MDOT_K];
#pragma unroll
  for (int j = 0; j < MDOT_K; ++j) { a[j] = 0.0; b[j] = 0.0; }
  GRID_LOOP(i, n) {
    const cd u = x[i];
#pragma unroll
    for (int j = 0; j < MDOT_K; ++j) {
      if (j < k) {
        const cd v = ys.p[j][i];
        a[j] += u.x * v.x + u.y * v.y;
        b[j] += u.y * v.x - u.x * v.y;
      }
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < MDOT_K; ++j) {
    const double ra = wave_sum(a[j]), rb = wave_sum(b[j]);
    if (lane == 0) { sm[2 * j][w] = ra; sm[2 * j + 1][w] = rb; }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * k; t += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q < BLAS_THREADS / 64; ++q) s += sm[t][q];
    partial[(size_t)blockIdx.x * 2 * MDOT_K + t] = s;
  }
}

// y = (OW ? 0 : y) + sum_j a_j x_j, with NRM: per-block sums of |y|^2 of the result (one sweep)
template <bool OW, bool NRM>
__global__ void __launch_bounds__(BLAS_THREADS) k_maxpy_nrm(cd* y, int k, MVCoef a, MVPtrs xs, i64 n, double* partial) {
  double s2 = 0.0;
  GRID_LOOP(i, n) {
    cd acc = OW ? make_cd(0.0, 0.0) : y[i];
    for (int j = 0; j < k; ++j) acc = bcadd(acc, bcmul(a.a[j], xs.p[j][i]));
    y[i] = acc;
    if (NRM) s2 += acc.x * acc.x + acc.y * acc.y;
  }
  if constexpr (NRM) {
    __shared__ double sm[BLAS_THREADS / 64];
    s2 = wave_sum(s2);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s2;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int q = 0; q < BLAS_THREADS / 64; ++q) t += sm[q];
      partial[blockIdx.x] = t;
    }
  }
}

// CSR y = A x, one thread per row (rows of about one nonzero)
__global__ void k_csr_spmv(i64 m, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y) {
  GRID_LOOP(r, m) {
    cd acc = make_cd(0.0, 0.0);
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p) acc = bcadd(acc, bcmul(val[p], x[col[p]]));
    y[r] = acc;
  }
}

// CSR y = A x, L lanes per row: the lanes of a row read its nonzeros side by side, so a wave's
// loads of val / col are contiguous runs over 64 / L consecutive rows (one thread per row reads
// them at a stride of the row length: 4.5x below bandwidth on the 7-nonzero wave-system rows).
// The L partial sums meet through lane shuffles; lane 0 of the group stores.
template <int L>
__global__ void __launch_bounds__(BLAS_THREADS) k_csr_spmv_vec(i64 m, const i64* rowptr, const i64* col,
                                                               const cd* val, const cd* x, cd* y) {
  const int lane = threadIdx.x & (L - 1);
  const i64 groups = (i64)gridDim.x * (blockDim.x / L);
  for (i64 r = (i64)blockIdx.x * (blockDim.x / L) + threadIdx.x / L; r < m; r += groups) {
    const i64 p0 = rowptr[r], p1 = rowptr[r + 1];
    double ax = 0.0, ay = 0.0;
    for (i64 p = p0 + lane; p < p1; p += L) {
      const cd a = val[p], b = x[col[p]];
      ax = fma(a.x, b.x, fma(-a.y, b.y, ax));
      ay = fma(a.x, b.y, fma(a.y, b.x, ay));
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) {
      ax += __shfl_xor(ax, o, L);
      ay += __shfl_xor(ay, o, L);
    }
    if (lane == 0) y[r] = make_cd(ax, ay);
  }
}

hipError_t blas_set(cd* x, cd a, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_set, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, x, a, n);
  return hipGetLastError();
}
hipError_t blas_shift(cd* x, cd a, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_shift, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, x, a, n);
  return hipGetLastError();
}
hipError_t blas_copy(cd* y, const cd* x, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_copy, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, y, x, n);
  return hipGetLastError();
}
hipError_t blas_axpy(cd* y, cd a, const cd* x, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_axpy, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, y, a, x, n);
  return hipGetLastError();
}
hipError_t blas_aypx(cd* y, cd b, const cd* x, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_aypx, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, y, b, x, n);
  return hipGetLastError();
}
hipError_t blas_waxpy(cd* w, cd a, const cd* x, const cd* y, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_waxpy, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, w, a, x, y, n);
  return hipGetLastError();
}
hipError_t blas_pmult(cd* w, const cd* x, const cd* y, i64 n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_pmult, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, w, x, y, n);
  return hipGetLastError();
}
hipError_t blas_maxpy(cd* y, int k, const cd* a, const cd* const* xs, i64 n, hipStream_t s) {
  for (int j0 = 0; j0 < k; j0 += MV_MAX) {
    const int kk = k - j0 < MV_MAX ? k - j0 : MV_MAX;
    MVCoef c;
    MVPtrs p;
    for (int j = 0; j < kk; ++j) { c.a[j] = a[j0 + j]; p.p[j] = xs[j0 + j]; }
    if (n > 0) hipLaunchKernelGGL(k_maxpy, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, y, kk, c, p, n);
  }
  return hipGetLastError();
}
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                         hipStream_t s) {
  if (m <= 0) return hipSuccess;
  // lanes per row: the power of two at or above the mean row length, 1 .. 16
  const double mean = (double)nnz / (double)m;
  const int L = mean <= 1.5 ? 1 : mean <= 2.5 ? 2 : mean <= 4.5 ? 4 : mean <= 8.5 ? 8 : 16;
  const dim3 blk(BLAS_THREADS);
  switch (L) {
    case 1: hipLaunchKernelGGL(k_csr_spmv, dim3(nblocks(m)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 2: hipLaunchKernelGGL((k_csr_spmv_vec<2>), dim3(nblocks(m * 2)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 4: hipLaunchKernelGGL((k_csr_spmv_vec<4>), dim3(nblocks(m * 4)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 8: hipLaunchKernelGGL((k_csr_spmv_vec<8>), dim3(nblocks(m * 8)), blk, 0, s, m, rowptr, col, val, x, y); break;
    default: hipLaunchKernelGGL((k_csr_spmv_vec<16>), dim3(nblocks(m * 16)), blk, 0, s, m, rowptr, col, val, x, y);
  }
  return hipGetLastError();
}

// Synchronous reductions (the result is needed on the host, as in PETSc).
static hipError_t reduce(const cd* x, const cd* y, i64 n, int kind, double out[2], hipStream_t s) {
  static thread_local double* partial = nullptr;
  static thread_local double* hpart = nullptr;
  if (!partial) {
    hipError_t e = hipMalloc(&partial, sizeof(double) * 2 * RED_BLOCKS);
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&hpart, sizeof(double) * 2 * RED_BLOCKS);
    if (e != hipSuccess) return e;
  }
  unsigned nb = nblocks(n);
  if (nb > RED_BLOCKS) nb = RED_BLOCKS;
  hipLaunchKernelGGL(k_reduce, dim3(nb), dim3(BLAS_THREADS), 0, s, x, y, n, kind, partial);
  hipError_t e = hipMemcpyAsync(hpart, partial, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  double a = 0.0, b = 0.0;
  for (unsigned k = 0; k < nb; ++k) {
    if (kind == 3) a = fmax(a, hpart[2 * k]);
    else { a += hpart[2 * k]; b += hpart[2 * k + 1]; }
  }
  out[0] = a;
  out[1] = b;
  return hipSuccess;
}

hipError_t blas_maxpy_norm(cd* y, int k, const cd* a, const cd* const* xs, i64 n, bool overwrite, double* norm2,
                           hipStream_t s) {
  static thread_local double* partial = nullptr;
  static thread_local double* hpart = nullptr;
  if (norm2 && !partial) {
    hipError_t e = hipMalloc(&partial, sizeof(double) * RED_BLOCKS);
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&hpart, sizeof(double) * RED_BLOCKS);
    if (e != hipSuccess) return e;
  }
  unsigned nb = nblocks(n);
  if (nb > RED_BLOCKS) nb = RED_BLOCKS;
  if (k <= 0 && !overwrite) {
    if (!norm2) return hipSuccess;
    double v = 0.0;
    const hipError_t e = blas_norm(y, n, 1, &v, s);
    *norm2 = v * v;
    return e;
  }
  for (int j0 = 0; j0 < (k > 0 ? k : 1); j0 += MV_MAX) {
    const int kk = k - j0 < MV_MAX ? (k - j0 > 0 ? k - j0 : 0) : MV_MAX;
    MVCoef c;
    MVPtrs p;
    for (int j = 0; j < kk; ++j) { c.a[j] = a[j0 + j]; p.p[j] = xs[j0 + j]; }
    const bool ow = overwrite && j0 == 0, last = j0 + MV_MAX >= k, nrm = norm2 && last;
    if (n <= 0) break;
    const dim3 g(nb), blk(BLAS_THREADS);
    if (ow && nrm) hipLaunchKernelGGL((k_maxpy_nrm<true, true>), g, blk, 0, s, y, kk, c, p, n, partial);
    else if (ow) hipLaunchKernelGGL((k_maxpy_nrm<true, false>), g, blk, 0, s, y, kk, c, p, n, partial);
    else if (nrm) hipLaunchKernelGGL((k_maxpy_nrm<false, true>), g, blk, 0, s, y, kk, c, p, n, partial);
    else hipLaunchKernelGGL((k_maxpy_nrm<false, false>), g, blk, 0, s, y, kk, c, p, n, partial);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !norm2) return e;
  if (n <= 0) {
    *norm2 = 0.0;
    return hipSuccess;
  }
  e = hipMemcpyAsync(hpart, partial, sizeof(double) * nb, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  double t = 0.0;
  for (unsigned q = 0; q < nb; ++q) t += hpart[q];
  *norm2 = t;
  return hipSuccess;
}

hipError_t blas_dot(const cd* x, const cd* y, i64 n, cd* val, hipStream_t s) {
  double o[2];
  hipError_t e = reduce(x, y, n, 0, o, s);
  *val = make_cd(o[0], o[1]);
  return e;
}
hipError_t blas_norm(const cd* x, i64 n, int type, double* val, hipStream_t s) {
  double o[2];
  const int kind = type == 1 ? 1 : (type == 0 ? 2 : (type == 3 ? 3 : 1));
  hipError_t e = reduce(x, nullptr, n, kind, o, s);
  *val = kind == 1 ? sqrt(o[0]) : o[0];
  return e;
}

hipError_t blas_mdot(const cd* x, int k, const cd* const* ys, i64 n, cd* vals, hipStream_t s) {
  static thread_local double* partial = nullptr;
  static thread_local double* hpart = nullptr;
  const int NB = 512;
  if (!partial) {
    hipError_t e = hipMalloc(&partial, sizeof(double) * 2 * MDOT_K * NB);
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&hpart, sizeof(double) * 2 * MDOT_K * NB);
    if (e != hipSuccess) return e;
  }
  for (int j0 = 0; j0 < k; j0 += MDOT_K) {
    const int kk = k - j0 < MDOT_K ? k - j0 : MDOT_K;
    MVPtrs p;
    for (int j = 0; j < kk; ++j) p.p[j] = ys[j0 + j];
    unsigned nb = nblocks(n);
    if (nb > (unsigned)NB) nb = NB;
    hipLaunchKernelGGL(k_mdot, dim3(nb), dim3(BLAS_THREADS), 0, s, x, kk, p, n, partial);
    hipError_t e = hipMemcpyAsync(hpart, partial, sizeof(double) * 2 * MDOT_K * nb, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    for (int j = 0; j < kk; ++j) {
      double ra = 0.0, rb = 0.0;
      for (unsigned q = 0; q < nb; ++q) {
        ra += hpart[(size_t)q * 2 * MDOT_K + 2 * j];
        rb += hpart[(size_t)q * 2 * MDOT_K + 2 * j + 1];
      }
      vals[j0 + j] = make_cd(ra, rb);
    }
  }
  return hipSuccess;
}

}  // namespace cfp
