// cfp_three_pass_sq.hip -- the 3-sweep apply for cube grids whose side is n = R^2 with R not a
// power of two: the reference's default mesh 100^3 (R = 10; src/FftLinearSolver_3D.c:166-190,
// tests/CMakeLists.txt:39-42).  Same four-step y split as cfp_three_pass.hip (y = y2 + R y1,
// ky = k1 + R k2), built on the radix-R column FFTs of cfp_fft_device.h:
//
//   S1 k_sq_rows<fwd>: unit (z, y2) = rows y2 + R y1 of plane z (R rows x n): column mode, thread
//       = x, the R-point y1 DFT in registers; LDS transpose to row mode (R threads per row); the
//       n-point x FFT along each row k1; store back to rows y2 + R k1 (every value keeps its slot).
//   S2 k_sq_mid: unit (x tile, k1) = XT x times R y2 times n z: thread (x, z) takes the R rows
//       y2 + R k1, twiddles W_n^{y2 k1}, R-point y2 DFT in registers; LDS to column mode (column
//       x + XT k2, n/R threads per column), z FFT, symbol divide, inverse z FFT (conjugate
//       trick), LDS back, inverse y2 DFT, twiddle, store in place.
//   S3 k_sq_rows<inv>: S1 on the conjugate, x 1/N.
//
// The plane schedule (k_plane: x + y of one z-plane per workgroup) keeps 100 CUs busy at
// 100^3; here S1/S3 have n R = 1000 units of 1000 points and S2 (n / XT) R units, so every
// sweep fills all 256 CUs.  An apply moves 3 x (read + write) x 16 bytes per point.
#include "cfp_fft_device.h"
#include "cfp_three_pass.h"

namespace cfp {

namespace {
template <int N> struct SqCfg;
template <> struct SqCfg<100> { static constexpr int R = 10; };
}  // namespace

// S1 / S3.  N threads: column mode thread x, row mode (row k1 = tid / TPC, tpc = tid % TPC).
// CO (S3): load in column mode (each row read by consecutive lanes) and transpose to row mode
// through LDS, instead of the row-mode load (ten 160-byte pieces per row and instruction).
// Measured slower (r04v: 11.9 against 11.0 us with non-temporal stores, 11.75 against 11.1 with
// the default policy), not launched.
template <int N, bool INV, bool CO = false>
__global__ void __launch_bounds__(N) k_sq_rows(const cd* in, cd* out, const cd* tw, double scale) {
  constexpr int R = SqCfg<N>::R, TPC = N / R;
  static_assert(R * R == N, "n = R^2");
  // whole-complex exchanges, rows padded by one element; default cache policy for b and x
  // (16 MB each, Infinity-Cache resident between applies, as at 128^3)
  constexpr int F = F_PAD1;
  __shared__ __attribute__((aligned(16))) cd lds[R * (N + 1)];
  __shared__ cd tws[N];
  const int tid = threadIdx.x;
  const int z = blockIdx.x / R, y2 = blockIdx.x % R;
  const i64 plane = (i64)z * N * N;
  const int row = tid / TPC, tpc = tid % TPC;
  for (int i = tid; i < N; i += N) tws[i] = tw[i];  // published by the first exchange's barrier
  cd v[R];
  if constexpr (!INV) {
    const cd* src = in + plane + (i64)y2 * N + tid;  // column x = tid, rows y2 + R y1
#pragma unroll
    for (int m = 0; m < R; ++m) v[m] = gload<F>(src + (i64)R * N * m);
    dft_any<R>(v);  // v[k1]
    // column x -> row mode
#pragma unroll
    for (int m = 0; m < R; ++m) lds[lds_idx<N, true, R, F>(m, tid)] = v[m];
    xbarrier<F>();
#pragma unroll
    for (int m = 0; m < R; ++m) v[m] = lds[lds_idx<N, true, R, F>(row, tpc + m * TPC)];
    fft_stages<N, R, R, true, R, F>(v, lds, tws, row, tpc, false);  // v[t]: kx = tpc + TPC t
    cd* dst = out + plane + (i64)(y2 + R * row) * N + tpc;
#pragma unroll
    for (int t = 0; t < R; ++t) gstore<F>(dst + TPC * t, v[t]);
  } else {
    if constexpr (CO) {
      const cd* src = in + plane + (i64)y2 * N + tid;  // column kx = tid, rows y2 + R k1
#pragma unroll
      for (int m = 0; m < R; ++m) v[m] = cconj(gload<F>(src + (i64)R * N * m));
#pragma unroll
      for (int m = 0; m < R; ++m) lds[lds_idx<N, true, R, F>(m, tid)] = v[m];
      xbarrier<F>();
#pragma unroll
      for (int m = 0; m < R; ++m) v[m] = lds[lds_idx<N, true, R, F>(row, tpc + m * TPC)];
    } else {
      const cd* src = in + plane + (i64)(y2 + R * row) * N + tpc;  // row k1, points kx = tpc + TPC m
#pragma unroll
      for (int m = 0; m < R; ++m) v[m] = cconj(gload<F>(src + TPC * m));
    }
    fft_stages<N, R, R, true, R, F>(v, lds, tws, row, tpc, !CO);  // v[t]: x = tpc + TPC t
    // row mode -> column x = tid
    xbarrier<F>();
#pragma unroll
    for (int t = 0; t < R; ++t) lds[lds_idx<N, true, R, F>(row, tpc + t * TPC)] = v[t];
    xbarrier<F>();
#pragma unroll
    for (int m = 0; m < R; ++m) v[m] = lds[lds_idx<N, true, R, F>(m, tid)];
    dft_any<R>(v);  // v[y1]
    const double sy = -scale;
    cd* dst = out + plane + (i64)y2 * N + tid;
#pragma unroll
    for (int m = 0; m < R; ++m) gstore<F>(dst + (i64)R * N * m, make_cd(v[m].x * scale, v[m].y * sy));
  }
}

// S2.  XT N threads: y2 mode thread (xl = tid % XT, z = tid / XT); column mode (column
// c = tid % T = xl + XT k2, tz = tid / T, points z = tz + TPC m).
template <int N, int XT>
__global__ void __launch_bounds__(XT * N) k_sq_mid(cd* data, TPArgs a) {
  constexpr int R = SqCfg<N>::R, TPC = N / R, T = XT * R, NXT = N / XT;
  static_assert(N % XT == 0, "whole x tiles");
  constexpr int F = 0;
  // y2 mode <-> column mode transposes: rows of T + 1 (with T = 40 the 16 z of a wave's lanes
  // otherwise fall on 2 bank groups); the z FFT's own exchange uses fft_stages' T-wide rows
  constexpr int TP = T + 1;
  __shared__ __attribute__((aligned(16))) cd lds[TP * N];
  __shared__ cd tws[N];
  const int tid = threadIdx.x;
  // XCD-aware unit order: the workgroups of one XCD (blockIdx % 8, round-robin dispatch) take a
  // contiguous range of units, so the x tiles that share 128-byte lines (a 1,600-byte row holds
  // 6.25 tiles of 64 bytes) meet in one L2; in blockIdx order the unit moved 1.50 x 32 N bytes
  // of HBM traffic (profiles/r04_pmc_small.txt)
  constexpr int NU = NXT * R, PER = NU / 8, EXTRA = NU % 8;
  const int b = blockIdx.x, j = b & 7, i = b >> 3;
  const int u = j * PER + (j < EXTRA ? j : EXTRA) + i;
  const int xt = u % NXT, k1 = u / NXT;
  for (int i2 = tid; i2 < N; i2 += XT * N) tws[i2] = a.tw[i2];
  const int xl = tid % XT, z = tid / XT;
  const int c = tid % T, tz = tid / T;
  cd* col = data + (i64)z * N * N + (i64)R * k1 * N + xt * XT + xl;  // row y2 + R k1 at y2 = 0
  cd v[R];
#pragma unroll
  for (int m = 0; m < R; ++m) v[m] = col[(i64)N * m];
  __syncthreads();  // tws
#pragma unroll
  for (int m = 1; m < R; ++m) v[m] = cmul(v[m], tws[(m * k1) % N]);  // W_n^{y2 k1}
  dft_any<R>(v);  // v[k2]
  // y2 mode -> column mode: element (column xl + XT k2, z) at z (T + 1) + column
#pragma unroll
  for (int m = 0; m < R; ++m) lds[z * TP + xl + XT * m] = v[m];
  __syncthreads();
#pragma unroll
  for (int m = 0; m < R; ++m) v[m] = lds[(tz + TPC * m) * TP + c];
  fft_stages<N, R, R, false, T, F>(v, lds, tws, c, tz, false);  // v[t]: kz = tz + TPC t
  {
    const int kx = xt * XT + c % XT, ky = k1 + R * (c / XT);
    const cd cs = a.colsym[kx + (i64)N * ky];
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const cd d = cadd(cadd(cs, a.axsym[tz + TPC * t]), make_cd(1.0, 0.0));
      v[t] = cconj(cdiv_sym(v[t], d));
    }
  }
  fft_stages<N, R, R, false, T, F>(v, lds, tws, c, tz, false);  // v[t]: z = tz + TPC t (conjugate domain)
  __syncthreads();
#pragma unroll
  for (int t = 0; t < R; ++t) lds[(tz + TPC * t) * TP + c] = v[t];
  __syncthreads();
#pragma unroll
  for (int m = 0; m < R; ++m) v[m] = lds[z * TP + xl + XT * m];
  dft_any<R>(v);  // v[y2]
#pragma unroll
  for (int m = 0; m < R; ++m) {
    const cd w = m ? cmul(v[m], tws[(m * k1) % N]) : v[m];
    col[(i64)N * m] = cconj(w);
  }
}

bool three_pass_sq_supported(const i64 n[3]) { return n[0] == n[1] && n[1] == n[2] && n[0] == 100; }

template <int N, int XT>
static void launch_sq_mid(cd* data, const TPArgs& a, hipStream_t s) {
  constexpr int R = SqCfg<N>::R;
  hipLaunchKernelGGL((k_sq_mid<N, XT>), dim3((N / XT) * R), dim3(XT * N), 0, s, data, a);
}

hipError_t launch_three_pass_sq(int stage, int n, const cd* in, cd* out, const TPArgs& a, TPShape shape,
                                hipStream_t s) {
  if (n != 100) return hipErrorNotSupported;
  constexpr int N = 100, R = SqCfg<N>::R;
  if (stage == 1) {
    // shape.mid picks the S2 x tile: default 4 x (250 units, 64-byte runs), LANE64 2 x (500
    // units), LANE32 5 x (200 units)
    if (shape.mid == TP_MID_LANE64) launch_sq_mid<N, 2>(out, a, s);
    else if (shape.mid == TP_MID_LANE32) launch_sq_mid<N, 5>(out, a, s);
    else launch_sq_mid<N, 4>(out, a, s);
  } else if (stage == 0) {
    hipLaunchKernelGGL((k_sq_rows<N, false>), dim3(N * R), dim3(N), 0, s, in, out, a.tw, 1.0);
  } else {
    hipLaunchKernelGGL((k_sq_rows<N, true>), dim3(N * R), dim3(N), 0, s, in, out, a.tw, a.scale);
  }
  return hipGetLastError();
}

}  // namespace cfp
