// cfp_three_pass.hip -- the 3-sweep apply for 256^3 grids (PCApply in 96 N bytes instead of
// the 5-pass schedule's 160 N).
//
// The y transform is split four-step (Cooley-Tukey, ny = N1 * N2 = 64 * 4): with
// y = y2 + N2 y1 and k = k1 + N1 k2,
//   X[k1 + N1 k2] = sum_{y2} W_4^{y2 k2} W_256^{y2 k1} sum_{y1} W_64^{y1 k1} x[y2 + N2 y1].
// The inner 64-point DFT rides with the x transform, the outer 4-point DFT with the z
// transform, and every intermediate stays in the slot it was read from (y1 <-> k1, y2 <-> k2):
//
//   P1  k_tp_rows<fwd>: one z-plane, rows y2 + 4 y1 (64 rows, 256 KB): 64-point DFT down the
//       rows (column mode, lanes = x), LDS transpose, 256-point DFT along each row
//   P2  k_tp_mid: 16 x-columns x 4 rows y2 + 4 k1 x 256 z (256 KB): twiddle W_256^{y2 k1},
//       4-point DFT across the lanes of a quad (DPP), 256-point z DFT, divide by the separable
//       symbol at (kx, k1 + 64 k2, kz), then the same transforms on the conjugate (inverse)
//   P3  k_tp_rows<inv>: P1 on the conjugate, x 1/N
//
// Every global access is a contiguous run of >= 256 bytes (P1 and P3 read/write whole rows,
// P2 reads 4 rows x 16 x per wave instruction).  Workgroups are 1024 threads x 16 points
// (256 KB in VGPRs) with a split-LDS exchange buffer of 128-136 KB, so one per CU.
#include "cfp_fft_device.h"
#include "cfp_three_pass.h"

namespace cfp {

namespace {
constexpr int TN = 256;  // nx = ny = nz
constexpr int TN1 = 64, TN2 = 4;
constexpr int RS = TN + TN / 16;  // padded row stride of the row-mode LDS layout

// 4-point DFT across the lanes of an aligned quad: this lane's output index is k = lane & 3
__device__ __forceinline__ cd dft4_quad(cd v, int k) {
  const cd r0 = make_cd(quad_bcast<0>(v.x), quad_bcast<0>(v.y));
  const cd r1 = make_cd(quad_bcast<1>(v.x), quad_bcast<1>(v.y));
  const cd r2 = make_cd(quad_bcast<2>(v.x), quad_bcast<2>(v.y));
  const cd r3 = make_cd(quad_bcast<3>(v.x), quad_bcast<3>(v.y));
  const bool odd = k & 1;
  const cd s = odd ? csub(r0, r2) : cadd(r0, r2);
  const cd d13 = csub(r1, r3), s13 = cadd(r1, r3);
  const cd t = odd ? make_cd(d13.y, -d13.x) : s13;  // -i (r1 - r3) for odd k
  return k < 2 ? cadd(s, t) : csub(s, t);
}
}  // namespace

// Persistent: a workgroup walks units blockIdx.x, + gridDim.x, ... (one per CU).  Prefetching
// the next unit into VGPRs across LDS-only barriers was tried and lost: at 1024 threads the
// extra registers spill (profiles/r01_schedule_sweep.txt).
template <bool INV, int FLAGS>
__global__ void __launch_bounds__(1024) k_tp_rows(const cd* in, cd* out, TPArgs a, int nunits) {
  constexpr int F = FLAGS | F_SPLIT_LDS | F_LDS_SYNC;
  __shared__ __attribute__((aligned(16))) double lds[TN1 * RS];  // 136 KB: both layouts fit
  __shared__ cd tw_l[TN + TN1];                                  // W_256, then W_64
  const int tid = threadIdx.x;
  for (int i = tid; i < TN; i += 1024) tw_l[i] = a.tw256[i];
  for (int i = tid; i < TN1; i += 1024) tw_l[TN + i] = a.tw256[4 * i];
  const int x = tid & (TN - 1), ty = tid >> 8;  // phase A: column x, thread ty of 4
  const int r = tid >> 4, tx = tid & 15;        // phase C: row r, thread tx of 16
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    // unit u = (z, y2): rows y2 + 4 y1 of plane z
    const i64 plane = (i64)(u / TN2) * TN * TN;
    const int y2 = u % TN2;
    cd v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      v[m] = gload<FLAGS>(in + plane + x + (i64)TN * (y2 + TN2 * (ty + 4 * m)));
      if (INV) v[m] = cconj(v[m]);
    }
    // phase A: 64-point DFT over y1 for every x (column mode, 256 columns x 4 threads)
    fft_stages<TN1, 16, 4, false, TN, F>(v, lds, tw_l + TN, x, ty, true);  // v[m]: k1 = ty + 4 m
    // phase B: transpose to rows k1, thread (row r, tx) gets x = tx + 16 m
    lds_barrier();  // phase A's last LDS reads are done
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int m = 0; m < 16; ++m) lds[(ty + 4 * m) * RS + x + (x >> 4)] = half ? v[m].y : v[m].x;
      lds_barrier();
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int xx = tx + 16 * m;
        const double val = lds[r * RS + xx + (xx >> 4)];
        if (half) v[m].y = val; else v[m].x = val;
      }
      lds_barrier();
    }
    // phase C: 256-point DFT along row r (row mode, 64 rows x 16 threads)
    fft_stages<TN, 16, 16, true, TN1, F>(v, lds, tw_l, r, tx, true);  // v[m]: kx = tx + 16 m
    const double sc = a.scale, sy = INV ? -sc : sc;
    cd* dst = out + plane + (i64)TN * (y2 + TN2 * r) + tx;
#pragma unroll
    for (int m = 0; m < 16; ++m) gstore<FLAGS>(dst + 16 * m, make_cd(v[m].x * sc, v[m].y * sy));
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

template <int FLAGS>
__global__ void __launch_bounds__(1024) k_tp_mid(cd* data, TPArgs a) {
  constexpr int T = 64;  // columns per workgroup: 16 x times 4 y2 (quad = y2)
  __shared__ __attribute__((aligned(16))) double lds[T * TN];  // 128 KB (split exchange)
  __shared__ cd tw_l[TN];
  const int tid = threadIdx.x;
  for (int i = tid; i < TN; i += 1024) tw_l[i] = a.tw256[i];
  const int xt = blockIdx.x % (TN / 16), k1 = blockIdx.x / (TN / 16);
  const int c = tid & (T - 1), tz = tid >> 6;
  const int y2 = c & 3, xk = xt * 16 + (c >> 2);
  const i64 base = xk + (i64)TN * (y2 + TN2 * k1);
  const i64 zs = (i64)TN * TN;
  const cd w = a.tw256[(y2 * k1) & (TN - 1)];  // W_256^{y2 k1}

  cd v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = gload<FLAGS>(data + base + zs * (tz + 16 * m));
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = dft4_quad(cmul(v[m], w), y2);  // lane's y2 is now k2
  fft_stages<TN, 16, 16, false, T, FLAGS | F_SPLIT_LDS>(v, lds, tw_l, c, tz, true);  // kz = tz + 16 m

  const cd cs = a.colsym[xk + (i64)TN * (k1 + TN1 * y2)];
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const cd d = cadd(cadd(cs, a.axsym[tz + 16 * m]), make_cd(1.0, 0.0));
    v[m] = cconj(cdiv(v[m], d));
  }
  fft_stages<TN, 16, 16, false, T, FLAGS | F_SPLIT_LDS>(v, lds, tw_l, c, tz, false);
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = cmul(dft4_quad(v[m], y2), w);
#pragma unroll
  for (int m = 0; m < 16; ++m) gstore<FLAGS>(data + base + zs * (tz + 16 * m), cconj(v[m]));
}

bool three_pass_supported(const i64 n[3]) { return n[0] == TN && n[1] == TN && n[2] == TN; }

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

hipError_t launch_three_pass(int stage, const cd* in, cd* out, const TPArgs& a, hipStream_t s) {
  const int units = TN * TN2;  // P1/P3: z-planes x y2; P2: x-tiles x k1 (16 x 64)
  const unsigned pgrid = (unsigned)(units < cu_count() ? units : cu_count());
  switch (stage) {
    case 0: hipLaunchKernelGGL((k_tp_rows<false, F_NT_LD>), dim3(pgrid), dim3(1024), 0, s, in, out, a, units); break;
    case 1: hipLaunchKernelGGL((k_tp_mid<0>), dim3((TN / 16) * TN1), dim3(1024), 0, s, out, a); break;
    default: hipLaunchKernelGGL((k_tp_rows<true, F_NT_ST>), dim3(pgrid), dim3(1024), 0, s, in, out, a, units); break;
  }
  return hipGetLastError();
}

}  // namespace cfp
