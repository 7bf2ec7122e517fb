// seg.hip -- HBM access-pattern microbenchmark for pass-fusion planning (not product code).
// Copies a 256^3 complex-double grid (in -> out) with the load/store pattern of a candidate
// pass and reports the time; no arithmetic.  Patterns (n = 256, 16 values per thread):
//   kind 0 "rows":  NR rows of 256 x at fixed (y-block, z); thread = (tpc 16, row)
//   kind 1 "cols":  TX x-columns x NR consecutive rows x all 256 z; thread = (x, row, tz)
// xcd > 0: blocks that share 256-byte row segments (kind 1, TX < 16) are mapped to the same
// XCD at the same time (dispatch is round-robin over 8 XCDs).
#include <hip/hip_runtime.h>

typedef double2 cd;
static const int n = 256;

template <int TX, int NR>
__global__ void __launch_bounds__(TX * NR * 16) k_cols(const cd* __restrict__ in, cd* __restrict__ out, int xcd) {
  const int tid = threadIdx.x;
  const int xi = tid % TX, r = (tid / TX) % NR, tz = tid / (TX * NR);
  unsigned b = blockIdx.x;
  constexpr int G = 16 / TX;  // tiles that share a 256-byte segment
  if (xcd && G > 1) {
    // blocks 8q + c (q = 0..G-1 within a group of 8G) -> tiles G*(8*qq + c) + q
    const unsigned c = b % 8, q = (b / 8) % G, grp = b / (8 * G);
    b = (grp * 8 + c) * G + q;
  }
  const int xt = b % (n / TX), yt = b / (n / TX);
  const long long base = (long long)xt * TX + xi + (long long)n * (yt * NR + r);
  cd v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = in[base + (long long)n * n * (tz + 16 * m)];
#pragma unroll
  for (int m = 0; m < 16; ++m) out[base + (long long)n * n * (tz + 16 * m)] = v[m];
}

template <int NR>
__global__ void __launch_bounds__(16 * NR) k_rows(const cd* __restrict__ in, cd* __restrict__ out, int stride_rows) {
  const int tid = threadIdx.x;
  const int tpc = tid % 16, r = tid / 16;
  const int b = blockIdx.x;
  // block -> (z, y-group): rows y = y0 + r * stride_rows
  const int groups = n / NR;
  const int z = b / groups, g = b % groups;
  const int y = stride_rows == 1 ? g * NR + r : g + r * stride_rows;
  const long long base = (long long)n * (y + (long long)n * z) + tpc;
  cd v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = in[base + 16 * m];
#pragma unroll
  for (int m = 0; m < 16; ++m) out[base + 16 * m] = v[m];
}

extern "C" int seg_run(int kind, int tx, int nr, int xcd, const void* in, void* out, int iters, double* ms) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&]() -> int {
    if (kind == 0) {
      const int blocks = n * (n / nr);
      const int stride = xcd;  // reuse: row stride (1 = consecutive rows, else y-stride)
      if (nr == 8) hipLaunchKernelGGL(k_rows<8>, dim3(blocks), dim3(128), 0, 0, (const cd*)in, (cd*)out, stride ? stride : 1);
      else if (nr == 16) hipLaunchKernelGGL(k_rows<16>, dim3(blocks), dim3(256), 0, 0, (const cd*)in, (cd*)out, stride ? stride : 1);
      else if (nr == 32) hipLaunchKernelGGL(k_rows<32>, dim3(blocks), dim3(512), 0, 0, (const cd*)in, (cd*)out, stride ? stride : 1);
      else if (nr == 64) hipLaunchKernelGGL(k_rows<64>, dim3(blocks), dim3(1024), 0, 0, (const cd*)in, (cd*)out, stride ? stride : 1);
      else return 1;
      return 0;
    }
    const int blocks = (n / tx) * (n / nr);
#define L(TXV, NRV) \
  if (tx == TXV && nr == NRV) { hipLaunchKernelGGL((k_cols<TXV, NRV>), dim3(blocks), dim3(TXV * NRV * 16), 0, 0, (const cd*)in, (cd*)out, xcd); return 0; }
    L(16, 1) L(16, 2) L(16, 4) L(8, 2) L(8, 4) L(8, 8) L(4, 4) L(4, 8) L(4, 16) L(2, 16) L(32, 1) L(32, 2)
#undef L
    return 1;
  };
  if (launch()) return 1;
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) launch();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float t = 0;
  hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---------------------------------------------------------------------------------------------
// r04: the 3-sweep chain's three patterns as pure copies, for several
// intermediate layouts.  Within the 8 rows y2 + 8 k1 of one k1 (contiguous in every layout):
//   mode 0 natural   [y2][x]                 P2 unit: T/8 x times 8 y2 = 8 runs of T B per z
//   mode 1 blocked8  [x / 8][y2][x % 8]      P2 unit of 64 columns: one 1 KiB run per z
//   mode 2 blocked4  [x / 4][y2][x % 4]      P2 unit of 32 columns: one 512 B run per z
// P1: rows y2 + 8 y1 of a plane (32 x 4 KiB runs) -> rows k1 in the mode's layout (natural 4 KiB
// runs, blocked8 128 B, blocked4 64 B); P2 (in place): T columns x 256 z (T = 64: 1024 threads,
// one workgroup per CU; T = 32: 512 threads, two per CU); P3 (in place): P1's pattern reversed.
// Thread maps as in the kernels: P1/P3 512 threads = (tx 16, row 32), slots x = tx + 16 m; P2
// T x 16 threads = (column T, tz 16), slots z = tz + 16 m.
__device__ __forceinline__ long long blk_off(int mode, int k1, int y2, int x) {
  if (mode == 0) return 256LL * (y2 + 8 * k1) + x;
  const int XB = mode == 1 ? 8 : 4;
  return 2048LL * k1 + (long long)(x / XB) * (8 * XB) + y2 * XB + x % XB;
}
template <bool REV>
__global__ void __launch_bounds__(512) k_chain_rows(const cd* __restrict__ in, cd* __restrict__ out, int mode) {
  const int tid = threadIdx.x, tx = tid % 16, r = tid / 16;
  const int z = blockIdx.x / 8, y2 = blockIdx.x % 8;
  const long long plane = (long long)n * n * z;
  cd v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int x = tx + 16 * m;
    v[m] = in[plane + (REV ? blk_off(mode, r, y2, x) : 256LL * (y2 + 8 * r) + x)];
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int x = tx + 16 * m;
    out[plane + (REV ? 256LL * (y2 + 8 * r) + x : blk_off(mode, r, y2, x))] = v[m];
  }
}
template <int T>
__global__ void __launch_bounds__(T * 16) k_chain_mid(const cd* __restrict__ in, cd* __restrict__ out, int mode) {
  constexpr int XU = T / 8, NXT = 256 / XU;  // x per unit, x tiles
  const int tid = threadIdx.x, c = tid % T, tz = tid / T;
  const int xt = blockIdx.x % NXT, k1 = blockIdx.x / NXT;
  const int x = xt * XU + c % XU, y2 = c / XU;
  const long long col = (mode == 1 && XU == 8) || (mode == 2 && XU == 4) ? 2048LL * k1 + (long long)xt * T + c
                                                                         : blk_off(mode, k1, y2, x);
  cd v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = in[col + (long long)n * n * (tz + 16 * m)];
#pragma unroll
  for (int m = 0; m < 16; ++m) out[col + (long long)n * n * (tz + 16 * m)] = v[m];
}

// chain b -> x (P1), x -> x (P2), x -> x (P3), iters times, layout `mode`, P2 tile T (64 or 32);
// us[0..2] = mean per-kernel time (events between the kernels), us[3] = mean chain time without
extern "C" int seg_chain(int mode, int T, const void* b, void* x, int iters, double* us) {
  if (mode < 0 || mode > 2 || (T != 64 && T != 32)) return 1;
  hipEvent_t e[4];
  for (auto& q : e) (void)hipEventCreate(&q);
  float acc[3] = {0, 0, 0};
  const cd* bb = (const cd*)b;
  cd* xx = (cd*)x;
  auto mid = [&]() {
    if (T == 64) hipLaunchKernelGGL((k_chain_mid<64>), dim3(1024), dim3(1024), 0, 0, xx, xx, mode);
    else hipLaunchKernelGGL((k_chain_mid<32>), dim3(2048), dim3(512), 0, 0, xx, xx, mode);
  };
  for (int it = -1; it < iters; ++it) {
    (void)hipEventRecord(e[0], 0);
    hipLaunchKernelGGL((k_chain_rows<false>), dim3(2048), dim3(512), 0, 0, bb, xx, mode);
    (void)hipEventRecord(e[1], 0);
    mid();
    (void)hipEventRecord(e[2], 0);
    hipLaunchKernelGGL((k_chain_rows<true>), dim3(2048), dim3(512), 0, 0, xx, xx, mode);
    (void)hipEventRecord(e[3], 0);
    (void)hipEventSynchronize(e[3]);
    if (it < 0) continue;
    for (int k = 0; k < 3; ++k) {
      float t = 0;
      (void)hipEventElapsedTime(&t, e[k], e[k + 1]);
      acc[k] += t;
    }
  }
  for (int k = 0; k < 3; ++k) us[k] = 1e3 * acc[k] / iters;
  (void)hipEventRecord(e[0], 0);
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL((k_chain_rows<false>), dim3(2048), dim3(512), 0, 0, bb, xx, mode);
    mid();
    hipLaunchKernelGGL((k_chain_rows<true>), dim3(2048), dim3(512), 0, 0, xx, xx, mode);
  }
  (void)hipEventRecord(e[1], 0);
  (void)hipEventSynchronize(e[1]);
  float t = 0;
  (void)hipEventElapsedTime(&t, e[0], e[1]);
  us[3] = 1e3 * t / iters;
  for (auto& q : e) (void)hipEventDestroy(q);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
