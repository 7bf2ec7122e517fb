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
