// copy_probe.hip -- achievable copy rate for the apply's vector sizes (not product code): 16-byte
// elements, out of place, grid-stride with U loads in flight per thread, cache policy variants.
//   which = U (1, 2, 4, 8) + 16 * policy (0 plain, 1 nt loads, 2 nt stores, 3 both)
//         + 64 * blocks-per-CU index (0: 4, 1: 8, 2: 16) -- 256-thread workgroups
#include <hip/hip_runtime.h>

typedef double dv2 __attribute__((ext_vector_type(2)));

template <int U, int POL>
__global__ void __launch_bounds__(256) k_copy(const dv2* __restrict__ in, dv2* __restrict__ out, long n) {
  const long stride = (long)gridDim.x * blockDim.x * U;
  for (long i = (long)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
    dv2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * blockDim.x;
      if (j < n) v[u] = (POL & 1) ? __builtin_nontemporal_load(in + j) : in[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * blockDim.x;
      if (j < n) {
        if (POL & 2) __builtin_nontemporal_store(v[u], out + j);
        else out[j] = v[u];
      }
    }
  }
}

template <int U, int POL>
static void launch(const dv2* in, dv2* out, long n, int blocks) {
  hipLaunchKernelGGL((k_copy<U, POL>), dim3(blocks), dim3(256), 0, 0, in, out, n);
}

extern "C" int copy_probe(int which, const void* in, void* out, long n, int cus, int iters, float* ms) {
  const int U = which & 15, pol = (which >> 4) & 3, bsel = which >> 6;
  const int blocks = cus * (bsel == 0 ? 4 : bsel == 1 ? 8 : 16);
  auto go = [&]() -> int {
#define P(UU)                                                                      \
  if (U == UU) {                                                                  \
    switch (pol) {                                                                \
      case 0: launch<UU, 0>((const dv2*)in, (dv2*)out, n, blocks); return 0;      \
      case 1: launch<UU, 1>((const dv2*)in, (dv2*)out, n, blocks); return 0;      \
      case 2: launch<UU, 2>((const dv2*)in, (dv2*)out, n, blocks); return 0;      \
      default: launch<UU, 3>((const dv2*)in, (dv2*)out, n, blocks); return 0;     \
    }                                                                             \
  }
    P(1) P(2) P(4) P(8)
#undef P
    return 1;
  };
  if (go()) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 3;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) go();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float t = 0;
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}
