// stream_order.hip -- streaming-kernel unit orders on MI355X (r05m): does the XCD-contiguous unit
// order that helps the row sweeps also help the BLAS-1 kernels of the Krylov loop?  Not product
// code.  256 threads per workgroup, one complex double per thread per step, 268 MB vectors.
//   order 0: grid-stride (blockIdx order; what cfp_blas.hip's GRID_LOOP does)
//   order 1: grid-stride with the workgroup id remapped so that each XCD takes a contiguous eighth
//            of every round
//   order 2: one contiguous range per workgroup
//   kind 0: axpy y += a x (2 reads, 1 write); 1: dot x^H y (2 reads); 2: copy (1 read, 1 write)
#include <hip/hip_runtime.h>

typedef HIP_vector_type<double, 2> cd;
typedef long long i64;

__device__ __forceinline__ i64 wg_of(int order) {
  const int G = gridDim.x, b = blockIdx.x;
  return order == 1 ? (i64)(b & 7) * (G >> 3) + (b >> 3) : b;
}

template <int ORDER, int KIND>
__global__ void __launch_bounds__(256) k_stream(cd* y, const cd* x, i64 n, double* partial) {
  double acc = 0.0;
  const i64 G = gridDim.x;
  if (ORDER == 2) {
    const i64 per = (n + G - 1) / G, lo = per * blockIdx.x, hi = lo + per < n ? lo + per : n;
    for (i64 i = lo + threadIdx.x; i < hi; i += 256) {
      const cd u = x[i];
      if (KIND == 0) { cd v = y[i]; v.x += 0.5 * u.x; v.y += 0.5 * u.y; y[i] = v; }
      else if (KIND == 1) { const cd v = y[i]; acc += u.x * v.x + u.y * v.y; }
      else y[i] = u;
    }
  } else {
    for (i64 i = wg_of(ORDER) * 256 + threadIdx.x; i < n; i += G * 256) {
      const cd u = x[i];
      if (KIND == 0) { cd v = y[i]; v.x += 0.5 * u.x; v.y += 0.5 * u.y; y[i] = v; }
      else if (KIND == 1) { const cd v = y[i]; acc += u.x * v.x + u.y * v.y; }
      else y[i] = u;
    }
  }
  if (KIND == 1 && threadIdx.x == 0) partial[blockIdx.x] = acc;  // keeps the work live
}

extern "C" int stream_order(int order, int kind, int blocks, void* y, const void* x, long long n, void* partial,
                            int iters, float* ms) {
  auto launch = [&]() -> int {
#define L(O, K) hipLaunchKernelGGL((k_stream<O, K>), dim3(blocks), dim3(256), 0, 0, (cd*)y, (const cd*)x, n, (double*)partial)
    switch (order * 3 + kind) {
      case 0: L(0, 0); break; case 1: L(0, 1); break; case 2: L(0, 2); break;
      case 3: L(1, 0); break; case 4: L(1, 1); break; case 5: L(1, 2); break;
      case 6: L(2, 0); break; case 7: L(2, 1); break; case 8: L(2, 2); break;
      default: return 1;
    }
#undef L
    return 0;
  };
  if (launch()) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 3;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float t = 0;
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}
