// launch.hip -- per-launch cost on this box: back-to-back empty kernels (small / 1 KiB kernarg),
// and the same chains captured in a hipGraph (not part of the product)
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { char b[1024]; };
__global__ void k_empty(int* p) { if (p && threadIdx.x == 1024) p[0] = 1; }
__global__ void k_big(Big a, int* p) { if (p && threadIdx.x == 1024) p[0] = a.b[5]; }

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  Big big = {};
  const int n = 2000;
  for (int mode = 0; mode < 4; ++mode) {
    const bool graph = mode >= 2, bigk = mode & 1;
    hipGraphExec_t ge = nullptr;
    if (graph) {
      hipGraph_t g;
      (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
      for (int i = 0; i < 100; ++i) {
        if (bigk) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
        else hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
      }
      (void)hipStreamEndCapture(s, &g);
      (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipGraphLaunch(ge, s);
    }
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    if (graph) {
      for (int i = 0; i < n / 100; ++i) (void)hipGraphLaunch(ge, s);
    } else {
      for (int i = 0; i < n; ++i) {
        if (bigk) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
        else hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
      }
    }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%s %s kernarg: %.2f us per launch\n", graph ? "graph " : "stream", bigk ? "1KiB " : "small", ms * 1e3 / n);
  }
  return 0;
}
