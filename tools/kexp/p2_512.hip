// p2_512.hip -- variants of the 512^3 middle kernel P2 (k_tp_mid<.., 32, 16, 512, ..>) for its
// HBM-traffic question: 1.19 x 32 N per launch in the product.  Not product
// code.  Each variant runs P2 in place on a whole 512^3 grid.
//   which 0: the product (XCD-ordered persistent grid of 256 workgroups, default cache policy)
//   which 1: non-temporal stores (F_NT_ST)
//   which 2: 128 workgroups (half the units in flight per XCD: half the line working set)
//   which 3: 64 workgroups
//   which 4: blockIdx unit order (no XCD ordering)
// r05h probes (output invalid; where the time goes):
//   which 5: no workgroup barriers (F_WAVE_LDS: the exchanges race, LDS traffic kept)
//   which 6: no loads (synthetic points), 7: no stores, 8: neither (arithmetic + exchanges alone)
//   which 9: no z FFT / divide and no y2 DFT (loads, twiddles, stores: memory alone)
// blocked intermediate layouts (the P2 of the blocked / blocked32 shapes):
//   which 10: blocks of 8 x, memory alone; 11: blocks of 8 x, full kernel
//   which 12: blocks of 2 x, memory alone; 13: blocks of 2 x, full kernel
#define CFP_KEXP 1
#include "cfp_three_pass.hip"
namespace cfp {
thread_local LaunchStamp g_stamp;  // defined in cfp_plan.hip in the library
hipError_t launch_three_pass_sq(int, int, const cd*, cd*, const TPArgs&, TPShape, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace cfp

using namespace cfp;

extern "C" int p2_512(int which, void* data, const void* tw, const void* colsym, const void* axsym, int iters,
                      float* ms) {
  TPArgs a;
  a.tw = (const cd*)tw;
  a.colsym = (const cd*)colsym;
  a.axsym = (const cd*)axsym;
  a.scale = 1.0;
  constexpr int units = 256 * 32;
  cd* d = (cd*)data;
  auto launch = [&]() -> int {
    switch (which) {
      case 0: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 1: hipLaunchKernelGGL((k_tp_mid<F_NT_ST, 32, 16, 512, 16, true, 512, true>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 2: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true>), dim3(128), dim3(1024), 0, 0, d, a, units); return 0;
      case 3: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true>), dim3(64), dim3(1024), 0, 0, d, a, units); return 0;
      case 4: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, false>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 5: hipLaunchKernelGGL((k_tp_mid<F_WAVE_LDS, 32, 16, 512, 16, true, 512, true>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 6: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 0, PR_NO_LOAD>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 7: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 0, PR_NO_STORE>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 8: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 0, PR_NO_LOAD | PR_NO_STORE>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 9: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 0, PR_NO_ZMATH | PR_NO_Y2>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 10: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 8, PR_NO_ZMATH | PR_NO_Y2>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 11: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 8>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 12: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 2, PR_NO_ZMATH | PR_NO_Y2>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      case 13: hipLaunchKernelGGL((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 2>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      default: return 1;
    }
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
