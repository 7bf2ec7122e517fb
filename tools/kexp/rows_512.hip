// rows_512.hip -- timing probes of the 512^3 row sweeps P1 / P3 (k_tp_rows<.., 32, 512, ..>, the
// product instantiations of launch_rows_ab) and, for comparison, the 256^3 ones.  Not product code.
// Output of the probe variants is invalid.  b -> x out of place, as in the apply.
//   which = 10 * probe + sweep, sweep 0: P1 512, 1: P3 512, 2: P1 256, 3: P3 256
//   probe 0: product, 1: no loads, 2: no stores, 3: neither (arithmetic + exchanges alone),
//   4: memory alone (no DFTs, no transpose), 5: memory + transpose (no DFTs)
//   6: product with units in z-major order, 7: memory alone in z-major order
//   8: product in XCD unit order, 9: memory alone in XCD unit order
//   10: memory alone, XCD order, 256^3 sweeps on 256 workgroups (one per CU, as at 512^3)
#define CFP_KEXP 1
#include "cfp_three_pass.hip"
namespace cfp {
thread_local LaunchStamp g_stamp;  // defined in cfp_plan.hip in the library
hipError_t launch_three_pass_sq(int, int, const cd*, cd*, const TPArgs&, TPShape, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace cfp

using namespace cfp;

template <int PR, bool XCD = false>
static int launch_probe(int sweep, const cd* b, cd* x, const TPArgs& a, int g256 = 512) {
  constexpr int W = F_WAVE_LDS;
  switch (sweep) {
    case 0: hipLaunchKernelGGL((k_tp_rows<false, F_NT_LD | W, 32, 512, 16, true, true, 0, XCD, PR>), dim3(256), dim3(1024), 0, 0, b, x, a, 512 * 16); return 0;
    case 1: hipLaunchKernelGGL((k_tp_rows<true, F_NT_ST | W, 32, 512, 16, true, true, 0, XCD, PR>), dim3(256), dim3(1024), 0, 0, b, x, a, 512 * 16); return 0;
    case 2: hipLaunchKernelGGL((k_tp_rows<false, F_NT_LD | W, 32, 256, 16, true, true, 0, XCD, PR>), dim3(g256), dim3(512), 0, 0, b, x, a, 256 * 8); return 0;
    case 3: hipLaunchKernelGGL((k_tp_rows<true, F_NT_ST | W, 32, 256, 16, true, true, 0, XCD, PR>), dim3(g256), dim3(512), 0, 0, b, x, a, 256 * 8); return 0;
    default: return 1;
  }
}

extern "C" int rows_512(int which, const void* b, void* x, const void* tw, int iters, float* ms) {
  TPArgs a;
  a.tw = (const cd*)tw;
  a.scale = 1.0;
  const int sweep = which % 10, probe = which / 10;
  auto launch = [&]() -> int {
    const cd* bb = (const cd*)b;
    cd* xx = (cd*)x;
    switch (probe) {
      case 0: return launch_probe<0>(sweep, bb, xx, a);
      case 1: return launch_probe<PR_NO_LOAD>(sweep, bb, xx, a);
      case 2: return launch_probe<PR_NO_STORE>(sweep, bb, xx, a);
      case 3: return launch_probe<PR_NO_LOAD | PR_NO_STORE>(sweep, bb, xx, a);
      case 4: return launch_probe<PR_NO_ZMATH | PR_NO_XCHG>(sweep, bb, xx, a);
      case 5: return launch_probe<PR_NO_ZMATH>(sweep, bb, xx, a);
      case 6: return launch_probe<PR_ZMAJOR>(sweep, bb, xx, a);
      case 7: return launch_probe<PR_ZMAJOR | PR_NO_ZMATH | PR_NO_XCHG>(sweep, bb, xx, a);
      case 8: return launch_probe<0, true>(sweep, bb, xx, a);
      case 9: return launch_probe<PR_NO_ZMATH | PR_NO_XCHG, true>(sweep, bb, xx, a);
      case 10: return launch_probe<PR_NO_ZMATH | PR_NO_XCHG, true>(sweep, bb, xx, a, 256);
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
