// tp_probe.hip -- timing probes of the 3-sweep middle kernel (P2) at 256^3 (not product code).
// Built with CFP_KEXP, which is the only build that may instantiate k_tp_mid_sw with PROBE != 0
// (a probe drops part of the work, so its output is invalid).  Each launch runs P2 in place on
// the whole grid with the product's persistent grid (one 1024-thread workgroup per CU).
//   which < 64:  k_tp_mid_sw<64, 8, 256, which>   (PR_* bits of cfp_three_pass.hip)
//   which = 100: k_tp_mid<0, 64, 8, 256> (the DPP lane-DFT kernel)
//   which += 1000: one workgroup per unit instead of the persistent grid
#define CFP_KEXP 1
#include "cfp_three_pass.hip"
namespace cfp {
thread_local LaunchStamp g_stamp;  // defined in cfp_plan.hip in the library
// launch_three_pass routes 100^3 to cfp_three_pass_sq.hip, which this harness does not build
hipError_t launch_three_pass_sq(int, int, const cd*, cd*, const TPArgs&, TPShape, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace cfp

using namespace cfp;

// the product's P2 (LDS-DMA prefetch, non-temporal loads) with probe bits P
template <int P>
static void launch_sw(cd* d, const TPArgs& a, unsigned g) {
  hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, P, true, 256, 0, F_NT_LD>), dim3(g), dim3(1024), 0, 0, d, a, 1024);
}

extern "C" int tp_probe(int which, void* data, const void* tw, const void* colsym, const void* axsym, int iters,
                        float* ms) {
  TPArgs a;
  a.tw = (const cd*)tw;
  a.colsym = (const cd*)colsym;
  a.axsym = (const cd*)axsym;
  a.scale = 1.0;
  const unsigned g = which >= 1000 ? 1024u : 256u;
  which %= 1000;
  cd* d = (cd*)data;
  auto launch = [&]() -> int {
    switch (which) {
#define C(P) case P: launch_sw<P>(d, a, g); return 0;
      C(0) C(1) C(2) C(3) C(4) C(6) C(7) C(8) C(16) C(24) C(26) C(28) C(29) C(30) C(31) C(32)
#undef C
      case 100: hipLaunchKernelGGL((k_tp_mid<0, 64, 8, 256>), dim3(g), dim3(1024), 0, 0, d, a, 1024); return 0;
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
