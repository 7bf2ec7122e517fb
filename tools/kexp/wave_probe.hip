// wave_probe.hip -- timing probes and shape variants of the wave 3-sweep middle kernel (P2w,
// cfp_wave_three.hip) at 128^3 (not product code).  Built with CFP_KEXP, the only build that may
// instantiate k_wtp_mid with PROBE != 0 (a probe drops part of the work; its output is invalid).
//   which < 16:  k_wtp_mid<split LDS, which>  (WPR_* bits)
//   which = 100: k_wtp_mid<whole-complex LDS (128 KiB, one workgroup per CU), 0>
//   which = 200 + P: k_wtp_mid_ct<split LDS, P> (comps on lane bits 4-5, permlane solve; r04)
//   which = 300 + P: k_wtp_mid_ct2<split LDS, P> (ct's map between the exchanges only; r04)
//   which = 400 + P: k_wtp_mid_ct2<split LDS, P, LDS-DMA prefetch> (the r04m default)
//   which = 500 + P / 600 + P: k_wtp_mid_ct3<P> (8 points per thread, whole-complex) without / with the
//   whole-unit prefetch
#define CFP_KEXP 1
#include "cfp_wave_three.hip"

using namespace cfp;

extern "C" int wave_probe(int which, void* data, const void* tw, const void* tabx, const void* taby, const void* tabz,
                          double c0sq, int iters, float* ms) {
  WTPArgs a;
  a.tw = (const cd*)tw;
  a.wave.tab[0] = (const double2*)tabx;
  a.wave.tab[1] = (const double2*)taby;
  a.wave.tab[2] = (const double2*)tabz;
  a.wave.n[0] = a.wave.n[1] = a.wave.n[2] = 128;
  a.wave.c0sq = c0sq;
  a.wave.fused = 2;
  a.wave.ncomp = 4;
  a.scale = 1.0;
  cd* d = (cd*)data;
  const int units = 64 * 16;
  auto launch = [&]() -> int {
    switch (which) {
#define C(P) case P: hipLaunchKernelGGL((k_wtp_mid<true, P>), dim3(512), dim3(512), 0, 0, d, a, units); return 0;
      C(0) C(1) C(2) C(3) C(4) C(8) C(12) C(13) C(14) C(15)
#undef C
      case 100: hipLaunchKernelGGL((k_wtp_mid<false, 0>), dim3(256), dim3(512), 0, 0, d, a, units); return 0;
#define D(P) case 200 + P: hipLaunchKernelGGL((k_wtp_mid_ct<true, P>), dim3(512), dim3(512), 0, 0, d, a, units); return 0;
      D(0) D(1) D(2) D(3) D(4) D(8) D(12) D(13) D(14) D(15)
#undef D
#define E(P) case 300 + P: hipLaunchKernelGGL((k_wtp_mid_ct2<true, P>), dim3(512), dim3(512), 0, 0, d, a, units); return 0;
      E(0) E(1) E(2) E(3) E(4) E(8) E(12) E(13) E(14) E(15)
#undef E
#define G(P) case 400 + P: hipLaunchKernelGGL((k_wtp_mid_ct2<true, P, true>), dim3(512), dim3(512), 0, 0, d, a, units); return 0;
      G(0) G(1) G(3) G(8) G(15)
#undef G
#define H(P) case 500 + P: hipLaunchKernelGGL((k_wtp_mid_ct3<P, false>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      H(0) H(1) H(3) H(15)
#undef H
#define I(P) case 600 + P: hipLaunchKernelGGL((k_wtp_mid_ct3<P, true>), dim3(256), dim3(1024), 0, 0, d, a, units); return 0;
      I(0) I(1) I(3)
#undef I
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
