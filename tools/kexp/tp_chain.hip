// tp_chain.hip -- the 256^3 3-sweep apply chain (P1 b -> x, P2 on x, P3 x -> x) with the global
// cache policy of each launch selectable (not product code; every variant is a valid apply):
//   which = p1 + 4 * p2 + 16 * p3
//   p1: 0 NT loads (product), 1 plain, 2 NT loads + NT stores, 3 NT stores
//   p2: 0 plain stores (product), 1 NT stores
//   p3: 0 NT stores (product), 1 NT loads + NT stores, 2 plain
//   + 64: P1 and P3 with the lane-pair phase A; + 128: and the y2 k1 twiddle moved from P2 to P1 / P3
#define CFP_KEXP 1
#include "cfp_three_pass.hip"

using namespace cfp;

static bool g_lp = false;  // which bit 6: P1 / P3 with the lane-pair phase A (k_tp_rows<.., LP>)
static bool g_twy = false;  // which bit 7: the y2 k1 twiddle in P1 / P3 (k_tp_rows<.., TWY>), not in P2
template <int F>
static void p1(const cd* b, cd* x, const TPArgs& a) {
  if (g_twy)
    hipLaunchKernelGGL((k_tp_rows<false, F, 32, 256, 16, true, true, true>), dim3(512), dim3(512), 0, 0, b, x, a, 2048);
  else if (g_lp)
    hipLaunchKernelGGL((k_tp_rows<false, F, 32, 256, 16, true, true>), dim3(512), dim3(512), 0, 0, b, x, a, 2048);
  else
    hipLaunchKernelGGL((k_tp_rows<false, F, 32, 256>), dim3(512), dim3(512), 0, 0, b, x, a, 2048);
}
template <int F>
static void p3(cd* x, const TPArgs& a) {
  if (g_twy)
    hipLaunchKernelGGL((k_tp_rows<true, F, 32, 256, 16, true, true, true>), dim3(512), dim3(512), 0, 0, x, x, a, 2048);
  else if (g_lp)
    hipLaunchKernelGGL((k_tp_rows<true, F, 32, 256, 16, true, true>), dim3(512), dim3(512), 0, 0, x, x, a, 2048);
  else
    hipLaunchKernelGGL((k_tp_rows<true, F, 32, 256>), dim3(512), dim3(512), 0, 0, x, x, a, 2048);
}
template <int ST>
static void p2(cd* x, const TPArgs& a) {
  if (g_twy)
    hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 256, ST, false>), dim3(256), dim3(1024), 0, 0, x, a, 1024);
  else
    hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 256, ST>), dim3(256), dim3(1024), 0, 0, x, a, 1024);
}

extern "C" int tp_chain(int which, const void* b, void* x, const void* tw, const void* colsym, const void* axsym,
                        int iters, float* ms) {
  TPArgs a;
  a.tw = (const cd*)tw;
  a.colsym = (const cd*)colsym;
  a.axsym = (const cd*)axsym;
  a.scale = 1.0 / (256.0 * 256.0 * 256.0);
  const int q1 = which & 3, q2 = (which >> 2) & 3, q3 = (which >> 4) & 3;
  g_lp = (which >> 6) & 1;
  g_twy = (which >> 7) & 1;
  const cd* bb = (const cd*)b;
  cd* xx = (cd*)x;
  auto go = [&]() {
    TPArgs a1 = a;
    a1.scale = 1.0;
    switch (q1) {
      case 0: p1<F_NT_LD>(bb, xx, a1); break;
      case 1: p1<0>(bb, xx, a1); break;
      case 2: p1<F_NT_LD | F_NT_ST>(bb, xx, a1); break;
      default: p1<F_NT_ST>(bb, xx, a1);
    }
    if (q2 == 0) p2<0>(xx, a1);
    else p2<F_NT_ST>(xx, a1);
    switch (q3) {
      case 0: p3<F_NT_ST>(xx, a); break;
      case 1: p3<F_NT_LD | F_NT_ST>(xx, a); break;
      default: p3<0>(xx, a);
    }
  };
  go();
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
