// tp_chain.hip -- the 256^3 3-sweep apply chain (P1 b -> x, P2 on x, P3 x -> x) with the global
// cache policy of each launch selectable (not product code; every variant is a valid apply):
//   which = p1 + 4 * p2 + 16 * p3
//   p1: 0 NT loads (product), 1 plain, 2 NT loads + NT stores, 3 NT stores
//   p2: 0 plain stores (product), 1 NT stores
//   p3: 0 NT stores (product), 1 NT loads + NT stores, 2 plain
//   + 64: P1 and P3 with the lane-pair phase A
//   (+ 128, the y2 k1 twiddle moved from P2 to P1 / P3, was measured in r03z and removed)
//   + 4096: P2 loads non-temporally (its input is read once)
//   + 256 * w: P2 = k_tp_mid_w8 (8 waves, 32 points per thread), w = 1: no register prefetch, 2: 8 slots, 3: 16
#define CFP_KEXP 1
#include "cfp_three_pass.hip"
namespace cfp {
thread_local LaunchStamp g_stamp;  // defined in cfp_plan.hip in the library
// launch_three_pass routes 100^3 to cfp_three_pass_sq.hip, which this harness does not build
hipError_t launch_three_pass_sq(int, int, const cd*, cd*, const TPArgs&, TPShape, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace cfp

namespace cfp {

// ---------------------------------------------------------------------------------------------
// Experiment (r03z, not product code; profiles/r03z_tp_w8.txt): P2 on 8 waves (k_tp_mid_w8): the k_tp_mid_sw unit (64 columns c = x + 8 y2, 256 z) with
// 512 threads of 32 points, z = tz + 8 m (tz = the wave).  At two waves per SIMD a lane has 256
// VGPRs: the 32 points, the temporaries, and VPF register slots of the NEXT unit loaded while this
// one computes (k_tp_mid_sw's 16 points fill its 128 VGPRs, so only the LDS half-prefetch fits).
//   z forward, 256 = 32 x 8:  A: 32-point DFT over m per lane -> Y_tz[k'] (k' = 0..31), twiddle
//     W_256^(tz k'), [y2 DIF on permlane transposes], exchange E1 -> thread (c, t) holds k' = t + 8 j
//     for all 8 tz, B: 8-point DFTs over tz -> kz = t + 8 j + 32 k2 (register 8 j + k2).
//   divide by 1 + colsym + axsym[kz] (axsym staged in LDS: no global load between the register
//     prefetch and its use), conjugate.
//   z inverse (forward DFT on the conjugate), n = n_a + 32 n_b with n_a = t + 8 j, n_b = k2:
//     B': 8-point DFTs over k2 -> q_a (register 8 j + q_a), twiddle W_256^(n_a q_a), [y2 DIT],
//     exchange E2 -> thread (c, t') holds q_a = t' for all 32 n_a, A': 32-point DFT over n_a ->
//     z = t' + 8 q_b: the load layout.
// The y2 stages and their transposed register map are k_tp_mid_sw's (register r at lane L holds
// slot (r & 28) | L5 | 2 L4, column y2 position 4 r0 + 2 r1 + L3); the exchanges write each value
// from there.  PF: after E2 each wave DMAs slots 0..15 of its next unit into the exchange buffer.
namespace {
// 32-point forward DFT, natural order in and out: two 16-point DFTs and a radix-2 with W_32^k
__device__ __forceinline__ void dft32(cd* v) {
  constexpr double C32[8] = {1.0, 0.98078528040323044913, 0.92387953251128675613, 0.83146961230254523708,
                             0.70710678118654752440, 0.55557023301960222474, 0.38268343236508977173,
                             0.19509032201612826785};
  cd e[16], o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    e[i] = v[2 * i];
    o[i] = v[2 * i + 1];
  }
  dft_reg<16>(e);
  dft_reg<16>(o);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    cd t;
    if (k % 2 == 0) {
      t = twr<16>(o[k], k / 2);
    } else {  // (x + iy)(c - is), c = cos(2 pi k / 32), s = sin(2 pi k / 32)
      const double c = k < 8 ? C32[k] : -C32[16 - k], sn = k < 8 ? C32[8 - k] : C32[k - 8];
      t = make_cd(fma(o[k].x, c, o[k].y * sn), fma(o[k].y, c, -o[k].x * sn));
    }
    v[k] = cadd(e[k], t);
    v[k + 16] = csub(e[k], t);
  }
}
}  // namespace

template <bool PF, int VPF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
k_tp_mid_w8(cd* data, TPArgs a, int nunits) {
  constexpr int T = 64, N2 = 8, TN = 256, NX = 256, N1 = TN / N2, XT = T / N2, NXT = NX / XT, XB = 3;
  constexpr int P = 32;                 // points per thread
  constexpr int NPF = PF ? 16 : 0;      // slots 0 .. NPF-1: LDS prefetch
  static_assert(VPF >= 0 && NPF + VPF <= P, "prefetched slots");
  __shared__ __attribute__((aligned(16))) double lds[T * TN];  // split exchange / prefetch buffer
  __shared__ cd tw_l[TN];
  __shared__ cd ax_l[TN];
  const int tid = threadIdx.x;
  for (int i = tid; i < TN; i += 512) {
    tw_l[i] = a.tw[i];
    ax_l[i] = a.axsym[i];
  }
  __syncthreads();
  const int c0 = tid & 63, tz0 = tid >> 6;
  const i64 zs = (i64)NX << (a.lnyl ? a.lnyl : ilog2(TN));
  const auto idx = [](int i) {
    asm volatile("" : "+v"(i));
    return i;
  };
  const auto col_ptr = [&](int u, int c, int tz) {
    const int xt = u % NXT, k1 = u / NXT;
    return data + xt * XT + (c & (XT - 1)) + (i64)NX * ((c >> XB) + N2 * k1) + zs * tz;
  };
  const auto tw_y = [&](int u, int c) { return tw_l[((c >> XB) * (a.k1_off + u / NXT)) & (TN - 1)]; };
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const auto prefetch = [&](int u) {  // this wave's slots 0 .. NPF-1 of unit u -> LDS
    const int c = idx(c0), tz = idx(tz0);
    const cd* src = col_ptr(u, c, tz);
#pragma unroll
    for (int m = 0; m < NPF; ++m)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(src + zs * 8 * m), (lds_void_t*)(lds + (wv * NPF + m) * 128),
                                       16, 0, 0);
  };
  static_assert(!PF || 8 * NPF * 128 <= T * TN, "the prefetch fits the exchange buffer");
  cd pf[VPF > 0 ? VPF : 1];
  const auto vprefetch = [&](int u) {
    const int c = idx(c0), tz = idx(tz0);
    const cd* src = col_ptr(u, c, tz);
#pragma unroll
    for (int m = 0; m < VPF; ++m) pf[m] = src[zs * 8 * (NPF + m)];
  };
  if ((int)blockIdx.x < nunits) {
    if constexpr (PF) prefetch(blockIdx.x);
    if constexpr (VPF > 0) vprefetch(blockIdx.x);
  }
  // one split exchange: value v[r] goes to lds[wr(r)], then v[t] = lds[rd(t)]
  const auto xchg = [&](cd* v, auto wr, auto rd) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < P; ++r) lds[wr(r)] = h ? v[r].y : v[r].x;
      lds_barrier();
#pragma unroll
      for (int t = 0; t < P; ++t) {
        const double d = lds[rd(t)];
        if (h) v[t].y = d; else v[t].x = d;
      }
    }
  };
  // register r at lane c after the y2 stages: slot (r & 28) | L5 | 2 L4, column (c & 7) + 8 p
  const auto slot_of = [](int r, int c) { return (r & 28) | ((c >> 5) & 1) | (((c >> 4) & 1) << 1); };
  const auto colp_of = [](int r, int c) { return (c & 7) + 8 * (4 * (r & 1) + 2 * ((r >> 1) & 1) + ((c >> 3) & 1)); };

  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    cd v[P];
    cd cs;
    {
      const int c = idx(c0), tz = idx(tz0);
      const cd* src = col_ptr(u, c, tz);
#pragma unroll
      for (int m = NPF + VPF; m < P; ++m) v[m] = src[zs * 8 * m];
#pragma unroll
      for (int m = 0; m < VPF; ++m) v[NPF + m] = pf[m];
      const int k1 = a.k1_off + u / NXT, p = c >> XB;  // global k1; column y2 position -> frequency brev3(p)
      cs = a.colsym[(u % NXT) * XT + (c & (XT - 1)) + (i64)NX * (k1 + N1 * brev<N2>(p))];
      if constexpr (PF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA, loads and stores landed
#pragma unroll
        for (int m = 0; m < NPF; ++m) v[m] = fromv(*reinterpret_cast<const dv2*>(lds + (wv * NPF + m) * 128 + 2 * c));
      }
    }
    if constexpr (VPF > 0) {
      if (u + (int)gridDim.x < nunits) vprefetch(u + gridDim.x);
    }
    {
      const int c = idx(c0);
      const cd w = tw_y(u, c);
#pragma unroll
      for (int m = 0; m < P; ++m) v[m] = cmul(v[m], w);
    }
    dft32(v);  // A: v[k'] = Y_tz[k']
    {
      const int tz = idx(tz0);
#pragma unroll
      for (int k = 1; k < P; ++k) v[k] = cmul(v[k], tw_l[(tz * k) & (TN - 1)]);
    }
    {  // y2 DIF: natural positions in, bit-reversed frequencies out
      {
        const int c = idx(c0);
        dif_pairs<5, 1, true, P>(v, tw_l[(TN / 8) * ((c >> 3) & 3)]);  // W_8^{y2 & 3}
      }
      {
        const int c = idx(c0);
        dif_pairs<4, 2, true, P>(v, tw_l[(TN / 4) * ((c >> 3) & 1)]);  // W_4^{y2 & 1}
      }
      const int c = idx(c0);
      const double sg = (c & 8) ? -1.0 : 1.0;
#pragma unroll
      for (int r = 0; r < P; ++r) v[r] = bfly_l3(v[r], sg);
    }
    {  // E1: [k' (32)][tz (8)][column (64)]; thread (c, t) reads k' = t + 8 j, all tz
      const int c = idx(c0), tz = idx(tz0);
      xchg(
          v, [&](int r) { return (slot_of(r, c) * 8 + tz) * 64 + colp_of(r, c); },
          [&](int t) { return ((tz + 8 * (t >> 3)) * 8 + (t & 7)) * 64 + c; });
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) dft_reg<8>(v + 8 * j);  // B: register 8 j + k2 = kz t + 8 j + 32 k2
    {
      const int t = idx(tz0);
#pragma unroll
      for (int r = 0; r < P; ++r) {
        const cd d = cadd(cadd(cs, ax_l[t + 8 * (r >> 3) + 32 * (r & 7)]), make_cd(1.0, 0.0));
        v[r] = cconj(cdiv_sym(v[r], d));
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) dft_reg<8>(v + 8 * j);  // B': register 8 j + q_a, n_a = t + 8 j
    {
      const int t = idx(tz0);
#pragma unroll
      for (int r = 0; r < P; ++r)
        if (r & 7) v[r] = cmul(v[r], tw_l[((t + 8 * (r >> 3)) * (r & 7)) & (TN - 1)]);
    }
    {  // y2 DIT: bit-reversed positions in, natural out (k_tp_mid_sw's inverse stages)
      {
        const int c = idx(c0);
        const double sg = (c & 8) ? -1.0 : 1.0;
#pragma unroll
        for (int r = 0; r < P; ++r) v[r] = bfly_l3(v[r], sg);
      }
      {
        const int c = idx(c0);
        const cd w = tw_l[(TN / 4) * ((c >> 3) & 1)];
#pragma unroll
        for (int k = 0; k < P; ++k)
          if ((k & 2) == 0) swap_c<4>(v[k], v[k + 2]);
#pragma unroll
        for (int k = 0; k < P; ++k)
          if ((k & 2) == 0) {
            const cd x = v[k], y = cmul(v[k + 2], w);
            v[k] = cadd(x, y);
            v[k + 2] = csub(x, y);
          }
      }
      {
        const int c = idx(c0);
        const cd w = tw_l[(TN / 8) * ((c >> 3) & 1)];
#pragma unroll
        for (int k = 0; k < P; ++k)
          if ((k & 1) == 0) swap_c<5>(v[k], v[k + 1]);
#pragma unroll
        for (int k = 0; k < P; ++k)
          if ((k & 1) == 0) {
            cd y = cmul(v[k + 1], w);
            if (k & 2) y = mul_mi(y);
            const cd x = v[k];
            v[k] = cadd(x, y);
            v[k + 1] = csub(x, y);
          }
      }
    }
    {  // E2: [q_a (8)][n_a (32)][column (64)]; thread (c, t') reads q_a = t', all n_a
      const int c = idx(c0), tz = idx(tz0);
      xchg(
          v,
          [&](int r) {
            const int s = slot_of(r, c);
            return ((s & 7) * 32 + tz + 8 * (s >> 3)) * 64 + colp_of(r, c);
          },
          [&](int t) { return (tz * 32 + t) * 64 + c; });
    }
    if constexpr (PF) {
      lds_barrier();  // every wave has read the exchange buffer
      if (u + (int)gridDim.x < nunits) prefetch(u + gridDim.x);
    }
    dft32(v);  // A': v[q_b] = z = t' + 8 q_b (the load layout)
    {
      const int c = idx(c0), tz = idx(tz0);
      const cd w = tw_y(u, c);
      cd* dst = col_ptr(u, c, tz);
#pragma unroll
      for (int m = 0; m < P; ++m) dst[zs * 8 * m] = cconj(cmul(v[m], w));
    }
    if constexpr (!PF) lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

}  // namespace cfp

using namespace cfp;

static bool g_lp = false;  // which bit 6: P1 / P3 with the lane-pair phase A (k_tp_rows<.., LP>)
template <int F>
static void p1(const cd* b, cd* x, const TPArgs& a) {
  if (g_lp)
    hipLaunchKernelGGL((k_tp_rows<false, F, 32, 256, 16, true, true>), dim3(512), dim3(512), 0, 0, b, x, a, 2048);
  else
    hipLaunchKernelGGL((k_tp_rows<false, F, 32, 256>), dim3(512), dim3(512), 0, 0, b, x, a, 2048);
}
template <int F>
static void p3(cd* x, const TPArgs& a) {
  if (g_lp)
    hipLaunchKernelGGL((k_tp_rows<true, F, 32, 256, 16, true, true>), dim3(512), dim3(512), 0, 0, x, x, a, 2048);
  else
    hipLaunchKernelGGL((k_tp_rows<true, F, 32, 256>), dim3(512), dim3(512), 0, 0, x, x, a, 2048);
}
static bool g_p2nt = false;  // which bit 12: P2 with non-temporal loads (and LDS-DMA)
static int g_w8 = 0;  // which bits 8..9: P2 = k_tp_mid_w8 with 1: VPF 0, 2: VPF 8, 3: VPF 16
template <int ST>
static void p2(cd* x, const TPArgs& a) {
  if (g_p2nt)
    hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 256, ST, F_NT_LD>), dim3(256), dim3(1024), 0, 0, x, a, 1024);
  else if (g_w8 == 1)
    hipLaunchKernelGGL((k_tp_mid_w8<true, 0>), dim3(256), dim3(512), 0, 0, x, a, 1024);
  else if (g_w8 == 2)
    hipLaunchKernelGGL((k_tp_mid_w8<true, 8>), dim3(256), dim3(512), 0, 0, x, a, 1024);
  else if (g_w8 == 3)
    hipLaunchKernelGGL((k_tp_mid_w8<true, 16>), dim3(256), dim3(512), 0, 0, x, a, 1024);
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
  g_w8 = (which >> 8) & 3;
  g_p2nt = (which >> 12) & 1;
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
