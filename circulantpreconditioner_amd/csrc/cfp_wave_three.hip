// cfp_wave_three.hip -- the 3-sweep apply of the wave-system block-circulant plan on a 128^3
// grid (config 4; cfp_wave.hip's 5-sweep schedule serves every other grid).  The field is the
// reference's interleaved layout idx = 4 cell + comp (src/WaveSystem.cxx:112-113), 64 bytes per
// cell.  As in the scalar 3-sweep (cfp_three_pass.hip) the y transform is split four-step,
// here ny = N1 N2 = 16 x 8, y = y2 + 8 y1, ky = k1 + 16 k2:
//
//   P1w k_wtp_rows<fwd>: one z-plane's rows y2 + 8 y1 (16 rows x 128 cells x 4 comps = 128 KiB).
//       Column mode, one thread per column 4 x + comp: the 16-point y1 DFT in registers; LDS
//       transpose to 64 rows (k1, comp) with the 4 comps of a cell in adjacent lanes; the
//       128-point x DFT along each row.  Every intermediate stays in its slot (y1 <-> k1).
//   P2w k_wtp_mid: 2 cells x 4 comps x 8 y2 (64 columns, lane = comp + 4 y2 + 32 x) x 128 z of
//       one k1: twiddle W_128^{y2 k1}, 8-point y2 DFT across lane bits 2..4 (DPP lane ^ 4, ^ 8,
//       ds_swizzle lane ^ 16), 128-point z DFT, the arrowhead solve S(k)^-1 per frequency with
//       the 4 comps gathered from the lane quad (wave_point, cfp_fft_device.h), then the same
//       transforms on the conjugate (inverse).
//   P3w k_wtp_rows<inv>: P1w on the conjugate, x 1/N.
//
// An apply moves 3 x (read + write) x 64 bytes per cell instead of the 5-sweep schedule's 5 x.
#include <hip/hip_ext.h>

#include "cfp_fft_device.h"
#include "cfp_internal.h"
#include "cfp_lane.h"
#include "cfp_three_pass.h"

#ifndef CFP_WAVE_MID_XCD
#define CFP_WAVE_MID_XCD 1
#endif

namespace cfp {

namespace {

constexpr int WNX = 128, WNC = 4, WW = WNX * WNC;  // cells per row, comps, values per row
// TWR: the four-step twiddle W_128^{y2 k1} rides in P1w's stores and P3w's loads instead of P2w's
// loads and stores (it is constant along a P1w row and uniform per P3w slot)
#ifndef CFP_WAVE_TWR
#define CFP_WAVE_TWR 0
#endif
constexpr bool kWaveTwr = CFP_WAVE_TWR != 0;
constexpr int WN1 = 16, WN2 = 8;                   // y = y2 + WN2 y1
constexpr i64 WPLANE = (i64)WNX * WW;              // values per z-plane

__device__ __forceinline__ int launder(int i) {
  asm volatile("" : "+v"(i));
  return i;
}

// first radix of an n-point FFT done as r0 x PTS x ... x PTS (n = r0 PTS^k, r0 <= PTS)
constexpr int wr0_of(int n, int pts) { return n > pts ? wr0_of(n / pts, pts) : n; }

}  // namespace

// P1w / P3w.  512 threads, 16 points each; one unit = (z, y2); persistent over the units.
// FLAGS: the global load / store policy (F_NT_LD, F_NT_ST).  XCD: units in xcd_round_unit order
// (the grid a multiple of 8 workgroups).
// NP > 0 (P3w only): the Gram-Schmidt dots post_v[j]^H x of the stored points ride in the sweep
// (WTPArgs post_*), as in the scalar P3 (cfp_three_pass.hip): per unit the lanes' sums are wave
// reductions added to the wave's LDS slot, one partial per workgroup and value at the end.
template <bool INV, int FLAGS, bool XCD = false, int NP = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
k_wtp_rows(const cd* in, cd* out, WTPArgs a, int nunits) {
  constexpr bool POST = INV && NP > 0;
  constexpr int NPP = POST ? NP : 1;
  constexpr int NW = 512 / 64;
  __shared__ double post_l[POST ? 2 * NPP * NW : 1];
  __shared__ const cd* post_ptr_l[NPP];
  __shared__ int post_n_l[2];  // post_nv, post_self
  if constexpr (POST) {
    for (int i = threadIdx.x; i < 2 * NPP * NW; i += 512) post_l[i] = 0.0;
    if (threadIdx.x < NPP) post_ptr_l[threadIdx.x] = a.post_v[threadIdx.x];
    if (threadIdx.x == 0) {
      post_n_l[0] = a.post_nv;
      post_n_l[1] = a.post_self;
    }
    __syncthreads();
  }
  constexpr int PTS = 16, TR = WNX / PTS;  // row mode: 8 threads per (row, comp)
  constexpr int NROW = WN1 * WNC;          // 64 row-mode rows (k1, comp)
  constexpr int CS = WW + WW / 16;         // padded stride of the column-mode transpose rows
  constexpr int RS = WNX + WNX / 16;       // fft_stages' row-mode stride
  constexpr int F = F_SPLIT_LDS | F_LDS_SYNC | F_TW_GLOBAL;
  constexpr int LDS_D = WN1 * CS > NROW * RS ? WN1 * CS : NROW * RS;
  static_assert(WN1 == PTS, "the y1 DFT runs in registers");
  __shared__ __attribute__((aligned(16))) double lds[LDS_D];
  const int tid = threadIdx.x;
  const int c0 = tid;  // column mode: column 4 x + comp
  const int comp0 = tid & 3, tx0 = (tid >> 2) & (TR - 1), k0 = tid >> 5;  // row mode
  for (int it = blockIdx.x; it < nunits; it += gridDim.x) {
    const int u = XCD ? xcd_round_unit(it, gridDim.x, nunits) : it;
    const int z = u / WN2, y2 = u % WN2;
    cd v[PTS];
    {
      const int c = launder(c0);
      const cd* src = in + z * WPLANE + (i64)y2 * WW + c;
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(src + (i64)WN2 * WW * m);  // rows y2 + 8 m
      __builtin_amdgcn_sched_barrier(0);  // every load out before the first butterfly
      if (INV) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
        if constexpr (kWaveTwr) {  // slot m = k1: W_128^{y2 m}, uniform over the workgroup
#pragma unroll
          for (int m = 1; m < PTS; ++m) v[m] = cmul(v[m], a.tw[(y2 * m) & (WNX - 1)]);
        }
      }
      dft_any<PTS>(v);  // v[m]: k1 = m (forward) / y1 = m (inverse)
    }
    {
      // transpose: (slot m, column c) -> row m's comp of cell x = tx + TR t
      const int c = launder(c0), comp = launder(comp0), tx = launder(tx0), k = launder(k0);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) lds[m * CS + c + (c >> 4)] = half ? v[m].y : v[m].x;
        lds_barrier();
#pragma unroll
        for (int t = 0; t < PTS; ++t) {
          const int cc = WNC * (tx + TR * t) + comp;
          const double val = lds[k * CS + cc + (cc >> 4)];
          if (half) v[t].y = val; else v[t].x = val;
        }
        lds_barrier();
      }
    }
    {
      const int comp = launder(comp0), tx = launder(tx0), k = launder(k0);
      // a row's TR threads are lanes 32 k + 4 tx + comp of one wave and its LDS row is theirs:
      // the exchange waits for the wave's own LDS accesses only (F_WAVE_LDS, r04ab)
      fft_stages<WNX, PTS, wr0_of(WNX, PTS), true, NROW, F | F_WAVE_LDS>(v, lds, a.tw, k * WNC + comp, tx, true);  // v[t]: kx = tx + TR t
    }
    {
      const int comp = launder(comp0), tx = launder(tx0), k = launder(k0);
      const double sc = a.scale, sy = INV ? -sc : sc;
      cd* dst = out + z * WPLANE + (i64)(y2 + WN2 * k) * WW + WNC * tx + comp;
      if (kWaveTwr && !INV) {  // row k1 = k: W_128^{y2 k} (P1w scale is 1)
        const cd w = a.tw[(y2 * k) & (WNX - 1)];
#pragma unroll
        for (int t = 0; t < PTS; ++t) gstore<FLAGS>(dst + WNC * TR * t, cmul(v[t], w));
      } else {
#pragma unroll
        for (int t = 0; t < PTS; ++t) {
          v[t] = make_cd(v[t].x * sc, v[t].y * sy);
          gstore<FLAGS>(dst + WNC * TR * t, v[t]);
        }
      }
      if constexpr (POST) {
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const int pnv = ((volatile int*)post_n_l)[0], pself = ((volatile int*)post_n_l)[1];
        const i64 e0 = dst - out;
        constexpr int QB = 4;
#pragma unroll
        for (int j = 0; j < NPP; ++j) {
          if (j < pnv) {
            double sr = 0.0, si = 0.0;
            if ((pself >> j) & 1) {
#pragma unroll
              for (int t = 0; t < PTS; ++t) sr += v[t].x * v[t].x + v[t].y * v[t].y;
            } else {
              const cd* pv = ((const cd* volatile*)post_ptr_l)[j] + e0;
#pragma unroll
              for (int t0 = 0; t0 < PTS; t0 += QB) {
                cd q[QB];
#pragma unroll
                for (int t = 0; t < QB; ++t) q[t] = gload<F_NT_LD>(pv + WNC * TR * (t0 + t));
#pragma unroll
                for (int t = 0; t < QB; ++t) {
                  const cd w = v[t0 + t];
                  sr += q[t].x * w.x + q[t].y * w.y;
                  si += q[t].x * w.y - q[t].y * w.x;
                }
              }
            }
            sr = wave_sum_d(sr);
            si = wave_sum_d(si);
            if (lane == 0) {
              post_l[(2 * j) * NW + wv] += sr;
              post_l[(2 * j + 1) * NW + wv] += si;
            }
          }
        }
      }
    }
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
  if constexpr (POST) {
    // one partial per workgroup and value: the waves' sums in a fixed order
    __syncthreads();
    if (threadIdx.x < 2 * NPP) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < NW; ++q) t += post_l[threadIdx.x * NW + q];
      a.post_partial[(size_t)blockIdx.x * 16 + threadIdx.x] = t;
    }
  }
}

// P2w.  512 threads = 8 z-groups x 64 columns (one wave per z-group); 16 points per thread.
// PROBE != 0 only in tools/kexp (wave_probe.hip, built with CFP_KEXP): timing probes that drop
// a part of the work (output invalid); the product library instantiates PROBE = 0 only.
enum { WPR_NO_Y2 = 1, WPR_NO_SOLVE = 2, WPR_NO_LOAD = 4, WPR_NO_STORE = 8 };
template <bool XS, int PROBE = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
k_wtp_mid(cd* data, WTPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int XT = 2, T = WNC * WN2 * XT;  // 64 columns: lane = comp + 4 y2 + 32 xl
  constexpr int PTS = 16, TZ = WNX / PTS;    // 8 z-groups, kz = tz + 8 m
  constexpr int NXT = WNX / XT;              // x tiles
  constexpr int F = (XS ? F_SPLIT_LDS : 0) | F_LDS_SYNC;
  __shared__ __attribute__((aligned(16))) double lds[T * WNX * (XS ? 1 : 2)];
  __shared__ cd tw_l[WNX];
  const int tid = threadIdx.x;
  for (int i = tid; i < WNX; i += T * TZ) tw_l[i] = a.tw[i];
  const int c0 = tid & (T - 1), tz0 = tid / T;
  const i64 zs = WPLANE;
  const double c0sq = a.wave.c0sq;
  // the thread's first point and its y twiddles (rebuilt where used: nothing but the points
  // stays live across an FFT)
  struct Col {
    cd* p;
    int y2;
    cd w, w8;  // W_128^{y2 k1}; W_8^(y2 & 3)
  };
  const auto column = [&](int u) {
    const int c = launder(c0), tz = launder(tz0);
    Col q;
    const int xt = u % NXT, k1 = u / NXT;
    const int comp = c & 3, xl = c >> 5;
    q.y2 = (c >> 2) & (WN2 - 1);
    q.p = data + (i64)(q.y2 + WN2 * k1) * WW + (xt * XT + xl) * WNC + comp + zs * tz;
    q.w = a.tw[(q.y2 * k1) & (WNX - 1)];
    q.w8 = a.tw[(WNX / 8) * (q.y2 & 3)];
    return q;
  };
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    cd v[PTS];
    {
      const Col q = column(u);
      if constexpr (PROBE & WPR_NO_LOAD) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = make_cd((double)m, (double)q.y2);
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = q.p[zs * TZ * m];
      }
      __builtin_amdgcn_sched_barrier(0);
      // 8-point DIF over y2 = lane bits 2..4; lane y2 ends with frequency k2 = brev3(y2).
      // Each radix-2 stage is branch-free: the upper lane forms partner - own as fma(-1, own,
      // partner), the lower own + partner; the upper lanes' twiddle W_8^(y2 & 3) is 1 below.
      const double s4 = q.y2 & 4 ? -1.0 : 1.0, s2 = q.y2 & 2 ? -1.0 : 1.0, s1 = q.y2 & 1 ? -1.0 : 1.0;
      const bool mi = (q.y2 & 3) == 3;
      const cd w8 = q.y2 & 4 ? q.w8 : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        v[m] = cmul(v[m], q.w);
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd p = lane_xor16(v[m]);
        v[m] = cmul(make_cd(fma(s4, v[m].x, p.x), fma(s4, v[m].y, p.y)), w8);
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd p = lane_xor8(v[m]);
        cd t = make_cd(fma(s2, v[m].x, p.x), fma(s2, v[m].y, p.y));
        t = mi ? mul_mi(t) : t;
        const cd r = lane_xor4(t);
        v[m] = make_cd(fma(s1, t.x, r.x), fma(s1, t.y, r.y));
      }
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      fft_stages<WNX, PTS, wr0_of(WNX, PTS), false, T, F>(v, lds, tw_l, c, tz, true);  // v[m]: kz = tz + TZ m
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      const int xt = u % NXT, k1 = u / NXT;
      const int comp = c & 3, xl = c >> 5, y2 = (c >> 2) & (WN2 - 1);
      const int k2 = ((y2 & 1) << 2) | (y2 & 2) | (y2 >> 2);
      double2 pq[3];
      pq[0] = a.wave.tab[0][xt * XT + xl];
      pq[1] = a.wave.tab[1][k1 + WN1 * k2];
      pq[2] = make_double2(0.0, 0.0);
      const WaveCol wc = wave_col(pq, 2, comp, c0sq);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_SOLVE) {
          v[m] = cconj(v[m]);
          continue;
        }
        cd r[4];
        r[0] = make_cd(quad_bcast<0>(v[m].x), quad_bcast<0>(v[m].y));
        r[1] = make_cd(quad_bcast<1>(v[m].x), quad_bcast<1>(v[m].y));
        r[2] = make_cd(quad_bcast<2>(v[m].x), quad_bcast<2>(v[m].y));
        r[3] = make_cd(quad_bcast<3>(v[m].x), quad_bcast<3>(v[m].y));
        v[m] = cconj(wave_point(r, comp, 2, wc, a.wave.tab[2][tz + TZ * m], c0sq));
      }
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      fft_stages<WNX, PTS, wr0_of(WNX, PTS), false, T, F>(v, lds, tw_l, c, tz, false);
    }
    {
      const Col q = column(u);
      // forward DFT from the bit-reversed order back to natural (the inverse by conjugation),
      // branch-free as above
      const double s4 = q.y2 & 4 ? -1.0 : 1.0, s2 = q.y2 & 2 ? -1.0 : 1.0, s1 = q.y2 & 1 ? -1.0 : 1.0;
      const bool mi = (q.y2 & 3) == 3;
      const cd w8 = q.y2 & 4 ? q.w8 : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd r = lane_xor4(v[m]);
        cd t = make_cd(fma(s1, v[m].x, r.x), fma(s1, v[m].y, r.y));
        t = mi ? mul_mi(t) : t;
        const cd p = lane_xor8(t);
        v[m] = make_cd(fma(s2, t.x, p.x), fma(s2, t.y, p.y));
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) {
          v[m] = cmul(v[m], q.w);
          continue;
        }
        const cd t = cmul(v[m], w8);
        const cd p = lane_xor16(t);
        v[m] = cmul(make_cd(fma(s4, t.x, p.x), fma(s4, t.y, p.y)), q.w);
      }
      if constexpr (PROBE & WPR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x + v[m].y;
        if (acc == 1.2345e300) q.p[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) q.p[zs * TZ * m] = cconj(v[m]);
      }
    }
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

// P2w with the cell's 4 comps on the top lane bits (k_wtp_mid_ct, r04, the default).  Lane =
// y2 bit 0 (lane bit 0) + y2 bit 1 (bit 1) + xl (bit 2) + y2 bit 2 (bit 3) + comp (bits 4-5): a wave
// still reads 8 runs of 2 cells x 4 comps (128 B) per z.  The y2 stages are one DPP move each
// (quad_perm lane ^ 1, ^ 2; row_ror:8 for lane ^ 8) instead of ds_swizzle + two DPP moves, and the
// arrowhead solve transposes the comps into registers with v_permlane16/32_swap (lane bits 4-5 <->
// register bits 0-1, 8 swaps per double pair group): each lane then solves 4 whole cells in
// registers, once, where k_wtp_mid gathers the quad with 4 DPP broadcasts per value and every lane
// of the quad redoes the cell's reciprocal and sums.  Register r then holds comp r & 3 of slot
// (r & 12) | L4 | 2 L5; the transpose is undone before the inverse z FFT.
template <bool XS, int PROBE = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
k_wtp_mid_ct(cd* data, WTPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int XT = 2, T = WNC * WN2 * XT;  // 64 columns, one per lane
  constexpr int PTS = 16, TZ = WNX / PTS;    // 8 z-groups, kz = tz + 8 m
  constexpr int NXT = WNX / XT;
  constexpr int F = (XS ? F_SPLIT_LDS : 0) | F_LDS_SYNC;
  __shared__ __attribute__((aligned(16))) double lds[T * WNX * (XS ? 1 : 2)];
  __shared__ cd tw_l[WNX];
  const int tid = threadIdx.x;
  for (int i = tid; i < WNX; i += T * TZ) tw_l[i] = a.tw[i];
  const int c0 = tid & (T - 1), tz0 = tid / T;
  const i64 zs = WPLANE;
  const double c0sq = a.wave.c0sq;
  const auto y2_of = [](int l) { return (l & 3) | ((l >> 1) & 4); };
  struct Col {
    cd* p;
    int y2;
    cd w, w8;  // W_128^{y2 k1}; W_8^(y2 & 3)
  };
  const auto column = [&](int u) {
    const int c = launder(c0), tz = launder(tz0);
    Col q;
    const int xt = u % NXT, k1 = u / NXT;
    const int comp = c >> 4, xl = (c >> 2) & 1;
    q.y2 = y2_of(c);
    q.p = data + (i64)(q.y2 + WN2 * k1) * WW + (xt * XT + xl) * WNC + comp + zs * tz;
    q.w = a.tw[(q.y2 * k1) & (WNX - 1)];
    q.w8 = a.tw[(WNX / 8) * (q.y2 & 3)];
    return q;
  };
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    cd v[PTS];
    {
      const Col q = column(u);
      if constexpr (PROBE & WPR_NO_LOAD) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = make_cd((double)m, (double)q.y2);
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = q.p[zs * TZ * m];
      }
      __builtin_amdgcn_sched_barrier(0);
      // 8-point DIF over y2 (lane bits 3, 1, 0), branch-free as in k_wtp_mid; lane y2 ends with
      // frequency k2 = brev3(y2)
      const double s4 = q.y2 & 4 ? -1.0 : 1.0, s2 = q.y2 & 2 ? -1.0 : 1.0, s1 = q.y2 & 1 ? -1.0 : 1.0;
      const bool mi = (q.y2 & 3) == 3;
      const cd w8 = q.y2 & 4 ? q.w8 : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        v[m] = cmul(v[m], q.w);
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd p = lane_xor8(v[m]);
        v[m] = cmul(make_cd(fma(s4, v[m].x, p.x), fma(s4, v[m].y, p.y)), w8);
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd p = dpp_c<DPP_XOR2>(v[m]);
        cd t = make_cd(fma(s2, v[m].x, p.x), fma(s2, v[m].y, p.y));
        t = mi ? mul_mi(t) : t;
        const cd r = dpp_c<DPP_XOR1>(t);
        v[m] = make_cd(fma(s1, t.x, r.x), fma(s1, t.y, r.y));
      }
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      fft_stages<WNX, PTS, wr0_of(WNX, PTS), false, T, F>(v, lds, tw_l, c, tz, true);  // v[m]: kz = tz + TZ m
    }
    if constexpr (PROBE & WPR_NO_SOLVE) {
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
    } else {
      const int c = launder(c0), tz = launder(tz0);
      const int xt = u % NXT, k1 = u / NXT;
      const int y2 = y2_of(c), xl = (c >> 2) & 1;
      const int k2 = ((y2 & 1) << 2) | (y2 & 2) | (y2 >> 2);
      // the two non-fused axes, folded once per column (wave_col's algebra, every comp at once)
      const double2 px = a.wave.tab[0][xt * XT + xl], py = a.wave.tab[1][k1 + WN1 * k2];
      const double iex = 1.0 / (1.0 + px.x), iey = 1.0 / (1.0 + py.x);
      const double wx = px.y * iex, wy = py.y * iey;
      const double dnf = 1.0 + px.x + py.x + c0sq * (px.y * wx + py.y * wy);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
      const int sl = ((c >> 4) & 1) | (((c >> 5) & 1) << 1);  // slot bits 0-1 now on lane bits 4-5
#pragma unroll
      for (int g = 0; g < PTS / 4; ++g) {
        const double2 pk = a.wave.tab[2][tz + TZ * (4 * g + sl)];
        const double ef = 1.0 + pk.x;
        const double D2 = fma(dnf + pk.x, ef, c0sq * pk.y * pk.y);
        const double inv = rcp_nr(ef * D2);
        const double id = ef * ef * inv, ief = D2 * inv;
        const double wz = pk.y * ief;
        cd* r = v + 4 * g;
        const double tx = fma(wx, r[1].x, fma(wy, r[2].x, wz * r[3].x));
        const double ty = fma(wx, r[1].y, fma(wy, r[2].y, wz * r[3].y));
        const cd x0 = make_cd(fma(c0sq, ty, r[0].x) * id, fma(-c0sq, tx, r[0].y) * id);
        r[1] = make_cd(fma(px.y, x0.y, r[1].x) * iex, fma(-px.y, x0.x, r[1].y) * iex);
        r[2] = make_cd(fma(py.y, x0.y, r[2].x) * iey, fma(-py.y, x0.x, r[2].y) * iey);
        r[3] = make_cd(fma(pk.y, x0.y, r[3].x) * ief, fma(-pk.y, x0.x, r[3].y) * ief);
        r[0] = x0;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = cconj(r[j]);
      }
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      fft_stages<WNX, PTS, wr0_of(WNX, PTS), false, T, F>(v, lds, tw_l, c, tz, false);
    }
    {
      const Col q = column(u);
      const double s4 = q.y2 & 4 ? -1.0 : 1.0, s2 = q.y2 & 2 ? -1.0 : 1.0, s1 = q.y2 & 1 ? -1.0 : 1.0;
      const bool mi = (q.y2 & 3) == 3;
      const cd w8 = q.y2 & 4 ? q.w8 : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) continue;
        const cd r = dpp_c<DPP_XOR1>(v[m]);
        cd t = make_cd(fma(s1, v[m].x, r.x), fma(s1, v[m].y, r.y));
        t = mi ? mul_mi(t) : t;
        const cd p = dpp_c<DPP_XOR2>(t);
        v[m] = make_cd(fma(s2, t.x, p.x), fma(s2, t.y, p.y));
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & WPR_NO_Y2) {
          v[m] = cmul(v[m], q.w);
          continue;
        }
        const cd t = cmul(v[m], w8);
        const cd p = lane_xor8(t);
        v[m] = cmul(make_cd(fma(s4, t.x, p.x), fma(s4, t.y, p.y)), q.w);
      }
      if constexpr (PROBE & WPR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x + v[m].y;
        if (acc == 1.2345e300) q.p[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) q.p[zs * TZ * m] = cconj(v[m]);
      }
    }
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

// P2w with two lane maps (k_wtp_mid_ct2, r04): the global loads and stores use k_wtp_mid's map
// (lane = comp + 4 y2 + 32 xl: 4 lanes = one cell's 64 contiguous bytes), and the z FFT's
// exchange switches to k_wtp_mid_ct's map (fft_stages_perm: write the old column, read the new),
// where the y2 stages are single DPP moves and the comps sit on lane bits 4-5 for the permlane
// solve; the inverse exchange switches back.  The y2 DFT runs between the z FFTs (it commutes
// with them; the twiddle W_128^{y2 k1} is applied at the load and the store).  k_wtp_mid_ct
// keeps its map for the global accesses too, and pays for it there: 49.3 against 44.5 us with
// the y2 DFT and the solve dropped (profiles/r04_wave_probe.txt).
//
// PF (r04): the scalar P2's LDS-DMA prefetch.  The split exchange buffer (64 columns x 128 z x 8
// bytes) is idle from the inverse exchange's last read to the next unit's first exchange: right
// after that read each wave DMAs slots 0..7 of its columns of unit u + gridDim.x into it
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, lane-linear), so those loads fly during
// the last FFT stage, the twiddle and the stores; the next unit loads only slots 8..15 from HBM.
typedef __attribute__((address_space(3))) void wlds_void_t;
typedef __attribute__((address_space(1))) void wglb_void_t;
template <bool XS, int PROBE = 0, bool PF = false, bool XCD = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
k_wtp_mid_ct2(cd* data, WTPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int XT = 2, T = WNC * WN2 * XT;  // 64 columns, one per lane
  constexpr int PTS = 16, TZ = WNX / PTS;    // 8 z-groups, kz = tz + 8 m
  constexpr int NXT = WNX / XT;
  constexpr int F = (XS ? F_SPLIT_LDS : 0) | F_LDS_SYNC;
  __shared__ __attribute__((aligned(16))) double lds[T * WNX * (XS ? 1 : 2)];
  __shared__ cd tw_l[WNX];
  const int tid = threadIdx.x;
  for (int i = tid; i < WNX; i += T * TZ) tw_l[i] = a.tw[i];
  const int c0 = tid & (T - 1), tz0 = tid / T;
  const i64 zs = WPLANE;
  const double c0sq = a.wave.c0sq;
  // map B (between the exchanges): y2 bits on lane bits 0, 1, 3; xl on 2; comp on 4-5
  const auto y2_b = [](int l) { return (l & 3) | ((l >> 1) & 4); };
  // LDS column of (comp, y2, xl) = comp0 | (comp1 ^ xl) << 1 | y2 << 2 | xl << 5: the 32 lanes of
  // either half-wave hit 32 different bank pairs in both maps (with comp + 4 y2 + 32 xl, map B's
  // halves collide on xl)
  const auto lab_a = [](int l) { return l ^ ((l >> 4) & 2); };
  const auto lab_b = [&](int l) {
    const int xl = (l >> 2) & 1;
    return ((l >> 4) & 1) | ((((l >> 5) & 1) ^ xl) << 1) | (y2_b(l) << 2) | (xl << 5);
  };
  // map A (global accesses): this lane's first point and W_128^{y2 k1}
  const auto col_ptr = [&](int u, int c, int tz) {
    const int xt = u % NXT, k1 = u / NXT;
    return data + (i64)(((c >> 2) & (WN2 - 1)) + WN2 * k1) * WW + (xt * XT + (c >> 5)) * WNC + (c & 3) + zs * tz;
  };
  const auto tw_y = [&](int u, int c) { return a.tw[(((c >> 2) & (WN2 - 1)) * (u / NXT)) & (WNX - 1)]; };
  constexpr int NPF = PF ? 8 : 0;  // slots 0 .. NPF-1 come from the LDS prefetch
  static_assert(!PF || XS, "the prefetch fills the split exchange buffer");
  static_assert(!PF || (T * TZ / 64) * NPF * 128 <= T * WNX, "the prefetch fits the exchange buffer");
  const int wv = __builtin_amdgcn_readfirstlane(tid / 64);
  const auto prefetch = [&](int u) {  // this wave's slots 0 .. NPF-1 of unit u -> LDS
    const int c = launder(c0), tz = launder(tz0);
    const cd* src = col_ptr(u, c, tz);
#pragma unroll
    for (int m = 0; m < NPF; ++m)
      __builtin_amdgcn_global_load_lds((wglb_void_t*)(src + zs * TZ * m), (wlds_void_t*)(lds + (wv * NPF + m) * 128),
                                       16, 0, 0);
  };
  if constexpr (PF) {
    if ((int)blockIdx.x < nunits) prefetch(XCD ? xcd_round_unit(blockIdx.x, gridDim.x, nunits) : (int)blockIdx.x);
  }
  for (int it = blockIdx.x; it < nunits; it += gridDim.x) {
    const int u = XCD ? xcd_round_unit(it, gridDim.x, nunits) : it;
    cd v[PTS];
    {
      const int c = launder(c0), tz = launder(tz0);
      const cd* src = col_ptr(u, c, tz);
      if constexpr (PROBE & WPR_NO_LOAD) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = make_cd((double)m, (double)c);
      } else {
#pragma unroll
        for (int m = NPF; m < PTS; ++m) v[m] = src[zs * TZ * m];
        if constexpr (PF) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (and loads) landed
#pragma unroll
          for (int m = 0; m < NPF; ++m) {  // the DMA is lane-linear
            const int lane = launder(c0);
            v[m] = fromv(*reinterpret_cast<const dv2*>(lds + (wv * NPF + m) * 128 + 2 * lane));
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!kWaveTwr) {
        const cd w = tw_y(u, c);
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = cmul(v[m], w);
      }
    }
    {
      // 8-point DIF over y2 (map B lane bits 3, 1, 0), branch-free, between the z FFT's exchange and
      // its second stage; lane y2 ends with k2 = brev3(y2)
      const auto y2_dif = [&](cd* w_) {
        if constexpr (!(PROBE & WPR_NO_Y2)) {
          const int c = launder(c0);
          const int y2 = y2_b(c);
          const double s4 = y2 & 4 ? -1.0 : 1.0, s2 = y2 & 2 ? -1.0 : 1.0, s1 = y2 & 1 ? -1.0 : 1.0;
          const bool mi = (y2 & 3) == 3;
          const cd w8 = y2 & 4 ? tw_l[(WNX / 8) * (y2 & 3)] : make_cd(1.0, 0.0);
#pragma unroll
          for (int m = 0; m < PTS; ++m) {
            const cd p = lane_xor8(w_[m]);
            w_[m] = cmul(make_cd(fma(s4, w_[m].x, p.x), fma(s4, w_[m].y, p.y)), w8);
          }
#pragma unroll
          for (int m = 0; m < PTS; ++m) {
            const cd p = dpp_c<DPP_XOR2>(w_[m]);
            cd t = make_cd(fma(s2, w_[m].x, p.x), fma(s2, w_[m].y, p.y));
            t = mi ? mul_mi(t) : t;
            const cd r = dpp_c<DPP_XOR1>(t);
            w_[m] = make_cd(fma(s1, t.x, r.x), fma(s1, t.y, r.y));
          }
        }
      };
      const int c = launder(c0), tz = launder(tz0);
      // PF: not the first exchange of the kernel -- other waves may still read their prefetched slots
      fft_stages_perm<WNX, PTS, wr0_of(WNX, PTS), T, F>(v, lds, tw_l, lab_a(c), lab_b(c), tz, !PF, y2_dif);  // map B; kz = tz + TZ m
    }
    if constexpr (PROBE & WPR_NO_SOLVE) {
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
    } else {
      const int c = launder(c0), tz = launder(tz0);
      const int xt = u % NXT, k1 = u / NXT;
      const int y2 = y2_b(c), xl = (c >> 2) & 1;
      const int k2 = ((y2 & 1) << 2) | (y2 & 2) | (y2 >> 2);
      const double2 px = a.wave.tab[0][xt * XT + xl], py = a.wave.tab[1][k1 + WN1 * k2];
      const double iex = 1.0 / (1.0 + px.x), iey = 1.0 / (1.0 + py.x);
      const double wx = px.y * iex, wy = py.y * iey;
      const double dnf = 1.0 + px.x + py.x + c0sq * (px.y * wx + py.y * wy);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
      const int sl = ((c >> 4) & 1) | (((c >> 5) & 1) << 1);  // slot bits 0-1 now on lane bits 4-5
#pragma unroll
      for (int g = 0; g < PTS / 4; ++g) {
        const double2 pk = a.wave.tab[2][tz + TZ * (4 * g + sl)];
        const double ef = 1.0 + pk.x;
        const double D2 = fma(dnf + pk.x, ef, c0sq * pk.y * pk.y);
        const double inv = rcp_nr(ef * D2);
        const double id = ef * ef * inv, ief = D2 * inv;
        const double wz = pk.y * ief;
        cd* r = v + 4 * g;
        const double tx = fma(wx, r[1].x, fma(wy, r[2].x, wz * r[3].x));
        const double ty = fma(wx, r[1].y, fma(wy, r[2].y, wz * r[3].y));
        const cd x0 = make_cd(fma(c0sq, ty, r[0].x) * id, fma(-c0sq, tx, r[0].y) * id);
        r[1] = make_cd(fma(px.y, x0.y, r[1].x) * iex, fma(-px.y, x0.x, r[1].y) * iex);
        r[2] = make_cd(fma(py.y, x0.y, r[2].x) * iey, fma(-py.y, x0.x, r[2].y) * iey);
        r[3] = make_cd(fma(pk.y, x0.y, r[3].x) * ief, fma(-pk.y, x0.x, r[3].y) * ief);
        r[0] = x0;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = cconj(r[j]);
      }
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
    }
    if constexpr (!(PROBE & WPR_NO_Y2)) {
      // inverse (forward DFT on the conjugate): DIT from the bit-reversed order back to natural
      const int c = launder(c0);
      const int y2 = y2_b(c);
      const double s4 = y2 & 4 ? -1.0 : 1.0, s2 = y2 & 2 ? -1.0 : 1.0, s1 = y2 & 1 ? -1.0 : 1.0;
      const bool mi = (y2 & 3) == 3;
      const cd w8 = y2 & 4 ? tw_l[(WNX / 8) * (y2 & 3)] : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const cd r = dpp_c<DPP_XOR1>(v[m]);
        cd t = make_cd(fma(s1, v[m].x, r.x), fma(s1, v[m].y, r.y));
        t = mi ? mul_mi(t) : t;
        const cd p = dpp_c<DPP_XOR2>(t);
        v[m] = make_cd(fma(s2, t.x, p.x), fma(s2, t.y, p.y));
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const cd t = cmul(v[m], w8);
        const cd p = lane_xor8(t);
        v[m] = make_cd(fma(s4, t.x, p.x), fma(s4, t.y, p.y));
      }
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      const auto next = [&](cd*) {  // right after the exchange's last read: the buffer is free
        if constexpr (PF) {
          lds_barrier();  // every wave has read the exchange buffer
          if (it + (int)gridDim.x < nunits)
            prefetch(XCD ? xcd_round_unit(it + (int)gridDim.x, gridDim.x, nunits) : it + (int)gridDim.x);
        }
      };
      fft_stages_perm<WNX, PTS, wr0_of(WNX, PTS), T, F>(v, lds, tw_l, lab_b(c), lab_a(c), tz, false, next);  // map A again
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      cd* dst = col_ptr(u, c, tz);
      const cd w = tw_y(u, c);
      if constexpr (PROBE & WPR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x * w.x + v[m].y;
        if (acc == 1.2345e300) dst[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else if constexpr (kWaveTwr) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) dst[zs * TZ * m] = cconj(v[m]);
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) dst[zs * TZ * m] = cconj(cmul(v[m], w));
      }
    }
    if constexpr (!PF) lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

// P2w at 8 points per thread (k_wtp_mid_ct3, r04, measured and not kept: 79.3 us with the prefetch
// against 63.9 for k_wtp_mid_ct2, parity green; tools/kexp only): the two lane maps of k_wtp_mid_ct2 with the
// z FFT as 2 x 8 x 8 over 16 z-groups of the 64 columns (1,024 threads, 16 waves), whole-complex
// exchanges (128 KiB, one workgroup per CU) -- the shape that won at 128^3 for the scalar P2 --
// and, with PF, the WHOLE next unit DMA'd into the exchange buffer after the inverse FFT's last
// exchange (the buffer holds exactly one unit), so a unit starts with no HBM load in its path.
template <int PROBE = 0, bool PF = false>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_wtp_mid_ct3(cd* data, WTPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int XT = 2, T = WNC * WN2 * XT;  // 64 columns, one per lane
  constexpr int PTS = 8, TZ = WNX / PTS;     // 16 z-groups, kz = tz + 16 m
  constexpr int NXT = WNX / XT;
  constexpr int F = F_LDS_SYNC;  // whole-complex exchanges
  __shared__ __attribute__((aligned(16))) double lds[2 * T * WNX];
  __shared__ cd tw_l[WNX];
  const int tid = threadIdx.x;
  for (int i = tid; i < WNX; i += T * TZ) tw_l[i] = a.tw[i];
  const int c0 = tid & (T - 1), tz0 = tid / T;
  const i64 zs = WPLANE;
  const double c0sq = a.wave.c0sq;
  const auto y2_b = [](int l) { return (l & 3) | ((l >> 1) & 4); };
  const auto lab_a = [](int l) { return l ^ ((l >> 4) & 2); };
  const auto lab_b = [&](int l) {
    const int xl = (l >> 2) & 1;
    return ((l >> 4) & 1) | ((((l >> 5) & 1) ^ xl) << 1) | (y2_b(l) << 2) | (xl << 5);
  };
  const auto col_ptr = [&](int u, int c, int tz) {
    const int xt = u % NXT, k1 = u / NXT;
    return data + (i64)(((c >> 2) & (WN2 - 1)) + WN2 * k1) * WW + (xt * XT + (c >> 5)) * WNC + (c & 3) + zs * tz;
  };
  const auto tw_y = [&](int u, int c) { return a.tw[(((c >> 2) & (WN2 - 1)) * (u / NXT)) & (WNX - 1)]; };
  constexpr int NPF = PF ? PTS : 0;  // every slot of the next unit comes from the LDS prefetch
  static_assert(!PF || (T * TZ / 64) * NPF * 128 <= 2 * T * WNX, "the prefetch fits the exchange buffer");
  const int wv = __builtin_amdgcn_readfirstlane(tid / 64);
  const auto prefetch = [&](int u) {  // this wave's slots of unit u -> LDS (lane-linear)
    const int c = launder(c0), tz = launder(tz0);
    const cd* src = col_ptr(u, c, tz);
#pragma unroll
    for (int m = 0; m < NPF; ++m)
      __builtin_amdgcn_global_load_lds((wglb_void_t*)(src + zs * TZ * m), (wlds_void_t*)(lds + (wv * NPF + m) * 128),
                                       16, 0, 0);
  };
  if constexpr (PF) {
    if ((int)blockIdx.x < nunits) prefetch(blockIdx.x);
  }
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    cd v[PTS];
    {
      const int c = launder(c0), tz = launder(tz0);
      if constexpr (PROBE & WPR_NO_LOAD) {
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = make_cd((double)m, (double)c);
      } else if constexpr (PF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA landed
#pragma unroll
        for (int m = 0; m < PTS; ++m) {
          const int lane = launder(c0);
          v[m] = fromv(*reinterpret_cast<const dv2*>(lds + (wv * NPF + m) * 128 + 2 * lane));
        }
      } else {
        const cd* src = col_ptr(u, c, tz);
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = src[zs * TZ * m];
        __builtin_amdgcn_sched_barrier(0);
      }
      const cd w = tw_y(u, c);
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cmul(v[m], w);
    }
    {
      // 8-point DIF over y2 (map B lane bits 3, 1, 0) right after the first exchange
      const auto y2_dif = [&](cd* w_) {
        if constexpr (!(PROBE & WPR_NO_Y2)) {
          const int c = launder(c0);
          const int y2 = y2_b(c);
          const double s4 = y2 & 4 ? -1.0 : 1.0, s2 = y2 & 2 ? -1.0 : 1.0, s1 = y2 & 1 ? -1.0 : 1.0;
          const bool mi = (y2 & 3) == 3;
          const cd w8 = y2 & 4 ? tw_l[(WNX / 8) * (y2 & 3)] : make_cd(1.0, 0.0);
#pragma unroll
          for (int m = 0; m < PTS; ++m) {
            const cd p = lane_xor8(w_[m]);
            w_[m] = cmul(make_cd(fma(s4, w_[m].x, p.x), fma(s4, w_[m].y, p.y)), w8);
          }
#pragma unroll
          for (int m = 0; m < PTS; ++m) {
            const cd p = dpp_c<DPP_XOR2>(w_[m]);
            cd t = make_cd(fma(s2, w_[m].x, p.x), fma(s2, w_[m].y, p.y));
            t = mi ? mul_mi(t) : t;
            const cd r = dpp_c<DPP_XOR1>(t);
            w_[m] = make_cd(fma(s1, t.x, r.x), fma(s1, t.y, r.y));
          }
        }
      };
      const int c = launder(c0), tz = launder(tz0);
      // PF: not the first exchange of the kernel -- other waves may still read their prefetched slots
      fft_stages_perm<WNX, PTS, wr0_of(WNX, PTS), T, F>(v, lds, tw_l, lab_a(c), lab_b(c), tz, !PF, y2_dif);  // kz = tz + TZ m
    }
    if constexpr (PROBE & WPR_NO_SOLVE) {
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
    } else {
      const int c = launder(c0), tz = launder(tz0);
      const int xt = u % NXT, k1 = u / NXT;
      const int y2 = y2_b(c), xl = (c >> 2) & 1;
      const int k2 = ((y2 & 1) << 2) | (y2 & 2) | (y2 >> 2);
      const double2 px = a.wave.tab[0][xt * XT + xl], py = a.wave.tab[1][k1 + WN1 * k2];
      const double iex = 1.0 / (1.0 + px.x), iey = 1.0 / (1.0 + py.x);
      const double wx = px.y * iex, wy = py.y * iey;
      const double dnf = 1.0 + px.x + py.x + c0sq * (px.y * wx + py.y * wy);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
      const int sl = ((c >> 4) & 1) | (((c >> 5) & 1) << 1);  // slot bits 0-1 now on lane bits 4-5
#pragma unroll
      for (int g = 0; g < PTS / 4; ++g) {
        const double2 pk = a.wave.tab[2][tz + TZ * (4 * g + sl)];
        const double ef = 1.0 + pk.x;
        const double D2 = fma(dnf + pk.x, ef, c0sq * pk.y * pk.y);
        const double inv = rcp_nr(ef * D2);
        const double id = ef * ef * inv, ief = D2 * inv;
        const double wz = pk.y * ief;
        cd* r = v + 4 * g;
        const double tx = fma(wx, r[1].x, fma(wy, r[2].x, wz * r[3].x));
        const double ty = fma(wx, r[1].y, fma(wy, r[2].y, wz * r[3].y));
        const cd x0 = make_cd(fma(c0sq, ty, r[0].x) * id, fma(-c0sq, tx, r[0].y) * id);
        r[1] = make_cd(fma(px.y, x0.y, r[1].x) * iex, fma(-px.y, x0.x, r[1].y) * iex);
        r[2] = make_cd(fma(py.y, x0.y, r[2].x) * iey, fma(-py.y, x0.x, r[2].y) * iey);
        r[3] = make_cd(fma(pk.y, x0.y, r[3].x) * ief, fma(-pk.y, x0.x, r[3].y) * ief);
        r[0] = x0;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = cconj(r[j]);
      }
#pragma unroll
      for (int k = 0; k < PTS; ++k)
        if ((k & 2) == 0) swap_c<5>(v[k], v[k + 2]);
#pragma unroll
      for (int k = 0; k < PTS; k += 2) swap_c<4>(v[k], v[k + 1]);
    }
    if constexpr (!(PROBE & WPR_NO_Y2)) {
      // inverse (forward DFT on the conjugate): DIT from the bit-reversed order back to natural
      const int c = launder(c0);
      const int y2 = y2_b(c);
      const double s4 = y2 & 4 ? -1.0 : 1.0, s2 = y2 & 2 ? -1.0 : 1.0, s1 = y2 & 1 ? -1.0 : 1.0;
      const bool mi = (y2 & 3) == 3;
      const cd w8 = y2 & 4 ? tw_l[(WNX / 8) * (y2 & 3)] : make_cd(1.0, 0.0);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const cd r = dpp_c<DPP_XOR1>(v[m]);
        cd t = make_cd(fma(s1, v[m].x, r.x), fma(s1, v[m].y, r.y));
        t = mi ? mul_mi(t) : t;
        const cd p = dpp_c<DPP_XOR2>(t);
        v[m] = make_cd(fma(s2, t.x, p.x), fma(s2, t.y, p.y));
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const cd t = cmul(v[m], w8);
        const cd p = lane_xor8(t);
        v[m] = make_cd(fma(s4, t.x, p.x), fma(s4, t.y, p.y));
      }
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      const auto next = [&](cd*) {  // right after the last exchange's reads: the buffer is free
        if constexpr (PF) {
          lds_barrier();  // every wave has read the exchange buffer
          if (u + (int)gridDim.x < nunits) prefetch(u + gridDim.x);
        }
      };
      fft_stages_perm<WNX, PTS, wr0_of(WNX, PTS), T, F>(v, lds, tw_l, lab_b(c), lab_a(c), tz, false, NoMid(), next);
    }
    {
      const int c = launder(c0), tz = launder(tz0);
      cd* dst = col_ptr(u, c, tz);
      const cd w = tw_y(u, c);
      if constexpr (PROBE & WPR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x * w.x + v[m].y;
        if (acc == 1.2345e300) dst[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) dst[zs * TZ * m] = cconj(cmul(v[m], w));
      }
    }
    if constexpr (!PF) lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

bool wave_three_pass_supported(const i64 n[3], int ncomp) {
  return ncomp == WNC && n[0] == WNX && n[1] == WNX && n[2] == WNX;
}

static int wcu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

// a launch that stamps its own dispatch while the stand-in KSP times the apply (g_stamp set by
// run_wave from g_apply_stamp, cfp_internal.h): the apply's device time without event packets
#define WTP_LAUNCH(K, G, B, S, ...)                                                                   \
  do {                                                                                                \
    if (g_stamp.start || g_stamp.stop)                                                                \
      hipExtLaunchKernelGGL(K, G, B, 0, S, g_stamp.start, g_stamp.stop, 0, __VA_ARGS__);              \
    else                                                                                              \
      hipLaunchKernelGGL(K, G, B, 0, S, __VA_ARGS__);                                                 \
  } while (0)

hipError_t launch_wave_three_pass(int stage, const cd* in, cd* out, const WTPArgs& a, hipStream_t s,
                                  unsigned* grid_out) {
  // persistent grids, two 512-thread workgroups per CU (70 / 64 KiB of LDS each)
  const int g = 2 * wcu_count();
  if (stage == 1) {
    const int units = (WNX / 2) * WN1;  // x tiles x k1
    // the LDS-DMA prefetch (global_load_lds_dwordx4) takes 16-byte aligned addresses
    // units in XCD order, each XCD on whole k1 row blocks (r05q, profiles/r05q_mid_xcd_ab.txt:
    // P2w 64.9-65.0 against 65.5-66.2 us; the whole apply within the noise); -DCFP_WAVE_MID_XCD=0: A/B
    const unsigned gm = units < g ? units : g;
    if (((uintptr_t)out & 15) == 0 && CFP_WAVE_MID_XCD && gm % 8 == 0)
      WTP_LAUNCH((k_wtp_mid_ct2<true, 0, true, true>), dim3(gm), dim3(512), s, out, a, units);
    else if (((uintptr_t)out & 15) == 0)
      WTP_LAUNCH((k_wtp_mid_ct2<true, 0, true>), dim3(units < g ? units : g), dim3(512), s, out, a, units);
    else
      WTP_LAUNCH((k_wtp_mid_ct2<true>), dim3(units < g ? units : g), dim3(512), s, out, a, units);
  } else {
    const int units = WNX * WN2;  // z-planes x y2
    // P1w out of place: non-temporal loads keep b out of the 256 MB Infinity Cache, which then
    // still holds much of P1w's output for P2w (the scalar 3-sweep's policy, cfp_three_pass.hip)
    const dim3 gg(units < g ? units : g);
    // units in XCD order (CFP_ROWS_XCD) when the grid is a multiple of 8 workgroups
    const bool xo = CFP_ROWS_XCD != 0 && gg.x % 8 == 0;
    if (stage == 0 && in != out && xo)
      WTP_LAUNCH((k_wtp_rows<false, F_NT_LD, true>), gg, dim3(512), s, in, out, a, units);
    else if (stage == 0 && in != out)
      WTP_LAUNCH((k_wtp_rows<false, F_NT_LD>), gg, dim3(512), s, in, out, a, units);
    else if (stage == 0)
      WTP_LAUNCH((k_wtp_rows<false, 0>), gg, dim3(512), s, in, out, a, units);
    else if (a.post_nv > 0) {  // P3w with the dots
      if (a.post_nv > 4 || !a.post_partial || gg.x > 1024) return hipErrorInvalidValue;
      if (xo)
        WTP_LAUNCH((k_wtp_rows<true, F_NT_ST, true, 4>), gg, dim3(512), s, in, out, a, units);
      else
        WTP_LAUNCH((k_wtp_rows<true, F_NT_ST, false, 4>), gg, dim3(512), s, in, out, a, units);
    } else if (xo)
      WTP_LAUNCH((k_wtp_rows<true, F_NT_ST, true>), gg, dim3(512), s, in, out, a, units);
    else
      WTP_LAUNCH((k_wtp_rows<true, F_NT_ST>), gg, dim3(512), s, in, out, a, units);
    if (grid_out) *grid_out = gg.x;
  }
  return hipGetLastError();
}

}  // namespace cfp
