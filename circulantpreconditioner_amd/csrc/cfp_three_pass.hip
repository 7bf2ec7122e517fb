// cfp_three_pass.hip -- the 3-sweep apply for 256^3 grids (PCApply in 96 N bytes instead of
// the 5-pass schedule's 160 N).
//
// The y transform is split four-step (Cooley-Tukey, ny = N1 * N2, N1 = 64 or 32): with
// y = y2 + N2 y1 and k = k1 + N1 k2,
//   X[k1 + N1 k2] = sum_{y2} W_N2^{y2 k2} W_256^{y2 k1} sum_{y1} W_N1^{y1 k1} x[y2 + N2 y1].
// The inner N1-point DFT rides with the x transform, the outer N2-point DFT with the z
// transform, and every intermediate stays in the slot it was read from (y1 <-> k1, y2 <-> k2):
//
//   P1  k_tp_rows<fwd>: one z-plane, rows y2 + N2 y1 (N1 rows, N1 x 4 KB): N1-point DFT down
//       the rows (column mode, lanes = x), LDS transpose, 256-point DFT along each row
//   P2  k_tp_mid_sw (default) / k_tp_mid: T/N2 x-columns x N2 rows y2 + N2 k1 x 256 z: twiddle
//       W_256^{y2 k1}, N2-point DFT across lanes (k_tp_mid_sw: radix-2 stages on permlane
//       register transposes; k_tp_mid: DPP lane permutations; frequencies left bit-reversed),
//       256-point z DFT, divide by the separable symbol at (kx, k1 + N1 k2, kz), then the same
//       transforms on the conjugate (inverse)
//   P3  k_tp_rows<inv>: P1 on the conjugate, x 1/N
//
// P1/P3 workgroups are N1 x 16 threads x 16 points with a split-LDS exchange buffer of
// N1 x 2.1 KB: one per CU at N1 = 64, two at N1 = 32.  P2 holds T columns (T = 64: one
// 1024-thread workgroup per CU; T = 32: two of 512); its global runs are T/N2 x 16 bytes.
//
#include "cfp_fft_device.h"
#include "cfp_lane.h"
#include "cfp_three_pass.h"

#include <hip/hip_ext.h>

#ifndef CFP_REAL_MID_XCD
#define CFP_REAL_MID_XCD 1
#endif

// a launch that stamps its own dispatch while per-launch profiling is on (cfp_internal.h)
#define TP_LAUNCH(K, G, B, S, ...)                                                                    \
  do {                                                                                                \
    if (g_stamp.start || g_stamp.stop)                                                                \
      hipExtLaunchKernelGGL(K, G, B, 0, S, g_stamp.start, g_stamp.stop, 0, __VA_ARGS__);              \
    else                                                                                              \
      hipLaunchKernelGGL(K, G, B, 0, S, __VA_ARGS__);                                                 \
  } while (0)

namespace cfp {

namespace {

// Radix-2 butterflies across lanes.  The DIF forms take points in natural lane order and
// leave the frequencies bit-reversed; the DIT forms are the forward transform from that order
// back to natural order (used inside the conjugate trick for the inverse).
// 4 points over an aligned quad: lane q holds point q -> frequency brev2(q)
__device__ __forceinline__ cd dft4_dif(cd v, int q) {
  const cd p = dpp_c<DPP_XOR2>(v);
  cd t = (q & 2) ? csub(p, v) : cadd(v, p);
  if (q == 3) t = mul_mi(t);
  const cd r = dpp_c<DPP_XOR1>(t);
  return (q & 1) ? csub(r, t) : cadd(t, r);
}
// lane q holds frequency brev2(q) -> point q
__device__ __forceinline__ cd dft4_dit(cd v, int q) {
  const cd r = dpp_c<DPP_XOR1>(v);
  cd u = (q & 1) ? csub(r, v) : cadd(v, r);
  if (q == 3) u = mul_mi(u);
  const cd p = dpp_c<DPP_XOR2>(u);
  return (q & 2) ? csub(p, u) : cadd(u, p);
}
// The 8-point DFT over 8 aligned lanes (N2 = 8) is a lane-xor-4 radix-2 stage (twiddle
// W_8^(j & 3) on the upper half) followed by dft4_dif, and dft4_dit followed by the mirrored
// stage for the inverse; k_tp_mid runs each stage as its own sweep over the 16 slots, which
// keeps the kernel out of scratch.  Lane j ends up holding frequency brev3(j).
template <int N2>
__device__ __forceinline__ int brev(int j) {
  if constexpr (N2 == 16) return ((j & 1) << 3) | ((j & 2) << 1) | ((j & 4) >> 1) | (j >> 3);
  return N2 == 4 ? ((j & 1) << 1) | (j >> 1) : ((j & 1) << 2) | (j & 2) | (j >> 2);
}
// XCD-aware unit order of a persistent grid of G workgroups (G % 8 == 0, whole rounds): the
// workgroups of one XCD (blockIdx % 8, round-robin dispatch) take G / 8 consecutive units of a
// round, so units that share 128-byte lines run under one L2
__device__ __forceinline__ int xcd_unit(int it, int G) {
  const int b = it % G;
  return it - b + (b & 7) * (G >> 3) + (b >> 3);
}

// a byte load with the sweep's load policy (the fused stencil's row classes)
template <int FLAGS>
__device__ __forceinline__ unsigned char gload_u8(const unsigned char* p) {
  if constexpr ((FLAGS & F_NT_LD) != 0) return __builtin_nontemporal_load(p);
  return *p;
}

// first radix of an n-point FFT done as r0 x PTS x ... x PTS (n = r0 PTS^k, r0 <= PTS)
constexpr int r0_of(int n, int pts) { return n > pts ? r0_of(n / pts, pts) : n; }

}  // namespace

// P3's reads of the Krylov basis vectors for the fused dots (FUSE > 0): non-temporal, so the
// 256 MiB vectors do not push the next P1 output out of the Infinity Cache before P2 reads it
#ifndef CFP_POST_NT
#define CFP_POST_NT 1
#endif
constexpr int kPostLoadFlags = CFP_POST_NT ? F_NT_LD : 0;

// PROBE != 0 only in tools/kexp (tp_probe.hip, p2_512.hip, rows_512.hip, built with
// CFP_KEXP): timing probes that drop a
// part of the work (output invalid).  The product library instantiates PROBE = 0 only.
enum { PR_NO_Y2 = 1, PR_NO_ZMATH = 2, PR_NO_XCHG = 4, PR_NO_LOAD = 8, PR_NO_STORE = 16,
       PR_PRIO = 32 /* experiment, full work: s_setprio 1 for the second half of the waves */,
       PR_ZMAJOR = 64 /* experiment, full work (k_tp_rows): units in z-major order (the units of one
                         round share y2 and differ in z) */ };

// Persistent: a workgroup walks units blockIdx.x, + gridDim.x, ...  Prefetching the next unit
// into VGPRs across LDS-only barriers was tried and lost: at 1024 threads the extra registers
// spill (profiles/r01_schedule_sweep.txt); at 128^3 with 8 points per thread it fits (104
// VGPRs) and still lost, P1 20.7 -> 23.3 us with one workgroup per CU walking two units
// (profiles/r03m_128_three_sweep.md).  PTS points per thread (16 or 8); XS = the LDS exchanges
// split into real and imaginary halves (half the footprint, twice the barriers).
//
// LP (lane pair, N1 = 2 PTS): the two threads of a column x are lanes L and L + 32 of one wave
// (x = lane % 32 + 32 wave), so phase A's 32-point DFT is a 16-point DFT per lane (even / odd
// y1), the twiddle W_32^k on the odd lane, and a radix-2 across lane bit 5 on permlane32 swaps:
// no LDS exchange and no barrier pair in phase A.  Slot m then holds k1 = m % 8 + 8 ty + 16 (m / 8).
//
// BLK (blocked intermediate layout, r04): the N2 rows y2 + N2 k1 of one k1 (contiguous in every
// layout) hold [x / BLK][y2][x % BLK] instead of [y2][x], so a P2 unit of BLK x times N2 y2
// columns is one run of N2 BLK 16 bytes per z (1 KiB at BLK = 8); P1's stores and P3's loads
// become BLK x 16 B runs instead.  Only the intermediate between the sweeps changes; b and x
// stay natural.  BLK = 0: natural.  At 512^3 (N2 = 16) blocks of BLK = 2 x: 32-byte pieces for
// P1 / P3, 512-byte runs for P2's 2 x times 16 y2 tile.
// XCD: units in xcd_unit order (the host launches whole rounds), so the N2 units of one z-plane,
// whose blocked pieces share 128-byte lines, run under one L2.
//
// FUSE (r06, the stand-in GMRES's Krylov step; one GPU, natural layout): P1 (!INV) with FUSE = 1
// loads y = A b, A an x-row-local stencil (TPArgs pre_*): the neighbours b[i -+ 1] of a point are
// the same rows' lines, so the extra loads hit the caches and the sweep still reads b once from
// HBM.  P3 (INV) with FUSE = NP > 0 accumulates post_v[j]^H x over its stored points (j <
// a.post_nv <= NP; a NULL vector is x itself) across all its units and writes one partial per
// workgroup and value: the VecMDot that follows a PCApply in classical Gram-Schmidt, without the
// separate sweep that re-reads x.
template <bool INV, int FLAGS, int N1, int TN, int PTS = 16, bool XS = true, bool LP = false, int BLK = 0,
          bool XCD = false, int PROBE = 0, int FUSE = 0>
__global__ void __launch_bounds__(N1 * (TN / PTS)) __attribute__((amdgpu_waves_per_eu(4)))
k_tp_rows(const cd* in, cd* out, TPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int N2 = TN / N1, TR = TN / PTS, NT = N1 * TR, TY = N1 / PTS;
  constexpr bool PRE = !INV && FUSE == 1, POST = INV && FUSE > 0;
  constexpr int NP = POST ? FUSE : 1;
  static_assert(!POST || NP <= TP_POST_MAX, "post dots: at most TP_POST_MAX vectors");
  static_assert(FUSE == 0 || (BLK == 0 && PROBE == 0), "fused work: natural layout, product kernels");
  constexpr bool BL = BLK > 0;
  constexpr int BX = BL ? BLK : 1, BW = N2 * BX;  // x per block column, values per block column
  static_assert(!LP || (TY == 2 && TN % 32 == 0), "lane pairs: two threads per column, 32 columns per wave");
  static_assert(!BL || (TR % BX == 0 && ((N2 == 8 && (BX == 4 || BX == 8)) || (N2 == 16 && (BX == 2 || BX == 8)))),
                "blocked layout: 4 or 8 x times 8 y2, or 2 or 8 x times 16 y2");
  constexpr int RS = TN + TN / 16;  // padded row stride of the row-mode LDS layout
  constexpr int F = FLAGS | (XS ? F_SPLIT_LDS : 0) | F_LDS_SYNC;
  // F_WAVE_LDS in FLAGS: phase C's row-FFT exchanges wave-local (a row's TR threads are
  // consecutive lanes of one wave and its LDS row is theirs alone); phase A (columns spread over
  // waves) and the transposes keep workgroup barriers
  constexpr int FA = F & ~F_WAVE_LDS;
  static_assert(!(FLAGS & F_WAVE_LDS) || 64 % TR == 0, "wave-local rows: whole rows per wave");
  __shared__ __attribute__((aligned(16))) double lds[N1 * RS * (XS ? 1 : 2)];  // both layouts fit
  __shared__ cd tw_l[N1];  // W_N1 for phase A; phase C reads W_256 from global memory (L2 hits),
                           // which keeps it out of scratch (20 B/lane with the table in LDS)
  // PRE: the stencil's classes as dense 3-slot rows (x - 1, x, x + 1) and their slot masks
  __shared__ cd pre_tab_l[PRE ? 3 * TP_PRE_MAX_CLS : 1];
  __shared__ unsigned pre_mk_l[PRE ? TP_PRE_MAX_CLS + 1 : 1];  // [ncls]: slot masks, [MAX]: their union
  __shared__ const unsigned char* pre_cls_l[1];
  __shared__ cd pre_edge_l[PRE ? NT : 1];  // PRE: per wave, the edge neighbours its lanes loaded
  // POST: per wave and value, the running sum of its lanes' dot contributions
  __shared__ double post_l[POST ? 2 * NP * (NT / 64) : 1];
  __shared__ const cd* post_ptr_l[POST ? NP : 1];
  __shared__ int post_n_l[2];  // post_nv, post_self
  const int tid = threadIdx.x;
  if constexpr (POST) {
    for (int i = tid; i < 2 * NP * (NT / 64); i += NT) post_l[i] = 0.0;
    if (tid < NP) post_ptr_l[tid] = a.post_v[tid];
    if (tid == 0) {
      post_n_l[0] = a.post_nv;
      post_n_l[1] = a.post_self;
    }
  }
  for (int i = tid; i < N1; i += NT) tw_l[i] = a.tw[N2 * i];
  if constexpr (PRE) {
    for (int c = tid; c < a.pre_ncls; c += NT) {
      const unsigned mk = a.pre_mask[c];
      unsigned dense = 0;
      pre_tab_l[3 * c] = pre_tab_l[3 * c + 1] = pre_tab_l[3 * c + 2] = make_cd(0.0, 0.0);
      for (int k = 0; k < a.pre_nd; ++k)
        if ((mk >> k) & 1u) {
          const int slot = a.pre_off[k] + 1;
          pre_tab_l[3 * c + slot] = a.pre_tab[c * a.pre_nd + k];
          dense |= 1u << slot;
        }
      pre_mk_l[c] = dense;
    }
    if (tid == 0) {
      unsigned all = 0;
      for (int k = 0; k < a.pre_nd; ++k) all |= 1u << (a.pre_off[k] + 1);
      pre_mk_l[TP_PRE_MAX_CLS] = all | (a.pre_cls_x ? 8u : 0u);  // bit 3: classes by x alone
      pre_cls_l[0] = a.pre_cls_x ? a.pre_cls_x : a.pre_cls;
    }
  }
  if constexpr (LP || PRE || POST) __syncthreads();  // phase A reads tw_l (and the stencil) before any barrier
  // phase A: column x, thread ty of TY
  const int x0 = LP ? (tid & 31) + 32 * (tid >> 6) : tid % TN, ty0 = LP ? (tid >> 5) & 1 : tid / TN;
  const int r0 = tid / TR, tx0 = tid % TR;  // phase C: row r, thread tx of TR
  // fresh (laundered) index copies at every use, as in k_tp_mid: nothing but the points
  // stays live across an FFT
  const auto idx = [](int i) {
    asm volatile("" : "+v"(i));
    return i;
  };
  // rows of the chunked side (P1 output, P3 input): one GPU: nyl = TN, one chunk = natural
  const int lnyl = a.lnyl ? a.lnyl : ilog2(TN);
  const int nyl = 1 << lnyl;
  const auto crow = [&](int z, int y) -> i64 {
    return (i64)(y >> lnyl) * a.chunk + ((i64)z << lnyl) * TN + (i64)(y & (nyl - 1)) * TN;
  };
  // unit u = (z, y2): rows y2 + N2 y1 of (local) plane z; thread (column x, ty) loads rows
  // y2 + N2 (ty + TY m)
  const auto load = [&](int u, cd* v) {
    const int x = idx(x0), ty = idx(ty0);
    if constexpr ((PROBE & PR_NO_LOAD) != 0) {
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = make_cd(x + m, ty + u);
      return;
    }
    if (INV) {  // chunked rows: per-thread part + uniform part (nyl >= N2 TY)
      const cd* const src = BL ? in + crow(u / N2, N2 * ty) + (u % N2) * BX + (x / BX) * BW + x % BX
                               : in + crow(u / N2, u % N2 + N2 * ty) + x;
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(src + crow(0, N2 * TY * m));
    } else if constexpr (PRE) {
      // y = A b on the unit's rows.  With lane pairs (LP) lanes L and L + 1 of a wave hold x and
      // x + 1 of one row for L % 32 < 31, so a point's x-neighbours come from its neighbour lanes
      // (DPP wave_shr / wave_shl).  The neighbours across a wave's 32-column edge are loaded with
      // b, one per lane -- lane (ty, j < 16) the x - 1 edge of point j, (ty, 16 + j) the x + 1
      // edge -- and handed to the edge lanes through the wave's LDS slots: one memory round trip
      // per unit, as the plain load.  A neighbour outside the row is never used (its slot is
      // absent from the row's class), so its address is clamped into the row.
      static_assert(LP, "the fused stencil relies on the lane-pair layout");
      const i64 p0 = (i64)(u / N2) * TN * TN + (i64)TN * (u % N2 + N2 * ty);  // row of point 0
      const i64 i0 = p0 + x;
      const int l32 = (int)(threadIdx.x & 31), wv = (int)(threadIdx.x >> 6);
      // the slots any class uses, and the class array, from LDS at each use (kernel-argument
      // values would sit in SGPRs across the FFTs)
      const unsigned slots = ((volatile unsigned*)pre_mk_l)[TP_PRE_MAX_CLS];
      const bool hm = (slots & 1u) != 0, hp = (slots & 4u) != 0;
      const unsigned char* const cls = ((const unsigned char* const volatile*)pre_cls_l)[0];
      // classes by x alone (bit 3): one byte per thread (its column x), else one per point.
      // Every load here is non-temporal like b's: the edge and class lines must not stay in the
      // caches in place of this sweep's output, which P2 reads next.
      const bool by_x = (slots & 8u) != 0;
      int cl[PTS];
      const int clx = by_x ? (int)gload_u8<FLAGS>(cls + x) : 0;
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const i64 i = i0 + (i64)TN * N2 * TY * m;
        v[m] = gload<FLAGS>(in + i);
        cl[m] = by_x ? clx : (int)gload_u8<FLAGS>(cls + i);
      }
      cd edge = make_cd(0.0, 0.0);
      {
        const bool left = l32 < 16;
        int xe = left ? x - l32 - 1 : x - l32 + 32;
        xe = xe < 0 ? 0 : (xe > TN - 1 ? TN - 1 : xe);
        if ((left && hm) || (!left && hp)) edge = gload<FLAGS>(in + p0 + (i64)TN * N2 * TY * (l32 & 15) + xe);
      }
      __builtin_amdgcn_sched_barrier(0);
      cd* const el = pre_edge_l + 64 * wv;
      el[threadIdx.x & 63] = edge;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes are done
      __builtin_amdgcn_wave_barrier();
      // an absent diagonal has a zero coefficient in the dense table: fma(0, b, acc) = acc, so the
      // sum is the same as k_dia_spmv's, which skips it (finite b)
      const auto coefs = [&](int c, cd* t) {
        t[0] = pre_tab_l[3 * c];
        t[1] = pre_tab_l[3 * c + 1];
        t[2] = pre_tab_l[3 * c + 2];
      };
      cd tx[3];
      if (by_x) coefs(clx, tx);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        cd t[3];
        if (by_x) {
          t[0] = tx[0], t[1] = tx[1], t[2] = tx[2];
        } else {
          coefs(cl[m], t);
        }
        // the same fma sequence, in the same diagonal order, as k_dia_spmv: bit-identical to
        // MatMult on the row-class form
        double ax = 0.0, ay = 0.0;
        const auto acc = [&](cd q, cd b) {
          ax = fma(q.x, b.x, fma(-q.y, b.y, ax));
          ay = fma(q.x, b.y, fma(q.y, b.x, ay));
        };
        if (hm) {
          cd bm = dpp_c<DPP_WAVE_SHR1>(v[m]);
          if (l32 == 0) bm = el[32 * ty + m];
          acc(t[0], bm);
        }
        acc(t[1], v[m]);
        if (hp) {
          cd bp = dpp_c<DPP_WAVE_SHL1>(v[m]);
          if (l32 == 31) bp = el[32 * ty + 16 + m];
          acc(t[2], bp);
        }
        v[m] = make_cd(ax, ay);
      }
    } else {
      const cd* const src = in + (i64)(u / N2) * TN * TN + x + (i64)TN * (u % N2 + N2 * ty);  // + uniform
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(src + (i64)TN * N2 * TY * m);
    }
    // all loads go out before the first butterfly: with runtime strides the scheduler
    // otherwise starts the DFT after 9 of them and issues the rest a memory latency later
    // (P3 100 -> 93 us at 256^3)
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int it = blockIdx.x; it < nunits; it += gridDim.x) {
    int u = XCD ? xcd_unit(it, gridDim.x) : it;
    if constexpr ((PROBE & PR_ZMAJOR) != 0) u = (u % (nunits / N2)) * N2 + u / (nunits / N2);
    cd v[PTS];
    load(u, v);
    if (INV) {
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
    }
    const auto k1_of = [](int m, int ty) {
      return LP ? (m & (PTS / 2 - 1)) + (PTS / 2) * ty + PTS * (m / (PTS / 2)) : ty + TY * m;
    };
    if constexpr ((PROBE & PR_NO_ZMATH) != 0) {
    } else if constexpr (LP) {
      // phase A on lane pairs: E / O = the 16-point DFTs of the even / odd y1 (lanes ty = 0 / 1)
      dft_reg<PTS>(v);
      {
        const int ty = idx(ty0);
#pragma unroll
        for (int k = 1; k < PTS; ++k) v[k] = cmul(v[k], tw_l[k * ty]);  // W_32^k on the odd lane
      }
      // lane ty = 0 takes (E[k], W^k O[k]), lane ty = 1 (E[k+8], W^(k+8) O[k+8]) -> X[k], X[k+16]
#pragma unroll
      for (int k = 0; k < PTS / 2; ++k) swap_c<5>(v[k], v[k + PTS / 2]);
#pragma unroll
      for (int k = 0; k < PTS / 2; ++k) {
        const cd p = v[k], q = v[k + PTS / 2];
        v[k] = cadd(p, q);
        v[k + PTS / 2] = csub(p, q);
      }
    } else {
      // phase A: N1-point DFT over y1 for every x (column mode, TN columns x TY threads)
      const int x = idx(x0), ty = idx(ty0);
      fft_stages<N1, PTS, r0_of(N1, PTS), false, TN, FA>(v, lds, tw_l, x, ty, true);  // v[m]: k1 = ty + TY m
      lds_barrier();  // phase A's last LDS reads are done
    }
    // phase B: transpose to rows k1, thread (row r, tx) gets x = tx + TR m
    if constexpr (!(PROBE & PR_NO_XCHG)) {
      const int x = idx(x0), ty = idx(ty0), r = idx(r0), tx = idx(tx0);
      if constexpr (XS) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int m = 0; m < PTS; ++m) lds[k1_of(m, ty) * RS + x + (x >> 4)] = half ? v[m].y : v[m].x;
          lds_barrier();
#pragma unroll
          for (int m = 0; m < PTS; ++m) {
            const int xx = tx + TR * m;
            const double val = lds[r * RS + xx + (xx >> 4)];
            if (half) v[m].y = val; else v[m].x = val;
          }
          lds_barrier();
        }
      } else {
        cd* const lc = reinterpret_cast<cd*>(lds);
#pragma unroll
        for (int m = 0; m < PTS; ++m) lc[k1_of(m, ty) * RS + x + (x >> 4)] = v[m];
        lds_barrier();
#pragma unroll
        for (int m = 0; m < PTS; ++m) {
          const int xx = tx + TR * m;
          v[m] = lc[r * RS + xx + (xx >> 4)];
        }
        lds_barrier();
      }
    }
    {
      // phase C: TN-point DFT along row r (row mode, N1 rows x TR threads)
      const int r = idx(r0), tx = idx(tx0);
      if constexpr (!(PROBE & PR_NO_ZMATH))
        fft_stages<TN, PTS, r0_of(TN, PTS), true, N1, F | F_TW_GLOBAL>(v, lds, a.tw, r, tx, true);  // v[m]: kx = tx + TR m
    }
    {
      const int r = idx(r0), tx = idx(tx0);
      const double sc = a.scale, sy = INV ? -sc : sc;
      if constexpr ((PROBE & PR_NO_STORE) != 0) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x * sc + v[m].y * sy;
        if (acc == 1.2345e300) out[tx] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else if (BL && !INV) {  // blocked: kx = tx + TR m at (kx / BX) 64 + y2 BX + kx % BX of row block r
        cd* dst = out + crow(u / N2, N2 * r) + (u % N2) * BX + (tx / BX) * BW + tx % BX;
#pragma unroll
        for (int m = 0; m < PTS; ++m) gstore<FLAGS>(dst + TR * N2 * m, make_cd(v[m].x * sc, v[m].y * sy));
      } else {
        const i64 e0 = (INV ? (i64)(u / N2) * TN * TN + (i64)TN * (u % N2 + N2 * r) : crow(u / N2, u % N2 + N2 * r)) + tx;
        cd* dst = out + e0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) {
          v[m] = make_cd(v[m].x * sc, v[m].y * sy);
          gstore<FLAGS>(dst + TR * m, v[m]);
        }
        if constexpr (POST) {
          // post_v[j]^H x over the unit's stored points (the other vectors read 4 points at a
          // time), reduced over the wave and added to the wave's slot in LDS: nothing stays live
          // across the next unit's FFTs
          const int lane = tid & 63, wv = tid >> 6;
          const int pnv = ((volatile int*)post_n_l)[0], pself = ((volatile int*)post_n_l)[1];
          constexpr int QB = 4;
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            if (j < pnv) {
              double sr = 0.0, si = 0.0;
              if ((pself >> j) & 1) {
#pragma unroll
                for (int m = 0; m < PTS; ++m) sr += v[m].x * v[m].x + v[m].y * v[m].y;
              } else {
                // the vector's address from LDS at each use (a kernel-argument pointer would be
                // held in SGPRs across the FFTs, which already use all of them)
                const cd* pv = ((const cd* volatile*)post_ptr_l)[j] + e0;
#pragma unroll
                for (int m0 = 0; m0 < PTS; m0 += QB) {
                  cd q[QB];
#pragma unroll
                  for (int m = 0; m < QB; ++m) q[m] = gload<kPostLoadFlags>(pv + TR * (m0 + m));
#pragma unroll
                  for (int m = 0; m < QB; ++m) {
                    const cd w = v[m0 + m];
                    sr += q[m].x * w.x + q[m].y * w.y;
                    si += q[m].x * w.y - q[m].y * w.x;
                  }
                }
              }
              sr = wave_sum_d(sr);
              si = wave_sum_d(si);
              if (lane == 0) {
                post_l[(2 * j) * (NT / 64) + wv] += sr;
                post_l[(2 * j + 1) * (NT / 64) + wv] += si;
              }
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
    if (tid < 2 * NP) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < NT / 64; ++q) s += post_l[tid * (NT / 64) + q];
      a.post_partial[(size_t)blockIdx.x * 16 + tid] = s;
    }
  }
}


// Persistent over units u = (x-tile, k1); T columns per unit = T/N2 x values times N2 y2.
// Barriers wait for LDS only, so one unit's stores drain while the next unit loads.
// N2 = 16 (512^3, r04): one more radix-2 lane stage (lane ^ 8, twiddle W_16^(y2 & 7)) in front of
// the 8-point one.  XCD: units in xcd_unit order (the host launches whole rounds).
// BLK: the blocked layout of k_tp_rows<.., BLK> (BLK = XT: one run of T values per z; 512^3 with
// BLK = 8: the unit's 16 32-byte pieces of a z lie in one contiguous 2 KiB block, shared by the
// four x tiles of the block, which run under one L2 in XCD order).
template <int FLAGS, int T, int N2, int TN, int PTS = 16, bool XS = true, int NX = TN, bool XCD = false,
          int BLK = 0, int PROBE = 0>
__global__ void __launch_bounds__(T * (TN / PTS)) __attribute__((amdgpu_waves_per_eu(4)))
k_tp_mid(cd* data, TPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  constexpr int N1 = TN / N2, TZ = TN / PTS, NT = T * TZ, XT = T / N2, NXT = NX / XT;
  constexpr int F = FLAGS | (XS ? F_SPLIT_LDS : 0) | F_LDS_SYNC;
  static_assert(N2 == 4 || N2 == 8 || N2 == 16, "the y2 DFT runs across 4, 8 or 16 lanes");
  static_assert(BLK == 0 || (BLK % XT == 0 && NX % BLK == 0), "blocks of whole x tiles");
  __shared__ __attribute__((aligned(16))) double lds[T * TN * (XS ? 1 : 2)];
  __shared__ cd tw_l[TN];
  const int tid = threadIdx.x;
  for (int i = tid; i < TN; i += NT) tw_l[i] = a.tw[i];
  const int c0 = tid & (T - 1), tz0 = tid / T;
  // NX: row length (TN; the real plan's half spectrum: TN / 2).  Slab plans (a.lnyl): this rank's
  // z-pencil block [TN z][nyl][NX] with the global k1 range [k1_off, k1_off + nyl / N2)
  const i64 zs = (i64)NX << (a.lnyl ? a.lnyl : ilog2(TN));
  // Everything but the 16 points is rebuilt from laundered copies of the thread indices where
  // it is used: 128 VGPRs hold the points plus one radix-16 stage's twiddles, and an address,
  // twiddle or index kept live across the FFTs (or hoisted out of the unit loop) spills.
  struct Col {
    cd* col;  // this thread's first point; slot m adds the uniform zs * TZ m
    int y2, xk;
    cd w, w8, w16;  // W_TN^{y2 k1}; W_8^(y2 & 3) (N2 >= 8); W_16^(y2 & 7) (N2 = 16)
  };
  const auto column = [&](int u) {
    int c = c0, tz = tz0;
    asm volatile("" : "+v"(c), "+v"(tz));
    Col q;
    const int xt = u % NXT, k1 = u / NXT;
    q.y2 = c & (N2 - 1);
    q.xk = xt * XT + c / N2;
    q.col = BLK ? data + (i64)NX * N2 * k1 + (q.xk / BLK) * (N2 * BLK) + q.y2 * BLK + q.xk % BLK + zs * tz
                : data + q.xk + (i64)NX * (q.y2 + N2 * k1) + zs * tz;
    q.w = a.tw[(q.y2 * (a.k1_off + k1)) & (TN - 1)];  // global k1
    q.w8 = a.tw[(TN / 8) * (q.y2 & 3)];
    if constexpr (N2 == 16) q.w16 = a.tw[(TN / 16) * (q.y2 & 7)];
    return q;
  };
  for (int it = blockIdx.x; it < nunits; it += gridDim.x) {
    const int u = XCD ? xcd_unit(it, gridDim.x) : it;
    cd v[PTS];
    {
      const Col q = column(u);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr (PROBE & PR_NO_LOAD) v[m] = make_cd(c0 + m, tz0 + u);
        else v[m] = gload<FLAGS>(q.col + zs * TZ * m);
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m) {  // the lane DFT in two sweeps over the slots: fewer live temporaries
        v[m] = cmul(v[m], q.w);
        if constexpr ((PROBE & PR_NO_Y2) != 0) continue;
        if constexpr (N2 == 16) {  // dft16_dif's first stage
          const cd p = lane_xor8(v[m]);
          v[m] = (q.y2 & 8) ? cmul(csub(p, v[m]), q.w16) : cadd(v[m], p);
        }
        if constexpr (N2 >= 8) {  // dft8_dif's first stage
          const cd p = lane_xor4(v[m]);
          v[m] = (q.y2 & 4) ? cmul(csub(p, v[m]), q.w8) : cadd(v[m], p);
        }
      }
#pragma unroll
      for (int m = 0; m < PTS; ++m)
        if constexpr (!(PROBE & PR_NO_Y2)) v[m] = dft4_dif(v[m], q.y2 & 3);  // the lane now holds k2
    }
    {
      int c = c0, tz = tz0;
      asm volatile("" : "+v"(c), "+v"(tz));
      if constexpr (!(PROBE & PR_NO_ZMATH))
        fft_stages<TN, PTS, r0_of(TN, PTS), false, T, F>(v, lds, tw_l, c, tz, true);  // kz = tz + TZ m
    }
    {
      int c = c0, tz = tz0;
      asm volatile("" : "+v"(c), "+v"(tz));
      const int k1 = a.k1_off + u / NXT, y2 = c & (N2 - 1);  // global k1
      const cd cs = a.colsym[(u % NXT) * XT + c / N2 + (i64)NX * (k1 + N1 * brev<N2>(y2))];
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const cd d = cadd(cadd(cs, a.axsym[tz + TZ * m]), make_cd(1.0, 0.0));
        v[m] = (PROBE & PR_NO_ZMATH) ? cconj(v[m]) : cconj(cdiv_sym(v[m], d));
      }
      if constexpr (!(PROBE & PR_NO_ZMATH)) fft_stages<TN, PTS, r0_of(TN, PTS), false, T, F>(v, lds, tw_l, c, tz, false);
    }
    {
      const Col q = column(u);
#pragma unroll
      for (int m = 0; m < PTS; ++m)
        if constexpr (!(PROBE & PR_NO_Y2)) v[m] = dft4_dit(v[m], q.y2 & 3);
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        if constexpr ((PROBE & PR_NO_Y2) != 0) {
          v[m] = cmul(v[m], q.w);
          continue;
        }
        if constexpr (N2 >= 8) {  // dft8_dit's last stage
          const cd u = (q.y2 & 4) ? cmul(v[m], q.w8) : v[m];
          const cd p = lane_xor4(u);
          v[m] = (q.y2 & 4) ? csub(p, u) : cadd(u, p);
        }
        if constexpr (N2 == 16) {  // dft16_dit's last stage
          const cd u = (q.y2 & 8) ? cmul(v[m], q.w16) : v[m];
          const cd p = lane_xor8(u);
          v[m] = (q.y2 & 8) ? csub(p, u) : cadd(u, p);
        }
        v[m] = cmul(v[m], q.w);
      }
      if constexpr (PROBE & PR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < PTS; ++m) acc += v[m].x + v[m].y;
        if (acc == 1.2345e300) q.col[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else {
#pragma unroll
        for (int m = 0; m < PTS; ++m) gstore<FLAGS>(q.col + zs * TZ * m, cconj(v[m]));
      }
    }
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

// ---------------------------------------------------------------------------------------------
// P2 with the y2 DFT on register transposes (k_tp_mid_sw).  A wave is one z-group tz and all
// 64 columns c = x + XT * y2 of the tile (XT = 64 / N2), so the y2 bits are the top lane bits:
// N2 = 8: y2 = lane bits 3..5; N2 = 4: lane bits 4..5.  A radix-2 stage over lane bit 5 / 4
// transposes a register pair with v_permlane32_swap / v_permlane16_swap (lane bit <-> register
// bit, 2 swaps per double) and then runs a plain butterfly on the pair: no per-lane selects, no
// duplicated butterfly halves.  Lane bit 3 (N2 = 8 only) has no swap instruction: DPP row_ror:8
// brings the partner's value, and one fma with a per-lane sign forms sum or difference.
//
// The y2 DFT commutes with the z DFT, so it runs between the z transform's first radix-16 stage
// (per lane, over the 16 slots) and the LDS exchange; the exchange writes each value from its
// transposed register straight to its (column, z) place, so the transposes are never undone.
// Register r at lane L then holds slot s = (r & 12) | L5 | 2 L4 and y2 position
// p = 4 r0 + 2 r1 + L3 (N2 = 8) or p = 2 r0 + r1 (N2 = 4).  Forward: DIF, natural order in,
// bit-reversed frequencies out (the symbol index follows, as in k_tp_mid).  Inverse: DIT from
// the bit-reversed order back to natural, same register map, so the second exchange lands in
// the load layout.
namespace {
// partner across lane bit 3 (row_ror:8 inside each 16-lane row)
__device__ __forceinline__ double ror8_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), 0x128, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x128, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// radix-2 over lane bit 3 without twiddle: bit clear -> own + partner, set -> partner - own
__device__ __forceinline__ cd bfly_l3(cd v, double sgn) {
  return make_cd(fma(sgn, v.x, ror8_d(v.x)), fma(sgn, v.y, ror8_d(v.y)));
}
}  // namespace

// DIF stage over register pairs (k, k + D) after a swap on lane bit B: a + b, (a - b) w
// (TW = false: no twiddle)
template <int B, int D, bool TW = true, int NR = 16>
__device__ __forceinline__ void dif_pairs(cd* v, cd w) {
#pragma unroll
  for (int k = 0; k < NR; ++k)
    if ((k & D) == 0) swap_c<B>(v[k], v[k + D]);
#pragma unroll
  for (int k = 0; k < NR; ++k)
    if ((k & D) == 0) {
      const cd a = v[k], b = v[k + D];
      v[k] = cadd(a, b);
      v[k + D] = TW ? cmul(csub(a, b), w) : csub(a, b);
    }
}

//
// PF (prefetch): the exchange buffer is idle from the second exchange's last read to the next
// unit's first exchange, which is exactly where the next unit's data is needed.  Right after
// the second exchange each wave DMAs slots 0..7 of its columns of unit u + gridDim.x into that
// buffer (global_load_lds_dwordx4: 1 KiB per wave-instruction, lane-linear), so those loads
// fly during stage B', the twiddle and the stores; the next unit then loads only slots 8..15
// from HBM and reads 0..7 back from LDS.  Barriers stay LDS-only (no vmcnt), so the DMA is not
// drained early.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
// NX: x extent (row length in points) of the grid P2 runs on: TN for the complex apply, TN / 2
// for the real-data plan's half spectrum (cfp_real.hip); y and z are TN long.
// BL: the blocked intermediate layout of k_tp_rows<.., BLK = XT>: a unit's T columns c = x + XT y2
// are the run at block column xt of row block k1, for every z (T 16 bytes).
//
// T = 32 (r04): 512 threads, two workgroups per CU that run their barrier phases independently.
// A wave then holds two z groups of the 32 columns: lane = x (bits 0-1) + tz parity (bit 2) +
// y2 (bits 3-5), so y2 keeps lane bits 3-5 and every y2 stage below (permlane swaps on bits 5 and
// 4, DPP on bit 3) is the T = 64 code; c (the column x + 4 y2) and tz index memory and LDS,
// `lane` the lane bits.
// XCD (r04): units in xcd_unit order (whole rounds), so x tiles that share 128-byte lines run
// under one L2 (T = 32 natural layout: 64-byte tiles).
template <int T, int N2, int TN, int PROBE = 0, bool PF = false, int NX = TN, int ST = 0, int LD = 0, bool BL = false,
          bool XCD = false, int TAG = 0>
__global__ void __launch_bounds__(T * (TN / 16)) __attribute__((amdgpu_waves_per_eu(4)))
k_tp_mid_sw(cd* data, TPArgs a, int nunits) {
#ifndef CFP_KEXP
  static_assert(PROBE == 0, "timing probes are built in tools/kexp only");
#endif
  static_assert(T == 64 || (T == 32 && N2 == 8), "a wave = the 64 columns of one z group, or 32 columns of two");
  static_assert(N2 == 4 || N2 == 8, "y2 = the top 2 or 3 lane bits");
  static_assert(TN == 256, "z = 16 x 16: radix-16 stage A in registers, one exchange, radix-16 stage B");
  constexpr int N1 = TN / N2, TZ = TN / 16, NT = T * TZ, XT = T / N2, NXT = NX / XT;
  constexpr int XB = ilog2(XT);  // lane bits of x
  static_assert(NX % XT == 0, "whole x tiles");
  static_assert(!BL || (NX == TN && N2 == 8), "blocked layout: complex grid, 8 x times 8 y2");
  __shared__ __attribute__((aligned(16))) double lds[T * TN];  // split exchange
  __shared__ cd tw_l[TN];
  const int tid = threadIdx.x;
  for (int i = tid; i < TN; i += NT) tw_l[i] = a.tw[i];
  __syncthreads();  // the y2 stages read tw_l before the first exchange barrier
  const int lane0 = tid & 63;
  const int c0 = T == 64 ? lane0 : (lane0 & 3) | ((lane0 >> 3) << 2);
  const int tz0 = T == 64 ? tid / 64 : 2 * (tid >> 6) + ((lane0 >> 2) & 1);
  // rows of this rank's block [TN z][nyl][NX] (one GPU: nyl = TN); unit u = (x tile, local k1)
  const i64 zs = (i64)NX << (a.lnyl ? a.lnyl : ilog2(TN));
  const auto idx = [](int i) {
    asm volatile("" : "+v"(i));
    return i;
  };
  // this lane's first point and the twiddle W_TN^{y2 k1} (natural layout: x = c % XT, y2 = c / XT)
  const auto col_ptr = [&](int u, int c, int tz) {
    const int xt = u % NXT, k1 = u / NXT;
    if constexpr (BL) return data + (i64)NX * N2 * k1 + xt * T + c + zs * tz;
    return data + xt * XT + (c & (XT - 1)) + (i64)NX * ((c >> XB) + N2 * k1) + zs * tz;
  };
  const auto tw_y = [&](int u, int c) { return tw_l[((c >> XB) * (a.k1_off + u / NXT)) & (TN - 1)]; };
  constexpr int NPF = PF ? 8 : 0;  // slots 0 .. NPF-1 come from the LDS prefetch (exchange buffer)
  const int wv = __builtin_amdgcn_readfirstlane(tid / 64);
  if constexpr ((PROBE & PR_PRIO) != 0) {
    if (wv >= NT / 128) __builtin_amdgcn_s_setprio(1);
  }
  const auto prefetch = [&](int u) {  // this wave's slots 0 .. NPF-1 of unit u -> LDS
    const int c = idx(c0), tz = idx(tz0);
    const cd* src = col_ptr(u, c, tz);
#pragma unroll
    for (int m = 0; m < NPF; ++m)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(src + zs * TZ * m), (lds_void_t*)(lds + (wv * NPF + m) * 128),
                                       16, 0, (LD & F_NT_LD) ? 2 : 0);
  };
  static_assert(!PF || (NT / 64) * NPF * 128 <= T * TN, "the prefetch fits the exchange buffer");
  if constexpr (PF) {
    if ((int)blockIdx.x < nunits) prefetch(XCD ? xcd_unit(blockIdx.x, gridDim.x) : (int)blockIdx.x);
  }
  // split exchange from the transposed registers (first radix-16 stage done) to the column
  // layout: v[t] = point tz + 16 t of column c
  const auto exchange_t = [&](cd* v, bool first) {
    if constexpr (PROBE & PR_NO_XCHG) return;
    const int c = idx(c0), tz = idx(tz0), lane = idx(lane0);
    const int l3 = N2 == 8 ? ((lane >> 3) & 1) : 0, l4 = (lane >> 4) & 1, l5 = (lane >> 5) & 1;
    const int wbase = (tz * 16 + l5 + 2 * l4) * T + (c & (XT - 1)) + XT * l3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!(first && h == 0)) lds_barrier();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = N2 == 8 ? 4 * (r & 1) + 2 * ((r >> 1) & 1) : 2 * (r & 1) + ((r >> 1) & 1);
        const int off = (r & 12) * T + XT * (N2 == 8 ? p & 6 : p);
        lds[wbase + off] = h ? v[r].y : v[r].x;
      }
      lds_barrier();
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const double d = lds[(tz + TZ * t) * T + c];
        if (h) v[t].y = d; else v[t].x = d;
      }
    }
  };
  // second radix-16 stage (Ns = 16): twiddles W_TN^{tz t}, then the in-register DFT
  const auto stage_b = [&](cd* v) {
    if constexpr (PROBE & PR_NO_ZMATH) return;
    const int tz = idx(tz0);
#pragma unroll
    for (int t = 1; t < 16; ++t) v[t] = cmul(v[t], tw_l[tz * t]);
    dft_reg<16>(v);
  };
  const auto lane_sign = [&]() {  // +1 where lane bit 3 is clear, -1 where set
    const int lane = idx(lane0);
    return (lane & 8) ? -1.0 : 1.0;
  };

  for (int it = blockIdx.x; it < nunits; it += gridDim.x) {
    const int u = XCD ? xcd_unit(it, gridDim.x) : it;
    cd v[16];
    if constexpr (PROBE & PR_NO_LOAD) {
      const int c = idx(c0), tz = idx(tz0);
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = make_cd(c + m, tz + u);
    } else {
      const int c = idx(c0), tz = idx(tz0);
      const cd* src = col_ptr(u, c, tz);
#pragma unroll
      for (int m = NPF; m < 16; ++m) v[m] = gload<LD>(src + zs * TZ * m);  // LD: load policy
      if constexpr (PF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (and loads) landed
#pragma unroll
        for (int m = 0; m < NPF; ++m) {  // the DMA is lane-linear
          const int lane = idx(lane0);
          v[m] = fromv(*reinterpret_cast<const dv2*>(lds + (wv * NPF + m) * 128 + 2 * lane));
        }
      }
    }
    {
      const int c = idx(c0);
      const cd w = tw_y(u, c);
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = cmul(v[m], w);
    }
    if constexpr (!(PROBE & PR_NO_ZMATH)) dft_reg<16>(v);  // z stage A (Ns = 1: no twiddles), per lane
    // y2 DFT, DIF: natural positions in, bit-reversed frequencies out
    if constexpr (PROBE & PR_NO_Y2) {
    } else if constexpr (N2 == 8) {
      {
        const int lane = idx(lane0);
        dif_pairs<5, 1>(v, tw_l[(TN / 8) * ((lane >> 3) & 3)]);  // W_8^{y2 & 3}
      }
      {
        const int lane = idx(lane0);
        dif_pairs<4, 2>(v, tw_l[(TN / 4) * ((lane >> 3) & 1)]);  // W_4^{y2 & 1}
      }
      const double s = lane_sign();
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = bfly_l3(v[r], s);
    } else {
      {
        const int lane = idx(lane0);
        dif_pairs<5, 1>(v, tw_l[(TN / 4) * ((lane >> 4) & 1)]);  // W_4^{y2 & 1}
      }
      dif_pairs<4, 2, false>(v, make_cd(1.0, 0.0));
    }
    exchange_t(v, !PF);  // PF: other waves may still be reading their prefetched slots
    stage_b(v);  // v[m]: kz = tz + 16 m; column c = x + XT p
    {
      const int c = idx(c0), tz = idx(tz0);
      const int k1 = a.k1_off + u / NXT, p = c >> XB;  // global k1
      const cd cs = a.colsym[(u % NXT) * XT + (c & (XT - 1)) + (i64)NX * (k1 + N1 * brev<N2>(p))];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const cd d = cadd(cadd(cs, a.axsym[tz + TZ * m]), make_cd(1.0, 0.0));
        v[m] = (PROBE & PR_NO_ZMATH) ? cconj(v[m]) : cconj(cdiv_sym(v[m], d));
      }
    }
    if constexpr (!(PROBE & PR_NO_ZMATH)) dft_reg<16>(v);  // inverse (on the conjugate): z stage A
    // y2 DFT, DIT: bit-reversed positions in, natural out
    if constexpr (PROBE & PR_NO_Y2) {
    } else if constexpr (N2 == 8) {
      {
        const double s = lane_sign();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = bfly_l3(v[r], s);
      }
      {
        const int lane = idx(lane0);
        const cd w = tw_l[(TN / 4) * ((lane >> 3) & 1)];  // W_4^{p & 1}, p bit 0 = lane bit 3
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if ((k & 2) == 0) swap_c<4>(v[k], v[k + 2]);
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if ((k & 2) == 0) {
            const cd x = v[k], y = cmul(v[k + 2], w);
            v[k] = cadd(x, y);
            v[k + 2] = csub(x, y);
          }
      }
      {
        // W_8^{p & 3}: p bit 0 = lane bit 3, p bit 1 = register bit 1 -> W_8^{l3} (x -i if r1)
        const int lane = idx(lane0);
        const cd w = tw_l[(TN / 8) * ((lane >> 3) & 1)];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if ((k & 1) == 0) swap_c<5>(v[k], v[k + 1]);
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if ((k & 1) == 0) {
            cd y = cmul(v[k + 1], w);
            if (k & 2) y = mul_mi(y);
            const cd x = v[k];
            v[k] = cadd(x, y);
            v[k + 1] = csub(x, y);
          }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((k & 2) == 0) swap_c<4>(v[k], v[k + 2]);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((k & 2) == 0) {
          const cd x = v[k], y = v[k + 2];
          v[k] = cadd(x, y);
          v[k + 2] = csub(x, y);
        }
      // W_4^{p & 1}, p bit 0 = register bit 1
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((k & 1) == 0) swap_c<5>(v[k], v[k + 1]);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((k & 1) == 0) {
          const cd y = (k & 2) ? mul_mi(v[k + 1]) : v[k + 1];
          const cd x = v[k];
          v[k] = cadd(x, y);
          v[k + 1] = csub(x, y);
        }
    }
    exchange_t(v, false);
    if constexpr (PF) {
      lds_barrier();  // every wave has read the exchange buffer
      if (it + (int)gridDim.x < nunits) prefetch(XCD ? xcd_unit(it + gridDim.x, gridDim.x) : it + (int)gridDim.x);
    }
    stage_b(v);  // natural layout again: column c = x + XT y2, slot m = z
    {
      const int c = idx(c0), tz = idx(tz0);
      const cd w = tw_y(u, c);
      cd* dst = col_ptr(u, c, tz);
      if constexpr (PROBE & PR_NO_STORE) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < 16; ++m) acc += v[m].x * w.x + v[m].y;
        if (acc == 1.2345e300) dst[0] = make_cd(acc, 0.0);  // keeps the work live, never true
      } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) gstore<ST>(dst + zs * TZ * m, cconj(cmul(v[m], w)));  // ST: store policy
      }
    }
    if constexpr (!PF) lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}


bool three_pass_supported(const i64 n[3]) {
  return n[0] == n[1] && n[1] == n[2] && (n[0] == 128 || n[0] == 256 || n[0] == 512);
}

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

// persistent grid: per_cu workgroups per CU, at most one per unit
static unsigned grid_of(int units, int per_cu) {
  const int g = per_cu * cu_count();
  return (unsigned)(units < g ? units : g);
}
// the same for the XCD-ordered kernels (xcd_unit), whose rounds must be whole and a multiple of
// 8 workgroups: the largest power of two <= grid_of (units is a power of two), 0 if below 8
static unsigned grid_xcd(int units, int per_cu) {
  unsigned g = grid_of(units, per_cu), p = 1;
  while (2 * p <= g) p *= 2;
  return p >= 8 && units % p == 0 ? p : 0;
}

// ---------------------------------------------------------------------------------------------
// Real-data 3-sweep (cfp_real.hip, row f4) at 256^3: the half spectrum H = M x 256 x 256
// (M = 128) takes the complex schedule's four-step split of y with the x transform replaced by
// r2c / c2r (the even/odd split of k_rx):
//   P1r k_tp_rows_r2c<false>: one z-plane's rows y2 + 8 y1 (32 real rows of 2 KiB): r2c along x
//       (128-point FFT in row mode, mirror bin from the partner lane), LDS transpose, 32-point y1
//       DFT per kx (column mode), store H in slot layout; the Nyquist bins X[128] of the unit's
//       32 rows take the same y1 DFT (one wave, a direct 32-point DFT from LDS) into Q's slots
//   P2  k_tp_mid_sw<.., NX = 128> on H (y2 + z + divide + inverse), then the Nyquist column's
//       y2 + z + divide + inverse on Q (k_tp_mid on 8 columns of one k1: 32 small workgroups)
//   P3r k_tp_rows_r2c<true>: y1 inverse (H in column mode, Q by one wave from LDS), transpose,
//       c2r merge with Q, inverse 128-point FFT, x 2/N
// P1r/P3r move 8 N + 8 N bytes, P2 16 N: 32 N per apply against ~80 N for r2c + 3 half-spectrum
// passes + c2r.  (Folding the Nyquist column into P2 as a 17th x tile was measured slower: 544
// units on 256 CUs take a third round, P2 70 -> 89 us.  Until r04 the column took its own
// 3-launch y / z plan between P2 and P3r: 18.4 us of the 199 us apply.)
// 8 points per thread (512 threads): the even/odd split needs every point and its mirror live
// at once, which at 16 points per thread spills.
// At 128^3 (r03, AUTO there too): M = 64, y = y2 + 4 y1 (N1 = 32, N2 = 4), 256 threads; P2 is
// the lane-DFT k_tp_mid on the 64-wide half spectrum (NX = 64).
// MF: policy of the accesses to b (P1r loads) and x (P3r stores), which nothing in the apply
// reads again (the complex P1 / P3 policy, kP1Flags / kP3Flags); H and Q stay plain.
// OCC: waves per SIMD asked of the compiler (4: two 512-thread workgroups per CU; 6: three)
// WC: whole-complex LDS exchanges (ds_*_b128, one barrier pair per exchange instead of two;
// 70 KiB at M = 128, two workgroups per CU) instead of real / imaginary halves
// WL: wave-local FFT exchanges.  A row's TPC threads are consecutive lanes of one wave, and in
// column mode a wave takes 16 whole columns (lane = 16 ty + column) instead of 64 columns of one
// ty: the row FFT's and the y1 DFT's exchanges (3 of the unit's 5; 12 of its 18 barriers with
// split exchanges) then wait for the wave's own LDS accesses only; the two transposes keep their
// workgroup barriers.  Column-mode LDS rows are M + 16 doubles apart (the four ty rows of a
// wave's store then fall on different bank halves).
template <bool INV, int M = 128, int N1 = 32, int N2 = 8, int NY = 256, int MF = 0, int OCC = 4, bool WC = false,
          bool WL = false>
__global__ void __launch_bounds__(N1 * (M / 8)) __attribute__((amdgpu_waves_per_eu(OCC)))
k_tp_rows_r2c(const double* in_r, cd* H, cd* Q, double* out_r, TPArgs a, int nunits) {
  constexpr int PTS = 8;
  constexpr int TPC = M / PTS;  // threads per row (row mode)
  constexpr int TY = N1 / PTS;  // 4 threads per column (column mode)
  constexpr int NT = N1 * TPC;
  constexpr int RS = M + M / 16;
  constexpr int TC = WL ? M + 16 : M;  // column-mode row stride of the y1 DFT's exchange
  static_assert(!WL || (64 % TPC == 0 && TY * 16 == 64 && M % 16 == 0), "wave-local: whole rows and 16 columns per wave");
  constexpr int F = (WC ? 0 : F_SPLIT_LDS) | F_LDS_SYNC;
  constexpr int FW = F | (WL ? F_WAVE_LDS : 0);  // the row FFT's and the y1 DFT's exchanges
  constexpr int LDS_D = (N1 * RS > N1 * TC ? N1 * RS : N1 * TC) * (WC ? 2 : 1);
  __shared__ __attribute__((aligned(16))) double lds[LDS_D];  // row layout; the column layout (N1 x TC) fits
  cd* const lc = reinterpret_cast<cd*>(lds);
  __shared__ cd tw_m[M];   // W_M (row FFT)
  __shared__ cd tw_1[N1];  // W_N1 (y1 DFT)
  __shared__ cd qy[N1];    // the unit's Nyquist bins over y1 (P1r: before its y1 DFT; P3r: after)
  const int tid = threadIdx.x;
  for (int i = tid; i < M; i += NT) tw_m[i] = a.tw[2 * i];
  for (int i = tid; i < N1; i += NT) tw_1[i] = a.tw[(2 * M / N1) * i];
  if constexpr (WL) __syncthreads();  // no workgroup barrier precedes the first wave-local FFT's twiddle reads
  const int r0 = tid / TPC, tpc0 = tid % TPC;  // row mode: row r (= y1), thread tpc
  // column mode: column kx, thread ty
  const int x0 = WL ? (tid >> 6) * 16 + (tid & 15) : tid % M, ty0 = WL ? (tid >> 4) & 3 : tid / M;
  const auto idx = [](int i) {
    asm volatile("" : "+v"(i));
    return i;
  };
  // row mode (row r, Z[k], k = tpc + TPC t) -> column mode (column kx, rows ty + TY m), with the
  // r2c even/odd split done on the way: each thread also reads its mirror bin Z[M - kx] of the
  // same rows from the transpose buffer (no cross-lane shuffles)
  const auto to_columns_r2c = [&](cd* v, int z, int y2) {
    const int r = idx(r0), tpc = idx(tpc0), x = idx(x0), ty = idx(ty0);
    const int xm = (M - x) & (M - 1);
    cd zm[PTS];
    if constexpr (WC) {
      lds_barrier();
#pragma unroll
      for (int t = 0; t < PTS; ++t) {
        const int k = tpc + TPC * t;
        lc[r * RS + k + (k >> 4)] = v[t];
      }
      lds_barrier();
#pragma unroll
      for (int m = 0; m < PTS; ++m) {
        const int row = (ty + TY * m) * RS;
        v[m] = lc[row + x + (x >> 4)];
        zm[m] = lc[row + xm + (xm >> 4)];
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        lds_barrier();
#pragma unroll
        for (int t = 0; t < PTS; ++t) {
          const int k = tpc + TPC * t;
          lds[r * RS + k + (k >> 4)] = h ? v[t].y : v[t].x;
        }
        lds_barrier();
#pragma unroll
        for (int m = 0; m < PTS; ++m) {
          const int row = (ty + TY * m) * RS;
          const double d = lds[row + x + (x >> 4)], dm = lds[row + xm + (xm >> 4)];
          if (h) { v[m].y = d; zm[m].y = dm; } else { v[m].x = d; zm[m].x = dm; }
        }
      }
    }
    lds_barrier();
    const cd w = a.tw[x];  // W_2M^kx
#pragma unroll
    for (int m = 0; m < PTS; ++m) {
      const cd e = make_cd(0.5 * (v[m].x + zm[m].x), 0.5 * (v[m].y - zm[m].y));
      const cd d = make_cd(v[m].x - zm[m].x, v[m].y + zm[m].y);  // Z[k] - conj Z[M-k]
      const cd o = make_cd(0.5 * d.y, -0.5 * d.x);                // d / 2i
      v[m] = cadd(e, cmul(w, o));
      if (x == 0) qy[ty + TY * m] = csub(e, o);  // Nyquist bin X[M] of row y1 = ty + TY m
    }
  };
  // column mode (column kx, rows y1 = ty + TY m, conjugated) -> row mode with the c2r merge: each
  // thread reads X[k] and its mirror X[M - k] of its row (X[M] = the Nyquist bin from Q)
  const auto to_rows_c2r = [&](cd* v, int z, int y2) {
    const int r = idx(r0), tpc = idx(tpc0), x = idx(x0), ty = idx(ty0);
    cd xm[PTS];
    if constexpr (WC) {
      lds_barrier();
#pragma unroll
      for (int m = 0; m < PTS; ++m) lc[(ty + TY * m) * RS + x + (x >> 4)] = cconj(v[m]);
      lds_barrier();
#pragma unroll
      for (int t = 0; t < PTS; ++t) {
        const int k = tpc + TPC * t, km = (M - k) & (M - 1);
        v[t] = lc[r * RS + k + (k >> 4)];
        xm[t] = lc[r * RS + km + (km >> 4)];
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        lds_barrier();
#pragma unroll
        for (int m = 0; m < PTS; ++m) lds[(ty + TY * m) * RS + x + (x >> 4)] = h ? -v[m].y : v[m].x;
        lds_barrier();
#pragma unroll
        for (int t = 0; t < PTS; ++t) {
          const int k = tpc + TPC * t, km = (M - k) & (M - 1);
          const double d = lds[r * RS + k + (k >> 4)], dm = lds[r * RS + km + (km >> 4)];
          if (h) { v[t].y = d; xm[t].y = dm; } else { v[t].x = d; xm[t].x = dm; }
        }
      }
    }
    lds_barrier();
    if (tpc == 0) xm[0] = qy[r];  // k = 0: the mirror is the Nyquist bin (row r's y1 inverse, from LDS)
#pragma unroll
    for (int t = 0; t < PTS; ++t) {
      const int k = tpc + TPC * t;
      const cd e = make_cd(0.5 * (v[t].x + xm[t].x), 0.5 * (v[t].y - xm[t].y));
      const cd d = make_cd(0.5 * (v[t].x - xm[t].x), 0.5 * (v[t].y + xm[t].y));
      const cd o = cmul(d, cconj(a.tw[k]));               // (X[k] - conj X[M-k]) W^-k / 2
      v[t] = cconj(make_cd(e.x - o.y, e.y + o.x));        // E + i O, conjugated: inverse by conjugation
    }
  };
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    const int z = u / N2, y2 = u % N2;
    cd v[PTS];
    if constexpr (!INV) {
      {
        const int r = idx(r0), tpc = idx(tpc0);
        const cd* src = reinterpret_cast<const cd*>(in_r) + ((i64)z * NY + y2 + N2 * r) * M + tpc;
#pragma unroll
        for (int t = 0; t < PTS; ++t) v[t] = gload<MF>(src + TPC * t);
        __builtin_amdgcn_sched_barrier(0);  // all loads out before the first butterfly
        fft_stages<M, PTS, r0_of(M, PTS), true, N1, FW>(v, lds, tw_m, r, tpc, true);  // 128 = 2 x 8 x 8; v[t] = Z[tpc + TPC t]
      }
      to_columns_r2c(v, z, y2);
      {
        const int x = idx(x0), ty = idx(ty0);
        fft_stages<N1, PTS, r0_of(N1, PTS), false, TC, FW>(v, lds, tw_1, x, ty, true);  // 32 = 4 x 8; v[m]: k1 = ty + TY m
        cd* dst = H + ((i64)z * NY + y2 + N2 * ty) * M + x;
#pragma unroll
        for (int m = 0; m < PTS; ++m) dst[(i64)N2 * TY * M * m] = v[m];
      }
      if constexpr (WL) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // qy: written by this wave's x = 0 lanes
      if (tid < N1) {  // the Nyquist column's y1 DFT (qy is visible: fft_stages held barriers; with WL
                       // the x = 0 lanes that wrote it are lanes 0, 16, 32, 48 of this same wave)
        const int k = idx(tid);
        cd acc = make_cd(0.0, 0.0);
#pragma unroll 8
        for (int j = 0; j < N1; ++j) acc = cadd(acc, cmul(qy[j], tw_1[(j * k) & (N1 - 1)]));
        Q[(i64)z * NY + y2 + N2 * k] = acc;  // slot layout, k1 = k
      }
    } else {
      cd qk = make_cd(0.0, 0.0);  // the Nyquist column, k1 = tid (first wave), from the middle launch
      if (tid < N1) qk = Q[(i64)z * NY + y2 + N2 * idx(tid)];
      {
        const int x = idx(x0), ty = idx(ty0);
        const cd* src = H + ((i64)z * NY + y2 + N2 * ty) * M + x;
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = src[(i64)N2 * TY * M * m];
        __builtin_amdgcn_sched_barrier(0);  // all loads out before the first butterfly (measured neutral here)
#pragma unroll
        for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
        fft_stages<N1, PTS, r0_of(N1, PTS), false, TC, FW>(v, lds, tw_1, x, ty, true);  // v[m]: y1 = ty + TY m
      }
      if (tid < 64) {  // one wave: the Nyquist column's y1 inverse into qy (read by to_rows_c2r)
        if (tid < N1) qy[tid] = qk;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes before its reads
        cd acc = make_cd(0.0, 0.0);
        const int y1 = idx(tid) & (N1 - 1);
#pragma unroll 8
        for (int k = 0; k < N1; ++k) acc = cadd(acc, cmul(qy[k], cconj(tw_1[(y1 * k) & (N1 - 1)])));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane has read qy before it is overwritten
        if (tid < N1) qy[tid] = acc;
      }
      to_rows_c2r(v, z, y2);
      {
        const int r = idx(r0), tpc = idx(tpc0);
        fft_stages<M, PTS, r0_of(M, PTS), true, N1, FW>(v, lds, tw_m, r, tpc, true);
        const double sc = a.scale;
        cd* dst = reinterpret_cast<cd*>(out_r) + ((i64)z * NY + y2 + N2 * r) * M + tpc;
#pragma unroll
        for (int t = 0; t < PTS; ++t) gstore<MF>(dst + TPC * t, make_cd(v[t].x * sc, -v[t].y * sc));
      }
    }
    lds_barrier();  // the next unit's first exchange overwrites LDS
  }
}

hipError_t launch_three_pass_real(int stage, int n, const double* b, cd* H, cd* Q, double* x, const TPArgs& a,
                                  hipStream_t s, bool alt_rows) {
  if (stage == 3) {  // the Nyquist column Q [n z][n y]: P2 on its N2 columns of each k1 (NX = 1)
    if (n == 128)
      hipLaunchKernelGGL((k_tp_mid<0, 4, 4, 128, 8, false, 1>), dim3(32), dim3(4 * 16), 0, s, Q, a, 32);
    else
      hipLaunchKernelGGL((k_tp_mid<0, 8, 8, 256, 4, false, 1>), dim3(32), dim3(8 * 64), 0, s, Q, a, 32);
    return hipGetLastError();
  }
  if (n == 128) {
    if (stage == 1) {  // x tiles of the 64-wide half spectrum (8 x times 4 y2) x k1
      constexpr int units = (64 / 8) * 32;
      hipLaunchKernelGGL((k_tp_mid<0, 32, 4, 128, 8, false, 64>), dim3(grid_of(units, 2)), dim3(512), 0, s, H, a,
                         units);
    } else {
      constexpr int units = 128 * 4;  // z-planes x y2
      const unsigned g = grid_of(units, 4);
      // wave-local FFT exchanges (WL) by default since r04ab; alt_rows: workgroup barriers
      if (stage == 0 && alt_rows)
        hipLaunchKernelGGL((k_tp_rows_r2c<false, 64, 32, 4, 128>), dim3(g), dim3(256), 0, s, b, H, Q, nullptr, a,
                           units);
      else if (stage == 0)
        hipLaunchKernelGGL((k_tp_rows_r2c<false, 64, 32, 4, 128, 0, 4, false, true>), dim3(g), dim3(256), 0, s, b, H,
                           Q, nullptr, a, units);
      else if (alt_rows)
        hipLaunchKernelGGL((k_tp_rows_r2c<true, 64, 32, 4, 128>), dim3(g), dim3(256), 0, s, nullptr, H, Q, x, a,
                           units);
      else
        hipLaunchKernelGGL((k_tp_rows_r2c<true, 64, 32, 4, 128, 0, 4, false, true>), dim3(g), dim3(256), 0, s, nullptr,
                           H, Q, x, a, units);
    }
    return hipGetLastError();
  }
  if (stage == 1) {
    constexpr int units = (128 / 8) * 32;  // x tiles of the half spectrum x k1
    // units in XCD order (whole rounds: 512 units, 256 workgroups; r05q, profiles/r05q_mid_xcd_ab.txt:
    // 5,713-5,736 against 5,639-5,681 real PCApply/s); -DCFP_REAL_MID_XCD=0: A/B
    const unsigned gx = CFP_REAL_MID_XCD ? grid_xcd(units, 1) : 0;
    if (gx)
      hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 128, 0, 0, false, true>), dim3(gx), dim3(1024), 0, s, H, a,
                         units);
    else
      hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 128>), dim3(grid_of(units, 1)), dim3(1024), 0, s, H, a,
                         units);
  } else {
    constexpr int units = 256 * 8;  // z-planes x y2
    const unsigned g = grid_of(units, 2);
    // the row FFT's and y1 DFT's exchanges wave-local (WL; r04aa: 5,720 against 5,343 real
    // PCApply/s, P1r 64 -> ~57 us); alt_rows (CFP_RSCHEDULE_THREE_ALT, A/B): workgroup barriers
    // blockIdx order (r05l: XCD order 5,641-5,704 against 5,699-5,701 real PCApply/s)
    if (stage == 0 && !alt_rows)  // P1r: 80 VGPRs, three workgroups per CU
      hipLaunchKernelGGL((k_tp_rows_r2c<false, 128, 32, 8, 256, F_NT_LD, 6, false, true>), dim3(grid_of(units, 3)),
                         dim3(512), 0, s, b, H, Q, nullptr, a, units);
    else if (stage == 0)
      hipLaunchKernelGGL((k_tp_rows_r2c<false, 128, 32, 8, 256, F_NT_LD, 6>), dim3(grid_of(units, 3)), dim3(512), 0, s, b,
                         H, Q, nullptr, a, units);
    else if (!alt_rows)
      hipLaunchKernelGGL((k_tp_rows_r2c<true, 128, 32, 8, 256, F_NT_ST, 4, true, true>), dim3(g), dim3(512), 0, s,
                         nullptr, H, Q, x, a, units);
    else
      hipLaunchKernelGGL((k_tp_rows_r2c<true, 128, 32, 8, 256, F_NT_ST, 4, true>), dim3(g), dim3(512), 0, s, nullptr, H, Q, x, a,
                         units);
  }
  return hipGetLastError();
}


// P1 load policy (r03, profiles/r03f_p1_inplace_ab.jsonl, r03g_p1_out_of_place_ab.jsonl):
// out of place, non-temporal loads (plain loads leave P2 at 153-160 us); in place (the direct
// solver's Un, Un), plain loads -- with NT loads of the lines it then overwrites, P1's output
// drops out of the Infinity Cache and P2 takes 143-145 us instead of 128.
constexpr int kP1Flags = F_NT_LD, kP1InPlaceFlags = 0;
// P3 store policy: non-temporal.  r03v A/B of all 24 P1 / P2 / P3 cache policies in the apply
// chain (tools/kexp/tp_chain.hip, profiles/r03v_tp_chain.txt): plain P3 stores 310 us against
// 314 us there, but +0.3-0.8 % in bench.py and -2 % inside GMRES (0.387 vs 0.379 ms per PCApply),
// so the measured policy stays.
constexpr int kP3Flags = F_NT_ST;
// 256^3, N1 = 32 (r03z, tools/kexp/run_tp_lp.py, profiles/r03z_tp_lp.txt, 3-sweep chain):
// P1 / P3 with the lane-pair phase A (no LDS exchange there): 310.8 -> 303.0 us.  Every executor
// (one GPU, slabs, pieces) runs it.  (Moving the four-step twiddle W_256^{y2 k1} from P2 into
// P1 / P3 lost: 313.1 us, P1 +9 us for its table loads, P2 -1 us; DESIGN.md.)
constexpr bool kRowsLP = true;
// P2 load policy (r03z, profiles/r03z_tp_p2nt.txt): non-temporal loads and LDS-DMA of its input,
// which nothing reads after it: chain 304.4 -> 300.7 us
constexpr int kP2LoadFlags = F_NT_LD;
// P1 / P3 phase C (the row FFT) with wave-local exchanges (r04ab): shape TP_MID_ROWSALT runs the
// other setting for A/B
constexpr bool kRowsWave = true;
// P1 / P3 units in XCD order at 256^3 and 512^3 (r05j, tools/kexp/run_rows_512.py,
// profiles/r05j_rows_probes.txt): each XCD walks whole z-planes of b / x, so an XCD's units read
// and write one contiguous region; 256^3 P1 93.8 -> 90.8 us, P3 90.4 -> 86.6 us; 512^3 P1 911 ->
// 884 us, P3 915 -> 866 us (the units of one plane in blockIdx order spread over all eight
// XCDs).  Whole apply (r05k, against a -DCFP_ROWS_XCD=0 build, alternating processes): 256^3
// 3,361-3,388 against 3,288-3,316 PCApply/s, 512^3 282.3-282.5 against 274.6-275.4.
constexpr bool kRowsXCD = CFP_ROWS_XCD != 0;

// P1F / P3F: P1's load and P3's store policy out of place (kP1Flags / kP3Flags; 0 = plain)
// WR: phase C's exchanges wave-local (F_WAVE_LDS)
template <int N1, int TN, int PER_CU, int PTS = 16, bool XS = true, bool LP = false, int BL = 0, bool XCD = false,
          int P1F = kP1Flags, int P3F = kP3Flags, bool WR = kRowsWave>
static void launch_rows(int stage, const cd* in, cd* out, const TPArgs& a, hipStream_t s) {
  constexpr int units = TN * (TN / N1);  // z-planes x y2
  constexpr int W = WR ? F_WAVE_LDS : 0;
  const unsigned g = XCD ? grid_xcd(units, PER_CU) : grid_of(units, PER_CU);
  if constexpr (XCD) {
    if (g == 0) {  // fewer than 8 workgroups: the same kernel in plain unit order
      launch_rows<N1, TN, PER_CU, PTS, XS, LP, BL, false, P1F, P3F, WR>(stage, in, out, a, s);
      return;
    }
  }
  const dim3 blk(N1 * (TN / PTS));
  if (stage == 0 && in == out)  // in place (the direct solver's Un, Un)
    TP_LAUNCH((k_tp_rows<false, kP1InPlaceFlags | W, N1, TN, PTS, XS, LP, BL, XCD>), dim3(g), blk, s, in, out, a, units);
  else if (stage == 0)
    TP_LAUNCH((k_tp_rows<false, P1F | W, N1, TN, PTS, XS, LP, BL, XCD>), dim3(g), blk, s, in, out, a, units);
  else
    TP_LAUNCH((k_tp_rows<true, P3F | W, N1, TN, PTS, XS, LP, BL, XCD>), dim3(g), blk, s, in, out, a, units);
}
// the default row sweeps, or (alt, shape TP_MID_ROWSALT) the same with the other phase-C exchanges;
// units in XCD order (kRowsXCD)
template <int N1, int TN, int PER_CU, int PTS, bool XS, bool LP, int P1F = kP1Flags, int P3F = kP3Flags,
          bool XCD = kRowsXCD>
static void launch_rows_ab(bool alt, int stage, const cd* in, cd* out, const TPArgs& a, hipStream_t s) {
  if (alt) launch_rows<N1, TN, PER_CU, PTS, XS, LP, 0, XCD, P1F, P3F, !kRowsWave>(stage, in, out, a, s);
  else launch_rows<N1, TN, PER_CU, PTS, XS, LP, 0, XCD, P1F, P3F, kRowsWave>(stage, in, out, a, s);
}

template <int T, int N2, int TN, int PER_CU, int PTS = 16, bool XS = true>
static void launch_mid(cd* data, const TPArgs& a, hipStream_t s) {
  constexpr int units = (TN / (T / N2)) * (TN / N2);  // x-tiles x k1
  TP_LAUNCH((k_tp_mid<0, T, N2, TN, PTS, XS>), dim3(grid_of(units, PER_CU)), dim3(T * (TN / PTS)), s, data, a, units);
}

template <int N2, int TN, bool PF = false, bool BL = false, int T = 64>
static void launch_mid_sw(cd* data, const TPArgs& a, hipStream_t s) {
  constexpr int units = (TN / (T / N2)) * (TN / N2);
  if constexpr (T == 64 && N2 == 8 && TN == 256 && PF && !BL) {
    if (a.krylov) {  // the default 256^3 P2 inside the stand-in KSP: same kernel, TAG 1 (TPArgs::krylov)
      TP_LAUNCH((k_tp_mid_sw<T, N2, TN, 0, PF, TN, 0, kP2LoadFlags, BL, false, 1>), dim3(grid_of(units, 64 / T)),
                dim3(T * (TN / 16)), s, data, a, units);
      return;
    }
  }
  TP_LAUNCH((k_tp_mid_sw<T, N2, TN, 0, PF, TN, 0, kP2LoadFlags, BL>), dim3(grid_of(units, 64 / T)),
            dim3(T * (TN / 16)), s, data, a, units);
}

bool three_pass_slab_supported(const i64 n[3], int P) {
  // N1 = 32 rows per P1 unit, k1 split over the ranks (P | 32); P3 reads chunk rows N2 apart
  // per thread and N2 TY = 2 N2 apart per slot (nyl >= 2 N2: 256^3 N2 = 8, 512^3 N2 = 16)
  const bool cube = n[0] == n[1] && n[1] == n[2] && (n[0] == 256 || n[0] == 512);
  return cube && P >= 1 && P <= 16 && (32 % P) == 0;
}

int three_pass_slab_n2(i64 n) { return n == 512 ? 16 : 8; }

hipError_t launch_three_pass_slab(int stage, int n, const cd* in, cd* out, const TPArgs& a, int nzl, hipStream_t s) {
  if (n == 512) {
    // 512^3 (r05): N1 = 32 x N2 = 16 as on one GPU; P2 on this rank's [512 z][nyl][512 x] block
    // (2 x times 16 y2 tiles of its nyl / 16 k1, XCD order), P1 / P3 on the local planes through
    // the per-peer chunks, one 1024-thread workgroup per CU
    constexpr int W = kRowsWave ? F_WAVE_LDS : 0;
    if (stage == 1) {
      const int nk1 = (1 << a.lnyl) / 16;  // local k1 values
      const int units = 256 * nk1;         // x tiles x local k1
      const unsigned g = grid_xcd(units, 1);
      if (g) TP_LAUNCH((k_tp_mid<0, 32, 16, 512, 16, true, 512, true>), dim3(g), dim3(1024), s, out, a, units);
      else TP_LAUNCH((k_tp_mid<0, 32, 16, 512, 16, true, 512, false>), dim3(grid_of(units, 1)), dim3(1024), s, out, a,
                     units);
    } else {
      const int units = nzl * 16;  // local z-planes x y2
      // XCD order when the rounds are whole and fill the chip (r05l, profiles/r05l_rows_xcd_ab.txt:
      // P = 8 local kernels 423-431 against 439-445 us; P = 16 in 4 pieces of 128 units: 274-276
      // against 256-258 us, so not below a full round)
      const unsigned gx = kRowsXCD && units >= (int)grid_of(1 << 30, 1) ? grid_xcd(units, 1) : 0;
      const unsigned g = gx ? gx : grid_of(units, 1);
      if (stage == 0 && gx)
        TP_LAUNCH((k_tp_rows<false, F_NT_LD | W, 32, 512, 16, true, kRowsLP, 0, true>), dim3(g), dim3(1024), s, in, out, a, units);
      else if (stage == 0)
        TP_LAUNCH((k_tp_rows<false, F_NT_LD | W, 32, 512, 16, true, kRowsLP>), dim3(g), dim3(1024), s, in, out, a, units);
      else if (gx)
        TP_LAUNCH((k_tp_rows<true, F_NT_ST | W, 32, 512, 16, true, kRowsLP, 0, true>), dim3(g), dim3(1024), s, in, out, a, units);
      else
        TP_LAUNCH((k_tp_rows<true, F_NT_ST | W, 32, 512, 16, true, kRowsLP>), dim3(g), dim3(1024), s, in, out, a, units);
    }
    return hipGetLastError();
  }
  if (stage == 1) {
    const int nk1 = a.lnyl ? (1 << a.lnyl) / 8 : 32;  // local k1 values: nyl / N2
    const int units = 32 * nk1;                        // x tiles x local k1
    if (((uintptr_t)out & 15) == 0)  // the LDS-DMA prefetch needs 16-byte addresses
      hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, true, 256, 0, kP2LoadFlags>), dim3(grid_of(units, 1)), dim3(1024), 0, s,
                         out, a, units);
    else
      hipLaunchKernelGGL((k_tp_mid_sw<64, 8, 256, 0, false, 256, 0, kP2LoadFlags>), dim3(grid_of(units, 1)), dim3(1024), 0, s,
                         out, a, units);
  } else {
    const int units = nzl * 8;  // local z-planes x y2
    // XCD order when the rounds are whole and fill the chip (as at 512^3)
    const unsigned gx = kRowsXCD && units >= (int)grid_of(1 << 30, 2) ? grid_xcd(units, 2) : 0;
    const unsigned g = gx ? gx : grid_of(units, 2);
    constexpr int W = kRowsWave ? F_WAVE_LDS : 0;
    if (stage == 0 && gx)
      hipLaunchKernelGGL((k_tp_rows<false, F_NT_LD | W, 32, 256, 16, true, kRowsLP, 0, true>), dim3(g), dim3(512), 0, s,
                         in, out, a, units);
    else if (stage == 0)
      hipLaunchKernelGGL((k_tp_rows<false, F_NT_LD | W, 32, 256, 16, true, kRowsLP>), dim3(g), dim3(512), 0, s,
                         in, out, a, units);
    else if (gx)
      hipLaunchKernelGGL((k_tp_rows<true, F_NT_ST | W, 32, 256, 16, true, kRowsLP, 0, true>), dim3(g), dim3(512), 0, s,
                         in, out, a, units);
    else
      hipLaunchKernelGGL((k_tp_rows<true, F_NT_ST | W, 32, 256, 16, true, kRowsLP>), dim3(g), dim3(512), 0, s,
                         in, out, a, units);
  }
  return hipGetLastError();
}

// The default 256^3 row sweeps with the stand-in GMRES's Krylov work fused in (TPArgs pre_* /
// post_*): P1 on A b, P3 with the dots.  Same grids and unit order as launch_rows_ab.
bool three_pass_fused_supported(int n, TPShape shape) { return n == 256 && shape.n1 == 0 && shape.mid == TP_MID_DEFAULT; }

template <bool XCD>
static void launch_rows_fused(int stage, const cd* in, cd* out, const TPArgs& a, hipStream_t s, unsigned g) {
  constexpr int W = kRowsWave ? F_WAVE_LDS : 0, units = 256 * 8;
  if (stage == 0)
    TP_LAUNCH((k_tp_rows<false, kP1Flags | W, 32, 256, 16, true, kRowsLP, 0, XCD, 0, 1>), dim3(g), dim3(512), s, in,
              out, a, units);
  else
    TP_LAUNCH((k_tp_rows<true, kP3Flags | W, 32, 256, 16, true, kRowsLP, 0, XCD, 0, TP_POST_MAX>), dim3(g), dim3(512),
              s, in, out, a, units);
}

hipError_t launch_three_pass_fused(int stage, int n, const cd* in, cd* out, const TPArgs& a, hipStream_t s,
                                   unsigned* grid_out) {
  if (n != 256 || (stage != 0 && stage != 2)) return hipErrorNotSupported;
  if (stage == 0 && (!a.pre_cls || in == out || a.pre_ncls < 1 || a.pre_ncls > TP_PRE_MAX_CLS || a.pre_nd < 1 ||
                     a.pre_nd > 3))
    return hipErrorInvalidValue;
  if (stage == 2 && (a.post_nv < 1 || a.post_nv > TP_POST_MAX || !a.post_partial)) return hipErrorInvalidValue;
  constexpr int units = 256 * 8;
  const unsigned gx = kRowsXCD ? grid_xcd(units, 2) : 0;
  const unsigned g = gx ? gx : grid_of(units, 2);
  if (grid_out) *grid_out = g;
  if (gx) launch_rows_fused<true>(stage, in, out, a, s, g);
  else launch_rows_fused<false>(stage, in, out, a, s, g);
  return hipGetLastError();
}

bool three_pass_shape_valid(int n1, int mid, i64 n) {
  if (mid == TP_MID_ROWSALT) return n1 == 0;
  if (n1 == 16) return n == 128 && mid >= TP_MID_DEFAULT && mid <= TP_MID_SWAP64;
  return (n1 == 0 || n1 == 32 || n1 == 64) && (mid >= 0 && mid <= TP_MID_SWAP32X) &&
         !(mid >= TP_MID_BLOCKED && n1 == 64);
}

hipError_t launch_three_pass(int stage, int n, const cd* in, cd* out, const TPArgs& a, TPShape shape,
                             hipStream_t s) {
  // TP_MID_ROWSALT: the default shape with the other phase-C exchanges in P1 / P3 (A/B)
  const bool ra = shape.mid == TP_MID_ROWSALT;
  if (ra) shape.mid = TP_MID_DEFAULT;
  if (n == 100) return launch_three_pass_sq(stage, n, in, out, a, shape, s);
  if (n == 512) {
    // 512^3 (r04): N1 = 32 x N2 = 16.  P1 / P3: 32 rows of 512 (16 points per thread, 1024
    // threads, split exchanges: 136 KiB, one per CU).  P2: the z FFT of 512 bounds the tile to 32
    // columns (128 KiB split exchange) = 2 x times 16 y2, 32-byte runs; units in XCD order so
    // the 4 tiles of a 128-byte line share an L2.  96 N bytes per apply against 160 N.
    // shape.mid = blocked: blocks of 2 x (P2 reads one 512-byte run per z; P1 / P3 in XCD order,
    // so the 16 y2 units of a plane share their lines' L2); blocked32: blocks of 8 x (P1 / P3
    // move whole 128-byte lines, P2's 32-byte pieces of a z lie in one 2 KiB block); lane64: P1 /
    // P3 phase A through LDS.
    const bool bl = shape.mid == TP_MID_BLOCKED, bl8 = shape.mid == TP_MID_BLOCKED32;
    if (stage == 1) {
      constexpr int units = (512 / 2) * 32;
      const unsigned g = grid_xcd(units, 1);  // whole rounds of a power of two >= 8
      if (g == 0) return hipErrorNotSupported;
      if (bl) TP_LAUNCH((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 2>), dim3(g), dim3(1024), s, out, a, units);
      else if (bl8) TP_LAUNCH((k_tp_mid<0, 32, 16, 512, 16, true, 512, true, 8>), dim3(g), dim3(1024), s, out, a, units);
      else TP_LAUNCH((k_tp_mid<0, 32, 16, 512, 16, true, 512, true>), dim3(g), dim3(1024), s, out, a, units);  // NT loads: 204 against 262 /s (r04y)
    } else if (bl) {
      launch_rows<32, 512, 1, 16, true, kRowsLP, 2, true>(stage, in, out, a, s);
    } else if (bl8) {
      launch_rows<32, 512, 1, 16, true, kRowsLP, 8>(stage, in, out, a, s);
    } else if (shape.mid == TP_MID_LANE64) {  // A/B: phase A through LDS
      launch_rows<32, 512, 1>(stage, in, out, a, s);
    } else {  // lane-pair phase A (no LDS exchange there)
      launch_rows_ab<32, 512, 1, 16, true, kRowsLP>(ra, stage, in, out, a, s);
    }
    return hipGetLastError();
  }
  if (n == 128) {
    // 128^3, n1 = 32 (N1 = 32 x N2 = 4; AUTO from r03m to r04), 8 points per thread and whole-complex LDS
    // exchanges (one barrier pair per exchange instead of two): P1/P3 512 threads, 69 KiB (2 per
    // CU); P2 32 columns = 8 x times 4 y2 (128-byte runs), 512 threads, 64 KiB (2 per CU).
    // shape.mid = lane64 keeps the round-2 kernels (16 points per thread, split exchanges, P2
    // 64 columns) for A/B: 15.9k against 18.4k applies/s, the 5-pass schedule 17.3k
    // (profiles/r03m_128_three_sweep.md).
    // Default since r04: y split 16 x 8 -- P1/P3 units of 16 rows (1,024 units, 256 threads, four
    // workgroups per CU, lane-pair phase A, 13.2 against 17.0 us); P2 below.  21,475 against
    // 18,520 applies/s for the r03 split 32 x 4 (n1 = 32) in the same process
    // (profiles/r04_schedule_ab.jsonl).
    const int n1 = shape.n1 ? shape.n1 : (shape.mid == TP_MID_LANE64 || shape.mid == TP_MID_SWAP64 ? 32 : 16);
    if (n1 == 16) {
      // P2 default (r04z): 32 columns = 4 x times 8 y2 (64-byte tiles, 512 units, two 512-thread
      // workgroups per CU, 8 points, whole-complex) in XCD order, so the two tiles of a 128-byte
      // line meet in one L2: 21,475 /s; in blockIdx order 19,130.  A/B: lane32 = 64 columns,
      // 8 points, whole-complex (1,024 threads; 21,070-21,150 /s); lane64 = 64 columns, 16
      // points, split (20,530 /s); swap64 = 64 columns, 16 points, whole-complex (20,750 /s)
      if (stage == 1) {
        if (shape.mid == TP_MID_LANE32) launch_mid<64, 8, 128, 1, 8, false>(out, a, s);
        else if (shape.mid == TP_MID_LANE64) launch_mid<64, 8, 128, 1>(out, a, s);
        else if (shape.mid == TP_MID_SWAP64) launch_mid<64, 8, 128, 1, 16, false>(out, a, s);
        else {
          constexpr int units = (128 / 4) * 16;
          const unsigned g = grid_xcd(units, 2);
          if (g) TP_LAUNCH((k_tp_mid<0, 32, 8, 128, 8, false, 128, true>), dim3(g), dim3(512), s, out, a, units);
          else launch_mid<32, 8, 128, 2, 8, false>(out, a, s);
        }
      } else {
        // blockIdx order (r05k: XCD order 21,370-21,420 against 21,630-21,700 PCApply/s; one
        // round of units whose b and x stay in the Infinity Cache)
        launch_rows_ab<16, 128, 4, 8, false, true, 0, 0, false>(ra, stage, in, out, a, s);
      }
      return hipGetLastError();
    }
    if (shape.mid == TP_MID_LANE64) {
      if (stage == 1) launch_mid<64, 4, 128, 2>(out, a, s);
      else launch_rows<32, 128, 4>(stage, in, out, a, s);
    } else {
      // 128^3: b and x (32 MiB each) stay in the 256 MiB Infinity Cache between applies, so P1
      // loads and P3 stores keep the default policy (shape.mid = swap64: the 256^3 NT policy, A/B)
      if (stage == 1) launch_mid<32, 4, 128, 2, 8, false>(out, a, s);
      else if (shape.mid == TP_MID_SWAP64) launch_rows<32, 128, 2, 8, false>(stage, in, out, a, s);
      else launch_rows<32, 128, 2, 8, false, false, 0, false, 0, 0>(stage, in, out, a, s);
    }
    return hipGetLastError();
  }
  // 256^3.  Default shape = the measured best: N1 = 32, P2 tiles of 64 columns (8 x times 8 y2,
  // 128-byte runs) with the y2 DFT on permlane transposes and the LDS-DMA prefetch of half the
  // next unit (k_tp_mid_sw<.., PF>; r02 A/B in the apply chain, profiles/r02e_p2_ab.txt: 138 us
  // without the prefetch, 144 us for the DPP lane kernel, 128 us with it), persistent grids.  The
  // other shapes are selected per plan (cfp_plan_set_three_pass_shape) for tests and measurements.
  const int n1 = shape.n1 == 64 ? 64 : 32;
  const bool t32 = shape.mid == TP_MID_LANE32;
  // the LDS-DMA prefetch (global_load_lds_dwordx4) takes 16-byte aligned addresses: a buffer that
  // is only 8-byte aligned runs the same kernel without it
  const bool pf_ok = ((uintptr_t)out & 15) == 0;
  if (shape.mid == TP_MID_BLOCKED) {  // N1 = 32, blocked intermediate layout (k_tp_rows<.., 8>)
    if (stage != 1) launch_rows<32, 256, 2, 16, true, kRowsLP, 8>(stage, in, out, a, s);
    else if (pf_ok) launch_mid_sw<8, 256, true, true>(out, a, s);
    else launch_mid_sw<8, 256, false, true>(out, a, s);
    return hipGetLastError();
  }
  if (shape.mid == TP_MID_SWAP32X) {  // natural layout; P2 = 32 columns in XCD order, two per CU
    if (stage != 1) {
      launch_rows<32, 256, 2, 16, true, kRowsLP>(stage, in, out, a, s);
    } else {
      constexpr int units = (256 / 4) * 32;
      const unsigned g = grid_xcd(units, 2);
      if (g == 0) return hipErrorNotSupported;
      if (pf_ok)
        TP_LAUNCH((k_tp_mid_sw<32, 8, 256, 0, true, 256, 0, kP2LoadFlags, false, true>), dim3(g), dim3(512), s, out, a,
                  units);
      else
        TP_LAUNCH((k_tp_mid_sw<32, 8, 256, 0, false, 256, 0, kP2LoadFlags, false, true>), dim3(g), dim3(512), s, out, a,
                  units);
    }
    return hipGetLastError();
  }
  if (shape.mid == TP_MID_BLOCKED32) {  // blocks of 4 x; P2 = 32 columns, two workgroups per CU
    // P1 / P3 in XCD order: the 8 y2 units of a plane share the 128-byte lines of their 64-byte
    // pieces (r04d without it: P3 130.6 us against 90.8 natural)
    if (stage != 1) launch_rows<32, 256, 2, 16, true, kRowsLP, 4, true>(stage, in, out, a, s);
    else if (pf_ok) launch_mid_sw<8, 256, true, true, 32>(out, a, s);
    else launch_mid_sw<8, 256, false, true, 32>(out, a, s);
    return hipGetLastError();
  }
  if (stage == 1) {
    if ((shape.mid == TP_MID_SWAP64_PF || shape.mid == TP_MID_DEFAULT) && pf_ok) {
      if (n1 == 64) launch_mid_sw<4, 256, true>(out, a, s);
      else launch_mid_sw<8, 256, true>(out, a, s);
    } else if (shape.mid == TP_MID_SWAP64 || shape.mid == TP_MID_SWAP64_PF || shape.mid == TP_MID_DEFAULT) {
      if (n1 == 64) launch_mid_sw<4, 256>(out, a, s);
      else launch_mid_sw<8, 256>(out, a, s);
    } else if (n1 == 64) {
      if (t32) launch_mid<32, 4, 256, 2>(out, a, s);
      else launch_mid<64, 4, 256, 1>(out, a, s);
    } else if (t32) {
      launch_mid<32, 8, 256, 2>(out, a, s);
    } else {
      launch_mid<64, 8, 256, 1>(out, a, s);
    }
  } else if (n1 == 64) {
    launch_rows<64, 256, 1>(stage, in, out, a, s);
  } else {
    launch_rows_ab<32, 256, 2, 16, true, kRowsLP>(ra, stage, in, out, a, s);
  }
  return hipGetLastError();
}

}  // namespace cfp
