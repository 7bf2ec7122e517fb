// cfp_fft_device.h -- device code of the fast axis-pass FFT (gfx950).  Included by
// cfp_kernels.hip (product dispatch) and by tools/kexp (variant timing harness).
//
// Stockham autosort FFT of length N = R0 * PTS^(S-1) per column.  TPC = N/PTS threads own
// one column; thread tpc keeps register slot m = point tpc + m*TPC on input and on output,
// so a forward transform's output feeds an inverse transform straight from registers.
// Stage s (radix r, Ns = product of earlier radices) maps butterfly j:
//   in : data[j + t*N/r] * W_{Ns r}^{(j mod Ns) t}      out: data[(j/Ns)*Ns*r + (j mod Ns) + t*Ns]
// Inter-stage exchanges go through LDS; every other step is in VGPRs.
#pragma once
#include "cfp_internal.h"

namespace cfp {

// -------------------------------------------------------------- variant flags
enum : int {
  F_SPLIT_LDS = 1,  // exchange real and imaginary parts separately (half the LDS footprint)
  F_TW_GLOBAL = 2,  // twiddles from the global table (L1/L2) instead of an LDS copy
  F_NT = 4,         // non-temporal global loads and stores
  F_REV = 8,        // walk the tiles in reverse block order
  F_NT_LD = 16,     // non-temporal global loads only
  F_NT_ST = 32,     // non-temporal global stores only
  F_LDS_SYNC = 64,  // exchange barriers wait for LDS only (global loads may stay in flight)
  F_OCC4 = 128,     // ask the compiler for 4 waves per SIMD (<= 128 VGPRs)
  F_SYM_LDS = 256,  // fused pass: stage the per-point symbol table in LDS next to the twiddles
  F_OCC8 = 512,     // ask the compiler for 8 waves per SIMD (<= 64 VGPRs)
  F_PAD1 = 1024,    // row-mode LDS rows padded by one element (n + 1) instead of n / 16
  F_WAVE_LDS = 2048,  // every exchange stays inside one wave (its columns' threads and LDS region
                      // belong to one wave): the exchange barriers become wave-local LDS waits
};
__host__ __device__ constexpr int waves_req(int flags, int mode) {
  return mode == PASS_FUSED_WAVE ? 1 : ((flags & F_OCC8) ? 8 : ((flags & F_OCC4) ? 4 : 1));
}

// Workgroup barrier that waits only for this wave's LDS accesses: global loads issued earlier
// (a prefetch of the next work unit) stay in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int FLAGS>
__device__ __forceinline__ void xbarrier() {
  // a wave's LDS accesses complete in order: waiting for its own is enough when no other wave
  // touches the region (the asm's memory clobber keeps the compiler from moving LDS accesses)
  if (FLAGS & F_WAVE_LDS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if (FLAGS & F_LDS_SYNC) lds_barrier();
  else __syncthreads();
}

// blockIdx -> unit of a persistent grid of G workgroups, G a multiple of 8 (the host checks):
// workgroups reach the XCDs round-robin (blockIdx % 8), and each XCD takes a contiguous eighth
// of every whole round of G units; a last, partial round keeps blockIdx order
__device__ __forceinline__ int xcd_round_unit(int it, int G, int n) {
  const int b = it % G, base = it - b;
  return base + G <= n ? base + (b & 7) * (G >> 3) + (b >> 3) : it;
}

// ------------------------------------------------------------------ complex helpers
__device__ __forceinline__ cd cadd(cd a, cd b) { return make_cd(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd csub(cd a, cd b) { return make_cd(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cd cmul(cd a, cd b) {
  return make_cd(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ cd cconj(cd a) { return make_cd(a.x, -a.y); }
// a / b = (a * conj(b)) / |b|^2, the complex VecPointwiseDivide of the reference
// (src/FftLinearSolver_3D.c:174).  A zero divisor gives 0, as PETSc's VecPointwiseDivide does
// (third-party semantics, PETSc src/vec/vec/impls/seq/bvec2.c): a singular symbol's null modes
// are dropped instead of turning the whole result into inf / NaN.
__device__ __forceinline__ bool cnonzero(cd b) { return b.x != 0.0 || b.y != 0.0; }
__device__ __forceinline__ cd cdiv(cd a, cd b) {
  const double den = cnonzero(b) ? 1.0 / fma(b.x, b.x, b.y * b.y) : 0.0;
  return make_cd(fma(a.x, b.x, a.y * b.y) * den, fma(a.y, b.x, -a.x * b.y) * den);
}

// a / b for the symbol divide: the hardware reciprocal refined by one Newton step instead of
// the IEEE division sequence (3 instead of ~12 VALU ops per point).  Measured on MI355X over
// 2^20 values spread across 60 binades (tools/kexp/rcp_check.hip): v_rcp_f64 alone 4.6e-8
// relative, after one step 2.2e-15, after two 1.1e-16 -- one step is 5 orders of magnitude
// inside the 1e-10 parity bar.  Valid for normal |b|^2 (a transport symbol has Re b >= 1).
__device__ __forceinline__ double rcp_nr(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}
__device__ __forceinline__ cd cdiv_sym(cd a, cd b) {
  const double den = cnonzero(b) ? rcp_nr(fma(b.x, b.x, b.y * b.y)) : 0.0;  // zero divisor -> 0
  return make_cd(fma(a.x, b.x, a.y * b.y) * den, fma(a.y, b.x, -a.x * b.y) * den);
}

#define CFP_C1 0.92387953251128675613  // cos(pi/8)
#define CFP_S1 0.38268343236508977173  // sin(pi/8)
#define CFP_H 0.70710678118654752440   // sqrt(1/2)

// v * W_R^k with W_R = exp(-2 pi i / R), R in {2,4,8,16}.  R and k are compile-time
// constants after unrolling, so every branch folds and trivial factors cost nothing.
template <int R>
__device__ __forceinline__ cd twr(cd v, int k) {
  const int e = (k * (16 / R)) & 15;  // exponent in units of 2 pi / 16
  const double x = v.x, y = v.y;
  switch (e) {
    case 0: return v;
    case 4: return make_cd(y, -x);                       // -i
    case 8: return make_cd(-x, -y);                      // -1
    case 12: return make_cd(-y, x);                      // +i
    case 2: return make_cd((x + y) * CFP_H, (y - x) * CFP_H);
    case 6: return make_cd((y - x) * CFP_H, -(x + y) * CFP_H);
    case 10: return make_cd(-(x + y) * CFP_H, (x - y) * CFP_H);
    case 14: return make_cd((x - y) * CFP_H, (x + y) * CFP_H);
    // odd multiples of pi/8: (x + iy)(c + i s), c = cos(2 pi e/16), s = -sin(2 pi e/16)
    case 1: return make_cd(fma(x, CFP_C1, y * CFP_S1), fma(y, CFP_C1, -x * CFP_S1));
    case 3: return make_cd(fma(x, CFP_S1, y * CFP_C1), fma(y, CFP_S1, -x * CFP_C1));
    case 5: return make_cd(fma(-x, CFP_S1, y * CFP_C1), fma(-y, CFP_S1, -x * CFP_C1));
    case 7: return make_cd(fma(-x, CFP_C1, y * CFP_S1), fma(-y, CFP_C1, -x * CFP_S1));
    case 9: return make_cd(fma(-x, CFP_C1, -y * CFP_S1), fma(-y, CFP_C1, x * CFP_S1));
    case 11: return make_cd(fma(-x, CFP_S1, -y * CFP_C1), fma(-y, CFP_S1, x * CFP_C1));
    case 13: return make_cd(fma(x, CFP_S1, -y * CFP_C1), fma(y, CFP_S1, x * CFP_C1));
    default: return make_cd(fma(x, CFP_C1, -y * CFP_S1), fma(y, CFP_C1, x * CFP_S1));  // 15
  }
}

__host__ __device__ constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }
__host__ __device__ constexpr int bitrev(int i, int bits) {
  return bits == 0 ? 0 : (((i & 1) << (bits - 1)) | bitrev(i >> 1, bits - 1));
}

// In-register forward DFT of R points, natural order in and out (radix-2 DIT, unrolled).
template <int R>
__device__ __forceinline__ void dft_reg(cd* v) {
  constexpr int LB = ilog2(R);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int j = bitrev(i, LB);
    if (i < j) { cd t = v[i]; v[i] = v[j]; v[j] = t; }
  }
#pragma unroll
  for (int len = 2; len <= R; len <<= 1) {
    const int half = len >> 1;
#pragma unroll
    for (int i = 0; i < R; i += len) {
#pragma unroll
      for (int k = 0; k < half; ++k) {
        cd u = v[i + k];
        cd t = twr<R>(v[i + k + half], k * (R / len));
        v[i + k] = cadd(u, t);
        v[i + k + half] = csub(u, t);
      }
    }
  }
}

// cos / sin(2 pi j / R), j = 0 .. R-1, for the odd in-register radices
template <int R> struct OddTab;
template <> struct OddTab<3> {
  static constexpr double C[3] = {1.0, -0.5, -0.5};
  static constexpr double S[3] = {0.0, 0.86602540378443864676, -0.86602540378443864676};
};
template <> struct OddTab<5> {
  static constexpr double C[5] = {1.0, 0.30901699437494742410, -0.80901699437494742410, -0.80901699437494742410,
                                  0.30901699437494742410};
  static constexpr double S[5] = {0.0, 0.95105651629515357212, 0.58778525229247312917, -0.58778525229247312917,
                                  -0.95105651629515357212};
};
template <> struct OddTab<7> {
  static constexpr double C[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429, -0.90096886790241912624,
                                  -0.90096886790241912624, -0.22252093395631440429, 0.62348980185873353053};
  static constexpr double S[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702, 0.43388373911755812048,
                                  -0.43388373911755812048, -0.97492791218182360702, -0.78183148246802980871};
};

// forward DFT of an odd R in registers, natural order: pairs a_t = x_t + x_{R-t},
// b_t = x_t - x_{R-t};  y_k = x_0 + sum a_t cos(2 pi k t / R) - i sum b_t sin(2 pi k t / R),
// y_{R-k} the same with +i.
template <int R>
__device__ __forceinline__ void dft_odd(cd* v) {
  constexpr int H = (R - 1) / 2;
  cd a[H], b[H];
#pragma unroll
  for (int t = 1; t <= H; ++t) {
    a[t - 1] = cadd(v[t], v[R - t]);
    b[t - 1] = csub(v[t], v[R - t]);
  }
  cd y0 = v[0];
#pragma unroll
  for (int t = 0; t < H; ++t) y0 = cadd(y0, a[t]);
  cd out[R];
  out[0] = y0;
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    double cr = v[0].x, ci = v[0].y, sr = 0.0, si = 0.0;
#pragma unroll
    for (int t = 1; t <= H; ++t) {
      const double c = OddTab<R>::C[(k * t) % R], sn = OddTab<R>::S[(k * t) % R];
      cr = fma(a[t - 1].x, c, cr);
      ci = fma(a[t - 1].y, c, ci);
      sr = fma(b[t - 1].x, sn, sr);
      si = fma(b[t - 1].y, sn, si);
    }
    // -i (sr + i si) = si - i sr
    out[k] = make_cd(cr + si, ci - sr);
    out[R - k] = make_cd(cr - si, ci + sr);
  }
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = out[k];
}

// 10 = 2 x 5, decimation in time: X[k] = E[k] + W10^k O[k], X[k+5] = E[k] - W10^k O[k] with
// E, O the 5-point DFTs of the even and odd samples
__device__ __forceinline__ void dft10(cd* v) {
  cd e[5], o[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    e[i] = v[2 * i];
    o[i] = v[2 * i + 1];
  }
  dft_odd<5>(e);
  dft_odd<5>(o);
  constexpr double c36 = 0.80901699437494742410, s36 = 0.58778525229247312917;
  constexpr double c72 = 0.30901699437494742410, s72 = 0.95105651629515357212;
  const double wr[5] = {1.0, c36, c72, -c72, -c36}, wi[5] = {0.0, -s36, -s72, -s72, -s36};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const cd t = k == 0 ? o[0] : cmul(o[k], make_cd(wr[k], wi[k]));
    v[k] = cadd(e[k], t);
    v[k + 5] = csub(e[k], t);
  }
}

// in-register DFT of any radix the fast pass uses: 2^k, odd 3 / 5 / 7, 10
template <int R>
__device__ __forceinline__ void dft_any(cd* v) {
  if constexpr ((R & (R - 1)) == 0) dft_reg<R>(v);
  else if constexpr (R == 10) dft10(v);
  else dft_odd<R>(v);
}

__host__ __device__ constexpr bool is_pow2c(int v) { return v > 0 && (v & (v - 1)) == 0; }
// log_b(v) when v is an exact power of b, else -1
__host__ __device__ constexpr int ilogb_exact(int v, int b) {
  return v == 1 ? 0 : (v % b != 0 ? -1 : (ilogb_exact(v / b, b) < 0 ? -1 : 1 + ilogb_exact(v / b, b)));
}

__device__ __forceinline__ i64 pt_off(const Side& s, int k) {
  return (i64)(k >> s.seg_shift) * s.seg_stride + (i64)(k & (s.seg_len - 1)) * s.pt_stride;
}
// point offset in a pass of length N: powers of two may be segmented (slab chunks, four-step
// halves); other lengths are plain strided columns (the host only routes those here)
template <int N>
__device__ __forceinline__ i64 kpt_off(const Side& s, int k) {
  if constexpr (is_pow2c(N)) return pt_off(s, k);
  else return (i64)k * s.pt_stride;
}
__device__ __forceinline__ i64 col_base(const Side& s, i64 g, i64 inner_n) {
  return (g % inner_n) * s.inner_stride + (g / inner_n) * s.outer_stride;
}

typedef double dv2 __attribute__((ext_vector_type(2)));
template <int FLAGS>
__device__ __forceinline__ cd gload(const cd* p) {
  if (FLAGS & (F_NT | F_NT_LD)) {
    dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p));
    return make_cd(v.x, v.y);
  }
  return *p;
}
// plain 16-byte load / store as a native vector (a HIP_vector_type assignment is a memcpy, which
// keeps register arrays of cd on the stack when they are filled in one loop and used in another)
__device__ __forceinline__ dv2 ldv(const cd* p) { return *reinterpret_cast<const dv2*>(p); }
__device__ __forceinline__ void stv(cd* p, dv2 v) { *reinterpret_cast<dv2*>(p) = v; }
__device__ __forceinline__ dv2 tov(cd v) {
  dv2 w;
  w.x = v.x;
  w.y = v.y;
  return w;
}
__device__ __forceinline__ cd fromv(dv2 v) { return make_cd(v.x, v.y); }

template <int FLAGS>
__device__ __forceinline__ void gstore(cd* p, cd v) {
  if (FLAGS & (F_NT | F_NT_ST)) {
    dv2 w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<dv2*>(p));
  } else {
    *p = v;
  }
}

struct KArgs {
  Side in, out;
  i64 inner_n;
  i64 ncols;  // columns of the pass (the last tile of a non-power-of-two pass may be partial)
  double scale;
  const cd* tw;
  const cd* colsym;
  const cd* axsym;
  const cd* diag;
  WaveSym wave;
  Tw4 tw4;
};

// W_n^e of a long axis' four-step twiddle (e < n <= 4096^2)
__device__ __forceinline__ cd tw4_at(const Tw4& t, i64 e) { return cmul(t.hi[e >> 12], t.lo[e & 4095]); }

// ------------------------------------------------------------ wave-system block symbol
// The periodic version of the wave-system operator (src/WaveSystem.cxx:92-176, 4 unknowns
// per cell: pressure, then the 3 momentum components) is block-circulant; its symbol at
// frequency theta is the arrowhead matrix
//   S = [ 1 + sum_d p_d    i c0^2 q_x   i c0^2 q_y   i c0^2 q_z ]
//       [ i q_x            1 + p_x      0            0          ]
//       [ i q_y            0            1 + p_y      0          ]
//       [ i q_z            0            0            1 + p_z    ]
// (p_d = kappa_d c0 (1 - cos theta_d), q_d = kappa_d sin theta_d, kappa_d = dt / h_d), so
// S^-1 r is: eliminate the momentum rows, solve the pressure row, back-substitute.  The two
// axes that are not transformed by the fused pass are constant along a column: their part is
// folded once per column (WaveCol); per point one reciprocal remains (wave_point).
struct WaveCol {
  double den;     // 1 + sum_nf p_d + c0^2 sum_nf q_d^2 / (1 + p_d)   (nf: non-fused axes)
  double w[3];    // q_d / (1 + p_d) for the non-fused axes, 0 for the fused one
  double qm, iem; // this lane's momentum row (comp = 1 + dm): q_dm and 1 / (1 + p_dm)
  bool mine_fused;
};

__device__ __forceinline__ WaveCol wave_col(const double2 pq[3], int fused, int comp, double c0sq) {
  WaveCol wc;
  wc.den = 1.0;
  wc.qm = 0.0;
  wc.iem = 1.0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const double ie = 1.0 / (1.0 + pq[d].x);
    const double w = pq[d].y * ie;
    const bool nf = d != fused;
    wc.w[d] = nf ? w : 0.0;
    if (nf) wc.den += pq[d].x + c0sq * pq[d].y * w;
    if (comp == 1 + d) { wc.qm = pq[d].y; wc.iem = ie; }
  }
  wc.mine_fused = comp == 1 + fused;
  return wc;
}

// component `comp` of S^-1 r at one point; pk = (p, q) of the fused axis at that point
__device__ __forceinline__ cd wave_point(const cd r[4], int comp, int f, const WaveCol& wc, double2 pk, double c0sq) {
  const double ef = 1.0 + pk.x;
  // den = den_nf + p_f + c0^2 q_f^2 / ef; with D2 = den * ef one reciprocal gives both 1/den
  // and 1/ef:  inv = 1 / (ef * D2),  1/den = ef^2 inv,  1/ef = D2 inv
  const double D2 = fma(wc.den + pk.x, ef, c0sq * pk.y * pk.y);
  const double inv = rcp_nr(ef * D2);  // ef >= 1, D2 >= 1
  const double id = ef * ef * inv, ief = D2 * inv;
  const double wf = pk.y * ief;
  cd t = make_cd(0.0, 0.0);
#pragma unroll
  for (int d = 0; d < 3; ++d) {  // weights select on the (uniform) fused axis, r is not indexed
    const double w = d == f ? wf : wc.w[d];
    t.x = fma(w, r[d + 1].x, t.x);
    t.y = fma(w, r[d + 1].y, t.y);
  }
  const cd x0 = make_cd(fma(c0sq, t.y, r[0].x) * id, fma(-c0sq, t.x, r[0].y) * id);
  cd rc = r[1];
#pragma unroll
  for (int j = 2; j < 4; ++j)
    if (comp == j) rc = r[j];
  const double qc = wc.mine_fused ? pk.y : wc.qm, iec = wc.mine_fused ? ief : wc.iem;
  const cd xm = make_cd(fma(qc, x0.y, rc.x) * iec, fma(-qc, x0.x, rc.y) * iec);
  return comp == 0 ? x0 : xm;
}

// reference version (generic kernel): the same algebra without the per-column hoisting
__device__ __forceinline__ cd wave_solve(const cd r[4], int comp, const double2 pq[3], double c0sq) {
  double ie[3];
  double den = 1.0 + pq[0].x + pq[1].x + pq[2].x;
  cd t = make_cd(0.0, 0.0);
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    ie[d] = 1.0 / (1.0 + pq[d].x);
    const double w = pq[d].y * ie[d];
    den = fma(c0sq * pq[d].y, w, den);
    t.x = fma(w, r[d + 1].x, t.x);
    t.y = fma(w, r[d + 1].y, t.y);
  }
  const double id = 1.0 / den;
  const cd x0 = make_cd(fma(c0sq, t.y, r[0].x) * id, fma(-c0sq, t.x, r[0].y) * id);
  cd rc = r[1];
  double qc = pq[0].y, iec = ie[0];
#pragma unroll
  for (int j = 2; j < 4; ++j)
    if (comp == j) { rc = r[j]; qc = pq[j - 1].y; iec = ie[j - 1]; }
  const cd xm = make_cd(fma(qc, x0.y, rc.x) * iec, fma(-qc, x0.x, rc.y) * iec);
  return comp == 0 ? x0 : xm;
}

// lane J of each aligned quad of lanes, broadcast to the quad (DPP quad_perm, VALU only)
template <int J>
__device__ __forceinline__ double quad_bcast(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), J * 0x55, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), J * 0x55, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// (p, q) of the two non-fused axes for the cell of column group `cell`
__device__ __forceinline__ void wave_cell_sym(const WaveSym& w, i64 cell, double2 pq[3]) {
  i64 idx[3] = {0, 0, 0};
  if (w.fused == 2) { idx[0] = cell % w.n[0]; idx[1] = cell / w.n[0]; }
  else if (w.fused == 1) { idx[0] = cell % w.n[0]; idx[2] = cell / w.n[0]; }
  else { idx[1] = cell % w.n[1]; idx[2] = cell / w.n[1]; }
#pragma unroll
  for (int d = 0; d < 3; ++d) pq[d] = d == w.fused ? make_double2(0.0, 0.0) : w.tab[d][idx[d]];
}

template <int N, int PTS, int R0>
struct Shape {
  static constexpr int TPC = N / PTS;
  static constexpr int QQ = PTS / R0;
  static constexpr int S = 1 + ilogb_exact(N / R0, PTS);
  static_assert(N % R0 == 0 && ilogb_exact(N / R0, PTS) >= 0, "N must be R0 * PTS^k");
  static_assert(PTS % R0 == 0, "R0 must divide PTS");
};

// LDS index of element idx of the workgroup's column c (row mode pads every 16 elements, or
// with F_PAD1 one element per row)
template <int N, bool ROW, int T, int FLAGS = 0>
__device__ __forceinline__ int lds_idx(int c, int idx) {
  if constexpr (FLAGS & F_PAD1) return ROW ? c * (N + 1) + idx : idx * T + c;
  constexpr int RS = N + N / 16;
  return ROW ? c * RS + idx + (idx >> 4) : idx * T + c;
}

// One LDS exchange: every thread writes its K values to positions wpos(k), then reads its
// PTS values from positions rpos(t).  `first` skips the barrier that protects the previous
// exchange's reads.  With F_SPLIT_LDS the real and imaginary halves go through a
// double-typed buffer one after the other.
template <int N, bool ROW, int T, int FLAGS, int K, int PTS, class WP, class RP>
__device__ __forceinline__ void exchange(void* ldsv, cd* vals, WP wpos, cd* dst, RP rpos, int c, bool first) {
  // vals may alias dst: all writes of a half complete (barrier) before its reads
  if (!first) xbarrier<FLAGS>();
  if (FLAGS & F_SPLIT_LDS) {
    double* lds = (double*)ldsv;
#pragma unroll
    for (int k = 0; k < K; ++k) lds[lds_idx<N, ROW, T, FLAGS>(c, wpos(k))] = vals[k].x;
    xbarrier<FLAGS>();
#pragma unroll
    for (int t = 0; t < PTS; ++t) dst[t].x = lds[lds_idx<N, ROW, T, FLAGS>(c, rpos(t))];
    xbarrier<FLAGS>();
#pragma unroll
    for (int k = 0; k < K; ++k) lds[lds_idx<N, ROW, T, FLAGS>(c, wpos(k))] = vals[k].y;
    xbarrier<FLAGS>();
#pragma unroll
    for (int t = 0; t < PTS; ++t) dst[t].y = lds[lds_idx<N, ROW, T, FLAGS>(c, rpos(t))];
  } else {
    cd* lds = (cd*)ldsv;
#pragma unroll
    for (int k = 0; k < K; ++k) lds[lds_idx<N, ROW, T, FLAGS>(c, wpos(k))] = vals[k];
    xbarrier<FLAGS>();
#pragma unroll
    for (int t = 0; t < PTS; ++t) dst[t] = lds[lds_idx<N, ROW, T, FLAGS>(c, rpos(t))];
  }
}

// All stages of one forward column FFT (registers in, registers out, natural order).
// `first` = no earlier LDS exchange in this kernel (skips one barrier).
template <int N, int PTS, int R0, bool ROW, int T, int FLAGS>
__device__ __forceinline__ void fft_stages(cd* v, void* lds, const cd* tws, int c, int tpc, bool first) {
  typedef Shape<N, PTS, R0> SH;
  constexpr int TPC = SH::TPC, QQ = SH::QQ, S = SH::S;
  if constexpr (S == 1) {
    dft_any<R0>(v);
    return;
  } else {
    // stage 0 (radix R0, Ns = 1, no twiddles): butterfly q works in place on slots
    // {q + t*QQ}; butterfly j = tpc + q*TPC writes data[j*R0 + t] from slot q + t*QQ
#pragma unroll
    for (int q = 0; q < QQ; ++q) {
      cd u[R0];
#pragma unroll
      for (int t = 0; t < R0; ++t) u[t] = v[q + t * QQ];
      dft_any<R0>(u);
#pragma unroll
      for (int t = 0; t < R0; ++t) v[q + t * QQ] = u[t];
    }
    exchange<N, ROW, T, FLAGS, PTS, PTS>(
        lds, v, [&](int k) { return (tpc + (k % QQ) * TPC) * R0 + (k / QQ); }, v,
        [&](int t) { return tpc + t * TPC; }, c, first);
    int Ns = R0;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      const int jm = tpc % Ns;  // Ns is a constant after unrolling: a mask for powers of two
      const int step = N / (Ns * PTS);
#pragma unroll
      for (int t = 1; t < PTS; ++t) v[t] = cmul(v[t], tws[jm * t * step]);
      dft_any<PTS>(v);
      if (s < S - 1) {
        const int o = (tpc / Ns) * Ns * PTS + jm;
        const int NsC = Ns;
        exchange<N, ROW, T, FLAGS, PTS, PTS>(
            lds, v, [&](int t) { return o + t * NsC; }, v, [&](int t) { return tpc + t * TPC; }, c, false);
      }
      Ns *= PTS;
    }
  }
}

// Two-stage column FFT (N = R0 PTS) whose exchange also permutes the columns: the thread writes
// its stage-0 values to column cw and reads column cr for stage 1, so the lane -> column map can
// change at the exchange (cfp_wave_three.hip: memory-friendly lanes for the global accesses,
// register-transposable lanes for the arrowhead solve).  cw and cr must be permutations of the
// same columns among the threads of one tpc; with cw == cr this is fft_stages.
// `mid(v)` runs right after the exchange, before stage 1's twiddles (a column-wise step in the
// new lane map that commutes with the FFT).
struct NoMid {
  __device__ void operator()(cd*) const {}
};
// With S > 2 stages the later exchanges stay in the new map (column cr); `last(v)` runs right
// after the last exchange's reads (the exchange buffer is then free; S = 2: after mid).
template <int N, int PTS, int R0, int T, int FLAGS, class MID = NoMid, class LAST = NoMid>
__device__ __forceinline__ void fft_stages_perm(cd* v, void* ldsv, const cd* tws, int cw, int cr, int tpc, bool first,
                                                MID mid = MID(), LAST last = LAST()) {
  typedef Shape<N, PTS, R0> SH;
  constexpr int TPC = SH::TPC, QQ = SH::QQ, S = SH::S;
  static_assert(S >= 2, "at least one exchange");
#pragma unroll
  for (int q = 0; q < QQ; ++q) {
    cd u[R0];
#pragma unroll
    for (int t = 0; t < R0; ++t) u[t] = v[q + t * QQ];
    dft_any<R0>(u);
#pragma unroll
    for (int t = 0; t < R0; ++t) v[q + t * QQ] = u[t];
  }
  const auto wpos = [&](int k) { return (tpc + (k % QQ) * TPC) * R0 + (k / QQ); };
  const auto rpos = [&](int t) { return tpc + t * TPC; };
  if (!first) xbarrier<FLAGS>();
  if constexpr ((FLAGS & F_SPLIT_LDS) != 0) {
    double* lds = (double*)ldsv;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h) xbarrier<FLAGS>();
#pragma unroll
      for (int k = 0; k < PTS; ++k) lds[lds_idx<N, false, T, FLAGS>(cw, wpos(k))] = h ? v[k].y : v[k].x;
      xbarrier<FLAGS>();
#pragma unroll
      for (int t = 0; t < PTS; ++t) {
        const double d = lds[lds_idx<N, false, T, FLAGS>(cr, rpos(t))];
        if (h) v[t].y = d; else v[t].x = d;
      }
    }
  } else {
    cd* lds = (cd*)ldsv;
#pragma unroll
    for (int k = 0; k < PTS; ++k) lds[lds_idx<N, false, T, FLAGS>(cw, wpos(k))] = v[k];
    xbarrier<FLAGS>();
#pragma unroll
    for (int t = 0; t < PTS; ++t) v[t] = lds[lds_idx<N, false, T, FLAGS>(cr, rpos(t))];
  }
  mid(v);
  if constexpr (S == 2) last(v);
  int Ns = R0;
#pragma unroll
  for (int s = 1; s < S; ++s) {
    const int jm = tpc % Ns;  // Ns is a constant after unrolling
    const int step = N / (Ns * PTS);
#pragma unroll
    for (int t = 1; t < PTS; ++t) v[t] = cmul(v[t], tws[jm * t * step]);
    dft_any<PTS>(v);
    if (s < S - 1) {
      const int o = (tpc / Ns) * Ns * PTS + jm;
      const int NsC = Ns;
      exchange<N, false, T, FLAGS, PTS, PTS>(
          ldsv, v, [&](int t) { return o + t * NsC; }, v, [&](int t) { return tpc + t * TPC; }, cr, false);
      if (s == S - 2) last(v);
    }
    Ns *= PTS;
  }
}

template <int N, int PTS, int R0, bool ROW, int T, int MODE, int FLAGS>
__global__ void __launch_bounds__(T*(N / PTS)) __attribute__((amdgpu_waves_per_eu(waves_req(FLAGS, MODE))))
k_axis_fast(const cd* in, cd* out, KArgs a) {
  typedef Shape<N, PTS, R0> SH;
  constexpr int TPC = SH::TPC;
  constexpr int NT = T * TPC;
  constexpr int LDS_N = ROW ? T * (N + N / 16) : T * N;
  constexpr bool NEED_LDS = SH::S > 1;
  constexpr bool TW_LDS = NEED_LDS && !(FLAGS & F_TW_GLOBAL);
  __shared__ __attribute__((aligned(16))) double lds_raw[NEED_LDS ? ((FLAGS & F_SPLIT_LDS) ? LDS_N : 2 * LDS_N) : 2];
  __shared__ cd tws_lds[TW_LDS ? N : 1];
  constexpr bool SYM_LDS = NEED_LDS && MODE == PASS_FUSED_SEP && (FLAGS & F_SYM_LDS);
  __shared__ cd axs_lds[SYM_LDS ? N : 1];

  const int tid = threadIdx.x;
  int c, tpc;
  if (ROW) { tpc = tid % TPC; c = tid / TPC; }
  else { c = tid % T; tpc = tid / T; }
  const unsigned blk = (FLAGS & F_REV) ? (gridDim.x - 1 - blockIdx.x) : blockIdx.x;
  // a partial last tile (non-power-of-two passes): its spare columns recompute the last column
  // and store nothing; they still take part in every barrier
  // (power-of-two passes always hold whole tiles: the host checks ncols % T, no guard code)
  constexpr bool GUARD = !is_pow2c(N);
  const i64 g0 = (i64)blk * T + c;
  const bool live = !GUARD || g0 < a.ncols;
  const i64 g = live ? g0 : a.ncols - 1;
  // point k = tpc + m*TPC: the bits of tpc and of m*TPC are disjoint and seg_len is a power
  // of two, so pt_off(k) = pt_off(tpc) + pt_off(m*TPC).  The first part is per thread (one
  // 64-bit VGPR base), the second is uniform per slot m (scalar ALU), so an access costs one
  // 64-bit add instead of two 64-bit multiplies.
  const i64 bin = col_base(a.in, g, a.inner_n) + kpt_off<N>(a.in, tpc);
  const i64 bout = col_base(a.out, g, a.inner_n) + kpt_off<N>(a.out, tpc);
  const cd* pin = in + bin;
  cd* pout = out + bout;

  // the column loads go out first; the table copies (L2 hits) queue behind them, so a wave's
  // HBM requests never wait on a twiddle round trip
  cd v[PTS];
#pragma unroll
  for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(pin + kpt_off<N>(a.in, m * TPC));

  const cd* tws = a.tw;
  if constexpr (TW_LDS) {
    for (int i = tid; i < N; i += NT) tws_lds[i] = a.tw[i];
    tws = tws_lds;
  }
  // fused separable pass: this column's symbol sum and (F_SYM_LDS) the per-point table, loaded
  // with the twiddles instead of after the forward transform
  const cd* axs = a.axsym;
  cd cs_early = make_cd(0.0, 0.0);
  if constexpr (MODE == PASS_FUSED_SEP) {
    cs_early = a.colsym[g];
    if constexpr (SYM_LDS) {
      for (int i = tid; i < N; i += NT) axs_lds[i] = a.axsym[i];
      axs = axs_lds;
    }
  }
  if (MODE == PASS_INV) {
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
  }
  if constexpr (MODE == PASS_INV) {
    if (a.tw4.lo) {  // uniform: the inverse of a long axis' first half, pre-twiddle
      const i64 k1 = (g / a.tw4.kdiv) % a.tw4.n1;
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cmul(v[m], tw4_at(a.tw4, k1 * (tpc + m * TPC)));
    }
  }
  // the twiddle table copy is published by the first exchange's barrier
  fft_stages<N, PTS, R0, ROW, T, FLAGS>(v, lds_raw, tws, c, tpc, true);

  if constexpr (MODE == PASS_FUSED_WAVE) {
    // the 4 components of a cell are columns 4j..4j+3: lanes of one quad (T % 4 == 0)
    double2 pc[3];
    wave_cell_sym(a.wave, g >> 2, pc);
    const int comp = c & 3;
    const double c0sq = a.wave.c0sq;
    const WaveCol wc = wave_col(pc, a.wave.fused, comp, c0sq);
    // the fused pass runs along the last non-trivial axis: z for 3-D grids
    const int f = a.wave.fused;
    const double2* tf = f == 0 ? a.wave.tab[0] : (f == 1 ? a.wave.tab[1] : a.wave.tab[2]);
#pragma unroll
    for (int m = 0; m < PTS; ++m) {
      const double2 pk = tf[tpc + m * TPC];
      cd r[4];
      r[0] = make_cd(quad_bcast<0>(v[m].x), quad_bcast<0>(v[m].y));
      r[1] = make_cd(quad_bcast<1>(v[m].x), quad_bcast<1>(v[m].y));
      r[2] = make_cd(quad_bcast<2>(v[m].x), quad_bcast<2>(v[m].y));
      r[3] = make_cd(quad_bcast<3>(v[m].x), quad_bcast<3>(v[m].y));
      v[m] = cconj(wave_point(r, comp, f, wc, pk, c0sq));
    }
    fft_stages<N, PTS, R0, ROW, T, FLAGS>(v, lds_raw, tws, c, tpc, false);
  }
  if (MODE == PASS_FUSED_SEP || MODE == PASS_FUSED_DIAG) {
    const cd cs = cs_early;
#pragma unroll
    for (int m = 0; m < PTS; ++m) {
      const int k = tpc + m * TPC;
      cd d;
      if (MODE == PASS_FUSED_SEP) {
        d = cadd(cadd(cs, axs[k]), make_cd(1.0, 0.0));
        v[m] = cconj(cdiv_sym(v[m], d));
      } else {
        d = a.diag[bin + kpt_off<N>(a.in, m * TPC)];
        v[m] = cconj(cdiv(v[m], d));
      }
    }
    fft_stages<N, PTS, R0, ROW, T, FLAGS>(v, lds_raw, tws, c, tpc, false);
  }
  if constexpr (MODE == PASS_FWD) {
    if (a.tw4.lo) {  // uniform: a long axis' first half, post-twiddle W_n^{k1 m2}
      const i64 k1 = (g / a.tw4.kdiv) % a.tw4.n1;
#pragma unroll
      for (int m = 0; m < PTS; ++m) v[m] = cmul(v[m], tw4_at(a.tw4, k1 * (tpc + m * TPC)));
    }
  }
  const bool conj_out = (MODE != PASS_FWD);
  const double sc = a.scale;
  if (GUARD && !live) return;  // after the last barrier
  if (sc == 1.0) {  // uniform: no 1/N on this pass, only the conjugation of the inverse
#pragma unroll
    for (int m = 0; m < PTS; ++m)
      gstore<FLAGS>(pout + kpt_off<N>(a.out, m * TPC), make_cd(v[m].x, conj_out ? -v[m].y : v[m].y));
    return;
  }
  const double sy = conj_out ? -sc : sc;
#pragma unroll
  for (int m = 0; m < PTS; ++m)
    gstore<FLAGS>(pout + kpt_off<N>(a.out, m * TPC), make_cd(v[m].x * sc, v[m].y * sy));
}

}  // namespace cfp
