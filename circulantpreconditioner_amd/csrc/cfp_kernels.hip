// cfp_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the circulant FFT preconditioner.
//
// One kernel family does all of the FFT work: an *axis pass* that transforms a batch of
// columns of one grid axis (x: contiguous rows, y/z: strided columns), optionally fused
// with the reference's pointwise divide and 1/N scale:
//
//   reference (src/FftLinearSolver_3D.c:166-190)      this file
//   MatMult(FFT_MAT, b, b_hat)      -> 3 passes       x-fwd, y-fwd, z-fwd  -+ the last forward
//   VecPointwiseDivide(b_hat,...)   -> fused          z: DFT ./Diag IDFT   -+ pass, the divide and
//   MatMultTranspose(FFT_MAT, ...)  -> 3 passes       y-inv, x-inv*(1/N)      the first inverse
//   VecScale(X, 1./size)            -> fused                                  pass are one kernel
//
// so one PCApply is 5 sweeps over HBM instead of the reference's 6 FFT sweeps plus 2
// vector sweeps.
//
// Fast path (n a power of two, 16..1024): Stockham autosort FFT.  Each thread owns PTS
// points of one column in VGPRs and runs radix-PTS butterflies in registers; stages
// exchange through LDS; the twiddle table W_n is staged in LDS once per workgroup.
// Strided axes (y, z) give each workgroup T consecutive columns, so every wave-wide load
// or store moves T*16 contiguous bytes per row of the tile; the contiguous axis (x) gives
// each workgroup whole rows.
// Generic path (any n <= 4096, incl. primes): LDS-resident mixed-radix Stockham with
// direct O(r) sums per output, used for sizes the fast path does not instantiate.
#include "cfp_internal.h"

namespace cfp {

// ------------------------------------------------------------------ complex helpers
__device__ __forceinline__ cd cadd(cd a, cd b) { return make_cd(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd csub(cd a, cd b) { return make_cd(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cd cmul(cd a, cd b) {
  return make_cd(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ cd cconj(cd a) { return make_cd(a.x, -a.y); }
// a / b = (a * conj(b)) / |b|^2, the complex VecPointwiseDivide of the reference (:174)
__device__ __forceinline__ cd cdiv(cd a, cd b) {
  double den = 1.0 / fma(b.x, b.x, b.y * b.y);
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

__device__ __forceinline__ i64 pt_off(const Side& s, int k) {
  return (i64)(k >> s.seg_shift) * s.seg_stride + (i64)(k & (s.seg_len - 1)) * s.pt_stride;
}
__device__ __forceinline__ i64 col_base(const Side& s, i64 g, i64 inner_n) {
  return (g % inner_n) * s.inner_stride + (g / inner_n) * s.outer_stride;
}

struct KArgs {
  Side in, out;
  i64 inner_n;
  double scale;
  const cd* tw;
  const cd* colsym;
  const cd* axsym;
  const cd* diag;
};

// ----------------------------------------------------------------- fast path
// Shape of one column FFT: N = R0 * PTS^(S-1); TPC = N/PTS threads per column, each
// holding PTS points.  Register slot m of thread tpc always holds point tpc + m*TPC on
// input and output (natural order), so a forward transform's output can feed an inverse
// transform straight from registers (the fused middle pass).
template <int N, int PTS, int R0>
struct Shape {
  static constexpr int TPC = N / PTS;
  static constexpr int QQ = PTS / R0;
  static constexpr int S = 1 + (ilog2(N / R0) / ilog2(PTS));
  static_assert(R0 * (1 << (ilog2(PTS) * (S - 1))) == N, "N must be R0 * PTS^k");
};

// Stockham stages.  Stage s (radix r, Ns = product of earlier radices) maps butterfly j:
//   in  : data[j + t*N/r] * W_{Ns r}^{(j mod Ns) t}
//   out : data[(j/Ns)*Ns*r + (j mod Ns) + t*Ns]
template <int N, int PTS, int R0, bool ROW, int T>
__device__ __forceinline__ void fft_stages(cd* v, cd* lds, const cd* tws, int c, int tpc, bool sync_first) {
  typedef Shape<N, PTS, R0> SH;
  constexpr int TPC = SH::TPC, QQ = SH::QQ, S = SH::S;
  constexpr int RS = N + N / 16;  // padded row stride (row mode)
  auto L = [&](int idx) -> int { return ROW ? c * RS + idx + (idx >> 4) : idx * T + c; };
  if constexpr (S == 1) {
    dft_reg<R0>(v);
    return;
  } else {
    if (sync_first) __syncthreads();
#pragma unroll
    for (int q = 0; q < QQ; ++q) {
      cd u[R0];
#pragma unroll
      for (int t = 0; t < R0; ++t) u[t] = v[q + t * QQ];
      dft_reg<R0>(u);
      const int j = tpc + q * TPC;
#pragma unroll
      for (int t = 0; t < R0; ++t) lds[L(j * R0 + t)] = u[t];
    }
    __syncthreads();
    int Ns = R0;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      cd u[PTS];
#pragma unroll
      for (int t = 0; t < PTS; ++t) u[t] = lds[L(tpc + t * TPC)];
      const int jm = tpc & (Ns - 1);
      const int step = N / (Ns * PTS);
#pragma unroll
      for (int t = 1; t < PTS; ++t) u[t] = cmul(u[t], tws[jm * t * step]);
      dft_reg<PTS>(u);
      if (s == S - 1) {
#pragma unroll
        for (int t = 0; t < PTS; ++t) v[t] = u[t];
      } else {
        __syncthreads();
        const int o = (tpc / Ns) * Ns * PTS + jm;
#pragma unroll
        for (int t = 0; t < PTS; ++t) lds[L(o + t * Ns)] = u[t];
        __syncthreads();
      }
      Ns *= PTS;
    }
  }
}

template <int N, int PTS, int R0, bool ROW, int T, int MODE>
__global__ void __launch_bounds__(T*(N / PTS)) k_axis_fast(const cd* in, cd* out, KArgs a) {
  typedef Shape<N, PTS, R0> SH;
  constexpr int TPC = SH::TPC;
  constexpr int NT = T * TPC;
  constexpr int LDS_N = ROW ? T * (N + N / 16) : T * N;
  __shared__ cd lds[SH::S > 1 ? LDS_N : 1];
  __shared__ cd tws[SH::S > 1 ? N : 1];

  const int tid = threadIdx.x;
  int c, tpc;
  if (ROW) { tpc = tid % TPC; c = tid / TPC; }
  else { c = tid % T; tpc = tid / T; }
  const i64 g = (i64)blockIdx.x * T + c;
  const i64 bin = col_base(a.in, g, a.inner_n);
  const i64 bout = col_base(a.out, g, a.inner_n);

  if constexpr (SH::S > 1) {
    for (int i = tid; i < N; i += NT) tws[i] = a.tw[i];
  }

  cd v[PTS];
#pragma unroll
  for (int m = 0; m < PTS; ++m) v[m] = in[bin + pt_off(a.in, tpc + m * TPC)];
  if (MODE == PASS_INV) {
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
  }
  fft_stages<N, PTS, R0, ROW, T>(v, lds, tws, c, tpc, false);

  if (MODE == PASS_FUSED_SEP || MODE == PASS_FUSED_DIAG) {
    cd cs = make_cd(0.0, 0.0);
    if (MODE == PASS_FUSED_SEP) cs = a.colsym[g];
#pragma unroll
    for (int m = 0; m < PTS; ++m) {
      const int k = tpc + m * TPC;
      cd d;
      if (MODE == PASS_FUSED_SEP) {
        d = cadd(cadd(cs, a.axsym[k]), make_cd(1.0, 0.0));
      } else {
        d = a.diag[bin + pt_off(a.in, k)];
      }
      v[m] = cconj(cdiv(v[m], d));
    }
    fft_stages<N, PTS, R0, ROW, T>(v, lds, tws, c, tpc, true);
  }
  const bool conj_out = (MODE != PASS_FWD);
  const double sc = a.scale;
  const double sy = conj_out ? -sc : sc;
#pragma unroll
  for (int m = 0; m < PTS; ++m) {
    out[bout + pt_off(a.out, tpc + m * TPC)] = make_cd(v[m].x * sc, v[m].y * sy);
  }
}

// Per-N configuration: (PTS, R0, T_col).  Row mode packs 256 threads' worth of rows.
template <int N> struct Cfg;
template <> struct Cfg<16> { static constexpr int PTS = 4, R0 = 4, TCOL = 16; };
template <> struct Cfg<32> { static constexpr int PTS = 8, R0 = 4, TCOL = 16; };
template <> struct Cfg<64> { static constexpr int PTS = 8, R0 = 8, TCOL = 16; };
template <> struct Cfg<128> { static constexpr int PTS = 16, R0 = 8, TCOL = 16; };
template <> struct Cfg<256> { static constexpr int PTS = 16, R0 = 16, TCOL = 16; };
template <> struct Cfg<512> { static constexpr int PTS = 16, R0 = 2, TCOL = 8; };
template <> struct Cfg<1024> { static constexpr int PTS = 16, R0 = 4, TCOL = 4; };

template <int N>
struct FastCfg {
  static constexpr int PTS = Cfg<N>::PTS, R0 = Cfg<N>::R0, TCOL = Cfg<N>::TCOL;
  static constexpr int TPC = N / PTS;
  static constexpr int TROW = (256 / TPC) > 0 ? (256 / TPC) : 1;
};

static bool is_pow2(i64 v) { return v > 0 && (v & (v - 1)) == 0; }

static bool row_mode(const PassDesc& p) {
  return p.inner_n == 1 && p.in.pt_stride == 1 && p.out.pt_stride == 1 && p.in.seg_len == p.n &&
         p.out.seg_len == p.n;
}

static int fast_tile(const PassDesc& p) {
  switch (p.n) {
#define CFP_TILE(NN) \
  case NN: return row_mode(p) ? FastCfg<NN>::TROW : FastCfg<NN>::TCOL;
    CFP_TILE(16) CFP_TILE(32) CFP_TILE(64) CFP_TILE(128) CFP_TILE(256) CFP_TILE(512) CFP_TILE(1024)
#undef CFP_TILE
    default: return 0;
  }
}

bool fast_path_supported(const PassDesc& p) {
  const int T = fast_tile(p);
  if (T == 0) return false;
  if (!is_pow2(p.in.seg_len) || !is_pow2(p.out.seg_len)) return false;
  if (p.in.seg_shift < 0 || p.out.seg_shift < 0) return false;
  if (p.ncols % T != 0) return false;
  if (!row_mode(p)) {
    if (p.inner_n % T != 0) return false;
    if (p.in.inner_stride != 1 || p.out.inner_stride != 1) return false;
  }
  return true;
}

template <int N, bool ROW, int MODE>
static hipError_t launch_fast_t(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  typedef FastCfg<N> C;
  constexpr int T = ROW ? C::TROW : C::TCOL;
  const unsigned blocks = (unsigned)(p.ncols / T);
  hipLaunchKernelGGL((k_axis_fast<N, C::PTS, C::R0, ROW, T, MODE>), dim3(blocks), dim3(T * C::TPC), 0, s, in,
                     out, a);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_fast_n(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  const bool row = row_mode(p);
#define CFP_M(ROWV)                                                               \
  switch (p.mode) {                                                               \
    case PASS_FWD: return launch_fast_t<N, ROWV, PASS_FWD>(p, in, out, a, s);     \
    case PASS_INV: return launch_fast_t<N, ROWV, PASS_INV>(p, in, out, a, s);     \
    case PASS_FUSED_SEP: return launch_fast_t<N, ROWV, PASS_FUSED_SEP>(p, in, out, a, s); \
    default: return launch_fast_t<N, ROWV, PASS_FUSED_DIAG>(p, in, out, a, s);    \
  }
  if (row) { CFP_M(true) } else { CFP_M(false) }
#undef CFP_M
}

// ----------------------------------------------------------------- generic path
#define CFP_GEN_THREADS 256
#define CFP_MAX_FACTORS 32

struct GArgs {
  KArgs k;
  int n;
  int ncol_per_block;
  i64 ncols;
  int nfac;
  int fac[CFP_MAX_FACTORS];
};

__device__ __forceinline__ i64 pt_off_gen(const Side& s, int k) {
  return (i64)(k / s.seg_len) * s.seg_stride + (i64)(k % s.seg_len) * s.pt_stride;
}

__device__ void gen_fft(cd*& A, cd*& B, const GArgs& g, int G) {
  const int n = g.n;
  int Ns = 1;
  for (int f = 0; f < g.nfac; ++f) {
    const int r = g.fac[f];
    const int nr = n / r;
    const int st1 = n / (Ns * r);
    for (int i = threadIdx.x; i < G * n; i += blockDim.x) {
      const int c = i / n, o = i - c * n;
      const int q = o / Ns;
      const int t = q % r;
      const int jm = o % Ns;
      const int j = (q / r) * Ns + jm;
      const cd* col = A + c * n;
      cd acc = make_cd(0.0, 0.0);
      // exponent of W_n for input s: s * (jm*st1 + t*nr)  (mod n)
      const int inc = (int)(((long long)jm * st1 + (long long)t * nr) % n);
      int e = 0;
      for (int sidx = 0; sidx < r; ++sidx) {
        acc = cadd(acc, cmul(col[j + sidx * nr], g.k.tw[e]));
        e += inc;
        if (e >= n) e -= n;
      }
      B[c * n + o] = acc;
    }
    __syncthreads();
    cd* tmp = A; A = B; B = tmp;
    Ns *= r;
  }
}

__global__ void __launch_bounds__(CFP_GEN_THREADS) k_axis_generic(const cd* in, cd* out, GArgs g, int mode) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  cd* sm = reinterpret_cast<cd*>(smem_raw);
  const int n = g.n, G = g.ncol_per_block;
  cd* A = sm;
  cd* B = sm + (size_t)G * n;
  const i64 g0 = (i64)blockIdx.x * G;
  for (int i = threadIdx.x; i < G * n; i += blockDim.x) {
    const int c = i / n, k = i - c * n;
    const i64 gg = g0 + c;
    cd v = make_cd(0.0, 0.0);
    if (gg < g.ncols) v = in[col_base(g.k.in, gg, g.k.inner_n) + pt_off_gen(g.k.in, k)];
    if (mode == PASS_INV) v = cconj(v);
    A[i] = v;
  }
  __syncthreads();
  gen_fft(A, B, g, G);
  if (mode == PASS_FUSED_SEP || mode == PASS_FUSED_DIAG) {
    for (int i = threadIdx.x; i < G * n; i += blockDim.x) {
      const int c = i / n, k = i - c * n;
      const i64 gg = g0 + c;
      if (gg >= g.ncols) continue;
      cd d;
      if (mode == PASS_FUSED_SEP) d = cadd(cadd(g.k.colsym[gg], g.k.axsym[k]), make_cd(1.0, 0.0));
      else d = g.k.diag[col_base(g.k.in, gg, g.k.inner_n) + pt_off_gen(g.k.in, k)];
      A[i] = cconj(cdiv(A[i], d));
    }
    __syncthreads();
    gen_fft(A, B, g, G);
  }
  const double sc = g.k.scale;
  const double sy = (mode != PASS_FWD) ? -sc : sc;
  for (int i = threadIdx.x; i < G * n; i += blockDim.x) {
    const int c = i / n, k = i - c * n;
    const i64 gg = g0 + c;
    if (gg < g.ncols) out[col_base(g.k.out, gg, g.k.inner_n) + pt_off_gen(g.k.out, k)] = make_cd(A[i].x * sc, A[i].y * sy);
  }
}

static int factorize(int n, int* fac) {
  int nf = 0;
  static const int pref[] = {16, 8, 4, 2, 3, 5, 7};
  for (int r : pref) {
    while (n % r == 0 && n > 1 && nf < CFP_MAX_FACTORS) { fac[nf++] = r; n /= r; }
  }
  for (int p = 11; n > 1 && nf < CFP_MAX_FACTORS; p += 2) {
    while (n % p == 0) { fac[nf++] = p; n /= p; }
    if ((long long)p * p > n && n > 1) { fac[nf++] = n; n = 1; }
  }
  return nf;
}

static const size_t kGenericMaxLds = 160 * 1024;

static hipError_t launch_generic(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  if (p.n < 1 || p.n > 4096) return hipErrorInvalidValue;
  GArgs g;
  g.k = a;
  g.n = p.n;
  g.ncols = p.ncols;
  g.nfac = p.n == 1 ? 0 : factorize(p.n, g.fac);
  int G = 2048 / p.n;
  if (G < 1) G = 1;
  if (G > 64) G = 64;
  if ((i64)G > p.ncols) G = (int)p.ncols;
  g.ncol_per_block = G;
  const size_t lds = (size_t)2 * G * p.n * sizeof(cd);
  if (lds > kGenericMaxLds) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_axis_generic, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGenericMaxLds);
    attr_set = true;
  }
  const i64 blocks = (p.ncols + G - 1) / G;
  hipLaunchKernelGGL(k_axis_generic, dim3((unsigned)blocks), dim3(CFP_GEN_THREADS), lds, s, in, out, g, p.mode);
  return hipGetLastError();
}

hipError_t launch_axis_pass(const PassDesc& p, const cd* in, cd* out, const cd* tw, hipStream_t s) {
  KArgs a;
  a.in = p.in;
  a.out = p.out;
  a.inner_n = p.inner_n;
  a.scale = p.scale;
  a.tw = tw;
  a.colsym = p.colsym;
  a.axsym = p.axsym;
  a.diag = p.diag;
  if (p.ncols <= 0) return hipSuccess;
  if (fast_path_supported(p)) {
    switch (p.n) {
      case 16: return launch_fast_n<16>(p, in, out, a, s);
      case 32: return launch_fast_n<32>(p, in, out, a, s);
      case 64: return launch_fast_n<64>(p, in, out, a, s);
      case 128: return launch_fast_n<128>(p, in, out, a, s);
      case 256: return launch_fast_n<256>(p, in, out, a, s);
      case 512: return launch_fast_n<512>(p, in, out, a, s);
      case 1024: return launch_fast_n<1024>(p, in, out, a, s);
      default: break;
    }
  }
  return launch_generic(p, in, out, a, s);
}

// ----------------------------------------------------------------- elementwise kernels
#define CFP_EW_THREADS 256

__global__ void k_pointwise_divide(cd* w, const cd* x, const cd* y, i64 n) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
    w[i] = cdiv(x[i], y[i]);
}
__global__ void k_scale(cd* x, cd alpha, i64 n) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
    x[i] = cmul(x[i], alpha);
}
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// SURVEY.md §8d synthetic input: Re, Im ~ U[-1,1) from SplitMix64(seed ^ 2i), (seed ^ 2i+1)
__global__ void k_fill_uniform(cd* x, i64 n, uint64_t seed, i64 offset) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    const uint64_t gi = (uint64_t)(i + offset);
    const uint64_t a = splitmix64(seed ^ (2 * gi)), b = splitmix64(seed ^ (2 * gi + 1));
    x[i] = make_cd((double)(a >> 11) * 0x1.0p-52 - 1.0, (double)(b >> 11) * 0x1.0p-52 - 1.0);
  }
}
// build_diag_mat_vec_3D (src/FftLinearSolver_3D.c:136-164), all three Kronecker tilings in
// one sweep: Diag[i] = ((lx*cx[ix] + ly*cy[iy]) + lz*cz[iz]) + 1
__global__ void k_build_diag(cd* d, const cd* cx, const cd* cy, const cd* cz, i64 nx, i64 ny, i64 nz, cd lx, cd ly,
                             cd lz) {
  const i64 N = nx * ny * nz;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (i64)gridDim.x * blockDim.x) {
    const i64 ix = i % nx, iy = (i / nx) % ny, iz = i / (nx * ny);
    cd s = cmul(cx[ix], lx);
    s = cadd(s, cmul(cy[iy], ly));
    s = cadd(s, cmul(cz[iz], lz));
    d[i] = cadd(s, make_cd(1.0, 0.0));
  }
}

static unsigned ew_blocks(i64 n) {
  i64 b = (n + CFP_EW_THREADS - 1) / CFP_EW_THREADS;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

hipError_t launch_pointwise_divide(cd* w, const cd* x, const cd* y, i64 n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pointwise_divide, dim3(ew_blocks(n)), dim3(CFP_EW_THREADS), 0, s, w, x, y, n);
  return hipGetLastError();
}
hipError_t launch_scale(cd* x, cd alpha, i64 n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scale, dim3(ew_blocks(n)), dim3(CFP_EW_THREADS), 0, s, x, alpha, n);
  return hipGetLastError();
}
hipError_t launch_fill_uniform(cd* x, i64 n, uint64_t seed, i64 offset, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_uniform, dim3(ew_blocks(n)), dim3(CFP_EW_THREADS), 0, s, x, n, seed, offset);
  return hipGetLastError();
}
hipError_t launch_build_diag_separable(cd* diag, const cd* cx, const cd* cy, const cd* cz, i64 nx, i64 ny, i64 nz,
                                       cd lx, cd ly, cd lz, hipStream_t s) {
  const i64 N = nx * ny * nz;
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_build_diag, dim3(ew_blocks(N)), dim3(CFP_EW_THREADS), 0, s, diag, cx, cy, cz, nx, ny, nz, lx,
                     ly, lz);
  return hipGetLastError();
}

}  // namespace cfp
