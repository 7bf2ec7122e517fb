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
// Mixed-radix path (any n <= 4096, incl. primes; the reference's own 10, 100, 10x25x40 ...):
// LDS-resident Stockham, one specialised radix (8, 4, 2, 3, 5, 7) per stage, butterflies
// staged in VGPRs so the stages run in place in one LDS buffer.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "cfp_fft_device.h"

namespace cfp {

// Per-(N, layout, role) configuration of the fast kernel: points per thread (PTS), first
// stage radix (R0), columns (column mode) or rows (row mode) per workgroup (T) and variant
// FLAGS (cfp_fft_device.h).  Roles: 0 = forward pass, 1 = inverse pass, 2 = fused middle
// pass.  Shapes are the winners of isolated-kernel timing (tools/kexp/run_kexp.py); the
// load/store cache policy per role is the winner of an exhaustive whole-apply sweep
// (tools/kexp/run_sweep.py: every pass reads the previous pass's output, as in an apply),
// profiles/r01_kexp_sweep.txt: non-temporal loads where a pass reads data that is cold in
// the caches (the first pass reads b), non-temporal stores on the inverse passes.
template <int N, bool ROW, int ROLE> struct Cfg;
#define CFP_CFG(NN, ROWV, ROLE, P, R, TT, F)                               \
  template <> struct Cfg<NN, ROWV, ROLE> {                                 \
    static constexpr int PTS = P, R0 = R, T = TT, FLAGS = F, TPC = NN / P; \
  };
#define LD F_NT_LD
#define ST F_NT_ST
#define SPL F_SPLIT_LDS
// role:     fwd=0 inv=1 fused=2
//      N     row  role PTS R0  T   FLAGS
CFP_CFG(16, false, 0, 4, 4, 16, 0)
CFP_CFG(16, false, 1, 4, 4, 16, ST)
CFP_CFG(16, false, 2, 4, 4, 16, LD)
CFP_CFG(16, true, 0, 4, 4, 64, LD)
CFP_CFG(16, true, 1, 4, 4, 64, ST)
CFP_CFG(16, true, 2, 4, 4, 64, LD)
CFP_CFG(32, false, 0, 8, 4, 16, 0)
CFP_CFG(32, false, 1, 8, 4, 16, ST)
CFP_CFG(32, false, 2, 8, 4, 16, LD)
CFP_CFG(32, true, 0, 8, 4, 64, LD)
CFP_CFG(32, true, 1, 8, 4, 64, ST)
CFP_CFG(32, true, 2, 8, 4, 64, LD)
CFP_CFG(64, false, 0, 8, 8, 16, 0)
CFP_CFG(64, false, 1, 8, 8, 16, ST)
CFP_CFG(64, false, 2, 8, 8, 16, LD)
CFP_CFG(64, true, 0, 8, 8, 32, LD)
CFP_CFG(64, true, 1, 8, 8, 32, ST)
CFP_CFG(64, true, 2, 8, 8, 32, LD)
CFP_CFG(128, false, 0, 8, 2, 16, 0)
CFP_CFG(128, false, 1, 8, 2, 16, ST)
CFP_CFG(128, false, 2, 8, 2, 16, LD)
CFP_CFG(128, true, 0, 16, 8, 32, LD)
CFP_CFG(128, true, 1, 16, 8, 32, ST)
CFP_CFG(128, true, 2, 16, 8, 32, LD)
CFP_CFG(256, false, 0, 8, 4, 16, 0)
CFP_CFG(256, false, 1, 8, 4, 16, ST)
CFP_CFG(256, false, 2, 16, 16, 16, SPL | LD | F_OCC4)
CFP_CFG(256, true, 0, 8, 4, 8, LD)
CFP_CFG(256, true, 1, 8, 4, 8, ST)
CFP_CFG(256, true, 2, 8, 4, 8, LD)
CFP_CFG(512, false, 0, 16, 2, 16, SPL | LD)
CFP_CFG(512, false, 1, 16, 2, 16, SPL | ST)
CFP_CFG(512, false, 2, 8, 8, 8, LD)
CFP_CFG(512, true, 0, 16, 2, 8, LD)
CFP_CFG(512, true, 1, 16, 2, 8, ST)
CFP_CFG(512, true, 2, 16, 2, 8, LD)
CFP_CFG(1024, false, 0, 16, 4, 8, SPL | LD)
CFP_CFG(1024, false, 1, 16, 4, 8, SPL | ST)
CFP_CFG(1024, false, 2, 16, 4, 8, SPL | LD)
CFP_CFG(1024, true, 0, 16, 4, 4, SPL | LD)
CFP_CFG(1024, true, 1, 16, 4, 4, SPL | ST)
CFP_CFG(1024, true, 2, 16, 4, 4, SPL | LD)
// non-power-of-two lengths the reference uses (its ctests run 10, 10^2, 10^3 and 100^3; its
// default mesh is 100^3): radix-10 register stages, N = R0 * 10^(S-1)
CFP_CFG(10, false, 0, 10, 10, 64, 0)
CFP_CFG(10, false, 1, 10, 10, 64, ST)
CFP_CFG(10, false, 2, 10, 10, 64, LD)
CFP_CFG(10, true, 0, 10, 10, 64, LD)
CFP_CFG(10, true, 1, 10, 10, 64, ST)
CFP_CFG(10, true, 2, 10, 10, 64, LD)
CFP_CFG(20, false, 0, 10, 2, 32, 0)
CFP_CFG(20, false, 1, 10, 2, 32, ST)
CFP_CFG(20, false, 2, 10, 2, 32, LD)
CFP_CFG(20, true, 0, 10, 2, 32, LD)
CFP_CFG(20, true, 1, 10, 2, 32, ST)
CFP_CFG(20, true, 2, 10, 2, 32, LD)
CFP_CFG(50, false, 0, 10, 5, 64, 0)
CFP_CFG(50, false, 1, 10, 5, 64, ST)
CFP_CFG(50, false, 2, 10, 5, 64, LD)
CFP_CFG(50, true, 0, 10, 5, 64, LD)
CFP_CFG(50, true, 1, 10, 5, 64, ST)
CFP_CFG(50, true, 2, 10, 5, 64, LD)
CFP_CFG(100, false, 0, 10, 10, 32, 0)
CFP_CFG(100, false, 1, 10, 10, 32, ST)
CFP_CFG(100, false, 2, 10, 10, 16, LD)  // r03: T = 8, 32, 64 measured 1-3 % slower (profiles/r03l_t100.txt)
CFP_CFG(100, true, 0, 10, 10, 32, LD)
CFP_CFG(100, true, 1, 10, 10, 32, ST)
CFP_CFG(100, true, 2, 10, 10, 32, LD)
CFP_CFG(200, false, 0, 10, 2, 16, 0)
CFP_CFG(200, false, 1, 10, 2, 16, ST)
CFP_CFG(200, false, 2, 10, 2, 16, LD)
CFP_CFG(200, true, 0, 10, 2, 16, LD)
CFP_CFG(200, true, 1, 10, 2, 16, ST)
CFP_CFG(200, true, 2, 10, 2, 16, LD)
#undef SPL
#undef ST
#undef LD
#undef CFP_CFG

constexpr int role_of(int mode) { return mode == PASS_FWD ? 0 : (mode == PASS_INV ? 1 : 2); }

static bool is_pow2(i64 v) { return v > 0 && (v & (v - 1)) == 0; }

// row mode = the transform axis is contiguous (x); columns may be any 2-D set of rows
static bool row_mode(const PassDesc& p) {
  return p.in.pt_stride == 1 && p.out.pt_stride == 1 && p.in.seg_len == p.n && p.out.seg_len == p.n;
}

template <int NN>
static int tile_of(bool r, int role) {
  if (r) return role == 0 ? Cfg<NN, true, 0>::T : (role == 1 ? Cfg<NN, true, 1>::T : Cfg<NN, true, 2>::T);
  return role == 0 ? Cfg<NN, false, 0>::T : (role == 1 ? Cfg<NN, false, 1>::T : Cfg<NN, false, 2>::T);
}

static int fast_tile(const PassDesc& p) {
  const bool r = row_mode(p);
  const int role = role_of(p.mode);
  switch (p.n) {
#define CFP_TILE(NN) \
  case NN: return tile_of<NN>(r, role);
    CFP_TILE(16) CFP_TILE(32) CFP_TILE(64) CFP_TILE(128) CFP_TILE(256) CFP_TILE(512) CFP_TILE(1024)
    CFP_TILE(10) CFP_TILE(20) CFP_TILE(50) CFP_TILE(100) CFP_TILE(200)
#undef CFP_TILE
    default: return 0;
  }
}

bool fast_path_supported(const PassDesc& p) {
  const int T = fast_tile(p);
  if (T == 0) return false;
  if (!is_pow2(p.n)) {
    // radix-10 lengths: unsegmented sides only; any column count (the kernel guards a partial
    // last tile) and any inner grouping (every column computes its own base)
    if (p.in.seg_len < p.n || p.out.seg_len < p.n) return false;
    if (!row_mode(p) && (p.in.inner_stride != 1 || p.out.inner_stride != 1)) return false;
    if (p.mode == PASS_FUSED_WAVE && (row_mode(p) || T % 4 != 0 || p.wave.ncomp != 4 || p.ncols % 4 != 0))
      return false;
    return true;
  }
  if (!is_pow2(p.in.seg_len) || !is_pow2(p.out.seg_len)) return false;
  if (p.in.seg_shift < 0 || p.out.seg_shift < 0) return false;
  if (p.ncols % T != 0) return false;
  if (!row_mode(p)) {
    // a tile of T columns covers whole inner groups or lies inside one
    if (p.inner_n % T != 0 && T % p.inner_n != 0) return false;
    if (p.in.inner_stride != 1 || p.out.inner_stride != 1) return false;
  } else if (p.mode == PASS_FUSED_WAVE) {
    return false;
  }
  // the fast fused wave pass gathers a cell from the 4 lanes of a quad: 3-D only
  if (p.mode == PASS_FUSED_WAVE && (T % 4 != 0 || p.wave.ncomp != 4)) return false;
  return true;
}

template <int N, bool ROW, int MODE>
static hipError_t launch_fast_t(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  typedef Cfg<N, ROW, role_of(MODE)> C;
  const unsigned blocks = (unsigned)((p.ncols + C::T - 1) / C::T);
  hipLaunchKernelGGL((k_axis_fast<N, C::PTS, C::R0, ROW, C::T, MODE, C::FLAGS>), dim3(blocks), dim3(C::T * C::TPC),
                     0, s, in, out, a);
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
    case PASS_FUSED_DIAG: return launch_fast_t<N, ROWV, PASS_FUSED_DIAG>(p, in, out, a, s); \
    default: break;                                                               \
  }
  if (row) { CFP_M(true) } else {
    CFP_M(false)
    if (p.mode == PASS_FUSED_WAVE) return launch_fast_t<N, false, PASS_FUSED_WAVE>(p, in, out, a, s);
  }
#undef CFP_M
  return hipErrorInvalidValue;
}

// ----------------------------------------------------------------- mixed-radix path
// Any n <= 4096 (the reference's own sizes are 10, 100, 10x25x40, ...; its default Cartesian
// mesh is 100^3): an LDS-resident Stockham FFT with one radix per stage (8, 4, 2, 3, 5, 7 as
// specialised in-register butterflies, any other prime as a direct sum).  A block owns G
// columns (G a power of two in column mode, so the coalesced load / store of G consecutive
// columns splits its index with a shift); stages ping-pong between two LDS buffers with one
// barrier each; every runtime division (butterfly -> column, j mod Ns, row-mode index ->
// column) is a multiply by a 40-bit magic number.  The symbol / wave solve of the fused modes
// runs between the forward and the (conjugated) second transform, as in the fast path.
#define CFP_MR_THREADS 256
#define CFP_MR_MAXF 24
#define CFP_MR_POINTS 2048  // target points per block (one LDS buffer: 32 KiB)
#define CFP_MR_MAXPTS 2048  // most points per block of the in-place stages (larger: ping-pong)
#define CFP_MR_U 8          // most global loads in flight per thread (batched load loops)

struct MRStage {
  int r;         // radix
  int m;         // n / r butterflies per column
  int ns;        // product of the earlier radices
  int step;      // n / (ns r): twiddle W_n^{(j mod ns) step t}
  uint64_t m_M;  // magic of m
  uint64_t ns_M; // magic of ns
};

struct MRArgs {
  KArgs k;
  int n, G, gshift, L;  // points per column, columns per block, log2 G (column mode), LDS column stride
  uint64_t G_M;         // magic of G when G is not a power of two (column mode, 3-component cells)
  i64 ncols;
  int nst;
  MRStage st[CFP_MR_MAXF];
  uint64_t n_M;                 // magic of n (row-mode index split)
  uint64_t segin_M, segout_M;   // magic of the sides' segment lengths (split sides)
  int tw_lds;                   // twiddle table copied into LDS
  int pingpong;                 // a prime radix above 7: stages go A -> B (else in place, one buffer)
  int nbuf;                     // LDS buffers of G * L points (2 for ping-pong or the wave solve)
};

// f(integral_constant<int, 0>) ... f(integral_constant<int, U-1>): the batched loops' slot index is
// a front-end constant, so their register arrays never become stack (scratch) arrays
#define CFP_INLINE __attribute__((always_inline))
template <int U, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (U > 0) {
    static_for<U - 1>(f);
    f(std::integral_constant<int, U - 1>{});
  }
}

__host__ __device__ inline uint64_t mr_magic(uint32_t d) { return ((1ull << 40) + d - 1) / d; }
// floor(u / d) for u * d < 2^40 (u < 2^20, d <= 4096 here)
__device__ __forceinline__ uint32_t mr_div(uint32_t u, uint64_t M) { return (uint32_t)(((uint64_t)u * M) >> 40); }

__device__ __forceinline__ i64 mr_pt_off(const Side& s, int k, uint64_t segM) {
  if (k < s.seg_len) return (i64)k * s.pt_stride;  // unsplit side (or the first segment)
  const uint32_t q = mr_div((uint32_t)k, segM);
  return (i64)q * s.seg_stride + (i64)(k - (int)q * s.seg_len) * s.pt_stride;
}

// the odd specialised radices (OddTab / dft_odd) are in cfp_fft_device.h, shared with the fast path
template <int R>
__device__ __forceinline__ void dft_small(cd* v) {
  if constexpr (R == 2 || R == 4 || R == 8) dft_reg<R>(v);
  else dft_odd<R>(v);
}

// one Stockham stage of compile-time radix R: A -> B, every butterfly of the block's columns
template <int R>
__device__ __forceinline__ void mr_stage(const cd* __restrict__ A, cd* __restrict__ B, const MRStage& S,
                                         const cd* tw, int G, int L) {
  const int nb = G * S.m;
  for (int b = threadIdx.x; b < nb; b += CFP_MR_THREADS) {
    const int c = (int)mr_div((uint32_t)b, S.m_M);
    const int j = b - c * S.m;
    const int q = (int)mr_div((uint32_t)j, S.ns_M);
    const int jm = j - q * S.ns;
    const cd* a = A + c * L + j;
    cd v[R];
    v[0] = a[0];
    const int e = jm * S.step;
#pragma unroll
    for (int t = 1; t < R; ++t) v[t] = cmul(a[t * S.m], tw[e * t]);
    dft_small<R>(v);
    cd* o = B + c * L + q * S.ns * R + jm;
#pragma unroll
    for (int t = 0; t < R; ++t) o[t * S.ns] = v[t];
  }
}

// the same stage in place: every butterfly of this thread is read and transformed in VGPRs,
// then (after a barrier) written back -- one LDS buffer instead of two, so twice the blocks
// per CU.  QMAX bounds the butterflies per thread for blocks of at most CFP_MR_MAXPTS points.
template <int R>
__device__ __forceinline__ void mr_stage_inplace(cd* A, const MRStage& S, const cd* tw, int G, int L) {
  constexpr int QMAX = (CFP_MR_MAXPTS / R + CFP_MR_THREADS - 1) / CFP_MR_THREADS;
  const int nb = G * S.m;
  cd v[QMAX][R];
  int opos[QMAX];
#pragma unroll
  for (int qq = 0; qq < QMAX; ++qq) {
    const int b = threadIdx.x + qq * CFP_MR_THREADS;
    opos[qq] = -1;
    if (b < nb) {
      const int c = (int)mr_div((uint32_t)b, S.m_M);
      const int j = b - c * S.m;
      const int q = (int)mr_div((uint32_t)j, S.ns_M);
      const int jm = j - q * S.ns;
      const cd* a = A + c * L + j;
      v[qq][0] = a[0];
      const int e = jm * S.step;
#pragma unroll
      for (int t = 1; t < R; ++t) v[qq][t] = cmul(a[t * S.m], tw[e * t]);
      dft_small<R>(v[qq]);
      opos[qq] = c * L + q * S.ns * R + jm;
    }
  }
  __syncthreads();
#pragma unroll
  for (int qq = 0; qq < QMAX; ++qq) {
    if (opos[qq] >= 0) {
      cd* o = A + opos[qq];
#pragma unroll
      for (int t = 0; t < R; ++t) o[t * S.ns] = v[qq][t];
    }
  }
}

// a prime radix above 7: direct sums, W_R^{kt} = W_n^{((k t) mod R) m}
__device__ __forceinline__ void mr_stage_prime(const cd* __restrict__ A, cd* __restrict__ B, const MRStage& S,
                                               const cd* tw, int G, int L, int n) {
  const int R = S.r;
  const int nb = G * S.m * R;  // one output per thread iteration
  for (int i = threadIdx.x; i < nb; i += CFP_MR_THREADS) {
    const int b = i / R, k = i - b * R;
    const int c = (int)mr_div((uint32_t)b, S.m_M);
    const int j = b - c * S.m;
    const int q = (int)mr_div((uint32_t)j, S.ns_M);
    const int jm = j - q * S.ns;
    const cd* a = A + c * L + j;
    cd acc = make_cd(0.0, 0.0);
    for (int t = 0; t < R; ++t) {
      int ex = jm * S.step * t + ((k * t) % R) * S.m;
      if (ex >= n) ex -= n;
      acc = cadd(acc, cmul(a[t * S.m], tw[ex]));
    }
    B[c * L + q * S.ns * R + jm + k * S.ns] = acc;
  }
}

// all stages; the result ends in *X (the buffers are swapped as the stages go)
__device__ __forceinline__ void mr_fft(cd*& X, cd*& Y, const MRArgs& g, const cd* tw) {
  if (!g.pingpong) {
    for (int s = 0; s < g.nst; ++s) {
      const MRStage& S = g.st[s];
      switch (S.r) {
        case 2: mr_stage_inplace<2>(X, S, tw, g.G, g.L); break;
        case 3: mr_stage_inplace<3>(X, S, tw, g.G, g.L); break;
        case 4: mr_stage_inplace<4>(X, S, tw, g.G, g.L); break;
        case 5: mr_stage_inplace<5>(X, S, tw, g.G, g.L); break;
        case 7: mr_stage_inplace<7>(X, S, tw, g.G, g.L); break;
        default: mr_stage_inplace<8>(X, S, tw, g.G, g.L); break;
      }
      __syncthreads();
    }
    return;
  }
  for (int s = 0; s < g.nst; ++s) {
    const MRStage& S = g.st[s];
    switch (S.r) {
      case 2: mr_stage<2>(X, Y, S, tw, g.G, g.L); break;
      case 3: mr_stage<3>(X, Y, S, tw, g.G, g.L); break;
      case 4: mr_stage<4>(X, Y, S, tw, g.G, g.L); break;
      case 5: mr_stage<5>(X, Y, S, tw, g.G, g.L); break;
      case 7: mr_stage<7>(X, Y, S, tw, g.G, g.L); break;
      case 8: mr_stage<8>(X, Y, S, tw, g.G, g.L); break;
      default: mr_stage_prime(X, Y, S, tw, g.G, g.L, g.n); break;
    }
    __syncthreads();
    cd* t = X;
    X = Y;
    Y = t;
  }
}

// U = loads in flight per thread in the batched loops, sized to the block (2 / 4 / 8 for blocks of
// up to 512 / 1024 / more points) so a small block does not issue clamped duplicates
template <bool ROW, int U>
__global__ void __launch_bounds__(CFP_MR_THREADS) k_axis_mixed(const cd* in, cd* out, MRArgs g, int mode) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  __shared__ i64 base_in[64], base_out[64];
  const int n = g.n, G = g.G, L = g.L;
  cd* X = reinterpret_cast<cd*>(smem_raw);
  cd* Y = X + (size_t)G * L;  // second buffer (ping-pong stages, the wave solve's output)
  const cd* tw = g.k.tw;
  if (g.tw_lds) {  // batched: up to U global loads in flight per thread
    cd* t = X + (size_t)(g.nbuf * G * L);
    // clamped indices: the surplus slots copy tw[n-1] onto itself, so neither loop branches
    for (int i0 = threadIdx.x; i0 < n; i0 += CFP_MR_THREADS * U) {
      dv2 v[U];
      static_for<U>([&](auto u) CFP_INLINE { v[u] = ldv(g.k.tw + min(i0 + u * CFP_MR_THREADS, n - 1)); });
      static_for<U>([&](auto u) CFP_INLINE { stv(t + min(i0 + u * CFP_MR_THREADS, n - 1), v[u]); });
    }
    tw = t;
  }
  const i64 g0 = (i64)blockIdx.x * G;
  if (threadIdx.x < G) {
    const i64 gg = g0 + threadIdx.x;
    base_in[threadIdx.x] = gg < g.ncols ? col_base(g.k.in, gg, g.k.inner_n) : 0;
    base_out[threadIdx.x] = gg < g.ncols ? col_base(g.k.out, gg, g.k.inner_n) : 0;
  }
  __syncthreads();
  const int total = G * n;
  auto split = [&](int i, int& c, int& k) {
    if (ROW) { c = (int)mr_div((uint32_t)i, g.n_M); k = i - c * n; }
    else if (g.gshift >= 0) { k = i >> g.gshift; c = i & (G - 1); }
    else { k = (int)mr_div((uint32_t)i, g.G_M); c = i - k * G; }
  };
  // the column loads are batched U per thread (all in flight before the first LDS store):
  // a block of 2,048 points is one round trip to HBM instead of 8 dependent ones
  // (the loads are unconditional -- a clamped index, and base_in = 0 for a missing column -- so
  // the compiler issues them back to back without branches; the second loop drops the extras)
  // (surplus slots of the last batch repeat the last point: the same value to the same LDS slot)
  for (int i0 = threadIdx.x; i0 < total; i0 += CFP_MR_THREADS * U) {
    dv2 v[U];
    int cc[U], kk[U];
    static_for<U>([&](auto u) CFP_INLINE {
      split(min(i0 + u * CFP_MR_THREADS, total - 1), cc[u], kk[u]);
      v[u] = ldv(in + base_in[cc[u]] + mr_pt_off(g.k.in, kk[u], g.segin_M));  // base 0 for a missing column
    });
    static_for<U>([&](auto u) CFP_INLINE {
      const int c = cc[u], k = kk[u];
      cd v1 = g0 + c < g.ncols ? fromv(v[u]) : make_cd(0.0, 0.0);
      if (mode == PASS_INV) v1 = cconj(v1);
      if (mode == PASS_INV && g.k.tw4.lo) v1 = cmul(v1, tw4_at(g.k.tw4, ((g0 + c) / g.k.tw4.kdiv % g.k.tw4.n1) * k));
      stv(X + c * L + k, tov(v1));
    });
  }
  __syncthreads();
  mr_fft(X, Y, g, tw);
  if (mode == PASS_FUSED_WAVE) {
    // columns nc*j .. nc*j+nc-1 of the block are the nc = dim+1 components of one cell
    // (G % nc == 0, g0 % nc == 0); the missing momentum rows of dim < 3 are zero, and the
    // absent axes' symbol entries (n_d = 1) are p = q = 0, so the 4x4 algebra serves them
    const int nc = g.k.wave.ncomp;
    constexpr int UW = 4;  // symbol-table loads batched UW points per thread (clamped, unconditional)
    for (int i0 = threadIdx.x; i0 < total; i0 += CFP_MR_THREADS * UW) {
      dv2 pq[UW][3];
      int cu[UW], ku[UW];
      const WaveSym& w = g.k.wave;
      static_for<UW>([&](auto u) CFP_INLINE {
        split(min(i0 + u * CFP_MR_THREADS, total - 1), cu[u], ku[u]);
        const i64 cell = (g0 + cu[u] < g.ncols ? g0 + cu[u] : g0) / nc;
        // (p, q) per axis: the fused axis at frequency k, the other two at the cell's column
        // (wave_cell_sym); an absent axis (n = 1) reads its single entry (0, 0)
        i64 idx[3];
        if (w.fused == 2) { idx[0] = cell % w.n[0]; idx[1] = cell / w.n[0]; idx[2] = ku[u]; }
        else if (w.fused == 1) { idx[0] = cell % w.n[0]; idx[1] = ku[u]; idx[2] = cell / w.n[0]; }
        else { idx[0] = ku[u]; idx[1] = cell % w.n[1]; idx[2] = cell / w.n[1]; }
#pragma unroll
        for (int d = 0; d < 3; ++d) pq[u][d] = ldv(w.tab[d] + idx[d]);
      });
      static_for<UW>([&](auto u) CFP_INLINE {  // (Y is write-only here: surplus slots repeat the same value)
        const int c = cu[u], k = ku[u];
        const int comp = c % nc;
        const int cb = c - comp;
        cd r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = j < nc ? X[(cb + j) * L + k] : make_cd(0.0, 0.0);
        cd res = make_cd(0.0, 0.0);
        const double2 pq3[3] = {fromv(pq[u][0]), fromv(pq[u][1]), fromv(pq[u][2])};
        if (g0 + c < g.ncols) res = cconj(wave_solve(r, comp, pq3, w.c0sq));
        stv(Y + c * L + k, tov(res));
      });
    }
    __syncthreads();
    cd* t = X;
    X = Y;
    Y = t;
    mr_fft(X, Y, g, tw);
  } else if (mode == PASS_FUSED_SEP || mode == PASS_FUSED_DIAG) {
    // symbol loads batched like the column loads
    for (int i0 = threadIdx.x; i0 < total; i0 += CFP_MR_THREADS * U) {
      // a read-modify-write: the surplus slots must not repeat a point, they skip the store
      dv2 d[U];
      int pos[U];
      static_for<U>([&](auto u) CFP_INLINE {  // unconditional loads at clamped indices, as above
        int c, k;
        split(min(i0 + u * CFP_MR_THREADS, total - 1), c, k);
        const i64 gg = g0 + c;
        const bool ok = i0 + u * CFP_MR_THREADS < total && gg < g.ncols;
        pos[u] = ok ? c * L + k : -1;
        if (mode == PASS_FUSED_SEP) d[u] = ldv(g.k.colsym + (ok ? gg : g0)) + ldv(g.k.axsym + k);
        else d[u] = ldv(g.k.diag + base_in[c] + mr_pt_off(g.k.in, k, g.segin_M));
      });
      static_for<U>([&](auto u) CFP_INLINE {
        if (pos[u] < 0) return;
        const cd xv = fromv(ldv(X + pos[u]));
        cd r;
        if (mode == PASS_FUSED_SEP) r = cconj(cdiv_sym(xv, cadd(fromv(d[u]), make_cd(1.0, 0.0))));
        else r = cconj(cdiv(xv, fromv(d[u])));
        stv(X + pos[u], tov(r));
      });
    }
    __syncthreads();
    mr_fft(X, Y, g, tw);
  }
  const double sc = g.k.scale;
  const double sy = (mode != PASS_FWD) ? -sc : sc;
  for (int i = threadIdx.x; i < total; i += CFP_MR_THREADS) {
    int c, k;
    split(i, c, k);
    if (g0 + c < g.ncols) {
      cd v = X[c * L + k];
      if (mode == PASS_FWD && g.k.tw4.lo) v = cmul(v, tw4_at(g.k.tw4, ((g0 + c) / g.k.tw4.kdiv % g.k.tw4.n1) * k));
      out[base_out[c] + mr_pt_off(g.k.out, k, g.segout_M)] = make_cd(v.x * sc, v.y * sy);
    }
  }
}

static int factorize(int n, int* fac) {
  int nf = 0;
  while (n % 8 == 0 && n > 1 && nf < CFP_MR_MAXF) { fac[nf++] = 8; n /= 8; }
  static const int pref[] = {4, 2, 3, 5, 7};
  for (int r : pref) {
    while (n % r == 0 && n > 1 && nf < CFP_MR_MAXF) { fac[nf++] = r; n /= r; }
  }
  for (int p = 11; n > 1 && nf < CFP_MR_MAXF; p += 2) {
    while (n % p == 0) { fac[nf++] = p; n /= p; }
    if ((long long)p * p > n && n > 1) { fac[nf++] = n; n = 1; }
  }
  return nf;
}

static const size_t kMixedMaxLds = 160 * 1024 - 2 * 64 * sizeof(i64);  // minus the static base_in/base_out

static hipError_t launch_generic(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  if (p.n < 1 || p.n > 4096) return hipErrorNotSupported;
  const bool row = p.in.pt_stride == 1 && p.out.pt_stride == 1 && p.in.seg_len >= p.n && p.out.seg_len >= p.n;
  MRArgs g;
  std::memset(&g, 0, sizeof(g));
  g.k = a;
  g.n = p.n;
  g.ncols = p.ncols;
  int fac[CFP_MR_MAXF];
  g.nst = p.n == 1 ? 0 : factorize(p.n, fac);
  int G = CFP_MR_POINTS / p.n;  // points per block (block-size sweep: DESIGN.md, mixed-radix pass)
  if (G < 1) G = 1;
  if (G > 64) G = 64;
  if (!row) {  // power of two for the shift split
    int q = 1;
    while (q * 2 <= G) q *= 2;
    G = q;
  }
  if ((i64)G > p.ncols) {
    G = (int)p.ncols;
    if (!row) {
      int q = 1;
      while (q * 2 <= G) q *= 2;
      G = q;
    }
  }
  if (p.mode == PASS_FUSED_WAVE) {  // whole cells (ncomp columns) per block
    const int nc = p.wave.ncomp;
    if (nc < 2 || nc > 4 || p.ncols % nc != 0) return hipErrorInvalidValue;
    if (nc == 3) {  // 3 * 2^j columns; the column-mode index split divides by a magic number
      int q = 3;
      while (q * 2 <= G) q *= 2;
      G = q;
    } else {
      if (G < nc) G = nc;
      G &= ~(nc - 1);
    }
  }
  g.G = G;
  g.gshift = is_pow2(G) ? ilog2(G) : -1;
  g.G_M = mr_magic((uint32_t)G);
  g.L = row ? p.n : p.n + 1;
  int ns = 1;
  for (int i = 0; i < g.nst; ++i) {
    MRStage& S = g.st[i];
    S.r = fac[i];
    S.m = p.n / fac[i];
    S.ns = ns;
    S.step = p.n / (ns * fac[i]);
    S.m_M = mr_magic((uint32_t)S.m);
    S.ns_M = mr_magic((uint32_t)ns);
    ns *= fac[i];
  }
  g.n_M = mr_magic((uint32_t)p.n);
  g.segin_M = mr_magic((uint32_t)(p.in.seg_len > 0 ? p.in.seg_len : 1));
  g.segout_M = mr_magic((uint32_t)(p.out.seg_len > 0 ? p.out.seg_len : 1));
  g.pingpong = 0;
  for (int i = 0; i < g.nst; ++i)
    if (fac[i] > 8) g.pingpong = 1;
  if (G * p.n > CFP_MR_MAXPTS) g.pingpong = 1;
  g.nbuf = (g.pingpong || p.mode == PASS_FUSED_WAVE) ? 2 : 1;
  size_t lds = (size_t)g.nbuf * G * g.L * sizeof(cd);
  g.tw_lds = lds + (size_t)p.n * sizeof(cd) <= 96 * 1024 ? 1 : 0;
  if (g.tw_lds) lds += (size_t)p.n * sizeof(cd);
  if (lds > kMixedMaxLds) return hipErrorInvalidConfiguration;
  static bool attr_set = false;
  if (!attr_set) {
    const void* kf[] = {(const void*)k_axis_mixed<true, 2>, (const void*)k_axis_mixed<true, 4>,
                        (const void*)k_axis_mixed<true, 8>, (const void*)k_axis_mixed<false, 2>,
                        (const void*)k_axis_mixed<false, 4>, (const void*)k_axis_mixed<false, 8>};
    for (const void* f : kf) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMixedMaxLds);
    (void)hipGetLastError();  // a refused attribute must not surface as this launch's error
    attr_set = true;
  }
  const i64 blocks = (p.ncols + G - 1) / G;
  const int pts = G * p.n;
  const dim3 gr((unsigned)blocks), bl(CFP_MR_THREADS);
#define CFP_MR_LAUNCH(ROWV)                                                                          \
  if (pts <= 2 * CFP_MR_THREADS) hipLaunchKernelGGL((k_axis_mixed<ROWV, 2>), gr, bl, lds, s, in, out, g, p.mode); \
  else if (pts <= 4 * CFP_MR_THREADS) hipLaunchKernelGGL((k_axis_mixed<ROWV, 4>), gr, bl, lds, s, in, out, g, p.mode); \
  else hipLaunchKernelGGL((k_axis_mixed<ROWV, 8>), gr, bl, lds, s, in, out, g, p.mode);
  if (row) { CFP_MR_LAUNCH(true) } else { CFP_MR_LAUNCH(false) }
#undef CFP_MR_LAUNCH
  return hipGetLastError();
}

hipError_t launch_axis_pass(const PassDesc& p, const cd* in, cd* out, const cd* tw, hipStream_t s) {
  KArgs a;
  a.in = p.in;
  a.out = p.out;
  a.inner_n = p.inner_n;
  a.ncols = p.ncols;
  a.scale = p.scale;
  a.tw = tw;
  a.colsym = p.colsym;
  a.axsym = p.axsym;
  a.diag = p.diag;
  a.wave = p.wave;
  a.tw4 = p.tw4;
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
      case 10: return launch_fast_n<10>(p, in, out, a, s);
      case 20: return launch_fast_n<20>(p, in, out, a, s);
      case 50: return launch_fast_n<50>(p, in, out, a, s);
      case 100: return launch_fast_n<100>(p, in, out, a, s);
      case 200: return launch_fast_n<200>(p, in, out, a, s);
      default: break;
    }
  }
  return launch_generic(p, in, out, a, s);
}

// ----------------------------------------------------------------- plane pass
// The x and y DFTs of one whole n x n z-plane per workgroup (n * n/PTS <= 1024 threads, the
// plane staged through LDS: PlaneCfg), so the apply of an
// n^2 x n_z grid is 3 sweeps -- plane forward, the fused z pass, plane inverse -- instead of 5.
// At the reference's default mesh (100^3) the five passes are launch-cost bound (11-15 us for a
// 32 MB sweep that sits in the Infinity Cache; profiles/r02r_100_kernel_stats.md).
//   forward: rows (thread = row y, points x = t + m TPC, row mode) -> x DFT -> transpose through
//            LDS -> columns (thread = column kx, points y) -> y DFT -> coalesced store along kx
//   inverse: the mirror (conjugated input, column y DFT first, row x DFT, conjugate * scale)
// SPLIT: the plane moves through LDS in real / imaginary halves (n (n + n/16) doubles), else
// whole complex values with rows padded by one element (n (n + 1) complex: 158 KiB at n = 100)
template <int N> struct PlaneCfg;
template <> struct PlaneCfg<32> { static constexpr int PTS = 8, R0 = 4; static constexpr bool SPLIT = false; };
template <> struct PlaneCfg<64> { static constexpr int PTS = 8, R0 = 8; static constexpr bool SPLIT = false; };
template <> struct PlaneCfg<100> { static constexpr int PTS = 10, R0 = 10; static constexpr bool SPLIT = false; };
template <> struct PlaneCfg<128> { static constexpr int PTS = 16, R0 = 8; static constexpr bool SPLIT = true; };

// static LDS of k_plane<N>: the plane buffer plus the twiddle table.  It must fit one gfx950
// CU's 160 KiB (k_plane<100> uses 163,200 of the 163,840 bytes); this library builds for gfx950
// only (Makefile --offload-arch=gfx950), and a config change that overflows fails to compile.
template <int N>
constexpr size_t plane_lds_bytes() {
  return (PlaneCfg<N>::SPLIT ? sizeof(double) * N * (N + N / 16) : sizeof(double) * 2 * N * (N + 1)) +
         sizeof(cd) * N;
}
constexpr size_t kGfx950LdsBytes = 160 * 1024;
static_assert(plane_lds_bytes<32>() <= kGfx950LdsBytes, "k_plane<32> exceeds the CU's LDS");
static_assert(plane_lds_bytes<64>() <= kGfx950LdsBytes, "k_plane<64> exceeds the CU's LDS");
static_assert(plane_lds_bytes<100>() <= kGfx950LdsBytes, "k_plane<100> exceeds the CU's LDS");
static_assert(plane_lds_bytes<128>() <= kGfx950LdsBytes, "k_plane<128> exceeds the CU's LDS");

// element (y, x) of the plane at LDS y * N + x
template <int N, int PTS, int FLAGS, class WP, class RP>
__device__ __forceinline__ void plane_transpose(double* lds, cd* v, WP wpos, RP rpos) {
  xbarrier<FLAGS>();  // the previous exchange's reads
  if constexpr (!(FLAGS & F_SPLIT_LDS)) {
    cd* l = (cd*)lds;
#pragma unroll
    for (int m = 0; m < PTS; ++m) l[wpos(m)] = v[m];
    xbarrier<FLAGS>();
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = l[rpos(m)];
    return;
  }
#pragma unroll
  for (int m = 0; m < PTS; ++m) lds[wpos(m)] = v[m].x;
  xbarrier<FLAGS>();
#pragma unroll
  for (int m = 0; m < PTS; ++m) v[m].x = lds[rpos(m)];
  xbarrier<FLAGS>();
#pragma unroll
  for (int m = 0; m < PTS; ++m) lds[wpos(m)] = v[m].y;
  xbarrier<FLAGS>();
#pragma unroll
  for (int m = 0; m < PTS; ++m) v[m].y = lds[rpos(m)];
}

template <int N, bool INV>
__global__ void __launch_bounds__(N*(N / PlaneCfg<N>::PTS)) k_plane(const cd* in, cd* out, const cd* tw, double scale) {
  constexpr int PTS = PlaneCfg<N>::PTS, R0 = PlaneCfg<N>::R0, TPC = N / PTS, NT = N * TPC;
  // the forward pass reads b (cold); the inverse writes x (not read again by this apply)
  constexpr bool SPLIT = PlaneCfg<N>::SPLIT;
  constexpr int FLAGS = (SPLIT ? F_SPLIT_LDS : F_PAD1) | (INV ? F_NT_ST : F_NT_LD);
  __shared__ __attribute__((aligned(16))) double lds[SPLIT ? N * (N + N / 16) : 2 * N * (N + 1)];
  __shared__ cd tws[N];
  const int tid = threadIdx.x;
  const int ry = tid / TPC, rt = tid % TPC;  // row mode: row y, points x = rt + m TPC
  const int cx = tid % N, ct = tid / N;      // column mode: column x, points y = ct + m TPC
  const i64 base = (i64)blockIdx.x * N * N;
  const cd* pin = in + base;
  cd* pout = out + base;
  cd v[PTS];
  if (!INV) {
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(pin + ry * N + rt + m * TPC);
  } else {
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = gload<FLAGS>(pin + (ct + m * TPC) * N + cx);
  }
  for (int i = tid; i < N; i += NT) tws[i] = tw[i];  // published by the first exchange's barrier
  if (!INV) {
    fft_stages<N, PTS, R0, true, N, FLAGS>(v, lds, tws, ry, rt, true);
    plane_transpose<N, PTS, FLAGS>(
        lds, v, [&](int m) { return ry * N + rt + m * TPC; }, [&](int m) { return (ct + m * TPC) * N + cx; });
    fft_stages<N, PTS, R0, false, N, FLAGS>(v, lds, tws, cx, ct, false);
#pragma unroll
    for (int m = 0; m < PTS; ++m) gstore<FLAGS>(pout + (ct + m * TPC) * N + cx, v[m]);
  } else {
#pragma unroll
    for (int m = 0; m < PTS; ++m) v[m] = cconj(v[m]);
    fft_stages<N, PTS, R0, false, N, FLAGS>(v, lds, tws, cx, ct, true);
    plane_transpose<N, PTS, FLAGS>(
        lds, v, [&](int m) { return (ct + m * TPC) * N + cx; }, [&](int m) { return ry * N + rt + m * TPC; });
    fft_stages<N, PTS, R0, true, N, FLAGS>(v, lds, tws, ry, rt, false);
    const double sy = -scale;
#pragma unroll
    for (int m = 0; m < PTS; ++m) gstore<FLAGS>(pout + ry * N + rt + m * TPC, make_cd(v[m].x * scale, v[m].y * sy));
  }
}

// gated on the static_asserts above (the kernels are only built when they fit gfx950's LDS)
bool plane_supported(i64 n) { return n == 32 || n == 64 || n == 100 || n == 128; }

template <int N>
static hipError_t launch_plane_t(bool inverse, i64 planes, const cd* in, cd* out, const cd* tw, double scale,
                                 hipStream_t s) {
  constexpr int NT = N * (N / PlaneCfg<N>::PTS);
  if (inverse) hipLaunchKernelGGL((k_plane<N, true>), dim3((unsigned)planes), dim3(NT), 0, s, in, out, tw, scale);
  else hipLaunchKernelGGL((k_plane<N, false>), dim3((unsigned)planes), dim3(NT), 0, s, in, out, tw, scale);
  return hipGetLastError();
}

hipError_t launch_plane_pass(bool inverse, int n, i64 planes, const cd* in, cd* out, const cd* tw, double scale,
                             hipStream_t s) {
  if (planes <= 0) return hipSuccess;
  switch (n) {
    case 32: return launch_plane_t<32>(inverse, planes, in, out, tw, scale, s);
    case 64: return launch_plane_t<64>(inverse, planes, in, out, tw, scale, s);
    case 100: return launch_plane_t<100>(inverse, planes, in, out, tw, scale, s);
    case 128: return launch_plane_t<128>(inverse, planes, in, out, tw, scale, s);
    default: return hipErrorNotSupported;
  }
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

// the symbol divide of a grid whose long axes are split (no short axis to fuse it into):
// x[i] /= ((sx[ix] + sy[iy]) + sz[iz]) + 1, the reference's summation order, position-indexed
__global__ void k_sym_divide_positions(cd* x, const cd* sx, const cd* sy, const cd* sz, i64 nx, i64 ny, i64 N) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (i64)gridDim.x * blockDim.x) {
    const i64 ix = i % nx, iy = (i / nx) % ny, iz = i / (nx * ny);
    const cd d = cadd(cadd(cadd(sx[ix], sy[iy]), sz[iz]), make_cd(1.0, 0.0));
    x[i] = cdiv(x[i], d);
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
hipError_t launch_sym_divide_positions(cd* x, const cd* sx, const cd* sy, const cd* sz, i64 nx, i64 ny, i64 nz,
                                       hipStream_t s) {
  const i64 N = nx * ny * nz;
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sym_divide_positions, dim3(ew_blocks(N)), dim3(CFP_EW_THREADS), 0, s, x, sx, sy, sz, nx, ny, N);
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
