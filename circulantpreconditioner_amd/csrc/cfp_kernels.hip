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
CFP_CFG(1024, true, 0, 16, 4, 4, LD)
CFP_CFG(1024, true, 1, 16, 4, 4, ST)
CFP_CFG(1024, true, 2, 16, 4, 4, LD)
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
    // a tile of T columns covers whole inner groups or lies inside one
    if (p.inner_n % T != 0 && T % p.inner_n != 0) return false;
    if (p.in.inner_stride != 1 || p.out.inner_stride != 1) return false;
  } else if (p.mode == PASS_FUSED_WAVE) {
    return false;
  }
  if (p.mode == PASS_FUSED_WAVE && T % 4 != 0) return false;
  return true;
}

template <int N, bool ROW, int MODE>
static hipError_t launch_fast_t(const PassDesc& p, const cd* in, cd* out, const KArgs& a, hipStream_t s) {
  typedef Cfg<N, ROW, role_of(MODE)> C;
  const unsigned blocks = (unsigned)(p.ncols / C::T);
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
  if (mode == PASS_FUSED_WAVE) {
    // columns 4j..4j+3 of the block are the 4 components of one cell (G % 4 == 0)
    for (int i = threadIdx.x; i < G * n; i += blockDim.x) {
      const int c = i / n, k = i - c * n;
      const i64 gg = g0 + c;
      if (gg >= g.ncols) continue;
      double2 pq[3];
      wave_cell_sym(g.k.wave, gg >> 2, pq);
      pq[g.k.wave.fused] = g.k.wave.tab[g.k.wave.fused][k];
      cd r[4];
      const int c4 = c & ~3;
      for (int j = 0; j < 4; ++j) r[j] = A[(c4 + j) * n + k];
      B[i] = cconj(wave_solve(r, c & 3, pq, g.k.wave.c0sq));
    }
    __syncthreads();
    cd* tmp = A; A = B; B = tmp;
    gen_fft(A, B, g, G);
  }
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
  if (p.mode == PASS_FUSED_WAVE) {  // whole cells (4 columns) per block
    if (G < 4) G = 4;
    G &= ~3;
    if (p.ncols % 4 != 0) return hipErrorInvalidValue;
  }
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
  a.wave = p.wave;
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
