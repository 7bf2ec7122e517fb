// cfp_internal.h -- shared device/host definitions of the MI355X circulant FFT library.
//
// Data model: complex double, interleaved (re, im) = double2,
// grid index i = ix + nx*(iy + ny*iz) (x fastest), i.e. row-major {nz, ny, nx} as the
// reference's MatCreateFFT(..., dims={nz,ny,nx}) (src/PCSHELLFft_3D.cxx:34-35).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cfp {

typedef double2 cd;
typedef long long i64;

// Per-launch profiling of the apply (cfp_plan_profile_begin / cfp_plan_time_passes): while
// `start` is set, the 3-sweep launch sites (cfp_three_pass.hip) stamp their dispatch itself with
// hipExtLaunchKernel's start / stop events, i.e. the kernel's own execution as rocprofv3 sees
// it.  Separate event packets between back-to-back kernels leave the device idle for ~4-5 us
// each, which inflated every measured pass by that much (profiles/r03z_256_kernel_stats.md).
struct LaunchStamp {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchStamp g_stamp;
// The stand-in KSP's PCApply timing (ksp_gmres.cpp): while set, an apply whose steps are all
// 3-sweep kernels stamps its first kernel's start into `start` and its last kernel's end into
// `stop` (hits = 2): the apply's device time without event packets around it.
struct ApplyStamp {
  hipEvent_t start = nullptr, stop = nullptr;
  int hits = 0;
};
extern thread_local ApplyStamp g_apply_stamp;

// How the points of one FFT column are addressed on one side (input or output) of an
// axis pass.  Column g (0 <= g < ncols) starts at
//     base(g) = (g % inner_n) * inner_stride + (g / inner_n) * outer_stride
// and point k (0 <= k < n) of that column sits at
//     base(g) + (k >> seg_shift) * seg_stride + (k & seg_mask) * pt_stride.
// An unsplit axis has seg_len = n (seg_shift large).  A split axis is what the slab
// transposes of the multi-GPU path produce: the y axis cut into P segments of n/P points,
// each segment in its own peer chunk.
struct Side {
  i64 inner_stride;
  i64 outer_stride;
  i64 pt_stride;
  i64 seg_stride;
  int seg_shift;  // log2(seg_len) when seg_len is a power of two, else -1 (generic kernel only)
  int seg_len;
};

enum PassMode : int {
  PASS_FWD = 0,         // out = scale * DFT(in)             (forward, e^{-})
  PASS_INV = 1,         // out = scale * IDFT(in)            (backward, e^{+}, unnormalised)
  PASS_FUSED_SEP = 2,   // out = scale * IDFT( DFT(in) / (colsym[g] + axsym[k]) )
  PASS_FUSED_DIAG = 3,  // out = scale * IDFT( DFT(in) / diag[same addressing as in] )
  PASS_FUSED_WAVE = 4,  // out = scale * IDFT( S(k)^-1 DFT(in) ), S = the 4x4 wave-system block
                        // symbol; the 4 components of a cell are 4 consecutive columns
  // launches of the 3-sweep schedule (cfp_three_pass.hip); reported, not dispatched here
  PASS_TP_ROWS_FWD = 5,  // x DFT + the 64-point stage of the y DFT
  PASS_TP_MID = 6,       // 4-point y stage + z DFT, symbol, and their inverses
  PASS_TP_ROWS_INV = 7,  // inverse of PASS_TP_ROWS_FWD, x 1/N
  // long axes (n = n1 n2 > 4096, four-step) with no short axis to fuse: the symbol divide as
  // its own sweep over the position-ordered spectrum (cfp_plan.hip); reported, not dispatched
  PASS_SYM_DIVIDE = 8,
  // plane schedule (n_x = n_y small): x and y DFTs of whole z-planes in one launch
  PASS_PLANE_FWD = 9,
  PASS_PLANE_INV = 10,
};

// Four-step twiddle of a long axis split n = n1 n2 (index k1 + n1 k2): the length-n2 pass over
// k2 multiplies its output m2 of column group k1 by W_n^{k1 m2} (forward), or its input by the
// same factor after the inverse's conjugation.  k1 = (g / kdiv) % n1 for column g;
// W_n^e = hi[e >> 12] * lo[e & 4095].
struct Tw4 {
  const cd* lo = nullptr;  // W_n^j, j < 4096   (NULL: no four-step twiddle on this pass)
  const cd* hi = nullptr;  // W_n^{4096 i}, i <= n / 4096
  i64 kdiv = 1;
  int n1 = 1;
};

// Separable parts of the wave-system block symbol (cfp_wave.hip): for axis d and frequency
// index k, p = kappa_d c0 (1 - cos theta), q = kappa_d sin theta, theta = 2 pi k / n_d.
struct WaveSym {
  const double2* tab[3];  // [n_d] (p, q) per axis
  i64 n[3];               // grid sizes (cells)
  double c0sq;            // c0^2
  int fused;              // axis transformed by the fused pass
  int ncomp;              // unknowns per cell: dim + 1 (pressure, dim momentum components)
};

struct PassDesc {
  int n;          // points per column (FFT length along the axis)
  i64 ncols;      // number of columns
  i64 inner_n;    // columns are enumerated inner-fastest: g = inner + inner_n * outer
  Side in, out;
  int mode;
  double scale;
  const cd* colsym;  // [ncols]   (PASS_FUSED_SEP)
  const cd* axsym;   // [n]       (PASS_FUSED_SEP)
  const cd* diag;    // addressed like `in` (PASS_FUSED_DIAG)
  WaveSym wave;      // PASS_FUSED_WAVE
  Tw4 tw4;           // four-step twiddle (PASS_FWD / PASS_INV of a long axis' first half)
};

__host__ __device__ inline cd make_cd(double x, double y) { cd r; r.x = x; r.y = y; return r; }

// Launchers (cfp_kernels.hip).  tw = forward twiddle table W_n[k] = exp(-2 pi i k / n), k < n.
hipError_t launch_axis_pass(const PassDesc& p, const cd* in, cd* out, const cd* tw, hipStream_t s);
bool fast_path_supported(const PassDesc& p);
// plane pass: the x and y DFTs of `planes` whole n x n z-planes in one launch (forward, or the
// conjugated inverse with `scale`); plane_supported(n) lists the built n
bool plane_supported(i64 n);
hipError_t launch_plane_pass(bool inverse, int n, i64 planes, const cd* in, cd* out, const cd* tw, double scale,
                             hipStream_t s);
hipError_t launch_pointwise_divide(cd* w, const cd* x, const cd* y, i64 n, hipStream_t s);
hipError_t launch_scale(cd* x, cd alpha, i64 n, hipStream_t s);
hipError_t launch_fill_uniform(cd* x, i64 n, uint64_t seed, i64 offset, hipStream_t s);
hipError_t launch_build_diag_separable(cd* diag, const cd* cx, const cd* cy, const cd* cz, i64 nx, i64 ny,
                                       i64 nz, cd lx, cd ly, cd lz, hipStream_t s);
hipError_t launch_sym_divide_inplace(cd* x, const cd* colsym, const cd* axsym, i64 n, hipStream_t s);
// x[i] /= 1 + sx[ix] + sy[iy] + sz[iz] over an nx*ny*nz grid (position-indexed symbol tables)
hipError_t launch_sym_divide_positions(cd* x, const cd* sx, const cd* sy, const cd* sz, i64 nx, i64 ny, i64 nz,
                                       hipStream_t s);

}  // namespace cfp
