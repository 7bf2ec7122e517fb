// cfp_three_pass.h -- the 3-sweep apply for 128^3 and 256^3 grids (cfp_three_pass.hip).
#pragma once
#include "cfp_internal.h"

namespace cfp {

// Row sweeps (P1 / P3 of the scalar and wave 3-sweeps) with units in XCD order
// (r05j-r05l, cfp_three_pass.hip kRowsXCD; the real-data rows keep blockIdx order).
// -DCFP_ROWS_XCD=0 builds the blockIdx order for A/B.
#ifndef CFP_ROWS_XCD
#define CFP_ROWS_XCD 1
#endif

struct TPArgs {
  const cd* tw;      // W_n[k] = exp(-2 pi i k / n), n = the grid side (128 or 256)
  const cd* colsym;  // separable symbol, z fused: [kx + n ky] = s_x[kx] + s_y[ky] (global ky)
  const cd* axsym;   // [kz] = s_z[kz]
  double scale;      // P3 only: 1/N
  // z-slab layout (cfp_dist.hip); the defaults are one GPU's natural layout.
  //   P1 writes / P3 reads the per-peer exchange chunks: row y of local plane z at
  //   (y >> lnyl) * chunk + (z << lnyl) * n + (y & (nyl - 1)) * n;  P2 runs on [n z][nyl][nx]
  //   with the k1 range [k1_off, k1_off + nyl / N2) of the four-step split.
  int lnyl = 0;     // log2 of the rows per chunk (0: nyl = n, one chunk)
  i64 chunk = 0;    // elements per peer chunk
  int k1_off = 0;   // first global k1 of this rank (P2)
  // Fused Krylov work of the stand-in GMRES (one GPU, natural layout; r06, launch_three_pass_fused):
  // P1 reads A b instead of b, A an x-row-local stencil in row-class diagonal form (cfp_blas.h
  // DiaDesc: diagonals -1, 0, +1 only, no entry across an x-row end); P3 adds the workgroup partial
  // sums of post_v[j]^H x (j < post_nv; bit j of post_self: x itself, i.e. |x|^2) to post_partial
  // [blockIdx][2 j + re/im], the k_mdot layout (cfp_blas.hip k_mdot_finish).
  const unsigned char* pre_cls = nullptr;   // [N] row class
  const unsigned char* pre_cls_x = nullptr; // optional [n]: row r's class is pre_cls_x[r mod n]
  const unsigned char* pre_mask = nullptr;  // [ncls] diagonals present per class (bit k: pre_off[k])
  const cd* pre_tab = nullptr;              // [ncls][pre_nd] coefficients
  int pre_nd = 0, pre_ncls = 0;
  int pre_off[3] = {0, 0, 0};
  const cd* post_v[4] = {nullptr, nullptr, nullptr, nullptr};
  int post_nv = 0;
  int post_self = 0;  // bit j: post_v[j] is x itself (NULL)
  double* post_partial = nullptr;
  // 1: this apply runs inside the stand-in KSP (a fused Krylov step, cfp_plan_apply_ex, or a
  // PCApply the KSP times).  Its P2 is the same kernel under a second instantiation, so that a
  // kernel trace lists the in-solver P2 apart from the bare apply's (the two run at different
  // clocks); no effect on the work.
  int krylov = 0;
};


// kernel shape at 256^3 (cfp_plan_set_three_pass_shape); zeros = the measured default
// BLOCKED: SWAP64_PF with the blocked intermediate layout (k_tp_rows<.., 8>; N1 = 32 only);
// at 512^3 blocks of 2 x (one P2 tile)
// BLOCKED32: blocks of 4 x and the permlane P2 on 32 columns, two workgroups per CU; at 512^3
// blocks of 8 x (P1 / P3 move whole 128-byte lines; r05i)
// SWAP32X: the permlane P2 on 32 columns (4 x times 8 y2, natural layout: 64-byte tiles), two
// workgroups per CU, units in XCD order (r04)
// ROWSALT: the default shape (n1 = 0 only; 128^3, 256^3, 512^3) with P1 / P3's row-FFT exchanges
// the other way (workgroup barriers instead of wave-local, or the reverse: kRowsWave), for A/B
enum { TP_MID_DEFAULT = 0, TP_MID_LANE64 = 1, TP_MID_LANE32 = 2, TP_MID_SWAP64 = 3, TP_MID_SWAP64_PF = 4,
       TP_MID_BLOCKED = 5, TP_MID_BLOCKED32 = 6, TP_MID_SWAP32X = 7, TP_MID_ROWSALT = 8 };
struct TPShape {
  int n1 = 0;   // y split ny = n1 * n2: 0 (default 32), 32 or 64
  int mid = 0;  // TP_MID_* (DEFAULT = SWAP64_PF at 256^3)
};

// the fused stencil's limits (LDS table in P1)
#define TP_PRE_MAX_CLS 16
#define TP_POST_MAX 4
// stage 0 with the stencil (a.pre_*), 2 with the dots (a.post_*): 256^3 default shape only
bool three_pass_fused_supported(int n, TPShape shape);
hipError_t launch_three_pass_fused(int stage, int n, const cd* in, cd* out, const TPArgs& a, hipStream_t s,
                                   unsigned* grid_out);

bool three_pass_supported(const i64 n[3]);
// 100^3 (n = R^2, R = 10: cfp_three_pass_sq.hip); launch_three_pass routes n = 100 there.
// shape.mid picks its middle kernel's x tile: DEFAULT 4 x, LANE64 2 x, LANE32 5 x
bool three_pass_sq_supported(const i64 n[3]);
hipError_t launch_three_pass_sq(int stage, int n, const cd* in, cd* out, const TPArgs& a, TPShape shape,
                                hipStream_t s);
// n: the grid side (0: any); n1 = 16 (y split 16 x 8) is built for 128^3 only
bool three_pass_shape_valid(int n1, int mid, i64 n = 0);
// stage 0: P1 (in -> out), 1: P2 (out in place), 2: P3 (in -> out)
hipError_t launch_three_pass(int stage, int n, const cd* in, cd* out, const TPArgs& a, TPShape shape,
                             hipStream_t s);
// z-slab rank of a 256^3 grid (cfp_dist.hip): stage 0 P1 on nzl local planes (in natural ->
// out chunked), 1 P2 on [256][nyl][256] in place, 2 P3 (in chunked -> out natural, x a.scale);
// the default shape (N1 = 32, permlane P2 with prefetch)
// the 3-sweep slab schedule: 256^3 and 512^3 with P | 32 ranks
bool three_pass_slab_supported(const i64 n[3], int P);
int three_pass_slab_n2(i64 n);  // rows y2 per k1 of the four-step y split (8 at 256, 16 at 512)
hipError_t launch_three_pass_slab(int stage, int n, const cd* in, cd* out, const TPArgs& a, int nzl, hipStream_t s);
// real-data plan at n^3, n = 128 or 256 (cfp_real.hip): stage 0 P1r (b -> H, Q), 1 P2 on H
// (n/2 x n x n, in place), 3 the same on the Nyquist column Q (n x n, kx = n/2, in place;
// a.colsym = its [ky] symbol), 2 P3r (H, Q -> x, x a.scale); a.tw = W_n, a.colsym =
// [kx + (n/2) ky], a.axsym = [kz].  P1r leaves Q after its y1 DFT, P3r takes it before its y1
// inverse (slot layout, as H).
hipError_t launch_three_pass_real(int stage, int n, const double* b, cd* H, cd* Q, double* x, const TPArgs& a,
                                  hipStream_t s, bool alt_rows = false);

// wave-system plan (cfp_wave_three.hip): the 3-sweep apply of the interleaved 4-component field
// (idx = 4 cell + comp) on a 128^3 grid, y split 16 x 8.  stage 0 P1w (in -> out), 1 P2w (out in
// place), 2 P3w (in -> out, x a.scale).  a.tw = W_128; a.wave: the (p, q) tables and c0^2.
struct WTPArgs {
  const cd* tw;
  WaveSym wave;
  double scale;
  // P3w with the Gram-Schmidt dots (r06, as the scalar P3's post_*): post_v[j]^H x over the
  // stored points for j < post_nv <= TP_POST_MAX (bit j of post_self: x itself), one partial per
  // workgroup and value into post_partial[block][16] (k_mdot's layout)
  const cd* post_v[4] = {nullptr, nullptr, nullptr, nullptr};
  int post_nv = 0, post_self = 0;
  double* post_partial = nullptr;
};
bool wave_three_pass_supported(const i64 n[3], int ncomp);
// grid_out (optional): the workgroups of the launch (the dots' partial count for stage 2)
hipError_t launch_wave_three_pass(int stage, const cd* in, cd* out, const WTPArgs& a, hipStream_t s,
                                  unsigned* grid_out = nullptr);

}  // namespace cfp
