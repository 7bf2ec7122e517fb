// kexp.hip -- timing harness for fast axis-pass kernel variants (not part of the product).
// Builds the same device code as the product (cfp_fft_device.h) with several shapes/flags
// and times them back to back in one process (methodology rule 24 of the HIP guide).
#include <cstring>

#include "../../circulantpreconditioner_amd/csrc/cfp_fft_device.h"

using namespace cfp;

template <int N, int P, int R, bool ROW, int T, int MODE, int FL>
static hipError_t launch_v(const cd* in, cd* out, const KArgs* a, i64 ncols) {
  hipLaunchKernelGGL((k_axis_fast<N, P, R, ROW, T, MODE, FL>), dim3((unsigned)(ncols / T)), dim3(T * (N / P)), 0,
                     nullptr, in, out, *a);
  return hipGetLastError();
}

struct Var {
  const char* name;
  int n, row, T, threads, mode, flags;
  hipError_t (*fn)(const cd*, cd*, const KArgs*, i64);
};

#define V(NN, P, R, ROWV, TT, MODE, FL) \
  {#NN "/pts" #P "/r0" #R "/" #ROWV "/T" #TT "/m" #MODE "/f" #FL, NN, ROWV, TT, TT * (NN / P), MODE, FL, \
   &launch_v<NN, P, R, ROWV, TT, MODE, FL>},

static const Var kVars[] = {
    // N = 256: row {0,16,32} = 0..2, col {0,16,32} = 3..5, fused split {1,17,33} = 6..8
    V(256, 8, 4, true, 8, 0, 0) V(256, 8, 4, true, 8, 0, 16) V(256, 8, 4, true, 8, 0, 32)
    V(256, 8, 4, false, 16, 0, 0) V(256, 8, 4, false, 16, 0, 16) V(256, 8, 4, false, 16, 0, 32)
    V(256, 16, 16, false, 16, 2, 1) V(256, 16, 16, false, 16, 2, 17) V(256, 16, 16, false, 16, 2, 33)
    // N = 512: row 9..11, col split 12..14, fused 15..17
    V(512, 16, 2, true, 8, 0, 0) V(512, 16, 2, true, 8, 0, 16) V(512, 16, 2, true, 8, 0, 32)
    V(512, 16, 2, false, 16, 0, 1) V(512, 16, 2, false, 16, 0, 17) V(512, 16, 2, false, 16, 0, 33)
    V(512, 8, 8, false, 8, 2, 0) V(512, 8, 8, false, 8, 2, 16) V(512, 8, 8, false, 8, 2, 32)
    // N = 128: row 18..20, col 21..23, fused 24..26
    V(128, 16, 8, true, 32, 0, 0) V(128, 16, 8, true, 32, 0, 16) V(128, 16, 8, true, 32, 0, 32)
    V(128, 8, 2, false, 16, 0, 0) V(128, 8, 2, false, 16, 0, 16) V(128, 8, 2, false, 16, 0, 32)
    V(128, 8, 2, false, 16, 2, 0) V(128, 8, 2, false, 16, 2, 16) V(128, 8, 2, false, 16, 2, 32)
    // N = 256 fused-pass shapes (27..36): non-split / split, PTS 16 / 8 / 4, T 8 / 16 / 32, LDS twiddles or global
    V(256, 16, 16, false, 8, 2, 16) V(256, 16, 16, false, 16, 2, 16) V(256, 8, 4, false, 16, 2, 16)
    V(256, 8, 4, false, 16, 2, 17) V(256, 8, 4, false, 8, 2, 16) V(256, 16, 16, false, 32, 2, 17)
    V(256, 16, 16, false, 16, 2, 19) V(256, 4, 4, false, 16, 2, 16) V(256, 8, 4, false, 32, 2, 17)
    V(256, 16, 16, false, 8, 2, 17)
    // reversed tile order (F_REV) of the product's 256 choices (37..41): x-fwd, y-fwd, fused, y-inv, x-inv
    V(256, 8, 4, true, 8, 0, 24) V(256, 8, 4, false, 16, 0, 8) V(256, 16, 16, false, 16, 2, 25)
    V(256, 8, 4, false, 16, 0, 40) V(256, 8, 4, true, 8, 0, 40)
    // fused 256 with the 4-wave occupancy request F_OCC4 (42..49): product (split, nt loads), T 32 / 8,
    // nt loads+stores, nt stores, PTS 8 split T 16, non-split, global twiddles
    V(256, 16, 16, false, 16, 2, 145) V(256, 16, 16, false, 32, 2, 145) V(256, 16, 16, false, 8, 2, 145)
    V(256, 16, 16, false, 16, 2, 133) V(256, 16, 16, false, 16, 2, 177) V(256, 8, 4, false, 16, 2, 145)
    V(256, 16, 16, false, 16, 2, 144) V(256, 16, 16, false, 16, 2, 147)
    // large rows (50..): 512 row T 8 nt-ld (product) / split / split T 4; 1024 row T 4 (product) /
    // split / split T 2 / split + global twiddles; 1024 column T 8 split (product) / T 4 / tw global
    V(512, 16, 2, true, 8, 0, 16) V(512, 16, 2, true, 8, 0, 17) V(512, 16, 2, true, 4, 0, 17)
    V(1024, 16, 4, true, 4, 0, 16) V(1024, 16, 4, true, 4, 0, 17) V(1024, 16, 4, true, 2, 0, 17)
    V(1024, 16, 4, true, 4, 0, 19) V(1024, 16, 4, false, 8, 0, 17) V(1024, 16, 4, false, 4, 0, 17)
    V(1024, 16, 4, false, 8, 0, 19)
    // x-fused order (60..): row-mode fused 256 shapes -- product (PTS 8, T 8, nt-ld), PTS 16 T 8 / 4 / 16
    // (nt-ld, split), 4-wave request, non-split
    V(256, 8, 4, true, 8, 2, 16) V(256, 16, 16, true, 8, 2, 17) V(256, 16, 16, true, 4, 2, 17)
    V(256, 16, 16, true, 16, 2, 17) V(256, 16, 16, true, 8, 2, 145) V(256, 16, 16, true, 8, 2, 16)
    V(256, 16, 16, true, 4, 2, 145) V(256, 8, 4, true, 16, 2, 16)
    // N = 512 whole-apply shapes (68..): fused split T 16 / +4-wave / PTS 8 T 16 / PTS 8 T 8 split /
    // PTS 16 T 8 split / product (PTS 8 T 8 nt-ld) / PTS 8 T 16 4-wave
    V(512, 16, 2, false, 16, 2, 17) V(512, 16, 2, false, 16, 2, 145) V(512, 8, 8, false, 16, 2, 17)
    V(512, 8, 8, false, 8, 2, 17) V(512, 16, 2, false, 8, 2, 17) V(512, 8, 8, false, 8, 2, 16)
    V(512, 8, 8, false, 16, 2, 145)
    // columns (75..80): product fwd (split nt-ld), PTS 8, T 32, product inv (split nt-st), PTS 8 inv, 4-wave
    V(512, 16, 2, false, 16, 0, 17) V(512, 8, 8, false, 16, 0, 17) V(512, 16, 2, false, 32, 0, 17)
    V(512, 16, 2, false, 16, 0, 33) V(512, 8, 8, false, 16, 0, 33) V(512, 16, 2, false, 16, 0, 145)
    // rows (81, 82): product fwd (nt-ld), inv (nt-st)
    V(512, 16, 2, true, 8, 0, 16) V(512, 16, 2, true, 8, 0, 32)
    // fused 256 at higher occupancy (83..): 8-wave request (F_OCC8 = 512) with PTS 8 T 16 / T 8 split,
    // PTS 4 T 16 split, PTS 8 T 16 split + global twiddles; PTS 8 T 32 split 4-wave
    V(256, 8, 4, false, 16, 2, 529) V(256, 8, 4, false, 8, 2, 529) V(256, 4, 4, false, 16, 2, 529)
    V(256, 8, 4, false, 16, 2, 531) V(256, 8, 4, false, 32, 2, 145)
};

extern "C" int kexp_count() { return (int)(sizeof(kVars) / sizeof(kVars[0])); }
extern "C" const char* kexp_name(int i) { return kVars[i].name; }
extern "C" int kexp_info(int i, int* n, int* row, int* T, int* threads, int* mode, int* flags) {
  const Var& v = kVars[i];
  *n = v.n; *row = v.row; *T = v.T; *threads = v.threads; *mode = v.mode; *flags = v.flags;
  return 0;
}

// time `iters` launches of variant i over a grid of n^3 (axis = row ? x : z), in place or not
extern "C" int kexp_time(int i, const double* in, double* out, const double* tw, const double* colsym,
                         const double* axsym, int iters, double* ms, int axis) {
  const Var& v = kVars[i];
  const i64 n = v.n, N = n * n * n;
  KArgs a;
  memset(&a, 0, sizeof(a));
  Side s;
  s.seg_len = (int)n;
  s.seg_shift = ilog2((int)n);
  s.seg_stride = 0;
  i64 ncols = N / n;
  if (v.row) { s.inner_stride = 0; s.outer_stride = n; s.pt_stride = 1; a.inner_n = 1; }
  else if (axis == 2) { s.inner_stride = 1; s.outer_stride = 0; s.pt_stride = n * n; a.inner_n = n * n; }
  else { s.inner_stride = 1; s.outer_stride = n * n; s.pt_stride = n; a.inner_n = n; }  // y axis
  a.in = s; a.out = s; a.scale = 1.0; a.ncols = ncols;
  a.tw = (const cd*)tw; a.colsym = (const cd*)colsym; a.axsym = (const cd*)axsym; a.diag = nullptr;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  v.fn((const cd*)in, (cd*)out, &a, ncols);  // warm-up
  hipEventRecord(e0, nullptr);
  for (int it = 0; it < iters; ++it) v.fn((const cd*)in, (cd*)out, &a, ncols);
  hipEventRecord(e1, nullptr);
  hipError_t e = hipEventSynchronize(e1);
  float t = 0;
  hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return e == hipSuccess ? (int)hipGetLastError() : (int)e;
}

// time `iters` chained applies: X b->x, Y x->x (y axis), Z x->x (z axis, fused), Y, X (all in place)
extern "C" int kexp_chain(int ix, int iy, int iz, int iy2, int ix2, const double* b, double* x, const double* tw, const double* colsym,
                          const double* axsym, int iters, double* ms) {
  const i64 n = kVars[ix].n, N = n * n * n;
  KArgs ax, ay, az;
  memset(&ax, 0, sizeof(ax));
  memset(&ay, 0, sizeof(ay));
  memset(&az, 0, sizeof(az));
  Side s;
  s.seg_len = (int)n; s.seg_shift = ilog2((int)n); s.seg_stride = 0;
  s.inner_stride = 0; s.outer_stride = n; s.pt_stride = 1; ax.in = ax.out = s; ax.inner_n = 1;
  s.inner_stride = 1; s.outer_stride = n * n; s.pt_stride = n; ay.in = ay.out = s; ay.inner_n = n;
  s.inner_stride = 1; s.outer_stride = 0; s.pt_stride = n * n; az.in = az.out = s; az.inner_n = n * n;
  for (KArgs* a : {&ax, &ay, &az}) {
    a->ncols = N / n;
    a->scale = 1.0; a->tw = (const cd*)tw; a->colsym = (const cd*)colsym; a->axsym = (const cd*)axsym; a->diag = nullptr;
  }
  const i64 nc = N / n;
  auto one = [&]() {
    kVars[ix].fn((const cd*)b, (cd*)x, &ax, nc);
    kVars[iy].fn((const cd*)x, (cd*)x, &ay, nc);
    kVars[iz].fn((const cd*)x, (cd*)x, &az, nc);
    kVars[iy2].fn((const cd*)x, (cd*)x, &ay, nc);
    kVars[ix2].fn((const cd*)x, (cd*)x, &ax, nc);
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  one();
  (void)hipEventRecord(e0, nullptr);
  for (int it = 0; it < iters; ++it) one();
  (void)hipEventRecord(e1, nullptr);
  hipError_t e = hipEventSynchronize(e1);
  float t = 0;
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return e == hipSuccess ? (int)hipGetLastError() : (int)e;
}

// time `iters` chained applies of `nst` steps: step i runs variant var[i] along axis ax[i]
// (0 = x rows, 1 = y columns, 2 = z columns); the first reads b, the rest work in place on x
extern "C" int kexp_chain_axes(int nst, const int* var, const int* axv, const double* b, double* x, const double* tw,
                               const double* colsym, const double* axsym, int iters, double* ms) {
  const i64 n = kVars[var[0]].n, N = n * n * n;
  KArgs a3[3];
  memset(a3, 0, sizeof(a3));
  Side s;
  s.seg_len = (int)n; s.seg_shift = ilog2((int)n); s.seg_stride = 0;
  s.inner_stride = 0; s.outer_stride = n; s.pt_stride = 1; a3[0].in = a3[0].out = s; a3[0].inner_n = 1;
  s.inner_stride = 1; s.outer_stride = n * n; s.pt_stride = n; a3[1].in = a3[1].out = s; a3[1].inner_n = n;
  s.inner_stride = 1; s.outer_stride = 0; s.pt_stride = n * n; a3[2].in = a3[2].out = s; a3[2].inner_n = n * n;
  for (KArgs& a : a3) {
    a.ncols = N / n;
    a.scale = 1.0; a.tw = (const cd*)tw; a.colsym = (const cd*)colsym; a.axsym = (const cd*)axsym; a.diag = nullptr;
    a.tw4.lo = a.tw4.hi = nullptr;
  }
  const i64 nc = N / n;
  auto one = [&]() {
    for (int i = 0; i < nst; ++i)
      kVars[var[i]].fn(i == 0 ? (const cd*)b : (const cd*)x, (cd*)x, &a3[axv[i]], nc);
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  one();
  (void)hipEventRecord(e0, nullptr);
  for (int it = 0; it < iters; ++it) one();
  (void)hipEventRecord(e1, nullptr);
  hipError_t e = hipEventSynchronize(e1);
  float t = 0;
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms = t / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return e == hipSuccess ? (int)hipGetLastError() : (int)e;
}
