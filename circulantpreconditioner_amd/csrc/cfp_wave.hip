// cfp_wave.hip -- the wave-system block-circulant plan (include/wave_system.h, SURVEY.md §8f
// row f2).  Same 5-sweep structure as the scalar plan, over the reference's interleaved
// layout idx = cell*nbComp + comp, nbComp = dim + 1 (src/WaveSystem.cxx:112-113,
// tests/WaveSystem_SphericalExplosion_impl_seq.cxx:19,57-68):
//
//   x pass   : columns (comp, y, z), point stride nbComp -- in 3-D a tile of 16 columns is
//              4 whole cells-rows x 4 components, i.e. 4 contiguous runs of 4*nx values
//   y, z pass: the scalar passes of a grid whose x extent is nbComp*nx (the components ride
//              along x as extra columns)
//   fused    : DFT along the last axis, per frequency the arrowhead solve, IDFT.  3-D: the 4
//              components are gathered from the lanes of one quad (DPP); 1-D / 2-D (2 or 3
//              components, the reference mains' default is a 2-D 50x50 grid): the mixed-radix
//              kernel gathers a cell's columns from LDS
//
// so an apply moves 5 x (read + write) x 64 bytes per cell and never materialises the 256-byte
// per-frequency block symbol (cfp_fft_device.h: wave_solve).
#include <hip/hip_runtime.h>

#include <cmath>
#include <map>
#include <memory>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/wave_system.h"
#include "cfp_blas.h"
#include "cfp_host.h"
#include "cfp_internal.h"
#include "cfp_three_pass.h"

using namespace cfp;

#define HIPCHK(expr)                                        \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return cfp::hip_error(_e, #expr); \
  } while (0)

struct cfp_wave_plan_s {
  int device = 0;
  i64 n[3] = {1, 1, 1};
  i64 N = 1;  // cells
  int dim = 3;
  int ncomp = 4;  // dim + 1 unknowns per cell
  std::map<int, cd*> tw;
  double2* tab[3] = {nullptr, nullptr, nullptr};
  bool has_sym = false;
  double c0 = 0.0;
  std::vector<int> axes;
  int fused = 0;
  int schedule = CFP_SCHEDULE_AUTO;  // AUTO: 3 sweeps where cfp_wave_three.hip serves the grid
  double* post_partial = nullptr;    // P3w's dot partials (cfp_wave_plan_apply_dots)
};

namespace {

struct Guard {
  int prev = -1;
  explicit Guard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~Guard() {
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

int ensure_tw(cfp_wave_plan_s* p, int n) {
  if (p->tw.count(n)) return CFP_SUCCESS;
  std::vector<cd> h = host_twiddles(n, -1);
  cd* d = nullptr;
  HIPCHK(hipMalloc(&d, sizeof(cd) * (size_t)n));
  HIPCHK(hipMemcpy(d, h.data(), sizeof(cd) * (size_t)n, hipMemcpyHostToDevice));
  p->tw[n] = d;
  return CFP_SUCCESS;
}

// the pass over `axis` of the interleaved 4-component field
PassDesc wave_pass(const cfp_wave_plan_s* p, int axis, int mode, double scale) {
  PassDesc d;
  d.n = (int)p->n[axis];
  if (axis == 0) {
    Side s;
    s.inner_stride = 1;
    s.outer_stride = p->ncomp * p->n[0];
    s.pt_stride = p->ncomp;
    s.seg_stride = 0;
    s.seg_len = (int)p->n[0];
    s.seg_shift = ilog2_exact(p->n[0]);
    d.in = d.out = s;
    d.inner_n = p->ncomp;
    d.ncols = p->ncomp * p->n[1] * p->n[2];
  } else {
    const i64 m[3] = {p->ncomp * p->n[0], p->n[1], p->n[2]};
    d.in = d.out = natural_side(axis, m);
    natural_cols(axis, m, &d.ncols, &d.inner_n);
  }
  d.mode = mode;
  d.scale = scale;
  d.colsym = d.axsym = d.diag = nullptr;
  for (int a = 0; a < 3; ++a) {
    d.wave.tab[a] = p->tab[a];
    d.wave.n[a] = p->n[a];
  }
  d.wave.c0sq = p->c0 * p->c0;
  d.wave.fused = p->fused;
  d.wave.ncomp = p->ncomp;
  return d;
}

int launch(cfp_wave_plan_s* p, const PassDesc& d, const cd* in, cd* out, hipStream_t s) {
  int rc = ensure_tw(p, d.n);
  if (rc) return rc;
  hipError_t e = launch_axis_pass(d, in, out, p->tw[d.n], s);
  return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "wave axis pass");
}

struct WStep {
  int axis, mode;
  bool from_b, scale;
  int tp = -1;  // >= 0: stage of the 3-sweep apply (cfp_wave_three.hip)
};

bool use_three(const cfp_wave_plan_s* p) {
  return p->schedule != CFP_SCHEDULE_FIVE_PASS && p->dim == 3 && wave_three_pass_supported(p->n, p->ncomp);
}

std::vector<WStep> wave_steps(const cfp_wave_plan_s* p) {
  std::vector<WStep> st;
  if (use_three(p)) {
    for (int k = 0; k < 3; ++k) st.push_back({k == 1 ? 2 : 0, PASS_FUSED_WAVE, k == 0, k == 2, k});
    return st;
  }
  const std::vector<int>& A = p->axes;
  if (A.empty()) {
    st.push_back({0, PASS_FUSED_WAVE, true, true});
    return st;
  }
  for (size_t i = 0; i + 1 < A.size(); ++i) st.push_back({A[i], PASS_FWD, i == 0, false});
  st.push_back({A.back(), PASS_FUSED_WAVE, A.size() == 1, A.size() == 1});
  for (int i = (int)A.size() - 2; i >= 0; --i) st.push_back({A[i], PASS_INV, false, i == 0});
  return st;
}

int run_wave(cfp_wave_plan_s* p, const cd* b, cd* x, hipStream_t s, std::vector<hipEvent_t>* ev,
             const WTPArgs* post = nullptr, unsigned* p3grid = nullptr) {
  if (!p->has_sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set (call cfp_wave_plan_set_symbol)");
  std::vector<WStep> st = wave_steps(p);
  const double invN = 1.0 / (double)p->N;
  for (size_t i = 0; i < st.size(); ++i) {
    const WStep& q = st[i];
    if (ev) HIPCHK(hipEventRecord((*ev)[i], s));
    if (q.tp >= 0) {
      WTPArgs a;
      a.tw = p->tw[128];
      a.wave = wave_pass(p, 2, PASS_FUSED_WAVE, 1.0).wave;
      a.wave.fused = 2;
      a.scale = q.scale ? invN : 1.0;
      if (post && q.tp == 2) {
        for (int j = 0; j < 4; ++j) a.post_v[j] = post->post_v[j];
        a.post_nv = post->post_nv;
        a.post_self = post->post_self;
        a.post_partial = post->post_partial;
      }
      if (!ev && g_apply_stamp.start) {  // the caller times the whole apply (stand-in KSP)
        if (i == 0) {
          g_stamp.start = g_apply_stamp.start;
          ++g_apply_stamp.hits;
        }
        if (i + 1 == st.size()) {
          g_stamp.stop = g_apply_stamp.stop;
          ++g_apply_stamp.hits;
        }
      }
      hipError_t e = launch_wave_three_pass(q.tp, q.from_b ? b : x, x, a, s, q.tp == 2 ? p3grid : nullptr);
      g_stamp = LaunchStamp{};
      if (e != hipSuccess) return hip_error(e, "wave 3-sweep launch");
      continue;
    }
    int rc = launch(p, wave_pass(p, q.axis, q.mode, q.scale ? invN : 1.0), q.from_b ? b : x, x, s);
    if (rc) return rc;
  }
  if (ev) HIPCHK(hipEventRecord((*ev)[st.size()], s));
  return CFP_SUCCESS;
}

int run_transform(cfp_wave_plan_s* p, bool inverse, const cd* in, cd* out, hipStream_t s) {
  // the symbol tables are not read by plain passes; the descriptor still carries them
  bool first = true;
  std::vector<int> axes = p->axes;
  if (axes.empty()) axes.push_back(0);
  for (int ax : axes) {
    int rc = launch(p, wave_pass(p, ax, inverse ? PASS_INV : PASS_FWD, 1.0), first ? in : out, out, s);
    if (rc) return rc;
    first = false;
  }
  return CFP_SUCCESS;
}

}  // namespace

extern "C" int cfp_wave_plan_create_dim(cfp_wave_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int dim,
                                        int device) {
  if (!plan) return set_error(CFP_ERR_ARG_NULL, "plan is NULL");
  *plan = nullptr;
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  if (dim < 1 || dim > 3) return set_error(CFP_ERR_ARG_OUTOFRANGE, "dim must be 1, 2 or 3 (got %d)", dim);
  if ((dim < 3 && nz != 1) || (dim < 2 && ny != 1))
    return set_error(CFP_ERR_ARG_SIZ, "a %d-D wave system has n = 1 along the axes above its dimension", dim);
  if (nx > 1024 || ny > 1024 || nz > 1024)
    return set_error(CFP_ERR_SUP, "wave plan: axis lengths above 1024 are not supported");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_error(CFP_ERR_ARG_OUTOFRANGE, "device %d out of range", device);
  Guard g(device);
  std::unique_ptr<cfp_wave_plan_s> p(new cfp_wave_plan_s);
  p->device = device;
  p->n[0] = nx;
  p->n[1] = ny;
  p->n[2] = nz;
  p->N = nx * ny * nz;
  p->dim = dim;
  p->ncomp = dim + 1;
  for (int a = 0; a < 3; ++a)
    if (p->n[a] > 1) p->axes.push_back(a);
  p->fused = p->axes.empty() ? 0 : p->axes.back();
  for (int a = 0; a < 3; ++a) {
    int rc = ensure_tw(p.get(), (int)p->n[a]);
    if (rc) return rc;
  }
  *plan = p.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_plan_create(cfp_wave_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int device) {
  return cfp_wave_plan_create_dim(plan, nx, ny, nz, 3, device);
}

extern "C" int cfp_wave_plan_destroy(cfp_wave_plan_t p) {
  if (!p) return CFP_SUCCESS;
  Guard g(p->device);
  for (auto& kv : p->tw) hipFree(kv.second);
  for (int a = 0; a < 3; ++a)
    if (p->tab[a]) hipFree(p->tab[a]);
  if (p->post_partial) hipFree(p->post_partial);
  delete p;
  return CFP_SUCCESS;
}

// p_d[k] = kappa_d c0 (1 - cos theta), q_d[k] = kappa_d sin theta, theta = 2 pi k / n_d
extern "C" int cfp_wave_plan_set_symbol(cfp_wave_plan_t p, const double kappa[3], double c0) {
  if (!p || !kappa) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!(c0 > 0.0)) return set_error(CFP_ERR_ARG_OUTOFRANGE, "c0 must be > 0");
  for (int a = 0; a < 3; ++a)
    if (!(kappa[a] >= 0.0)) return set_error(CFP_ERR_ARG_OUTOFRANGE, "kappa must be >= 0");
  Guard g(p->device);
  for (int a = 0; a < 3; ++a) {
    const i64 n = p->n[a];
    std::vector<double2> t((size_t)n);
    for (i64 k = 0; k < n; ++k) {
      const long double th = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
      t[(size_t)k] = make_double2((double)((long double)kappa[a] * c0 * (1.0L - cosl(th))),
                                  (double)((long double)kappa[a] * sinl(th)));
    }
    if (!p->tab[a]) HIPCHK(hipMalloc(&p->tab[a], sizeof(double2) * (size_t)n));
    HIPCHK(hipMemcpy(p->tab[a], t.data(), sizeof(double2) * (size_t)n, hipMemcpyHostToDevice));
  }
  p->c0 = c0;
  p->has_sym = true;
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_plan_apply(cfp_wave_plan_t p, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  Guard g(p->device);
  return run_wave(p, (const cd*)b, (cd*)x, (hipStream_t)stream, nullptr);
}

// x = S^{-1} b and dots[2 j + re/im] = v[j]^H x (v[j] NULL or x: |x|^2), dots a device array.
// On the 3-sweep schedule the dots ride in P3w's stores (*fused = 1, at most 4 vectors);
// otherwise the apply runs, then one multi-dot sweep (*fused = 0).
extern "C" int cfp_wave_plan_apply_dots(cfp_wave_plan_t p, const double* b, double* x, void* stream, int nv,
                                        const double* const* v, double* dots, int* fused) {
  if (!p || !b || !x || (nv > 0 && (!v || !dots))) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (nv < 0 || nv > 8) return set_error(CFP_ERR_ARG_OUTOFRANGE, "nv must be in 0..8");
  if (fused) *fused = 0;
  Guard g(p->device);
  hipStream_t s = (hipStream_t)stream;
  if (nv == 0) return run_wave(p, (const cd*)b, (cd*)x, s, nullptr);
  if (use_three(p) && nv <= 4) {
    if (!p->post_partial) HIPCHK(hipMalloc(&p->post_partial, sizeof(double) * 16 * 1024));
    WTPArgs post;
    for (int j = 0; j < nv; ++j) {
      post.post_v[j] = (const cd*)v[j];
      if (!v[j] || v[j] == x) post.post_self |= 1 << j;
    }
    post.post_nv = nv;
    post.post_partial = p->post_partial;
    unsigned gp = 0;
    int rc = run_wave(p, (const cd*)b, (cd*)x, s, nullptr, &post, &gp);
    if (rc) return rc;
    if (gp < 1 || gp > 1024) return set_error(CFP_ERR_LIB, "P3w grid out of range");
    hipError_t e = blas_mdot_finish(p->post_partial, (int)gp, nv, dots, s);
    if (e != hipSuccess) return hip_error(e, "dots finish");
    if (fused) *fused = 1;
    return CFP_SUCCESS;
  }
  int rc = run_wave(p, (const cd*)b, (cd*)x, s, nullptr);
  if (rc) return rc;
  const cd* ys[8];
  for (int j = 0; j < nv; ++j) ys[j] = (const cd*)v[j] == (const cd*)x ? nullptr : (const cd*)v[j];
  hipError_t e = blas_mdot_dev((const cd*)x, nv, ys, p->N * p->ncomp, dots, s);
  if (e != hipSuccess) return hip_error(e, "dots");
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_plan_forward(cfp_wave_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  Guard g(p->device);
  return run_transform(p, false, (const cd*)in, (cd*)out, (hipStream_t)stream);
}

extern "C" int cfp_wave_plan_backward(cfp_wave_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  Guard g(p->device);
  return run_transform(p, true, (const cd*)in, (cd*)out, (hipStream_t)stream);
}

extern "C" int cfp_wave_plan_set_schedule(cfp_wave_plan_t p, int schedule) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "plan is NULL");
  if (schedule != CFP_SCHEDULE_AUTO && schedule != CFP_SCHEDULE_FIVE_PASS && schedule != CFP_SCHEDULE_THREE_PASS)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "wave plan schedule must be AUTO, FIVE_PASS or THREE_PASS (got %d)",
                     schedule);
  if (schedule == CFP_SCHEDULE_THREE_PASS && !(p->dim == 3 && wave_three_pass_supported(p->n, p->ncomp)))
    return set_error(CFP_ERR_SUP, "the wave 3-sweep schedule needs a 3-D 128^3 grid");
  p->schedule = schedule;
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_plan_num_passes(cfp_wave_plan_t p, int* passes) {
  if (!p || !passes) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *passes = (int)wave_steps(p).size();
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_plan_time_passes(cfp_wave_plan_t p, const double* b, double* x, int iters, double* ms_out,
                                         void* stream) {
  if (!p || !b || !x || !ms_out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (iters < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "iters must be >= 1");
  Guard g(p->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t np = wave_steps(p).size();
  std::vector<double> acc(np, 0.0);
  std::vector<hipEvent_t> ev(np + 1);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  int rc = CFP_SUCCESS;
  for (int it = 0; it < iters && rc == CFP_SUCCESS; ++it) {
    rc = run_wave(p, (const cd*)b, (cd*)x, s, &ev);
    if (rc) break;
    hipError_t e = hipEventSynchronize(ev[np]);
    if (e != hipSuccess) {
      rc = hip_error(e, "event sync");
      break;
    }
    for (size_t i = 0; i < np; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
      acc[i] += ms;
    }
  }
  for (auto& e : ev) hipEventDestroy(e);
  if (rc) return rc;
  for (size_t i = 0; i < np; ++i) ms_out[i] = acc[i] / iters;
  return CFP_SUCCESS;
}
