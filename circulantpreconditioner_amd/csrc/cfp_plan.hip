// cfp_plan.hip -- host side of the single-GPU plan: pass schedule, symbol tables, C ABI.
//
// A plan replaces the reference's persistent PCSHELL state (struct FFTPrecTransportContext,
// src/PCSHELLFft_3D.hxx:8-21: FFT_MAT, Diag, b_hat, b_cartesien) with:
//   * the axis-pass schedule of one apply (cfp_kernels.hip),
//   * per-axis twiddle tables W_n (host long double -> device double),
//   * the symbol: separable tables (colsym over the fused axis' columns, axsym over its
//     points) generated once, or an explicit Diag vector for a general symbol.
// An apply reads b, writes x, and needs no scratch (x is the work buffer).
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/circulant_fft.h"
#include "cfp_blas.h"
#include "cfp_internal.h"
#include "cfp_host.h"
#include "cfp_three_pass.h"

using namespace cfp;

// ------------------------------------------------------------------ error plumbing
static thread_local std::string g_err;

namespace cfp {
int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
int hip_error(hipError_t e, const char* what) {
  return set_error(e == hipErrorOutOfMemory ? CFP_ERR_MEM : CFP_ERR_LIB, "%s: %s", what, hipGetErrorString(e));
}
}  // namespace cfp

#define HIPCHK(expr)                                     \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return cfp::hip_error(_e, #expr); \
  } while (0)

extern "C" const char* cfp_last_error(void) { return g_err.c_str(); }
extern "C" const char* cfp_version(void) { return "circulant_fft 0.1.0 (gfx950)"; }

extern "C" int cfp_device_count(int* count) {
  if (!count) return set_error(CFP_ERR_ARG_NULL, "count is NULL");
  HIPCHK(hipGetDeviceCount(count));
  return CFP_SUCCESS;
}

extern "C" int cfp_stream_sync(void* stream) {
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return CFP_SUCCESS;
}

extern "C" int cfp_device_copy(void* dst, const void* src, size_t bytes, void* stream) {
  if ((!dst || !src) && bytes) return set_error(CFP_ERR_ARG_NULL, "cfp_device_copy: NULL pointer");
  HIPCHK(cfp::blas_copy_bytes(dst, src, bytes, (hipStream_t)stream));
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ twiddles
namespace cfp {

std::vector<cd> host_twiddles(int n, int sign) {
  std::vector<cd> t((size_t)n);
  for (int k = 0; k < n; ++k) {
    long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
    t[k] = make_cd((double)cosl(a), (double)(sign * sinl(a)));
  }
  return t;
}

// 1 - e^{-2 pi i k / n}: the 1-D DFT of the transport column (1, -1, 0, ...)
std::vector<cd> host_transport_symbol(i64 n) {
  std::vector<cd> s((size_t)n, make_cd(0.0, 0.0));
  if (n <= 1) return s;
  for (i64 k = 0; k < n; ++k) {
    long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
    s[k] = make_cd((double)(1.0L - cosl(a)), (double)sinl(a));
  }
  return s;
}

int ilog2_exact(i64 v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1LL << l) < v) ++l;
  return l;
}

Side natural_side(int axis, const i64 n[3]) {
  Side s;
  const i64 nx = n[0], ny = n[1];
  s.seg_len = (int)n[axis];
  s.seg_shift = ilog2_exact(n[axis]);
  if (s.seg_shift < 0) s.seg_shift = 30;  // unused by the generic kernel
  s.seg_stride = 0;
  if (axis == 0) { s.inner_stride = 0; s.outer_stride = nx; s.pt_stride = 1; }
  else if (axis == 1) { s.inner_stride = 1; s.outer_stride = nx * ny; s.pt_stride = nx; }
  else { s.inner_stride = 1; s.outer_stride = 0; s.pt_stride = nx * ny; }
  if (ilog2_exact(n[axis]) < 0) s.seg_shift = -1;
  return s;
}

void natural_cols(int axis, const i64 n[3], i64* ncols, i64* inner_n) {
  const i64 N = n[0] * n[1] * n[2];
  *ncols = N / n[axis];
  *inner_n = axis == 0 ? 1 : (axis == 1 ? n[0] : n[0] * n[1]);
}

}  // namespace cfp

// ------------------------------------------------------------------ plan
struct cfp_plan_s {
  int device = 0;
  i64 n[3] = {1, 1, 1};
  i64 N = 1;
  std::map<int, cd*> tw;  // device forward twiddles per axis length
  int sym_kind = 0;       // 0 none, 1 separable, 2 explicit diag
  uint64_t sym_version = 0;  // bumped by every symbol setter (cfp_plan_symbol_version)
  cd* colsym = nullptr;   // separable: per column of the fused axis (sum over the other axes)
  cd* axsym = nullptr;    //            per point of the fused axis
  cd* diag = nullptr;     // explicit
  cd* host_stage = nullptr;  // device staging buffers for cfp_plan_apply_host
  // the 3-sweep intermediate of the blocked shapes (TP_MID_BLOCKED*): a sweep that changes the
  // layout cannot run in place (a unit's natural rows hold other units' blocked values), so
  // P1 writes and P3 reads this plan-owned buffer (N values, allocated on first use)
  cd* mid_buf = nullptr;
  // cfp_plan_apply_ex: the fused P3's workgroup partials (16 doubles per workgroup) and the
  // stencil output of the unfused fallback (N values), both allocated on first use
  double* post_partial = nullptr;
  cd* pre_buf = nullptr;
  // HIP-graph replay (cfp_plan_set_graph): one instantiated graph of the apply's launches per
  // (b, x) pair, captured on a private stream and launched into the caller's stream.  A graph
  // holds device pointers, not values: every setter that can move a buffer or change the
  // launch list drops them (graph_clear); a value written into a symbol or Diag buffer is seen.
  struct GraphEntry {
    const cd* b;
    cd* x;
    hipGraphExec_t exec;
  };
  bool graph_on = false;
  hipStream_t cap_stream = nullptr;
  std::vector<GraphEntry> graphs;
  std::vector<int> axes;     // non-trivial axes, x..z
  int fused_axis = 0;
  std::vector<cd> sym1d[3];  // separable: lambda_d * c_d_hat (host copies)
  i64 chunk_planes = 0;      // > 0: chunked x/y schedule (see apply_steps)
  int schedule = CFP_SCHEDULE_AUTO;
  TPShape tp_shape;          // 3-sweep kernel shape (cfp_plan_set_three_pass_shape)
  bool external_x = false;  // x transformed by the caller (real plan): y/z passes only, no 1/N
  // long axes (n > 4096): four-step split n = n1 n2, both <= 4096 (0: a short axis).  Their
  // spectrum stays in position order p = m1 + n1 m2 for frequency m = m2 + n2 m1.
  int split[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  cd* tw4lo[3] = {nullptr, nullptr, nullptr};
  cd* tw4hi[3] = {nullptr, nullptr, nullptr};
  cd* possym[3] = {nullptr, nullptr, nullptr};  // position-indexed symbols (the standalone divide)
  bool long_axes() const { return split[0][0] || split[1][0] || split[2][0]; }
  // profiling mode (cfp_plan_profile_begin/_end): every cfp_plan_apply records one event per
  // launch into its own slot, so per-launch times come from the caller's own timed applies
  std::vector<hipEvent_t> prof_ev;
  size_t prof_stride = 0, prof_cap = 0, prof_used = 0;
  size_t prof_every = 1, prof_calls = 0;  // record every prof_every-th apply (sampling)
};

namespace cfp {
thread_local LaunchStamp g_stamp;  // cfp_internal.h
thread_local ApplyStamp g_apply_stamp;
}  // namespace cfp
extern "C" void cfp_apply_stamp_clear(void) { cfp::g_apply_stamp.start = cfp::g_apply_stamp.stop = nullptr; }

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

int ensure_tw(cfp_plan_s* p, int n) {
  if (p->tw.count(n)) return CFP_SUCCESS;
  std::vector<cd> h = host_twiddles(n, -1);
  cd* d = nullptr;
  HIPCHK(hipMalloc(&d, sizeof(cd) * (size_t)n));
  HIPCHK(hipMemcpy(d, h.data(), sizeof(cd) * (size_t)n, hipMemcpyHostToDevice));
  p->tw[n] = d;
  return CFP_SUCCESS;
}

struct Step {
  int axis;
  int mode;    // PASS_* or -1 for the fused symbol pass
  bool from_b;
  bool scale;
  i64 z0, z1;  // z-plane range of an x or y pass (z1 < 0: whole grid)
  int tp = -1; // >= 0: stage of the 3-sweep schedule (cfp_three_pass.hip)
  int sub = 0; // long axis: 1 = the length-n2 half (with the twiddle), 2 = the length-n1 half;
               // 3 = the standalone symbol divide (no short axis to fuse)
};

// the 3-sweep schedule serves 100^3, 128^3, 256^3 and 512^3 grids with a separable symbol: on
// request, and by default (AUTO without chunking), where it beats the 5-pass schedule by ~18 % at
// 256^3, ~6 % at 128^3 and 7 % at 512^3 (262 against 246 PCApply/s), and the plane schedule by
// 18 % at 100^3 (27.6k against 23.3k PCApply/s; profiles/r04_schedule_ab.jsonl)
bool use_three_pass(const cfp_plan_s* p, bool diag_override) {
  const bool want = p->schedule == CFP_SCHEDULE_THREE_PASS ||
                    (p->schedule == CFP_SCHEDULE_AUTO && p->chunk_planes == 0 &&
                     (p->n[0] == 256 || p->n[0] == 128 || p->n[0] == 100 || p->n[0] == 512));
  if (!want || diag_override || p->sym_kind != 1 || p->external_x) return false;
  return three_pass_supported(p->n) || three_pass_sq_supported(p->n);
}

// the plane schedule (n_x = n_y in {32, 64, 100, 128}, n_z > 1): plane forward (x + y DFTs of
// whole z-planes), the fused z pass, plane inverse -- on request, and by default for 100^2, 64^2
// and 32^2 planes, where the five passes are launch-cost bound
bool use_plane(const cfp_plan_s* p) {
  if (p->external_x || p->long_axes() || p->n[0] != p->n[1] || !plane_supported(p->n[0]) || p->n[2] < 2)
    return false;
  if (p->schedule == CFP_SCHEDULE_PLANE) return true;
  // (128^2 planes lose to the 5 passes: 15,400 vs 17,100 PCApply/s, profiles/r02t_plane_schedule.md;
  // 32^2 planes win: 32^3 at 65,300-71,500 against 39,400-43,000, profiles/r06z2_plane32_ab.txt)
  return p->schedule == CFP_SCHEDULE_AUTO && p->chunk_planes == 0 &&
         (p->n[0] == 100 || p->n[0] == 64 || p->n[0] == 32);
}

// axis order of the 5-pass schedule: the last one is fused with the symbol
void order_axes(cfp_plan_s* p) {
  p->axes.clear();
  const int order_z[3] = {0, 1, 2}, order_y[3] = {0, 2, 1};
  // AUTO fuses y on large grids (512^3 5 passes: 4 % faster, profiles/r01_schedule_sweep.txt), z
  // otherwise -- and z on every grid the 3-sweep schedule serves, whose middle sweep reads the
  // z-fused tables (decided from the geometry alone: this runs before a symbol is set)
  const bool yf = p->schedule == CFP_SCHEDULE_FIVE_PASS_YFUSED ||
                  (p->schedule == CFP_SCHEDULE_AUTO && p->n[1] >= 512 && p->n[2] >= 512 && !three_pass_supported(p->n));
  const int* o = (yf && !p->long_axes()) ? order_y : order_z;
  std::vector<int> longs;
  for (int i = 0; i < 3; ++i) {
    if (p->n[o[i]] <= 1 || (p->external_x && o[i] == 0)) continue;
    if (p->split[o[i]][0]) longs.push_back(o[i]);
    else p->axes.push_back(o[i]);
  }
  // a long axis cannot carry the fused DFT / divide / IDFT pass: the last short axis does, and
  // the long axes run first; with no short axis the divide is a sweep of its own (fused_axis -1)
  p->fused_axis = p->axes.empty() ? (longs.empty() ? 0 : -1) : p->axes.back();
  p->axes.insert(p->axes.begin(), longs.begin(), longs.end());
}

// The apply schedule: forward passes over all non-trivial axes but the last, the fused
// DFT/divide/IDFT pass over the last one, then the inverse passes in reverse order; the
// 1/N scale rides on the final launch.  With chunking (3-D grids), the x and y passes run
// alternately over blocks of `chunk` z-planes, so the y pass reads planes the x pass has
// just written while they are still resident in the 256 MiB Infinity Cache (and the
// inverse pair likewise).
std::vector<Step> apply_steps(const cfp_plan_s* p, bool diag_override = false) {
  std::vector<Step> st;
  if (use_three_pass(p, diag_override)) {
    st.push_back({0, PASS_TP_ROWS_FWD, true, false, 0, -1, 0});
    st.push_back({2, PASS_TP_MID, false, false, 0, -1, 1});
    st.push_back({0, PASS_TP_ROWS_INV, false, true, 0, -1, 2});
    return st;
  }
  if (use_plane(p)) {
    st.push_back({3, PASS_PLANE_FWD, true, false, 0, -1, -1, 4});
    st.push_back({2, -1, false, false, 0, -1, -1, 0});
    st.push_back({3, PASS_PLANE_INV, false, true, 0, -1, -1, 4});
    return st;
  }
  const std::vector<int>& A = p->axes;
  if (A.empty()) {
    st.push_back({0, -1, true, true, 0, -1});  // N == 1: fused pass on a length-1 axis
    return st;
  }
  const bool chunked = p->chunk_planes > 0 && A.size() == 3 && A.back() == 2 && p->chunk_planes < p->n[2] &&
                       !p->long_axes();
  if (chunked) {
    const i64 C = p->chunk_planes, nz = p->n[2];
    for (i64 z = 0; z < nz; z += C) {
      const i64 z1 = z + C < nz ? z + C : nz;
      st.push_back({0, PASS_FWD, true, false, z, z1});
      st.push_back({1, PASS_FWD, false, false, z, z1});
    }
    st.push_back({2, -1, false, false, 0, -1});
    for (i64 z = 0; z < nz; z += C) {
      const i64 z1 = z + C < nz ? z + C : nz;
      st.push_back({1, PASS_INV, false, false, z, z1});
      st.push_back({0, PASS_INV, false, true, z, z1});
    }
    return st;
  }
  if (p->long_axes()) {
    // forward over every axis but the fused one (a long axis = its two halves), the fused pass
    // or the standalone divide, then the inverses in reverse order; 1/N on the last launch
    std::vector<int> nf;
    for (int a : A)
      if (a != p->fused_axis) nf.push_back(a);
    for (int a : nf) {
      if (p->split[a][0]) {
        st.push_back({a, PASS_FWD, st.empty(), false, 0, -1, -1, 1});
        st.push_back({a, PASS_FWD, false, false, 0, -1, -1, 2});
      } else {
        st.push_back({a, PASS_FWD, st.empty(), false, 0, -1, -1, 0});
      }
    }
    if (p->fused_axis >= 0) st.push_back({p->fused_axis, -1, st.empty(), false, 0, -1, -1, 0});
    else st.push_back({0, PASS_SYM_DIVIDE, false, false, 0, -1, -1, 3});
    for (int i = (int)nf.size() - 1; i >= 0; --i) {
      const int a = nf[i];
      if (p->split[a][0]) {
        st.push_back({a, PASS_INV, false, false, 0, -1, -1, 2});
        st.push_back({a, PASS_INV, false, false, 0, -1, -1, 1});
      } else {
        st.push_back({a, PASS_INV, false, false, 0, -1, -1, 0});
      }
    }
    st.back().scale = true;
    return st;
  }
  for (size_t i = 0; i + 1 < A.size(); ++i) st.push_back({A[i], PASS_FWD, i == 0, false, 0, -1});
  st.push_back({A.back(), -1, A.size() == 1, A.size() == 1, 0, -1});
  for (int i = (int)A.size() - 2; i >= 0; --i) st.push_back({A[i], PASS_INV, false, i == 0, 0, -1});
  return st;
}

// pass descriptor of a step; *offset = element offset of the step's first z-plane
PassDesc make_pass(const cfp_plan_s* p, const Step& q, int mode, double scale, i64* offset) {
  PassDesc d;
  d.n = (int)p->n[q.axis];
  natural_cols(q.axis, p->n, &d.ncols, &d.inner_n);
  d.in = natural_side(q.axis, p->n);
  d.out = d.in;
  d.mode = mode;
  d.scale = scale;
  d.colsym = p->colsym;
  d.axsym = p->axsym;
  d.diag = p->diag;
  *offset = 0;
  if (q.sub == 1 || q.sub == 2) {
    // long axis a = four-step halves over k = k1 + n1 k2; lower = positions of the axes below a
    const int a = q.axis;
    const i64 n1 = p->split[a][0], n2 = p->split[a][1];
    const i64 lower = a == 0 ? 1 : (a == 1 ? p->n[0] : p->n[0] * p->n[1]);
    const i64 upper = p->N / (lower * p->n[a]);
    Side sd;
    sd.seg_stride = 0;
    sd.inner_stride = 1;
    if (q.sub == 1) {  // DFT over k2: columns (lower, k1) contiguous, then the upper axes
      d.n = (int)n2;
      sd.pt_stride = n1 * lower;
      d.inner_n = lower * n1;
      sd.outer_stride = lower * p->n[a];
      d.ncols = lower * n1 * upper;
      d.tw4.lo = p->tw4lo[a];
      d.tw4.hi = p->tw4hi[a];
      d.tw4.kdiv = lower;
      d.tw4.n1 = (int)n1;
    } else {  // DFT over k1: columns (lower), then (m2, upper) with one stride lower * n1
      d.n = (int)n1;
      sd.pt_stride = lower;
      d.inner_n = lower;
      sd.outer_stride = lower * n1;
      d.ncols = lower * n2 * upper;
      if (lower == 1) sd.inner_stride = 0;
    }
    sd.seg_len = d.n;
    sd.seg_shift = ilog2_exact(d.n);
    d.in = d.out = sd;
    return d;
  }
  if (q.z1 >= 0 && q.axis < 2) {
    const i64 planes = q.z1 - q.z0;
    d.ncols = planes * (q.axis == 0 ? p->n[1] : p->n[0]);
    *offset = q.z0 * p->n[0] * p->n[1];
  }
  return d;
}

int step_mode(const cfp_plan_s* p, const Step& q, bool diag_override) {
  if (q.mode >= 0) return q.mode;
  return (diag_override || p->sym_kind == 2) ? PASS_FUSED_DIAG : PASS_FUSED_SEP;
}

// ev (profiling): 2 events per step, (*ev)[2 i] / [2 i + 1] = start / end of step i -- the 3-sweep
// kernels' own dispatch stamps, else events recorded around the step's launches
// fz (cfp_plan_apply_ex): the fused stencil (stage 0) and dots (stage 2) of the 3-sweep schedule;
// *p3grid = the workgroups of the fused P3 (its partials)
int run_apply(cfp_plan_s* p, const cd* diag_override, const cd* b, cd* x, hipStream_t s, std::vector<hipEvent_t>* ev,
              const TPArgs* fz = nullptr, unsigned* p3grid = nullptr) {
  if (!diag_override && p->sym_kind == 0)
    return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on plan (call cfp_plan_set_symbol_* first)");
  // no dispatch stamps into a graph being captured: a replay would record into events that
  // belong to other applies by then (the caller then times the apply by its own events)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
  if (capturing) {
    ev = nullptr;
    g_apply_stamp.start = g_apply_stamp.stop = nullptr;
  }
  std::vector<Step> st = apply_steps(p, diag_override != nullptr);
  const double invN = p->external_x ? 1.0 : 1.0 / (double)p->N;
  for (size_t i = 0; i < st.size(); ++i) {
    const Step& q = st[i];
    if (q.tp >= 0) {
      const int tn = (int)p->n[0];
      int trc = ensure_tw(p, tn);
      if (trc) return trc;
      TPArgs a;
      a.tw = p->tw[tn];
      a.colsym = p->colsym;
      a.axsym = p->axsym;
      a.scale = q.scale ? invN : 1.0;
      if (ev) {
        g_stamp = LaunchStamp{(*ev)[2 * i], (*ev)[2 * i + 1]};  // one kernel: stamp its dispatch
      } else if (g_apply_stamp.start) {  // the caller times the whole apply (stand-in KSP)
        if (i == 0) {
          g_stamp.start = g_apply_stamp.start;
          ++g_apply_stamp.hits;
        }
        if (i + 1 == st.size()) {
          g_stamp.stop = g_apply_stamp.stop;
          ++g_apply_stamp.hits;
        }
      }
      const cd* tin = q.from_b ? b : x;
      cd* tout = x;
      if ((tn == 256 || tn == 512) && (p->tp_shape.mid == TP_MID_BLOCKED || p->tp_shape.mid == TP_MID_BLOCKED32)) {
        if (!p->mid_buf) HIPCHK(hipMalloc(&p->mid_buf, sizeof(cd) * (size_t)p->N));
        if (q.tp == 2) tin = p->mid_buf;
        else tout = p->mid_buf;
      }
      hipError_t e;
      if (fz && q.tp == 0 && fz->pre_cls) {
        a.pre_cls = fz->pre_cls;
        a.pre_cls_x = fz->pre_cls_x;
        a.pre_mask = fz->pre_mask;
        a.pre_tab = fz->pre_tab;
        a.pre_nd = fz->pre_nd;
        a.pre_ncls = fz->pre_ncls;
        for (int k = 0; k < 3; ++k) a.pre_off[k] = fz->pre_off[k];
        e = launch_three_pass_fused(0, tn, tin, tout, a, s, nullptr);
      } else if (fz && q.tp == 2 && fz->post_nv > 0) {
        for (int j = 0; j < TP_POST_MAX; ++j) a.post_v[j] = fz->post_v[j];
        a.post_nv = fz->post_nv;
        a.post_self = fz->post_self;
        a.post_partial = fz->post_partial;
        e = launch_three_pass_fused(2, tn, tin, tout, a, s, p3grid);
      } else {
        a.krylov = fz != nullptr || g_apply_stamp.start != nullptr;  // an apply inside the stand-in KSP
        e = launch_three_pass(q.tp, tn, tin, tout, a, p->tp_shape, s);
      }
      g_stamp = LaunchStamp{};
      if (e != hipSuccess) return hip_error(e, "3-sweep launch");
      continue;
    }
    if (q.sub == 4) {
      const int pn = (int)p->n[0];
      int prc = ensure_tw(p, pn);
      if (prc) return prc;
      if (ev) HIPCHK(hipEventRecord((*ev)[2 * i], s));
      hipError_t e = launch_plane_pass(q.mode == PASS_PLANE_INV, pn, p->n[2], q.from_b ? b : x, x, p->tw[pn],
                                       q.scale ? invN : 1.0, s);
      if (e != hipSuccess) return hip_error(e, "plane pass launch");
      if (ev) HIPCHK(hipEventRecord((*ev)[2 * i + 1], s));
      continue;
    }
    if (q.sub == 3) {
      if (ev) HIPCHK(hipEventRecord((*ev)[2 * i], s));
      hipError_t e = launch_sym_divide_positions(x, p->possym[0], p->possym[1], p->possym[2], p->n[0], p->n[1],
                                                 p->n[2], s);
      if (e != hipSuccess) return hip_error(e, "symbol divide");
      if (ev) HIPCHK(hipEventRecord((*ev)[2 * i + 1], s));
      continue;
    }
    i64 off = 0;
    PassDesc d = make_pass(p, q, step_mode(p, q, diag_override != nullptr), q.scale ? invN : 1.0, &off);
    if (diag_override) d.diag = diag_override;
    int rc = ensure_tw(p, d.n);
    if (rc) return rc;
    if (ev) HIPCHK(hipEventRecord((*ev)[2 * i], s));
    hipError_t e = launch_axis_pass(d, (q.from_b ? b : x) + off, x + off, p->tw[d.n], s);
    if (e != hipSuccess) return hip_error(e, "axis pass launch");
    if (ev) HIPCHK(hipEventRecord((*ev)[2 * i + 1], s));
  }
  return CFP_SUCCESS;
}

int run_transform(cfp_plan_s* p, bool inverse, const cd* in, cd* out, hipStream_t s) {
  if (p->long_axes())
    return set_error(CFP_ERR_SUP, "forward / backward transforms of axes above 4096 are not exposed (their "
                                  "spectrum stays in four-step order inside the apply)");
  if (p->axes.empty()) {
    if (in != out) HIPCHK(hipMemcpyAsync(out, in, sizeof(cd), hipMemcpyDeviceToDevice, s));
    return CFP_SUCCESS;
  }
  bool first = true;
  for (int ax : p->axes) {
    i64 off = 0;
    PassDesc d = make_pass(p, Step{ax, inverse ? PASS_INV : PASS_FWD, first, false, 0, -1},
                           inverse ? PASS_INV : PASS_FWD, 1.0, &off);
    int rc = ensure_tw(p, d.n);
    if (rc) return rc;
    hipError_t e = launch_axis_pass(d, first ? in : out, out, p->tw[d.n], s);
    if (e != hipSuccess) return hip_error(e, "axis pass launch");
    first = false;
  }
  return CFP_SUCCESS;
}

constexpr size_t kMaxGraphs = 64;  // GMRES(30) applies the PC to ~32 distinct Krylov vectors

// A cached graph may still be running in the caller's stream (hipGraphLaunch is
// asynchronous), so the device is drained before any executable graph is destroyed.  The
// callers are setters and the 65th (b, x) pair, never the steady-state apply.
void graph_clear(cfp_plan_s* p) {
  if (p->graphs.empty()) return;
  hipDeviceSynchronize();
  for (auto& g : p->graphs) hipGraphExecDestroy(g.exec);
  p->graphs.clear();
}

void free_symbol(cfp_plan_s* p) {
  graph_clear(p);
  if (p->colsym) hipFree(p->colsym);
  if (p->axsym) hipFree(p->axsym);
  if (p->diag) hipFree(p->diag);
  p->colsym = p->axsym = p->diag = nullptr;
  for (int a = 0; a < 3; ++a) {
    if (p->possym[a]) hipFree(p->possym[a]);
    p->possym[a] = nullptr;
  }
  p->sym_kind = 0;
}

// frequency held at position q of a long axis: q = m1 + n1 m2 holds m = m2 + n2 m1
i64 long_freq(const cfp_plan_s* p, int a, i64 q) {
  const i64 n1 = p->split[a][0], n2 = p->split[a][1];
  return q / n1 + n2 * (q % n1);
}

std::complex<double> lamc(const double lam[6], int a) { return {lam[2 * a], lam[2 * a + 1]}; }

// Build colsym/axsym from per-axis host vectors s_d[k] = lambda_d * c_d_hat[k].
int upload_separable(cfp_plan_s* p, const std::vector<cd> s_nat[3]) {
  // the kernels index the symbol by position: a long axis holds frequency long_freq(q) at q
  std::vector<cd> s[3];
  for (int a = 0; a < 3; ++a) {
    s[a] = s_nat[a];
    if (p->split[a][0])
      for (i64 q = 0; q < p->n[a]; ++q) s[a][(size_t)q] = s_nat[a][(size_t)long_freq(p, a, q)];
  }
  if (p->fused_axis < 0) {  // no short axis: position-indexed tables for the standalone divide
    free_symbol(p);
    for (int a = 0; a < 3; ++a) {
      HIPCHK(hipMalloc(&p->possym[a], sizeof(cd) * (size_t)p->n[a]));
      HIPCHK(hipMemcpy(p->possym[a], s[a].data(), sizeof(cd) * (size_t)p->n[a], hipMemcpyHostToDevice));
    }
    for (int a = 0; a < 3; ++a) p->sym1d[a] = s_nat[a];
    p->sym_kind = 1;
    return CFP_SUCCESS;
  }
  const int f = p->fused_axis;
  const i64 nf = p->n[f];
  i64 ncols, inner_n;
  natural_cols(f, p->n, &ncols, &inner_n);
  std::vector<cd> col((size_t)ncols), ax((size_t)nf);
  // column g of axis f -> the coordinates of the other two axes
  for (i64 g = 0; g < ncols; ++g) {
    i64 idx[3];
    if (f == 0) { idx[0] = 0; idx[1] = g % p->n[1]; idx[2] = g / p->n[1]; }
    else if (f == 1) { idx[0] = g % p->n[0]; idx[1] = 0; idx[2] = g / p->n[0]; }
    else { idx[0] = g % p->n[0]; idx[1] = g / p->n[0]; idx[2] = 0; }
    // reference summation order: ((x + y) + z) + 1 with the fused axis' term added last
    double re = 0.0, im = 0.0;
    for (int a = 0; a < 3; ++a) {
      if (a == f) continue;
      re += s[a][(size_t)idx[a]].x;
      im += s[a][(size_t)idx[a]].y;
    }
    col[(size_t)g] = make_cd(re, im);
  }
  for (i64 k = 0; k < nf; ++k) ax[(size_t)k] = s[f][(size_t)k];
  free_symbol(p);
  HIPCHK(hipMalloc(&p->colsym, sizeof(cd) * (size_t)ncols));
  HIPCHK(hipMalloc(&p->axsym, sizeof(cd) * (size_t)nf));
  HIPCHK(hipMemcpy(p->colsym, col.data(), sizeof(cd) * (size_t)ncols, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(p->axsym, ax.data(), sizeof(cd) * (size_t)nf, hipMemcpyHostToDevice));
  for (int a = 0; a < 3; ++a) p->sym1d[a] = s_nat[a];
  p->sym_kind = 1;
  return CFP_SUCCESS;
}

int set_separable(cfp_plan_s* p, const std::vector<cd> hat[3], const double lam[6]) {
  std::vector<cd> s[3];
  for (int a = 0; a < 3; ++a) {
    std::complex<double> l = lamc(lam, a);
    s[a].resize(hat[a].size());
    for (size_t k = 0; k < hat[a].size(); ++k) {
      std::complex<double> c(hat[a][k].x, hat[a][k].y);
      // c * lambda as in vec_kronecker_product_identity_* (src/FftLinearSolver_3D.c:100,122)
      const double re = c.real() * l.real() - c.imag() * l.imag();
      const double im = c.real() * l.imag() + c.imag() * l.real();
      s[a][k] = make_cd(re, im);
    }
  }
  ++p->sym_version;
  return upload_separable(p, s);
}

}  // namespace

extern "C" int cfp_plan_create(cfp_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int device) {
  if (!plan) return set_error(CFP_ERR_ARG_NULL, "plan is NULL");
  *plan = nullptr;
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const int64_t dims_in[3] = {nx, ny, nz};
  int split[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  for (int a = 0; a < 3; ++a) {
    if (dims_in[a] <= 4096) continue;
    // four-step: n = n1 n2 with both halves <= 4096, as balanced as possible
    i64 best = 0;
    for (i64 d = 2; d <= 4096; ++d)
      if (dims_in[a] % d == 0 && dims_in[a] / d <= 4096) {
        const i64 o = dims_in[a] / d;
        if (best == 0 || std::llabs(d - o) < std::llabs(best - dims_in[a] / best)) best = d;
      }
    if (best == 0)
      return set_error(CFP_ERR_SUP, "axis length %lld is not a product of two factors <= 4096", (long long)dims_in[a]);
    split[a][0] = (int)best;
    split[a][1] = (int)(dims_in[a] / best);
  }
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_error(CFP_ERR_ARG_OUTOFRANGE, "device %d out of range", device);
  DeviceGuard dg(device);
  std::unique_ptr<cfp_plan_s> p(new cfp_plan_s);
  p->device = device;
  p->n[0] = nx; p->n[1] = ny; p->n[2] = nz;
  p->N = nx * ny * nz;
  std::memcpy(p->split, split, sizeof(split));
  order_axes(p.get());
  for (int a : p->axes) {
    if (p->split[a][0]) {
      int rc = ensure_tw(p.get(), p->split[a][0]);
      if (!rc) rc = ensure_tw(p.get(), p->split[a][1]);
      if (rc) return rc;
      // four-step twiddles W_n^j (j < 4096) and W_n^{4096 i} (i <= n / 4096), long double
      const i64 n = p->n[a];
      const i64 nhi = n / 4096 + 1;
      std::vector<cd> lo(4096), hi((size_t)nhi);
      const long double two_pi = 6.283185307179586476925286766559L;
      for (i64 j = 0; j < 4096; ++j) {
        const long double t = two_pi * (long double)j / (long double)n;
        lo[(size_t)j] = make_cd((double)cosl(t), (double)-sinl(t));
      }
      for (i64 i = 0; i < nhi; ++i) {
        const long double t = two_pi * (long double)((4096 * i) % n) / (long double)n;
        hi[(size_t)i] = make_cd((double)cosl(t), (double)-sinl(t));
      }
      HIPCHK(hipMalloc(&p->tw4lo[a], sizeof(cd) * 4096));
      HIPCHK(hipMalloc(&p->tw4hi[a], sizeof(cd) * (size_t)nhi));
      HIPCHK(hipMemcpy(p->tw4lo[a], lo.data(), sizeof(cd) * 4096, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(p->tw4hi[a], hi.data(), sizeof(cd) * (size_t)nhi, hipMemcpyHostToDevice));
      continue;
    }
    int rc = ensure_tw(p.get(), (int)p->n[a]);
    if (rc) return rc;
  }
  if (p->axes.empty()) {
    int rc = ensure_tw(p.get(), 1);
    if (rc) return rc;
  }
  *plan = p.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_destroy(cfp_plan_t p) {
  if (!p) return CFP_SUCCESS;
  DeviceGuard dg(p->device);
  free_symbol(p);
  for (auto& kv : p->tw) hipFree(kv.second);
  for (int a = 0; a < 3; ++a) {
    if (p->tw4lo[a]) hipFree(p->tw4lo[a]);
    if (p->tw4hi[a]) hipFree(p->tw4hi[a]);
  }
  if (p->host_stage) hipFree(p->host_stage);
  if (p->mid_buf) hipFree(p->mid_buf);
  if (p->post_partial) hipFree(p->post_partial);
  if (p->pre_buf) hipFree(p->pre_buf);
  graph_clear(p);
  if (p->cap_stream) hipStreamDestroy(p->cap_stream);
  for (auto& e : p->prof_ev) hipEventDestroy(e);
  delete p;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_symbol_version(cfp_plan_t p, uint64_t* version) {
  if (!p || !version) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *version = p->sym_version;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_set_symbol_transport(cfp_plan_t p, const double lam[6]) {
  if (!p || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  std::vector<cd> hat[3];
  for (int a = 0; a < 3; ++a) hat[a] = host_transport_symbol(p->n[a]);
  return set_separable(p, hat, lam);
}

extern "C" int cfp_plan_set_symbol_separable(cfp_plan_t p, const double* cx, const double* cy, const double* cz,
                                             const double lam[6]) {
  if (!p || !cx || !cy || !cz || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  std::vector<cd> hat[3];
  const double* src[3] = {cx, cy, cz};
  for (int a = 0; a < 3; ++a) {
    hat[a].resize((size_t)p->n[a]);
    std::memcpy(hat[a].data(), src[a], sizeof(cd) * (size_t)p->n[a]);
  }
  return set_separable(p, hat, lam);
}

extern "C" int cfp_plan_set_diag(cfp_plan_t p, const double* diag, int on_device) {
  if (!p || !diag) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (p->long_axes()) return set_error(CFP_ERR_SUP, "an explicit Diag needs axes <= 4096 (use a separable symbol)");
  DeviceGuard dg(p->device);
  free_symbol(p);
  ++p->sym_version;
  HIPCHK(hipMalloc(&p->diag, sizeof(cd) * (size_t)p->N));
  HIPCHK(hipMemcpy(p->diag, diag, sizeof(cd) * (size_t)p->N, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
  p->sym_kind = 2;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_get_diag(cfp_plan_t p, double* diag_dev, void* stream) {
  if (!p || !diag_dev) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  hipStream_t s = (hipStream_t)stream;
  if (p->sym_kind == 2) {
    HIPCHK(hipMemcpyAsync(diag_dev, p->diag, sizeof(cd) * (size_t)p->N, hipMemcpyDeviceToDevice, s));
    return CFP_SUCCESS;
  }
  if (p->sym_kind != 1) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set");
  cd* tmp[3] = {nullptr, nullptr, nullptr};
  for (int a = 0; a < 3; ++a) {
    HIPCHK(hipMalloc(&tmp[a], sizeof(cd) * (size_t)p->n[a]));
    HIPCHK(hipMemcpy(tmp[a], p->sym1d[a].data(), sizeof(cd) * (size_t)p->n[a], hipMemcpyHostToDevice));
  }
  const cd one = make_cd(1.0, 0.0);
  hipError_t e = launch_build_diag_separable((cd*)diag_dev, tmp[0], tmp[1], tmp[2], p->n[0], p->n[1], p->n[2], one,
                                             one, one, s);
  hipStreamSynchronize(s);
  for (int a = 0; a < 3; ++a) hipFree(tmp[a]);
  if (e != hipSuccess) return hip_error(e, "build diag");
  return CFP_SUCCESS;
}

// Graph mode: replay the captured launches of this (b, x) pair, or run the apply eagerly
// (which also builds anything allocated lazily, e.g. twiddle tables) and capture the same
// launch list for the next call.
static int graph_apply(cfp_plan_s* p, const cd* b, cd* x, hipStream_t s) {
  for (const auto& g : p->graphs)
    if (g.b == b && g.x == x) {
      HIPCHK(hipGraphLaunch(g.exec, s));
      return CFP_SUCCESS;
    }
  int rc = run_apply(p, nullptr, b, x, s, nullptr);
  if (rc) return rc;
  if (!p->cap_stream) HIPCHK(hipStreamCreateWithFlags(&p->cap_stream, hipStreamNonBlocking));
  HIPCHK(hipStreamBeginCapture(p->cap_stream, hipStreamCaptureModeThreadLocal));
  rc = run_apply(p, nullptr, b, x, p->cap_stream, nullptr);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(p->cap_stream, &g);
  if (rc || e != hipSuccess) {
    if (g) hipGraphDestroy(g);
    return rc ? rc : hip_error(e, "apply graph capture");
  }
  hipGraphExec_t exec = nullptr;
  e = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return hip_error(e, "apply graph instantiate");
  if (p->graphs.size() >= kMaxGraphs) {
    HIPCHK(hipDeviceSynchronize());  // the evicted graph may still be in flight
    hipGraphExecDestroy(p->graphs.front().exec);
    p->graphs.erase(p->graphs.begin());
  }
  p->graphs.push_back({b, x, exec});
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_set_graph(cfp_plan_t p, int on) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  DeviceGuard dg(p->device);
  graph_clear(p);
  p->graph_on = on != 0;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_apply(cfp_plan_t p, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  // profiling: this apply's own event slot (skipped if the schedule changed since begin)
  const bool sample = p->prof_cap && (p->prof_calls++ % p->prof_every) == 0;
  if (sample && p->prof_used < p->prof_cap && 2 * apply_steps(p).size() == p->prof_stride) {
    std::vector<hipEvent_t> ev(p->prof_ev.begin() + (long)(p->prof_used * p->prof_stride),
                               p->prof_ev.begin() + (long)((p->prof_used + 1) * p->prof_stride));
    ++p->prof_used;
    return run_apply(p, nullptr, (const cd*)b, (cd*)x, (hipStream_t)stream, &ev);
  }
  if (p->graph_on) return graph_apply(p, (const cd*)b, (cd*)x, (hipStream_t)stream);
  return run_apply(p, nullptr, (const cd*)b, (cd*)x, (hipStream_t)stream, nullptr);
}

// whether cfp_plan_apply_ex runs the stencil and the dots inside the apply's own sweeps
static bool apply_ex_fusable(const cfp_plan_s* p, const cfp_stencil_t* st, int nv) {
  bool pre_ok = !st || (st->x_local && st->nd >= 1 && st->nd <= 3 && st->ncls >= 1 && st->ncls <= TP_PRE_MAX_CLS);
  for (int k = 0; st && k < st->nd; ++k) pre_ok = pre_ok && st->off[k] >= -1 && st->off[k] <= 1;
  const bool cube = p->n[0] == p->n[1] && p->n[1] == p->n[2];
  return cube && use_three_pass(p, false) && three_pass_fused_supported((int)p->n[0], p->tp_shape) && pre_ok &&
         nv >= 0 && nv <= TP_POST_MAX;
}

extern "C" int cfp_plan_apply_ex_fusable(cfp_plan_t p, const cfp_stencil_t* pre, int post_nv, int* fusable) {
  if (!p || !fusable) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *fusable = apply_ex_fusable(p, pre, post_nv) ? 1 : 0;
  return CFP_SUCCESS;
}

// The Krylov step around one apply (circulant_fft.h cfp_apply_ex_t): y = A b in P1 and the dots
// in P3 of the 256^3 3-sweep schedule, or the stencil and the dots as their own kernels around a
// plain apply wherever that schedule or the stencil's shape does not allow the fusion.
extern "C" int cfp_plan_apply_ex(cfp_plan_t p, const double* b, double* x, void* stream, cfp_apply_ex_t* ex) {
  if (!p || !b || !x || !ex) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  const cfp_stencil_t* st = ex->pre;
  const int nv = ex->post_nv;
  if (nv < 0 || nv > 8) return set_error(CFP_ERR_ARG_OUTOFRANGE, "post_nv must be in 0..8");
  if (nv > 0 && !ex->post_out) return set_error(CFP_ERR_ARG_NULL, "post_out is NULL");
  if (st) {
    if (!st->cls || !st->mask || !st->tab) return set_error(CFP_ERR_ARG_NULL, "stencil arrays are NULL");
    if (st->nd < 1 || st->nd > DIA_MAX || st->ncls < 1 || st->ncls > 256)
      return set_error(CFP_ERR_ARG_OUTOFRANGE, "stencil: 1 <= nd <= 8, 1 <= ncls <= 256");
    if ((const void*)b == (const void*)x) return set_error(CFP_ERR_ARG_WRONG, "b and x must differ with a stencil");
  }
  ex->fused = 0;
  if (!st && nv == 0) return cfp_plan_apply(p, b, x, stream);
  DeviceGuard dg(p->device);
  hipStream_t s = (hipStream_t)stream;
  if (apply_ex_fusable(p, st, nv)) {
    TPArgs fz;
    if (st) {
      fz.pre_cls = st->cls;
      fz.pre_cls_x = st->cls_x;
      fz.pre_mask = st->mask;
      fz.pre_tab = (const cd*)st->tab;
      fz.pre_nd = st->nd;
      fz.pre_ncls = st->ncls;
      for (int k = 0; k < st->nd; ++k) fz.pre_off[k] = (int)st->off[k];
    }
    if (nv > 0) {
      if (!p->post_partial) HIPCHK(hipMalloc(&p->post_partial, sizeof(double) * 16 * 1024));
      for (int j = 0; j < nv; ++j) {
        fz.post_v[j] = (const cd*)ex->post_v[j];
        if (!ex->post_v[j] || ex->post_v[j] == x) fz.post_self |= 1 << j;
      }
      fz.post_nv = nv;
      fz.post_partial = p->post_partial;
    }
    unsigned g = 0;
    int rc = run_apply(p, nullptr, (const cd*)b, (cd*)x, s, nullptr, &fz, &g);
    if (rc) return rc;
    if (nv > 0) {
      if (g < 1 || g > 1024) return set_error(CFP_ERR_LIB, "fused P3 grid out of range");
      hipError_t e = blas_mdot_finish(p->post_partial, (int)g, nv, ex->post_out, s);
      if (e != hipSuccess) return hip_error(e, "dots finish");
    }
    ex->fused = 1;
    return CFP_SUCCESS;
  }
  const double* src = b;
  if (st) {
    if (!p->pre_buf) HIPCHK(hipMalloc(&p->pre_buf, sizeof(cd) * (size_t)p->N));
    DiaDesc d;
    for (int k = 0; k < st->nd; ++k) d.off[k] = st->off[k];
    d.nd = st->nd;
    d.ncls = st->ncls;
    hipError_t e = blas_dia_spmv(p->N, d, st->cls, st->mask, (const cd*)st->tab, (const cd*)b, p->pre_buf, s);
    if (e != hipSuccess) return hip_error(e, "stencil");
    src = (const double*)p->pre_buf;
  }
  int rc = cfp_plan_apply(p, src, x, stream);
  if (rc || nv == 0) return rc;
  const cd* ys[8];
  for (int j = 0; j < nv; ++j) ys[j] = (const cd*)ex->post_v[j];
  hipError_t e = blas_mdot_dev((const cd*)x, nv, ys, p->N, ex->post_out, s);
  if (e != hipSuccess) return hip_error(e, "dots");
  return CFP_SUCCESS;
}

static void profile_free(cfp_plan_s* p) {
  for (auto& e : p->prof_ev) hipEventDestroy(e);
  p->prof_ev.clear();
  p->prof_stride = p->prof_cap = p->prof_used = p->prof_calls = 0;
  p->prof_every = 1;
}

// Start recording per-launch events in every `every`-th call of cfp_plan_apply (the first,
// then every-th after it), at most `max_applies` of them.
extern "C" int cfp_plan_profile_begin(cfp_plan_t p, int max_applies, int every) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (max_applies < 1 || max_applies > 100000) return set_error(CFP_ERR_ARG_OUTOFRANGE, "max_applies out of range");
  if (every < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "every must be >= 1");
  DeviceGuard dg(p->device);
  profile_free(p);
  p->prof_stride = 2 * apply_steps(p).size();
  p->prof_ev.resize(p->prof_stride * (size_t)max_applies, nullptr);
  for (auto& e : p->prof_ev) {
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (r != hipSuccess) {
      profile_free(p);
      return hip_error(r, "hipEventCreate");
    }
  }
  p->prof_cap = (size_t)max_applies;
  p->prof_used = 0;
  p->prof_every = (size_t)every;
  p->prof_calls = 0;
  return CFP_SUCCESS;
}

// Stop recording; ms_out[i] = mean duration of launch i over the recorded applies (ms_out holds
// cfp_plan_num_passes entries), *applies = how many applies were recorded.
extern "C" int cfp_plan_profile_end(cfp_plan_t p, double* ms_out, int* applies) {
  if (!p || !ms_out || !applies) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!p->prof_cap) return set_error(CFP_ERR_ARG_WRONGSTATE, "profiling was not started");
  DeviceGuard dg(p->device);
  const size_t np = p->prof_stride / 2, used = p->prof_used;
  std::vector<double> acc(np, 0.0);
  int rc = CFP_SUCCESS;
  if (used > 0) {
    hipError_t e = hipEventSynchronize(p->prof_ev[used * p->prof_stride - 1]);
    if (e != hipSuccess) rc = hip_error(e, "event sync");
  }
  for (size_t a = 0; a < used && !rc; ++a)
    for (size_t i = 0; i < np; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, p->prof_ev[a * p->prof_stride + 2 * i], p->prof_ev[a * p->prof_stride + 2 * i + 1]);
      acc[i] += ms;
    }
  for (size_t i = 0; i < np; ++i) ms_out[i] = used ? acc[i] / (double)used : 0.0;
  *applies = (int)used;
  profile_free(p);
  return rc;
}

extern "C" int cfp_plan_apply_with_diag(cfp_plan_t p, const double* diag, const double* b, double* x, void* stream) {
  if (!p || !diag || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (p->long_axes()) return set_error(CFP_ERR_SUP, "an explicit Diag needs axes <= 4096 (use a separable symbol)");
  DeviceGuard dg(p->device);
  return run_apply(p, (const cd*)diag, (const cd*)b, (cd*)x, (hipStream_t)stream, nullptr);
}

// host b -> the plan's persistent device staging buffer (allocated once) -> in-place apply ->
// host x; every copy is checked (a failed copy is CFP_ERR_LIB, never stale data)
static int apply_host_impl(cfp_plan_s* p, const cd* diag, const double* b, double* x) {
  const size_t bytes = sizeof(cd) * (size_t)p->N;
  if (!p->host_stage) HIPCHK(hipMalloc(&p->host_stage, bytes));
  HIPCHK(hipMemcpy(p->host_stage, b, bytes, hipMemcpyHostToDevice));
  int rc = run_apply(p, diag, p->host_stage, p->host_stage, nullptr, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpy(x, p->host_stage, bytes, hipMemcpyDeviceToHost));
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_apply_host(cfp_plan_t p, const double* b, double* x) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  return apply_host_impl(p, nullptr, b, x);
}

extern "C" int cfp_plan_apply_with_diag_host(cfp_plan_t p, const double* diag_dev, const double* b, double* x) {
  if (!p || !diag_dev || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (p->long_axes()) return set_error(CFP_ERR_SUP, "an explicit Diag needs axes <= 4096 (use a separable symbol)");
  DeviceGuard dg(p->device);
  return apply_host_impl(p, (const cd*)diag_dev, b, x);
}

extern "C" int cfp_plan_forward(cfp_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  return run_transform(p, false, (const cd*)in, (cd*)out, (hipStream_t)stream);
}

extern "C" int cfp_plan_backward(cfp_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  DeviceGuard dg(p->device);
  return run_transform(p, true, (const cd*)in, (cd*)out, (hipStream_t)stream);
}

extern "C" int cfp_plan_set_chunking(cfp_plan_t p, int64_t chunk_planes) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  graph_clear(p);
  if (chunk_planes < 0) return set_error(CFP_ERR_ARG_OUTOFRANGE, "chunk_planes must be >= 0");
  p->chunk_planes = chunk_planes;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_set_schedule(cfp_plan_t p, int schedule) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (schedule < CFP_SCHEDULE_AUTO || schedule > CFP_SCHEDULE_PLANE)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "unknown schedule %d", schedule);
  if (schedule == CFP_SCHEDULE_PLANE &&
      (p->n[0] != p->n[1] || !plane_supported(p->n[0]) || p->n[2] < 2 || p->long_axes() || p->external_x))
    return set_error(CFP_ERR_SUP, "the plane schedule needs n_x = n_y in {64, 100, 128} and n_z > 1");
  if (schedule == CFP_SCHEDULE_THREE_PASS && !three_pass_supported(p->n) && !three_pass_sq_supported(p->n))
    return set_error(CFP_ERR_SUP, "the 3-sweep schedule needs a 100^3, 128^3, 256^3 or 512^3 grid");
  DeviceGuard dg(p->device);
  graph_clear(p);
  const int f_old = p->fused_axis;
  p->schedule = schedule;
  order_axes(p);
  // the separable tables are laid out for the fused axis: rebuild them if it moved
  if (p->sym_kind == 1 && p->fused_axis != f_old) {
    std::vector<cd> s[3] = {p->sym1d[0], p->sym1d[1], p->sym1d[2]};
    return upload_separable(p, s);
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_set_three_pass_shape(cfp_plan_t p, int n1, int mid) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  graph_clear(p);
  if (!three_pass_shape_valid(n1, mid, p->n[0] == p->n[1] && p->n[1] == p->n[2] ? p->n[0] : 0))
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "3-sweep shape n1=%d mid=%d is not one of the built shapes", n1, mid);
  p->tp_shape.n1 = n1;
  p->tp_shape.mid = mid;
  if ((p->n[0] == 256 || p->n[0] == 512) && (mid == TP_MID_BLOCKED || mid == TP_MID_BLOCKED32) && !p->mid_buf) {
    DeviceGuard g(p->device);
    HIPCHK(hipMalloc(&p->mid_buf, sizeof(cd) * (size_t)p->N));  // here, not inside a graph capture
  }
  return CFP_SUCCESS;
}

// internal (cfp_host.h): the real plan transforms x itself (r2c / c2r rows) and runs this
// plan's y/z passes over the half spectrum without the 1/N scale
extern "C" int cfp_plan_set_external_x(cfp_plan_t p, int on) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  DeviceGuard dg(p->device);
  graph_clear(p);
  const int f_old = p->fused_axis;
  p->external_x = on != 0;
  order_axes(p);
  if (p->axes.empty()) return set_error(CFP_ERR_SUP, "external x needs a non-trivial y or z axis");
  if (p->sym_kind == 1 && p->fused_axis != f_old) {
    std::vector<cd> s[3] = {p->sym1d[0], p->sym1d[1], p->sym1d[2]};
    return upload_separable(p, s);
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_num_passes(cfp_plan_t p, int* passes) {
  if (!p || !passes) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *passes = (int)apply_steps(p).size();
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_pass_info(cfp_plan_t p, int pass, int* axis, int* n, int64_t* ncols, int* mode, int* fast) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  std::vector<Step> st = apply_steps(p);
  if (pass < 0 || pass >= (int)st.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "pass index");
  if (st[pass].tp >= 0) {  // 3-sweep launches: axis 3 = "x + y stage 1", 4 = "y stage 2 + z"
    if (axis) *axis = st[pass].tp == 1 ? 4 : 3;
    if (n) *n = (int)p->n[0];
    if (ncols) *ncols = p->N / p->n[0];
    if (mode) *mode = st[pass].mode;
    if (fast) *fast = 1;
    return CFP_SUCCESS;
  }
  if (st[pass].sub == 4) {  // plane passes: axis 3 = "x + y"
    if (axis) *axis = 3;
    if (n) *n = (int)p->n[0];
    if (ncols) *ncols = p->n[2];
    if (mode) *mode = st[pass].mode;
    if (fast) *fast = 1;
    return CFP_SUCCESS;
  }
  if (st[pass].sub == 3) {  // the standalone symbol divide of an all-long grid
    if (axis) *axis = -1;
    if (n) *n = 1;
    if (ncols) *ncols = p->N;
    if (mode) *mode = PASS_SYM_DIVIDE;
    if (fast) *fast = 1;
    return CFP_SUCCESS;
  }
  const int m = step_mode(p, st[pass], false);
  i64 off = 0;
  PassDesc d = make_pass(p, st[pass], m, 1.0, &off);
  if (axis) *axis = st[pass].axis;
  if (n) *n = d.n;
  if (ncols) *ncols = d.ncols;
  if (mode) *mode = m;
  if (fast) *fast = fast_path_supported(d) ? 1 : 0;
  return CFP_SUCCESS;
}

extern "C" int cfp_plan_time_passes(cfp_plan_t p, const double* b, double* x, int iters, double* ms_out, void* stream) {
  if (!p || !b || !x || !ms_out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (iters < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "iters must be >= 1");
  DeviceGuard dg(p->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t np = apply_steps(p).size();
  std::vector<double> acc(np, 0.0);
  std::vector<hipEvent_t> ev(2 * np);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  int rc = CFP_SUCCESS;
  for (int it = 0; it < iters && rc == CFP_SUCCESS; ++it) {
    rc = run_apply(p, nullptr, (const cd*)b, (cd*)x, s, &ev);
    if (rc) break;
    hipError_t e = hipEventSynchronize(ev[2 * np - 1]);
    if (e != hipSuccess) { rc = hip_error(e, "event sync"); break; }
    for (size_t i = 0; i < np; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
      acc[i] += ms;
    }
  }
  for (auto& e : ev) hipEventDestroy(e);
  if (rc) return rc;
  for (size_t i = 0; i < np; ++i) ms_out[i] = acc[i] / iters;
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ vector kernels
extern "C" int cfp_pointwise_divide(double* w, const double* x, const double* y, int64_t n, void* stream) {
  if (!w || !x || !y) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  hipError_t e = launch_pointwise_divide((cd*)w, (const cd*)x, (const cd*)y, n, (hipStream_t)stream);
  return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "pointwise divide");
}

extern "C" int cfp_scale(double* x, double re, double im, int64_t n, void* stream) {
  if (!x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  hipError_t e = launch_scale((cd*)x, make_cd(re, im), n, (hipStream_t)stream);
  return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "scale");
}

extern "C" int cfp_fill_uniform(double* x, int64_t n, uint64_t seed, int64_t offset, void* stream) {
  if (!x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  hipError_t e = launch_fill_uniform((cd*)x, n, seed, offset, (hipStream_t)stream);
  return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "fill uniform");
}

extern "C" int cfp_build_diag_3d(double* diag, const double* cx, const double* cy, const double* cz, int64_t nx,
                                 int64_t ny, int64_t nz, const double lam[6], void* stream) {
  if (!diag || !cx || !cy || !cz || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  hipError_t e = launch_build_diag_separable((cd*)diag, (const cd*)cx, (const cd*)cy, (const cd*)cz, nx, ny, nz,
                                             make_cd(lam[0], lam[1]), make_cd(lam[2], lam[3]),
                                             make_cd(lam[4], lam[5]), (hipStream_t)stream);
  return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "build diag");
}

extern "C" int cfp_transport_symbol_1d(int64_t n, double* out) {
  if (!out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (n < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "n must be >= 1");
  std::vector<cd> s = host_transport_symbol(n);
  std::memcpy(out, s.data(), sizeof(cd) * (size_t)n);
  return CFP_SUCCESS;
}
