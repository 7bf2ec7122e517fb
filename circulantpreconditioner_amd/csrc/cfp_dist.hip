// cfp_dist.hip -- z-slab decomposition of the circulant apply over P GPUs.
//
// Replaces the FFTW-MPI slab transposes that PETSc's MATFFTW performs inside MatMult /
// MatMultTranspose when size > 1 (src/FftLinearSolver_3D.c:170,180).
// The y passes read/write the exchange chunks directly (no pack/unpack kernels): the
// forward y pass writes point ky of a column to chunk ky / nyl, the inverse y pass reads
// it back from there, so an all-to-all is a set of contiguous peer messages.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <complex>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/circulant_fft_dist.h"
#include "cfp_host.h"
#include "cfp_internal.h"
#include "cfp_three_pass.h"

using namespace cfp;

#define HIPCHK(expr)                                        \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return cfp::hip_error(_e, #expr); \
  } while (0)
#define NCCLCHK(expr)                                                                            \
  do {                                                                                           \
    ncclResult_t _r = (expr);                                                                    \
    if (_r != ncclSuccess) return cfp::set_error(CFP_ERR_LIB, "%s: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)

namespace {

struct SlabLayout {
  i64 nx, ny, nz;
  int P, r;
  i64 nzl, nyl, z0, y0, local, chunk, offset;
};

int make_layout(i64 nx, i64 ny, i64 nz, int P, int r, SlabLayout* L) {
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  if (P < 1 || r < 0 || r >= P) return set_error(CFP_ERR_ARG_OUTOFRANGE, "rank %d of %d", r, P);
  if (nz % P || ny % P)
    return set_error(CFP_ERR_ARG_SIZ, "slab decomposition needs nranks | nz and nranks | ny (nz=%lld ny=%lld P=%d)",
                     (long long)nz, (long long)ny, P);
  if (nx > 4096 || ny > 4096 || nz > 4096) return set_error(CFP_ERR_SUP, "axis lengths above 4096 unsupported");
  L->nx = nx; L->ny = ny; L->nz = nz; L->P = P; L->r = r;
  L->nzl = nz / P; L->nyl = ny / P;
  L->z0 = r * L->nzl; L->y0 = r * L->nyl;
  L->local = L->nzl * ny * nx;
  L->chunk = L->nzl * L->nyl * nx;
  L->offset = L->z0 * ny * nx;
  return CFP_SUCCESS;
}

Side side(i64 inner_stride, i64 outer_stride, i64 pt_stride, i64 seg_len, i64 seg_stride) {
  Side s;
  s.inner_stride = inner_stride;
  s.outer_stride = outer_stride;
  s.pt_stride = pt_stride;
  s.seg_len = (int)seg_len;
  s.seg_shift = ilog2_exact(seg_len);
  s.seg_stride = seg_stride;
  return s;
}

enum Buf { B_IN = 0, B_X = 1, B_W = 2 };

struct Step {
  bool exchange;
  PassDesc pass;  // kernel steps
  int src, dst;   // buffer ids
  int fused;      // 1 if this is the symbol pass
  int axis;       // 0, 1, 2 (kernel steps)
  int tp;         // >= 0: stage of the 3-sweep slab schedule (cfp_three_pass.hip)
};

// 256^3: 3 local sweeps per rank (x + y1 | y2 + z + symbol + inverses | inverse), the same two
// exchanges; otherwise 5 axis passes.  AUTO takes 3 sweeps for P <= 4 only: measured per rank
// (tools/slab_local_timing.py, profiles/r02i_slab_local.txt) 174 vs 219 us at P = 2 and 90 vs
// 119 us at P = 4, a tie at P = 8 (P2 has 128 units for 256 CUs) and a loss at P = 16.
bool slab_three(const SlabLayout& L, int schedule) {
  const i64 n[3] = {L.nx, L.ny, L.nz};
  if (schedule == CFP_SCHEDULE_FIVE_PASS || !three_pass_slab_supported(n, L.P)) return false;
  return schedule == CFP_SCHEDULE_THREE_PASS || L.P <= 4;
}

std::vector<Step> slab_steps(const SlabLayout& L, int schedule = CFP_SCHEDULE_AUTO) {
  std::vector<Step> st;
  if (slab_three(L, schedule)) {
    // P1 natural planes -> per-peer chunks (work), exchange into x as [nz][nyl][nx] (the rank's k1
    // rows), P2 in place, exchange back into work (chunks), P3 -> x natural, x 1/N
    auto tp = [&](int stage, int src, int dst) {
      Step s;
      std::memset(&s, 0, sizeof(s));
      s.exchange = false;
      s.tp = stage;
      s.axis = stage == 1 ? 2 : 0;
      s.pass.n = (int)L.nx;
      s.pass.mode = stage == 0 ? PASS_TP_ROWS_FWD : (stage == 1 ? PASS_TP_MID : PASS_TP_ROWS_INV);
      s.pass.scale = stage == 2 ? 1.0 / (double)(L.nx * L.ny * L.nz) : 1.0;
      s.src = src; s.dst = dst; s.fused = stage == 1;
      st.push_back(s);
    };
    auto ex = [&](int src, int dst) {
      Step s;
      std::memset(&s, 0, sizeof(s));
      s.exchange = true; s.src = src; s.dst = dst; s.tp = -1;
      st.push_back(s);
    };
    tp(0, B_IN, B_W);
    ex(B_W, B_X);
    tp(1, B_X, B_X);
    ex(B_X, B_W);
    tp(2, B_W, B_X);
    return st;
  }
  const i64 nx = L.nx, ny = L.ny, nz = L.nz, nzl = L.nzl, nyl = L.nyl;
  auto kern = [&](int axis, int n, i64 ncols, i64 inner_n, Side in, Side out, int mode, int src, int dst,
                  int fused) {
    Step s;
    s.exchange = false;
    s.axis = axis;
    s.pass.n = n; s.pass.ncols = ncols; s.pass.inner_n = inner_n;
    s.pass.in = in; s.pass.out = out; s.pass.mode = mode; s.pass.scale = 1.0;
    s.pass.colsym = s.pass.axsym = s.pass.diag = nullptr;
    s.src = src; s.dst = dst; s.fused = fused; s.tp = -1;
    st.push_back(s);
  };
  auto exch = [&](int src, int dst) {
    Step s;
    std::memset(&s, 0, sizeof(s));
    s.exchange = true; s.src = src; s.dst = dst; s.tp = -1;
    st.push_back(s);
  };
  const Side xs = side(0, nx, 1, nx, 0);                    // x rows of the local slab
  const Side ynat = side(1, nx * ny, nx, ny, 0);            // y columns, natural [nzl][ny][nx]
  const Side ysplit = side(1, nyl * nx, nx, nyl, L.chunk);  // y columns in per-peer chunks
  const Side zs = side(1, 0, nx * nyl, nz, 0);              // z columns of [nz][nyl][nx]
  int cur = B_IN;
  if (nx > 1) { kern(0, (int)nx, nzl * ny, 1, xs, xs, PASS_FWD, B_IN, B_X, 0); cur = B_X; }
  kern(1, (int)ny, nx * nzl, nx, ynat, ysplit, PASS_FWD, cur, B_W, 0);
  exch(B_W, B_X);
  kern(2, (int)nz, nx * nyl, nx * nyl, zs, zs, PASS_FUSED_SEP, B_X, B_X, 1);
  exch(B_X, B_W);
  kern(1, (int)ny, nx * nzl, nx, ysplit, ynat, PASS_INV, B_W, B_X, 0);
  if (nx > 1) kern(0, (int)nx, nzl * ny, 1, xs, xs, PASS_INV, B_X, B_X, 0);
  // 1/N on the last launch
  for (int i = (int)st.size() - 1; i >= 0; --i)
    if (!st[i].exchange) { st[i].pass.scale = 1.0 / (double)(nx * ny * nz); break; }
  return st;
}

// Per-rank device state shared by both executors.
struct SlabRank {
  SlabLayout L;
  int device = 0;
  std::map<int, cd*> tw;
  cd* colsym = nullptr;
  cd* colsym3 = nullptr;  // 3-sweep schedule: the global [kx + nx ky] table
  cd* axsym = nullptr;
  cd* work = nullptr;
  bool own_work = true;
  bool sym = false;
  int schedule = CFP_SCHEDULE_AUTO;
  double lam_[6] = {0, 0, 0, 0, 0, 0};
  std::vector<Step> steps;

  int init(const SlabLayout& lay, int dev) {
    L = lay;
    device = dev;
    int rc = set_steps(CFP_SCHEDULE_AUTO);
    if (rc) return rc;
    HIPCHK(hipMalloc(&work, sizeof(cd) * (size_t)L.local));
    return CFP_SUCCESS;
  }
  bool three() const { return !steps.empty() && steps[0].tp >= 0; }
  int set_steps(int sched) {
    schedule = sched;
    steps = slab_steps(L, sched);
    for (const Step& s : steps) {
      if (s.exchange || tw.count(s.pass.n)) continue;
      std::vector<cd> h = host_twiddles(s.pass.n, -1);
      cd* d = nullptr;
      HIPCHK(hipMalloc(&d, sizeof(cd) * h.size()));
      HIPCHK(hipMemcpy(d, h.data(), sizeof(cd) * h.size(), hipMemcpyHostToDevice));
      tw[s.pass.n] = d;
    }
    return sym ? set_transport(lam_) : CFP_SUCCESS;  // the new schedule's symbol tables
  }
  void release() {
    for (auto& kv : tw) hipFree(kv.second);
    tw.clear();
    if (colsym) hipFree(colsym);
    if (colsym3) hipFree(colsym3);
    if (axsym) hipFree(axsym);
    if (work && own_work) hipFree(work);
    colsym = colsym3 = axsym = work = nullptr;
  }
  // colsym over the z-pass columns g = ix + nx*iyl (global ky = y0 + iyl); axsym over kz
  int set_transport(const double lam[6]) {
    std::vector<cd> hat[3] = {host_transport_symbol(L.nx), host_transport_symbol(L.ny), host_transport_symbol(L.nz)};
    std::vector<cd> s[3];
    for (int a = 0; a < 3; ++a) {
      const double lr = lam[2 * a], li = lam[2 * a + 1];
      s[a].resize(hat[a].size());
      for (size_t k = 0; k < hat[a].size(); ++k) {
        const double cr = hat[a][k].x, ci = hat[a][k].y;
        s[a][k] = make_cd(cr * lr - ci * li, cr * li + ci * lr);
      }
    }
    const i64 ncols = L.nx * L.nyl;
    std::vector<cd> col((size_t)ncols);
    for (i64 g = 0; g < ncols; ++g) {
      const i64 ix = g % L.nx, ky = L.y0 + g / L.nx;
      col[(size_t)g] = make_cd(s[0][ix].x + s[1][ky].x, s[0][ix].y + s[1][ky].y);
    }
    if (!colsym) HIPCHK(hipMalloc(&colsym, sizeof(cd) * (size_t)ncols));
    if (!axsym) HIPCHK(hipMalloc(&axsym, sizeof(cd) * (size_t)L.nz));
    HIPCHK(hipMemcpy(colsym, col.data(), sizeof(cd) * (size_t)ncols, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(axsym, s[2].data(), sizeof(cd) * (size_t)L.nz, hipMemcpyHostToDevice));
    if (three()) {  // every rank holds the global column table: P2 indexes it with global ky
      std::vector<cd> g((size_t)(L.nx * L.ny));
      for (i64 ky = 0; ky < L.ny; ++ky)
        for (i64 ix = 0; ix < L.nx; ++ix)
          g[(size_t)(ix + L.nx * ky)] = make_cd(s[0][ix].x + s[1][ky].x, s[0][ix].y + s[1][ky].y);
      if (!colsym3) HIPCHK(hipMalloc(&colsym3, sizeof(cd) * g.size()));
      HIPCHK(hipMemcpy(colsym3, g.data(), sizeof(cd) * g.size(), hipMemcpyHostToDevice));
    }
    std::memcpy(lam_, lam, sizeof(lam_));
    sym = true;
    return CFP_SUCCESS;
  }
  cd* buf(int id, const cd* b, cd* x) const { return id == B_IN ? (cd*)b : (id == B_X ? x : work); }
  int launch(const Step& s, const cd* b, cd* x, hipStream_t st) const {
    if (s.tp >= 0) {
      TPArgs a;
      a.tw = tw.at((int)L.nx);
      a.colsym = colsym3;
      a.axsym = axsym;
      a.scale = s.pass.scale;
      a.lnyl = ilog2_exact(L.nyl);
      a.chunk = L.chunk;
      a.k1_off = (int)(L.r * (L.nyl / 8));  // N2 = 8 rows per k1
      hipError_t e = launch_three_pass_slab(s.tp, buf(s.src, b, x), buf(s.dst, b, x), a, (int)L.nzl, st);
      return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "slab 3-sweep launch");
    }
    PassDesc p = s.pass;
    if (s.fused) { p.colsym = colsym; p.axsym = axsym; }
    hipError_t e = launch_axis_pass(p, buf(s.src, b, x), buf(s.dst, b, x), tw.at(p.n), st);
    return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "slab axis pass");
  }
};

}  // namespace

struct cfp_dist_plan_s {
  SlabRank R;
  ncclComm_t comm = nullptr;
  // sampled per-phase events inside the caller's applies (as cfp_plan_profile_begin)
  std::vector<hipEvent_t> prof_ev;
  size_t prof_stride = 0, prof_cap = 0, prof_used = 0, prof_every = 1, prof_calls = 0;
};

static void dist_profile_free(cfp_dist_plan_s* p) {
  for (auto& e : p->prof_ev) hipEventDestroy(e);
  p->prof_ev.clear();
  p->prof_stride = p->prof_cap = p->prof_used = p->prof_calls = 0;
  p->prof_every = 1;
}

struct cfp_group_s {
  std::vector<SlabRank> R;
  std::vector<hipStream_t> streams;
};

extern "C" int cfp_slab_layout(int64_t nx, int64_t ny, int64_t nz, int P, int r, int64_t* out) {
  if (!out) return set_error(CFP_ERR_ARG_NULL, "out is NULL");
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  const int64_t v[8] = {L.nzl, L.nyl, L.z0, L.y0, L.local, L.chunk, L.offset, (int64_t)P};
  std::memcpy(out, v, sizeof(v));
  return CFP_SUCCESS;
}

extern "C" int cfp_slab_num_steps(int64_t nx, int64_t ny, int64_t nz, int P, int r, int* nsteps) {
  if (!nsteps) return set_error(CFP_ERR_ARG_NULL, "nsteps is NULL");
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  *nsteps = (int)slab_steps(L, CFP_SCHEDULE_FIVE_PASS).size();  // the axis-pass step list (host replays)
  return CFP_SUCCESS;
}

extern "C" int cfp_slab_step_info(int64_t nx, int64_t ny, int64_t nz, int P, int r, int i, int64_t* desc,
                                  double* scale) {
  if (!desc || !scale) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  const std::vector<Step> st = slab_steps(L, CFP_SCHEDULE_FIVE_PASS);
  if (i < 0 || i >= (int)st.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "step index");
  const Step& s = st[(size_t)i];
  const PassDesc& p = s.pass;
  const int64_t v[18] = {s.exchange ? 1 : 0, s.src, s.dst, s.exchange ? -1 : s.axis, s.exchange ? 0 : p.n,
                         s.exchange ? -1 : p.mode, s.exchange ? 0 : p.ncols, s.exchange ? 0 : p.inner_n,
                         p.in.inner_stride, p.in.outer_stride, p.in.pt_stride, p.in.seg_len, p.in.seg_stride,
                         p.out.inner_stride, p.out.outer_stride, p.out.pt_stride, p.out.seg_len, p.out.seg_stride};
  std::memcpy(desc, v, sizeof(v));
  *scale = s.exchange ? 1.0 : p.scale;
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int cfp_dist_get_unique_id(char* id_out) {
  if (!id_out) return set_error(CFP_ERR_ARG_NULL, "id_out is NULL");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_create(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                    const char* uid, int device) {
  if (!plan || !uid) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *plan = nullptr;
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<cfp_dist_plan_s> p(new cfp_dist_plan_s);
  rc = p->R.init(L, device);
  if (rc) { p->R.release(); return rc; }
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclResult_t nr = ncclCommInitRank(&p->comm, P, id, r);
  if (nr != ncclSuccess) {
    p->R.release();
    return set_error(CFP_ERR_LIB, "ncclCommInitRank: %s", ncclGetErrorString(nr));
  }
  *plan = p.release();
  return CFP_SUCCESS;
}

// Plan without a communicator: the caller performs the two exchanges itself between the
// three kernel segments (cfp_dist_plan_run_segment), e.g. with torch.distributed's RCCL.
extern "C" int cfp_dist_plan_create_external(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                             int device) {
  if (!plan) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *plan = nullptr;
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<cfp_dist_plan_s> p(new cfp_dist_plan_s);
  rc = p->R.init(L, device);
  if (rc) { p->R.release(); return rc; }
  *plan = p.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_work_buffer(cfp_dist_plan_t p, double** work) {
  if (!p || !work) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *work = (double*)p->R.work;
  return CFP_SUCCESS;
}

// use a caller-owned work buffer (local_size complex values) instead of the plan's own
extern "C" int cfp_dist_plan_set_work_buffer(cfp_dist_plan_t p, double* work) {
  if (!p || !work) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  if (p->R.work && p->R.own_work) hipFree(p->R.work);
  p->R.work = (cd*)work;
  p->R.own_work = false;
  return CFP_SUCCESS;
}

// segment 0: kernels before the first exchange (which sends work -> receives into x);
// segment 1: between the exchanges (the exchange after it sends x -> receives into work);
// segment 2: kernels after the second exchange.
extern "C" int cfp_dist_plan_run_segment(cfp_dist_plan_t p, int seg, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (seg < 0 || seg > 2) return set_error(CFP_ERR_ARG_OUTOFRANGE, "segment must be 0, 1 or 2");
  if (!p->R.sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  HIPCHK(hipSetDevice(p->R.device));
  int cur = 0;
  for (const Step& st : p->R.steps) {
    if (st.exchange) { ++cur; continue; }
    if (cur != seg) continue;
    int rc = p->R.launch(st, (const cd*)b, (cd*)x, (hipStream_t)stream);
    if (rc) return rc;
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_destroy(cfp_dist_plan_t p) {
  if (!p) return CFP_SUCCESS;
  hipSetDevice(p->R.device);
  dist_profile_free(p);
  if (p->comm) ncclCommDestroy(p->comm);
  p->R.release();
  delete p;
  return CFP_SUCCESS;
}

// schedule of the slab plan's local passes: CFP_SCHEDULE_AUTO (3 sweeps at 256^3 with P | 32),
// CFP_SCHEDULE_FIVE_PASS, or CFP_SCHEDULE_THREE_PASS (CFP_ERR_SUP where not supported)
static int slab_schedule_check(const SlabLayout& L, int schedule) {
  if (schedule != CFP_SCHEDULE_AUTO && schedule != CFP_SCHEDULE_FIVE_PASS && schedule != CFP_SCHEDULE_THREE_PASS)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "slab schedule must be AUTO, FIVE_PASS or THREE_PASS");
  const i64 n[3] = {L.nx, L.ny, L.nz};
  if (schedule == CFP_SCHEDULE_THREE_PASS && !three_pass_slab_supported(n, L.P))
    return set_error(CFP_ERR_SUP, "the 3-sweep slab schedule needs a 256^3 grid and nranks | 32");
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_set_schedule(cfp_dist_plan_t p, int schedule) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  int rc = slab_schedule_check(p->R.L, schedule);
  if (rc) return rc;
  HIPCHK(hipSetDevice(p->R.device));
  dist_profile_free(p);
  return p->R.set_steps(schedule);
}

extern "C" int cfp_group_set_schedule(cfp_group_t g, int schedule) {
  if (!g) return set_error(CFP_ERR_ARG_NULL, "NULL group");
  for (auto& R : g->R) {
    int rc = slab_schedule_check(R.L, schedule);
    if (rc) return rc;
    HIPCHK(hipSetDevice(R.device));
    rc = R.set_steps(schedule);
    if (rc) return rc;
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_set_symbol_transport(cfp_dist_plan_t p, const double lam[6]) {
  if (!p || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  return p->R.set_transport(lam);
}

extern "C" int cfp_dist_plan_local_size(cfp_dist_plan_t p, int64_t* n) {
  if (!p || !n) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *n = p->R.L.local;
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_num_phases(cfp_dist_plan_t p, int* n) {
  if (!p || !n) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *n = (int)p->R.steps.size();
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_phase_info(cfp_dist_plan_t p, int i, int* is_exchange, int* axis, int* n, int* mode) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (i < 0 || i >= (int)p->R.steps.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "phase index");
  const Step& s = p->R.steps[i];
  if (is_exchange) *is_exchange = s.exchange ? 1 : 0;
  if (axis) *axis = s.exchange ? -1 : s.axis;
  if (n) *n = s.exchange ? 0 : s.pass.n;
  if (mode) *mode = s.exchange ? -1 : s.pass.mode;
  return CFP_SUCCESS;
}

static int rccl_exchange(cfp_dist_plan_s* p, const cd* src, cd* dst, hipStream_t s) {
  const SlabLayout& L = p->R.L;
  const size_t cnt = (size_t)L.chunk * 2;  // doubles per peer message
  if (L.P > 1 && !p->comm)
    return set_error(CFP_ERR_ARG_WRONGSTATE, "plan made with cfp_dist_plan_create_external has no communicator");
  HIPCHK(hipMemcpyAsync(dst + L.r * L.chunk, src + L.r * L.chunk, sizeof(cd) * (size_t)L.chunk,
                        hipMemcpyDeviceToDevice, s));
  if (L.P == 1) return CFP_SUCCESS;
  NCCLCHK(ncclGroupStart());
  for (int q = 0; q < L.P; ++q) {
    if (q == L.r) continue;
    NCCLCHK(ncclSend(src + q * L.chunk, cnt, ncclDouble, q, p->comm, s));
    NCCLCHK(ncclRecv(dst + q * L.chunk, cnt, ncclDouble, q, p->comm, s));
  }
  NCCLCHK(ncclGroupEnd());
  return CFP_SUCCESS;
}

static int dist_apply(cfp_dist_plan_s* p, const cd* b, cd* x, hipStream_t s, std::vector<hipEvent_t>* ev) {
  if (!p->R.sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  for (size_t i = 0; i < p->R.steps.size(); ++i) {
    const Step& st = p->R.steps[i];
    if (ev) HIPCHK(hipEventRecord((*ev)[i], s));
    int rc;
    if (st.exchange) rc = rccl_exchange(p, p->R.buf(st.src, b, x), p->R.buf(st.dst, b, x), s);
    else rc = p->R.launch(st, b, x, s);
    if (rc) return rc;
  }
  if (ev) HIPCHK(hipEventRecord((*ev)[p->R.steps.size()], s));
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_apply(cfp_dist_plan_t p, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  const bool sample = p->prof_cap && (p->prof_calls++ % p->prof_every) == 0;
  if (sample && p->prof_used < p->prof_cap) {
    std::vector<hipEvent_t> ev(p->prof_ev.begin() + (long)(p->prof_used * p->prof_stride),
                               p->prof_ev.begin() + (long)((p->prof_used + 1) * p->prof_stride));
    ++p->prof_used;
    return dist_apply(p, (const cd*)b, (cd*)x, (hipStream_t)stream, &ev);
  }
  return dist_apply(p, (const cd*)b, (cd*)x, (hipStream_t)stream, nullptr);
}

// sampled phase events inside the caller's own applies (cfp_plan_profile_begin's contract)
extern "C" int cfp_dist_plan_profile_begin(cfp_dist_plan_t p, int max_applies, int every) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (max_applies < 1 || max_applies > 100000 || every < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "bad profile range");
  HIPCHK(hipSetDevice(p->R.device));
  dist_profile_free(p);
  p->prof_stride = p->R.steps.size() + 1;
  p->prof_ev.resize(p->prof_stride * (size_t)max_applies, nullptr);
  for (auto& e : p->prof_ev) {
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) {
      dist_profile_free(p);
      return hip_error(r, "hipEventCreate");
    }
  }
  p->prof_cap = (size_t)max_applies;
  p->prof_every = (size_t)every;
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_profile_end(cfp_dist_plan_t p, double* ms_out, int* applies) {
  if (!p || !ms_out || !applies) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!p->prof_cap) return set_error(CFP_ERR_ARG_WRONGSTATE, "profiling was not started");
  HIPCHK(hipSetDevice(p->R.device));
  const size_t np = p->prof_stride - 1, used = p->prof_used;
  std::vector<double> acc(np, 0.0);
  int rc = CFP_SUCCESS;
  if (used > 0) {
    hipError_t e = hipEventSynchronize(p->prof_ev[used * p->prof_stride - 1]);
    if (e != hipSuccess) rc = hip_error(e, "event sync");
  }
  for (size_t a = 0; a < used && !rc; ++a)
    for (size_t i = 0; i < np; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, p->prof_ev[a * p->prof_stride + i], p->prof_ev[a * p->prof_stride + i + 1]);
      acc[i] += ms;
    }
  for (size_t i = 0; i < np; ++i) ms_out[i] = used ? acc[i] / (double)used : 0.0;
  *applies = (int)used;
  dist_profile_free(p);
  return rc;
}

extern "C" int cfp_dist_plan_time_phases(cfp_dist_plan_t p, const double* b, double* x, int iters, double* ms_out,
                                         void* stream) {
  if (!p || !b || !x || !ms_out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (iters < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "iters must be >= 1");
  HIPCHK(hipSetDevice(p->R.device));
  const size_t np = p->R.steps.size();
  std::vector<hipEvent_t> ev(np + 1);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  std::vector<double> acc(np, 0.0);
  int rc = CFP_SUCCESS;
  for (int it = 0; it < iters && !rc; ++it) {
    rc = dist_apply(p, (const cd*)b, (cd*)x, (hipStream_t)stream, &ev);
    if (rc) break;
    if (hipEventSynchronize(ev[np]) != hipSuccess) { rc = set_error(CFP_ERR_LIB, "event sync"); break; }
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

// ------------------------------------------------------------------ single-process group
extern "C" int cfp_group_create(cfp_group_t* group, int64_t nx, int64_t ny, int64_t nz, int P, const int* devices) {
  if (!group || !devices) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *group = nullptr;
  std::unique_ptr<cfp_group_s> g(new cfp_group_s);
  g->R.resize((size_t)P);
  g->streams.resize((size_t)P, nullptr);
  for (int r = 0; r < P; ++r) {
    SlabLayout L;
    int rc = make_layout(nx, ny, nz, P, r, &L);
    if (!rc) {
      hipError_t e = hipSetDevice(devices[r]);
      if (e != hipSuccess) rc = hip_error(e, "hipSetDevice");
    }
    if (!rc) rc = g->R[r].init(L, devices[r]);
    if (!rc) {
      hipError_t e = hipStreamCreateWithFlags(&g->streams[r], hipStreamNonBlocking);
      if (e != hipSuccess) rc = hip_error(e, "hipStreamCreate");
    }
    if (rc) {
      for (int q = 0; q <= r; ++q) {
        g->R[q].release();
        if (g->streams[q]) hipStreamDestroy(g->streams[q]);
      }
      return rc;
    }
  }
  *group = g.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_group_destroy(cfp_group_t g) {
  if (!g) return CFP_SUCCESS;
  for (size_t r = 0; r < g->R.size(); ++r) {
    hipSetDevice(g->R[r].device);
    g->R[r].release();
    if (g->streams[r]) hipStreamDestroy(g->streams[r]);
  }
  delete g;
  return CFP_SUCCESS;
}

extern "C" int cfp_group_set_symbol_transport(cfp_group_t g, const double lam[6]) {
  if (!g || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  for (auto& R : g->R) {
    HIPCHK(hipSetDevice(R.device));
    int rc = R.set_transport(lam);
    if (rc) return rc;
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_group_apply(cfp_group_t g, const double* const* b, double* const* x) {
  if (!g || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  const int P = (int)g->R.size();
  for (auto& R : g->R)
    if (!R.sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the group");
  const size_t nsteps = g->R[0].steps.size();
  for (size_t i = 0; i < nsteps; ++i) {
    const Step& st = g->R[0].steps[i];
    if (!st.exchange) {
      for (int r = 0; r < P; ++r) {
        HIPCHK(hipSetDevice(g->R[r].device));
        int rc = g->R[r].launch(g->R[r].steps[i], (const cd*)b[r], (cd*)x[r], g->streams[r]);
        if (rc) return rc;
      }
    } else {
      for (int r = 0; r < P; ++r) {
        HIPCHK(hipSetDevice(g->R[r].device));
        HIPCHK(hipStreamSynchronize(g->streams[r]));
      }
      // rank r's chunk q goes to rank q's chunk r
      for (int r = 0; r < P; ++r) {
        const SlabRank& S = g->R[r];
        HIPCHK(hipSetDevice(S.device));
        const cd* src = S.buf(st.src, (const cd*)b[r], (cd*)x[r]);
        for (int q = 0; q < P; ++q) {
          const SlabRank& D = g->R[q];
          cd* dst = D.buf(st.dst, (const cd*)b[q], (cd*)x[q]);
          HIPCHK(hipMemcpyAsync(dst + r * D.L.chunk, src + q * S.L.chunk, sizeof(cd) * (size_t)S.L.chunk,
                                hipMemcpyDefault, g->streams[r]));
        }
      }
      for (int r = 0; r < P; ++r) {
        HIPCHK(hipSetDevice(g->R[r].device));
        HIPCHK(hipStreamSynchronize(g->streams[r]));
      }
    }
  }
  for (int r = 0; r < P; ++r) {
    HIPCHK(hipSetDevice(g->R[r].device));
    HIPCHK(hipStreamSynchronize(g->streams[r]));
  }
  return CFP_SUCCESS;
}
