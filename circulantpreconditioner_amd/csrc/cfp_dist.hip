// cfp_dist.hip -- z-slab decomposition of the circulant apply over P GPUs.
//
// Replaces the FFTW-MPI slab transposes that PETSc's MATFFTW performs inside MatMult /
// MatMultTranspose when size > 1 (src/FftLinearSolver_3D.c:170,180).
// The y passes read/write the exchange chunks directly (no pack/unpack kernels): the
// forward y pass writes point ky of a column to chunk ky / nyp, the inverse y pass reads
// it back from there, so an all-to-all is a set of contiguous peer messages.
//
// Pipelining (pieces K > 1).  A block of B = nzl / K local z-planes is a contiguous sub-block
// of every per-peer chunk ([nzl][nyp][nx]), so the forward all-to-all splits into K pieces:
// piece k carries block k of every chunk and can leave as soon as block k's x and y passes are
// done, while block k + 1's passes run.  The backward all-to-all mirrors it: block k's inverse
// y and x passes start when piece k has arrived.  The exchanges run on a second stream, ordered
// against the passes by events (each step names the one step of the other stream it waits
// for); every rank issues the same sequence of exchanges, so RCCL's ordering rule holds.  With
// K > 1 the exchanges land in a second work buffer W2, so that no pass writes memory a piece is
// still reading or receiving:
//   x fwd  b -> x (block k, natural)       y fwd  x -> W (block k of every chunk)
//   piece  W -> W2                         z      W2 -> W2 (fused symbol, [nz][nyp][nx])
//   piece  W2 -> W                         y inv  W -> x (block k),  x inv  x -> x (1/N)
// K = 1 keeps the round-2 layout (exchanges into x, one work buffer).
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
#include "cfp_rccl.h"
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

// Rank r holds z-planes [r nzl, (r + 1) nzl) in natural order (PETSC_DECIDE rows; P | nz) and,
// after the forward all-to-all, y rows [y0, y0 + nyl) of every plane (the z-pencil block).  The
// y rows are split as FFTW-MPI splits its transposed dimension: blocks of nyp = ceil(ny / P), so
// with P not dividing ny the last ranks hold fewer rows (possibly none).  Every per-peer chunk is
// nzl x nyp x nx (the rows past a peer's count are padding, never read), so the segment
// addressing of the y passes stays uniform and the z-pencil buffer is [nz][nyp][nx].
struct SlabLayout {
  i64 nx, ny, nz;
  int P, r;
  i64 nzl, nyl, z0, y0, local, chunk, offset;
  i64 nyp;   // y rows per chunk (ceil(ny / P)); nyl = this rank's valid rows <= nyp
  i64 work;  // elements of a work buffer: max(local, P chunk)
  bool padded() const { return nyp * P != ny; }
};

int make_layout(i64 nx, i64 ny, i64 nz, int P, int r, SlabLayout* L) {
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  if (P < 1 || r < 0 || r >= P) return set_error(CFP_ERR_ARG_OUTOFRANGE, "rank %d of %d", r, P);
  if (nz % P)
    return set_error(CFP_ERR_ARG_SIZ, "slab decomposition needs nranks | nz (whole z-planes per rank; nz=%lld P=%d)",
                     (long long)nz, P);
  if (nx > 4096 || ny > 4096 || nz > 4096) return set_error(CFP_ERR_SUP, "axis lengths above 4096 unsupported");
  L->nx = nx; L->ny = ny; L->nz = nz; L->P = P; L->r = r;
  L->nzl = nz / P;
  L->nyp = (ny + P - 1) / P;
  L->z0 = r * L->nzl;
  L->y0 = r * L->nyp;
  L->nyl = ny - L->y0 < 0 ? 0 : (ny - L->y0 < L->nyp ? ny - L->y0 : L->nyp);
  L->local = L->nzl * ny * nx;
  L->chunk = L->nzl * L->nyp * nx;
  L->work = L->local > P * L->chunk ? L->local : P * L->chunk;
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

// buffers of a step: the caller's b and x, the plan's work buffers W, W2, and the z-pencil
// copy of an explicit Diag (cfp_dist_plan_set_diag)
enum Buf { B_IN = 0, B_X = 1, B_W = 2, B_W2 = 3, B_D = 4 };
// step kinds (also the host-only description, include/circulant_fft_dist.h)
enum Kind { K_PASS = 0, K_EXCH = 1, K_TP = 2, K_REPACK = 3 };
// what a step list computes
enum ListKind { L_APPLY_SEP = 0, L_APPLY_DIAG = 1, L_FORWARD = 2, L_BACKWARD = 3, L_DIAG_T = 4 };

struct Step {
  int kind = K_PASS;
  int src = 0, dst = 0;
  i64 src_off = 0, dst_off = 0;  // element offset of the step's base in its buffers
  // K_PASS
  PassDesc pass{};
  int axis = 0;
  int fused = 0;  // 1: separable symbol tables, 2: explicit Diag (B_D, addressed like the input)
  // K_TP: stage of the 3-sweep schedule (cfp_three_pass.hip), local z-planes of the launch
  int tp = -1;
  int planes = 0;
  // K_EXCH: peer q gets src[q chunk + ex_off, + ex_cnt) and stores it at dst[rank chunk + ex_off]
  i64 ex_off = 0, ex_cnt = 0;
  // K_REPACK: `planes` natural planes [.][ny][nx] <-> per-peer chunks
  int to_chunks = 0;
  int wait = -1;  // the step of the other stream this one waits for (-1: none)
  int seg = 0;    // 0 before the first exchange, 1 between, 2 after (cfp_dist_plan_run_segment)
};

// 256^3: 3 local sweeps per rank (x + y1 | y2 + z + symbol + inverses | inverse), the same two
// exchanges; otherwise 5 axis passes.  AUTO takes 3 sweeps on every supported P.  Per rank
// (tools/slab_local_timing.py, exchanges skipped), 3 against 5 sweeps at 256^3: r02i
// (profiles/r02i_slab_local.txt) 174 / 219 us at P = 2, 90 / 119 at P = 4, a tie at P = 8 and a
// loss at P = 16, so AUTO was P <= 4 until r05; r05o (profiles/r05o_slab256_local.txt, with the
// lane-pair and XCD-ordered rows) 86 / 119 at P = 4, 56 / 63 at P = 8, 45 / 53 at P = 16.
// 512^3 (r05): 96 N / P local bytes against 160 N / P; P2 keeps 1,024 units
// for 256 CUs at P = 8.
bool slab_three(const SlabLayout& L, int schedule) {
  const i64 n[3] = {L.nx, L.ny, L.nz};
  if (schedule == CFP_SCHEDULE_FIVE_PASS || !three_pass_slab_supported(n, L.P)) return false;
  return true;
}

// AUTO pipeline depth: one piece on one rank and for slabs under 64 MiB (the exchanges are then
// a few MiB per peer, and the extra launches and events cost about what the overlap saves);
// else 4 pieces (512^3 over 8 ranks: 16 MiB per peer per piece, 16-plane blocks), or 2 when
// 4 does not divide the local planes.
int auto_pieces(const SlabLayout& L) {
  if (L.P == 1 || L.local < (i64(1) << 22)) return 1;
  if (L.nzl % 4 == 0 && L.nzl >= 8) return 4;
  if (L.nzl % 2 == 0) return 2;
  return 1;
}

int pieces_valid(const SlabLayout& L, int K) { return K >= 1 && K <= L.nzl && L.nzl % K == 0; }

std::vector<Step> slab_steps(const SlabLayout& L, int schedule, int K, int list) {
  std::vector<Step> st;
  // nyp: rows per chunk; nyl: the z-pencil rows this rank transforms (nyl <= nyp, padded layouts)
  const i64 nx = L.nx, ny = L.ny, nz = L.nz, nzl = L.nzl, nyl = L.nyl, nyp = L.nyp;
  const double invN = 1.0 / (double)(nx * ny * nz);
  const bool apply = list == L_APPLY_SEP || list == L_APPLY_DIAG;
  if (!apply) K = 1;
  const i64 B = nzl / K;  // planes per block
  // where the forward exchange lands (z-pencil buffer [nz][nyp][nx]): x if it fits (one piece,
  // no padding), else W2
  const int M = (K == 1 && !L.padded()) ? B_X : B_W2;
  int seg = 0;
  auto push = [&](Step s) {
    s.seg = seg;
    st.push_back(s);
    return (int)st.size() - 1;
  };
  auto exch = [&](int src, int dst, i64 k, int wait) {
    Step s;
    s.kind = K_EXCH; s.src = src; s.dst = dst;
    s.ex_off = k * B * nyp * nx; s.ex_cnt = B * nyp * nx;
    s.wait = wait;
    return push(s);
  };
  auto pass = [&](int axis, int n, i64 ncols, i64 inner_n, Side in, Side out, int mode, int src, i64 soff, int dst,
                  i64 doff, int fused, double scale, int wait) {
    Step s;
    s.kind = K_PASS; s.axis = axis;
    std::memset(&s.pass, 0, sizeof(s.pass));
    s.pass.n = n; s.pass.ncols = ncols; s.pass.inner_n = inner_n;
    s.pass.in = in; s.pass.out = out; s.pass.mode = mode; s.pass.scale = scale;
    s.src = src; s.dst = dst; s.src_off = soff; s.dst_off = doff; s.fused = fused; s.wait = wait;
    return push(s);
  };
  const Side xs = side(0, nx, 1, nx, 0);                    // x rows of the local slab
  const Side ynat = side(1, nx * ny, nx, ny, 0);            // y columns, natural [nzl][ny][nx]
  const Side ysplit = side(1, nyp * nx, nx, nyp, L.chunk);  // y columns in per-peer chunks
  const Side zs = side(1, 0, nx * nyp, nz, 0);              // z columns of [nz][nyp][nx]: the first nyl rows
  const i64 zcols_inner = nyl > 0 ? nx * nyl : 1;           // (no columns on a rank without rows)

  if (list == L_DIAG_T) {  // natural Diag slab -> chunks (W) -> exchange -> z-pencil copy (B_D)
    Step r;
    r.kind = K_REPACK; r.src = B_IN; r.dst = B_W; r.to_chunks = 1; r.planes = (int)nzl;
    push(r);
    seg = 1;
    exch(B_W, B_D, 0, 0);
    return st;
  }
  if (list == L_FORWARD || list == L_BACKWARD) {
    // the unnormalised 3-D DFT of the slab in natural order (FFTW-MPI's non-transposed
    // MatMult / MatMultTranspose): x, y -> chunks, exchange, z, exchange back, chunks -> natural
    const int mode = list == L_FORWARD ? PASS_FWD : PASS_INV;
    int cur = B_IN;
    if (nx > 1) { pass(0, (int)nx, nzl * ny, 1, xs, xs, mode, B_IN, 0, B_X, 0, 0, 1.0, -1); cur = B_X; }
    int y = pass(1, (int)ny, nx * nzl, nx, ynat, ysplit, mode, cur, 0, B_W, 0, 0, 1.0, -1);
    seg = 1;
    int e = exch(B_W, B_W2, 0, y);
    int z = pass(2, (int)nz, nx * nyl, zcols_inner, zs, zs, mode, B_W2, 0, B_W2, 0, 0, 1.0, e);
    seg = 2;
    e = exch(B_W2, B_W, 0, z);
    Step r;
    r.kind = K_REPACK; r.src = B_W; r.dst = B_X; r.to_chunks = 0; r.planes = (int)nzl; r.wait = e;
    push(r);
    return st;
  }

  const bool three = list == L_APPLY_SEP && slab_three(L, schedule);
  if (three) {
    // P1 natural planes -> per-peer chunks (W), exchange into the z-pencil buffer as
    // [nz][nyl][nx] (the rank's k1 rows), P2 in place, exchange back into W, P3 -> x natural, 1/N
    auto tp = [&](int stage, int src, i64 soff, int dst, i64 doff, int planes, int wait) {
      Step s;
      s.kind = K_TP; s.tp = stage; s.axis = stage == 1 ? 2 : 0;
      std::memset(&s.pass, 0, sizeof(s.pass));
      s.pass.n = (int)nx;
      s.pass.mode = stage == 0 ? PASS_TP_ROWS_FWD : (stage == 1 ? PASS_TP_MID : PASS_TP_ROWS_INV);
      s.pass.scale = stage == 2 ? invN : 1.0;
      s.src = src; s.dst = dst; s.src_off = soff; s.dst_off = doff; s.planes = planes;
      s.fused = stage == 1; s.wait = wait;
      return push(s);
    };
    std::vector<int> p1(K);
    for (i64 k = 0; k < K; ++k) p1[k] = tp(0, B_IN, k * B * ny * nx, B_W, k * B * nyp * nx, (int)B, -1);
    seg = 1;
    int last = -1;
    for (i64 k = 0; k < K; ++k) last = exch(B_W, M, k, p1[k]);
    const int mid = tp(1, M, 0, M, 0, 0, last);
    seg = 2;
    for (i64 k = 0; k < K; ++k) {
      const int e = exch(M, B_W, k, mid);
      tp(2, B_W, k * B * nyp * nx, B_X, k * B * ny * nx, (int)B, e);
    }
    return st;
  }
  const int fused = list == L_APPLY_DIAG ? 2 : 1;
  const int zmode = list == L_APPLY_DIAG ? PASS_FUSED_DIAG : PASS_FUSED_SEP;
  std::vector<int> yk(K);
  for (i64 k = 0; k < K; ++k) {
    const i64 nat = k * B * ny * nx;
    int cur = B_IN;
    if (nx > 1) { pass(0, (int)nx, B * ny, 1, xs, xs, PASS_FWD, B_IN, nat, B_X, nat, 0, 1.0, -1); cur = B_X; }
    yk[k] = pass(1, (int)ny, nx * B, nx, ynat, ysplit, PASS_FWD, cur, nat, B_W, k * B * nyp * nx, 0, 1.0, -1);
  }
  seg = 1;
  int last = -1;
  for (i64 k = 0; k < K; ++k) last = exch(B_W, M, k, yk[k]);
  const int z = pass(2, (int)nz, nx * nyl, zcols_inner, zs, zs, zmode, M, 0, M, 0, fused, 1.0, last);
  seg = 2;
  for (i64 k = 0; k < K; ++k) {
    const i64 nat = k * B * ny * nx;
    const int e = exch(M, B_W, k, z);
    // 1/N on the block's last launch
    pass(1, (int)ny, nx * B, nx, ysplit, ynat, PASS_INV, B_W, k * B * nyp * nx, B_X, nat, 0, nx > 1 ? 1.0 : invN, e);
    if (nx > 1) pass(0, (int)nx, B * ny, 1, xs, xs, PASS_INV, B_X, nat, B_X, nat, 0, invN, -1);
  }
  return st;
}

// natural planes [planes][ny][nx] <-> per-peer chunks: element (z, y, x) of the slab sits at
// (z ny + y) nx + x naturally and at (y / nyp) chunk + (z nyp + y % nyp) nx + x in the chunks.
// One thread per element; consecutive threads walk x, so both sides are coalesced.
__global__ void k_slab_repack(const cd* __restrict__ in, cd* __restrict__ out, i64 total, i64 nx, i64 ny, i64 nyp,
                              i64 chunk, int to_chunks) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (i64)gridDim.x * blockDim.x) {
    const i64 x = i % nx, row = i / nx;
    const i64 y = row % ny, z = row / ny;
    const i64 c = (y / nyp) * chunk + (z * nyp + y % nyp) * nx + x;
    if (to_chunks) out[c] = in[i];
    else out[i] = in[c];
  }
}

hipError_t launch_repack(const cd* in, cd* out, const SlabLayout& L, i64 planes, int to_chunks, hipStream_t s) {
  const i64 total = planes * L.ny * L.nx;
  if (total <= 0) return hipSuccess;
  const i64 want = (total + 255) / 256;
  const unsigned g = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(k_slab_repack, dim3(g), dim3(256), 0, s, in, out, total, L.nx, L.ny, L.nyp, L.chunk, to_chunks);
  return hipGetLastError();
}

// Per-rank device state shared by every executor.
struct SlabRank {
  SlabLayout L;
  int device = 0;
  std::map<int, cd*> tw;
  cd* colsym = nullptr;
  cd* colsym3 = nullptr;  // 3-sweep schedule: the global [kx + nx ky] table
  cd* axsym = nullptr;
  cd* work = nullptr;
  cd* work2 = nullptr;    // pieces > 1 and the transforms
  cd* diag_t = nullptr;   // z-pencil copy of an explicit Diag
  bool own_work = true, own_work2 = true;
  bool sym = false;       // separable symbol set
  bool diag = false;      // explicit Diag set (cfp_dist_plan_set_diag)
  int schedule = CFP_SCHEDULE_AUTO;
  int pieces_req = 0;     // 0 = AUTO
  double lam_[6] = {0, 0, 0, 0, 0, 0};
  std::vector<Step> steps;       // the apply
  std::vector<Step> diag_steps;  // the apply with the explicit Diag

  int init(const SlabLayout& lay, int dev) {
    L = lay;
    device = dev;
    int rc = set_steps(CFP_SCHEDULE_AUTO, 0);
    if (rc) return rc;
    HIPCHK(hipMalloc(&work, sizeof(cd) * (size_t)L.work));
    return CFP_SUCCESS;
  }
  int pieces() const { return pieces_req ? pieces_req : auto_pieces(L); }
  bool three() const { return !steps.empty() && steps[0].kind == K_TP; }
  int ensure_tw(int n) {
    if (tw.count(n)) return CFP_SUCCESS;
    std::vector<cd> h = host_twiddles(n, -1);
    cd* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(cd) * h.size()));
    HIPCHK(hipMemcpy(d, h.data(), sizeof(cd) * h.size(), hipMemcpyHostToDevice));
    tw[n] = d;
    return CFP_SUCCESS;
  }
  int ensure_work2() {
    if (!work2) {
      HIPCHK(hipMalloc(&work2, sizeof(cd) * (size_t)L.work));
      own_work2 = true;
    }
    return CFP_SUCCESS;
  }
  int set_steps(int sched, int pieces_request) {
    schedule = sched;
    pieces_req = pieces_request;
    const int K = pieces();
    steps = slab_steps(L, sched, K, L_APPLY_SEP);
    diag_steps = slab_steps(L, sched, K, L_APPLY_DIAG);
    for (const auto* list : {&steps, &diag_steps})
      for (const Step& s : *list)
        if (s.kind == K_PASS || s.kind == K_TP) {
          int rc = ensure_tw(s.pass.n);
          if (rc) return rc;
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
    if (work2 && own_work2) hipFree(work2);
    if (diag_t) hipFree(diag_t);
    colsym = colsym3 = axsym = work = work2 = diag_t = nullptr;
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
    const i64 ncols = L.nx * L.nyl;  // 0 on a rank past the last y row (padded layouts)
    std::vector<cd> col((size_t)(ncols > 0 ? ncols : 1));
    for (i64 g = 0; g < ncols; ++g) {
      const i64 ix = g % L.nx, ky = L.y0 + g / L.nx;
      col[(size_t)g] = make_cd(s[0][ix].x + s[1][ky].x, s[0][ix].y + s[1][ky].y);
    }
    if (!colsym) HIPCHK(hipMalloc(&colsym, sizeof(cd) * (size_t)(ncols > 0 ? ncols : 1)));
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
  // buffers the steps of `list` touch must exist
  int prepare(const std::vector<Step>& list) {
    for (const Step& s : list)
      if (s.src == B_W2 || s.dst == B_W2) return ensure_work2();
    return CFP_SUCCESS;
  }
  cd* buf(int id, const cd* b, cd* x) const {
    switch (id) {
      case B_IN: return (cd*)b;
      case B_X: return x;
      case B_W: return work;
      case B_W2: return work2;
      default: return diag_t;
    }
  }
  // a kernel step (pass, 3-sweep stage, repack) on stream st
  int launch(const Step& s, const cd* b, cd* x, hipStream_t st) const {
    const cd* in = buf(s.src, b, x) + s.src_off;
    cd* out = buf(s.dst, b, x) + s.dst_off;
    if (s.kind == K_TP) {
      TPArgs a;
      a.tw = tw.at((int)L.nx);
      a.colsym = colsym3;
      a.axsym = axsym;
      a.scale = s.pass.scale;
      a.lnyl = ilog2_exact(L.nyp);  // (the 3-sweep slab schedule is never padded: P | 32)
      a.chunk = L.chunk;
      a.k1_off = (int)(L.r * (L.nyp / three_pass_slab_n2(L.nx)));  // N2 rows per k1
      hipError_t e = launch_three_pass_slab(s.tp, (int)L.nx, in, out, a, s.planes, st);
      return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "slab 3-sweep launch");
    }
    if (s.kind == K_REPACK) {
      hipError_t e = launch_repack(in, out, L, s.planes, s.to_chunks, st);
      return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "slab repack");
    }
    PassDesc p = s.pass;
    if (p.ncols == 0) return CFP_SUCCESS;  // a rank without z-pencil rows (padded layouts)
    if (s.fused == 1) { p.colsym = colsym; p.axsym = axsym; }
    if (s.fused == 2) p.diag = diag_t;  // the z-pencil Diag, addressed like the pass input
    hipError_t e = launch_axis_pass(p, in, out, tw.at(p.n), st);
    return e == hipSuccess ? CFP_SUCCESS : hip_error(e, "slab axis pass");
  }
};

}  // namespace

struct cfp_dist_plan_s {
  SlabRank R;
  ncclComm_t comm = nullptr;
  bool own_comm = true;
  double timeout_s = kRcclDefaultTimeoutS;  // RCCL init / enqueue / finalize deadline
  double init_ms = 0.0;                     // wall time of the communicator's creation
  cfp_dist_exchange_fn xfn = nullptr;  // caller's exchange (cfp_dist_plan_set_exchange)
  void* xuser = nullptr;
  hipStream_t cstream = nullptr;  // exchange stream of the pipelined apply
  std::vector<hipEvent_t> step_ev;  // one completion event per step (cross-stream waits)
  // sampled per-step start/end events inside the caller's applies (as cfp_plan_profile_begin)
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

// ------------------------------------------------------------------ host-only descriptions
extern "C" int cfp_slab_work_size(int64_t nx, int64_t ny, int64_t nz, int P, int r, int64_t* n) {
  if (!n) return set_error(CFP_ERR_ARG_NULL, "n is NULL");
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  *n = L.work;
  return CFP_SUCCESS;
}

extern "C" int cfp_slab_layout(int64_t nx, int64_t ny, int64_t nz, int P, int r, int64_t* out) {
  if (!out) return set_error(CFP_ERR_ARG_NULL, "out is NULL");
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  const int64_t v[8] = {L.nzl, L.nyl, L.z0, L.y0, L.local, L.chunk, L.offset, (int64_t)P};
  std::memcpy(out, v, sizeof(v));
  return CFP_SUCCESS;
}

static int host_steps(int64_t nx, int64_t ny, int64_t nz, int P, int r, int schedule, int pieces, int list,
                      SlabLayout* L, std::vector<Step>* out) {
  int rc = make_layout(nx, ny, nz, P, r, L);
  if (rc) return rc;
  if (schedule < CFP_SCHEDULE_AUTO || schedule > CFP_SCHEDULE_THREE_PASS)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "slab schedule must be AUTO, FIVE_PASS or THREE_PASS");
  if (list < CFP_SLAB_LIST_APPLY || list > CFP_SLAB_LIST_DIAG)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "unknown step list %d", list);
  const int K = pieces == 0 ? auto_pieces(*L) : pieces;
  if (!pieces_valid(*L, K)) return set_error(CFP_ERR_ARG_OUTOFRANGE, "pieces must divide the local planes");
  const int lk = list == CFP_SLAB_LIST_APPLY ? L_APPLY_SEP
               : list == CFP_SLAB_LIST_APPLY_DIAG ? L_APPLY_DIAG
               : list == CFP_SLAB_LIST_FORWARD ? L_FORWARD
               : list == CFP_SLAB_LIST_BACKWARD ? L_BACKWARD : L_DIAG_T;
  *out = slab_steps(*L, schedule, K, lk);
  return CFP_SUCCESS;
}

extern "C" int cfp_slab_steps_count(int64_t nx, int64_t ny, int64_t nz, int P, int r, int schedule, int pieces,
                                    int list, int* nsteps) {
  if (!nsteps) return set_error(CFP_ERR_ARG_NULL, "nsteps is NULL");
  SlabLayout L;
  std::vector<Step> st;
  int rc = host_steps(nx, ny, nz, P, r, schedule, pieces, list, &L, &st);
  if (rc) return rc;
  *nsteps = (int)st.size();
  return CFP_SUCCESS;
}

static void describe(const SlabLayout& L, const Step& s, int64_t* desc, double* scale) {
  const PassDesc& p = s.pass;
  const bool ps = s.kind == K_PASS;
  const int64_t v[CFP_SLAB_DESC_LEN] = {
      s.kind, s.src, s.dst,
      s.kind == K_TP ? s.tp : (s.kind == K_REPACK ? s.to_chunks : (ps ? s.axis : -1)),
      (ps || s.kind == K_TP) ? p.n : 0, (ps || s.kind == K_TP) ? p.mode : -1,
      ps ? p.ncols : s.planes, ps ? p.inner_n : 0,
      ps ? p.in.inner_stride : 0, ps ? p.in.outer_stride : 0, ps ? p.in.pt_stride : 0, ps ? p.in.seg_len : 0,
      ps ? p.in.seg_stride : 0,
      ps ? p.out.inner_stride : 0, ps ? p.out.outer_stride : 0, ps ? p.out.pt_stride : 0, ps ? p.out.seg_len : 0,
      ps ? p.out.seg_stride : 0,
      s.src_off, s.dst_off, s.ex_off, s.ex_cnt, L.chunk, s.wait,
      s.kind == K_TP ? ilog2_exact(L.nyp) : 0, s.kind == K_TP ? (int64_t)(L.r * (L.nyp / three_pass_slab_n2(L.nx))) : 0,
      s.seg, s.fused};
  std::memcpy(desc, v, sizeof(v));
  *scale = (ps || s.kind == K_TP) ? p.scale : 1.0;
}

extern "C" int cfp_slab_steps_get(int64_t nx, int64_t ny, int64_t nz, int P, int r, int schedule, int pieces, int list,
                                  int i, int64_t* desc, double* scale) {
  if (!desc || !scale) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  SlabLayout L;
  std::vector<Step> st;
  int rc = host_steps(nx, ny, nz, P, r, schedule, pieces, list, &L, &st);
  if (rc) return rc;
  if (i < 0 || i >= (int)st.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "step index");
  describe(L, st[(size_t)i], desc, scale);
  return CFP_SUCCESS;
}

// the round-2 description: the five-pass list with one piece, 18 fields
extern "C" int cfp_slab_num_steps(int64_t nx, int64_t ny, int64_t nz, int P, int r, int* nsteps) {
  return cfp_slab_steps_count(nx, ny, nz, P, r, CFP_SCHEDULE_FIVE_PASS, 1, CFP_SLAB_LIST_APPLY, nsteps);
}

extern "C" int cfp_slab_step_info(int64_t nx, int64_t ny, int64_t nz, int P, int r, int i, int64_t* desc,
                                  double* scale) {
  if (!desc || !scale) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  int64_t d[CFP_SLAB_DESC_LEN];
  int rc = cfp_slab_steps_get(nx, ny, nz, P, r, CFP_SCHEDULE_FIVE_PASS, 1, CFP_SLAB_LIST_APPLY, i, d, scale);
  if (rc) return rc;
  std::memcpy(desc, d, 18 * sizeof(int64_t));
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ plan
extern "C" int cfp_dist_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int cfp_dist_get_unique_id(char* id_out) {
  if (!id_out) return set_error(CFP_ERR_ARG_NULL, "id_out is NULL");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return CFP_SUCCESS;
}

static int plan_new(int64_t nx, int64_t ny, int64_t nz, int P, int r, int device, std::unique_ptr<cfp_dist_plan_s>* out) {
  SlabLayout L;
  int rc = make_layout(nx, ny, nz, P, r, &L);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<cfp_dist_plan_s> p(new cfp_dist_plan_s);
  rc = p->R.init(L, device);
  if (rc) { p->R.release(); return rc; }
  *out = std::move(p);
  return CFP_SUCCESS;
}

// The plan's own communicator is non-blocking (cfp_rccl.h): its creation is polled against
// timeout_s, so a rank that never joins is an error (CFP_ERR_LIB, "timed out") and not a hang.
extern "C" int cfp_dist_plan_create_timeout(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                            const char* uid, int device, double timeout_s) {
  if (!plan || !uid) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *plan = nullptr;
  std::unique_ptr<cfp_dist_plan_s> p;
  int rc = plan_new(nx, ny, nz, P, r, device, &p);
  if (rc) return rc;
  if (timeout_s > 0) p->timeout_s = timeout_s;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  bool timed_out = false;
  const auto t0 = std::chrono::steady_clock::now();
  const ncclResult_t nr = rccl_init_rank(&p->comm, P, id, r, p->timeout_s, &timed_out);
  p->init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (nr != ncclSuccess) {
    p->R.release();
    if (timed_out)
      return set_error(CFP_ERR_LIB, "ncclCommInitRankConfig: timed out after %.1f s (rank %d of %d)", p->timeout_s, r, P);
    return set_error(CFP_ERR_LIB, "%s: %s (rank %d of %d)", rccl_blocking() ? "ncclCommInitRank" : "ncclCommInitRankConfig",
                     ncclGetErrorString(nr), r, P);
  }
  *plan = p.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_create(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                    const char* uid, int device) {
  return cfp_dist_plan_create_timeout(plan, nx, ny, nz, P, r, uid, device, kRcclDefaultTimeoutS);
}

// What RCCL this plan talks through: the rank count and rank its communicator reports
// (ncclCommCount / ncclCommUserRank; 0 / -1 without one), the library version
// (ncclGetVersion), the creation time, and the shared object the calls bind to.
extern "C" int cfp_dist_plan_rccl_info(cfp_dist_plan_t p, int* nranks, int* rank, int* version, double* init_ms,
                                       char* lib_path, int path_len) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  int cnt = 0, rk = -1;
  if (p->comm) {
    NCCLCHK(ncclCommCount(p->comm, &cnt));
    NCCLCHK(ncclCommUserRank(p->comm, &rk));
  }
  if (nranks) *nranks = cnt;
  if (rank) *rank = rk;
  if (init_ms) *init_ms = p->init_ms;
  if (version) NCCLCHK(ncclGetVersion(version));
  rccl_library_path(lib_path, path_len);
  return CFP_SUCCESS;
}

// Host-only: 1 when the library's communicators use the blocking protocol (CFP_RCCL_BLOCKING),
// 0 for the default non-blocking creation polled against a deadline.
extern "C" int cfp_rccl_blocking(int* blocking) {
  if (!blocking) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *blocking = rccl_blocking() ? 1 : 0;
  return CFP_SUCCESS;
}

// Host-only (no GPU, no communicator): the RCCL version and library this process resolved.
extern "C" int cfp_rccl_version(int* version, char* lib_path, int path_len) {
  if (!version) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  NCCLCHK(ncclGetVersion(version));
  rccl_library_path(lib_path, path_len);
  return CFP_SUCCESS;
}

// a communicator the caller owns (an ncclComm_t of P ranks whose rank r is this process)
extern "C" int cfp_dist_plan_create_with_comm(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                              void* nccl_comm, int device) {
  if (!plan || !nccl_comm) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *plan = nullptr;
  int cnt = 0, rk = 0;
  NCCLCHK(ncclCommCount((ncclComm_t)nccl_comm, &cnt));
  NCCLCHK(ncclCommUserRank((ncclComm_t)nccl_comm, &rk));
  if (cnt != P || rk != r) return set_error(CFP_ERR_ARG_WRONG, "communicator has rank %d of %d, expected %d of %d", rk, cnt, r, P);
  std::unique_ptr<cfp_dist_plan_s> p;
  int rc = plan_new(nx, ny, nz, P, r, device, &p);
  if (rc) return rc;
  p->comm = (ncclComm_t)nccl_comm;
  p->own_comm = false;
  *plan = p.release();
  return CFP_SUCCESS;
}

// Plan without a communicator: the caller performs the exchanges itself, either through a
// callback (cfp_dist_plan_set_exchange) inside cfp_dist_plan_apply, or step by step
// (cfp_dist_plan_num_steps / _step / _run_step).
extern "C" int cfp_dist_plan_create_external(cfp_dist_plan_t* plan, int64_t nx, int64_t ny, int64_t nz, int P, int r,
                                             int device) {
  if (!plan) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *plan = nullptr;
  std::unique_ptr<cfp_dist_plan_s> p;
  int rc = plan_new(nx, ny, nz, P, r, device, &p);
  if (rc) return rc;
  *plan = p.release();
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_set_exchange(cfp_dist_plan_t p, cfp_dist_exchange_fn fn, void* user) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  p->xfn = fn;
  p->xuser = user;
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_work_buffer(cfp_dist_plan_t p, double** work) {
  if (!p || !work) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *work = (double*)p->R.work;
  return CFP_SUCCESS;
}

// use a caller-owned work buffer (cfp_slab_work_size complex values) instead of the plan's own
extern "C" int cfp_dist_plan_set_work_buffer(cfp_dist_plan_t p, double* work) {
  return cfp_dist_plan_set_work_buffers(p, work, nullptr);
}

extern "C" int cfp_dist_plan_set_work_buffers(cfp_dist_plan_t p, double* work, double* work2) {
  if (!p || !work) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  HIPCHK(hipDeviceSynchronize());  // the plan's own buffers may still be in use by queued work
  if (p->R.work && p->R.own_work) hipFree(p->R.work);
  p->R.work = (cd*)work;
  p->R.own_work = false;
  if (work2) {
    if (p->R.work2 && p->R.own_work2) hipFree(p->R.work2);
    p->R.work2 = (cd*)work2;
    p->R.own_work2 = false;
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_destroy(cfp_dist_plan_t p) {
  if (!p) return CFP_SUCCESS;
  hipSetDevice(p->R.device);
  hipDeviceSynchronize();
  dist_profile_free(p);
  for (auto& e : p->step_ev) hipEventDestroy(e);
  if (p->cstream) hipStreamDestroy(p->cstream);
  if (p->comm && p->own_comm) rccl_destroy(p->comm, p->timeout_s);
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
    return set_error(CFP_ERR_SUP, "the 3-sweep slab schedule needs a 256^3 or 512^3 grid and nranks | 32");
  return CFP_SUCCESS;
}

static int pieces_check(const SlabLayout& L, int pieces) {
  if (pieces < 0 || (pieces > 0 && !pieces_valid(L, pieces)))
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "pieces (%d) must be 0 (AUTO) or divide the %lld local planes", pieces,
                     (long long)L.nzl);
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_set_schedule(cfp_dist_plan_t p, int schedule) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  int rc = slab_schedule_check(p->R.L, schedule);
  if (rc) return rc;
  HIPCHK(hipSetDevice(p->R.device));
  HIPCHK(hipDeviceSynchronize());
  dist_profile_free(p);
  return p->R.set_steps(schedule, p->R.pieces_req);
}

extern "C" int cfp_dist_plan_set_pieces(cfp_dist_plan_t p, int pieces) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  int rc = pieces_check(p->R.L, pieces);
  if (rc) return rc;
  HIPCHK(hipSetDevice(p->R.device));
  HIPCHK(hipDeviceSynchronize());
  dist_profile_free(p);
  return p->R.set_steps(p->R.schedule, pieces);
}

extern "C" int cfp_dist_plan_pieces(cfp_dist_plan_t p, int* pieces) {
  if (!p || !pieces) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *pieces = p->R.pieces();
  return CFP_SUCCESS;
}

extern "C" int cfp_group_set_schedule(cfp_group_t g, int schedule) {
  if (!g) return set_error(CFP_ERR_ARG_NULL, "NULL group");
  for (auto& R : g->R) {
    int rc = slab_schedule_check(R.L, schedule);
    if (rc) return rc;
    HIPCHK(hipSetDevice(R.device));
    rc = R.set_steps(schedule, R.pieces_req);
    if (rc) return rc;
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_group_set_pieces(cfp_group_t g, int pieces) {
  if (!g) return set_error(CFP_ERR_ARG_NULL, "NULL group");
  for (auto& R : g->R) {
    int rc = pieces_check(R.L, pieces);
    if (rc) return rc;
    HIPCHK(hipSetDevice(R.device));
    rc = R.set_steps(R.schedule, pieces);
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
  const bool ex = s.kind == K_EXCH;
  if (is_exchange) *is_exchange = ex ? 1 : 0;
  if (axis) *axis = ex ? -1 : s.axis;
  if (n) *n = ex ? 0 : s.pass.n;
  if (mode) *mode = ex ? -1 : s.pass.mode;
  return CFP_SUCCESS;
}

// One exchange piece: through the plan's RCCL communicator (grouped ncclSend / ncclRecv; the
// self chunk is a device copy), or through the caller's callback.
static int do_exchange(cfp_dist_plan_s* p, const Step& s, const cd* src, cd* dst, hipStream_t st) {
  const SlabLayout& L = p->R.L;
  if (p->xfn) {
    const int rc = p->xfn(p->xuser, (const double*)src, (double*)dst, L.chunk, s.ex_off, s.ex_cnt, (void*)st);
    return rc ? set_error(CFP_ERR_LIB, "exchange callback returned %d", rc) : CFP_SUCCESS;
  }
  if (L.P > 1 && !p->comm)
    return set_error(CFP_ERR_ARG_WRONGSTATE, "plan made with cfp_dist_plan_create_external has no communicator or exchange callback");
  const i64 self = L.r * L.chunk + s.ex_off;
  HIPCHK(hipMemcpyAsync(dst + self, src + self, sizeof(cd) * (size_t)s.ex_cnt, hipMemcpyDeviceToDevice, st));
  if (L.P == 1) return CFP_SUCCESS;
  const size_t cnt = (size_t)s.ex_cnt * 2;  // doubles per peer message
  NCCLCHK(ncclGroupStart());
  for (int q = 0; q < L.P; ++q) {
    if (q == L.r) continue;
    NCCLCHK(ncclSend(src + q * L.chunk + s.ex_off, cnt, ncclDouble, q, p->comm, st));
    NCCLCHK(ncclRecv(dst + q * L.chunk + s.ex_off, cnt, ncclDouble, q, p->comm, st));
  }
  // a non-blocking communicator may still be enqueueing: settle before the next call on it
  NCCLCHK(rccl_settle(p->comm, ncclGroupEnd(), p->timeout_s));
  return CFP_SUCCESS;
}

// Run a step list.  Kernels go to the caller's stream s.  With more than one piece the
// exchanges go to the plan's exchange stream; each cross-stream edge (Step::wait) is an event.
// ev (profiling): 2 events per step, recorded around it on the stream it runs on.
static int dist_run(cfp_dist_plan_s* p, const std::vector<Step>& steps, const cd* b, cd* x, hipStream_t s,
                    hipEvent_t* ev) {
  int rc = p->R.prepare(steps);
  if (rc) return rc;
  int nex = 0;
  for (const Step& st : steps) nex += st.kind == K_EXCH;
  const bool two = nex > 2;  // pieces: overlap on the exchange stream
  if (two) {
    if (!p->cstream) HIPCHK(hipStreamCreateWithFlags(&p->cstream, hipStreamNonBlocking));
    while (p->step_ev.size() < steps.size()) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      p->step_ev.push_back(e);
    }
  }
  for (size_t i = 0; i < steps.size(); ++i) {
    const Step& st = steps[i];
    const bool ex = st.kind == K_EXCH;
    hipStream_t q = (two && ex) ? p->cstream : s;
    if (two && st.wait >= 0) HIPCHK(hipStreamWaitEvent(q, p->step_ev[(size_t)st.wait], 0));
    if (ev) HIPCHK(hipEventRecord(ev[2 * i], q));
    rc = ex ? do_exchange(p, st, p->R.buf(st.src, b, x), p->R.buf(st.dst, b, x), q) : p->R.launch(st, b, x, q);
    if (rc) return rc;
    if (ev) HIPCHK(hipEventRecord(ev[2 * i + 1], q));
    if (two) HIPCHK(hipEventRecord(p->step_ev[i], q));
  }
  if (two) {  // the caller's stream sees the whole apply (the last exchange included)
    for (size_t i = steps.size(); i-- > 0;)
      if (steps[i].kind == K_EXCH) {
        HIPCHK(hipStreamWaitEvent(s, p->step_ev[i], 0));
        break;
      }
  }
  return CFP_SUCCESS;
}

static const std::vector<Step>& apply_list(const cfp_dist_plan_s* p) {
  return p->R.diag ? p->R.diag_steps : p->R.steps;
}

extern "C" int cfp_dist_plan_apply(cfp_dist_plan_t p, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!p->R.sym && !p->R.diag) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  HIPCHK(hipSetDevice(p->R.device));
  const std::vector<Step>& steps = apply_list(p);
  const bool sample = p->prof_cap && (p->prof_calls++ % p->prof_every) == 0;
  if (sample && p->prof_used < p->prof_cap && p->prof_stride == 2 * steps.size()) {
    hipEvent_t* ev = p->prof_ev.data() + p->prof_used * p->prof_stride;
    ++p->prof_used;
    return dist_run(p, steps, (const cd*)b, (cd*)x, (hipStream_t)stream, ev);
  }
  return dist_run(p, steps, (const cd*)b, (cd*)x, (hipStream_t)stream, nullptr);
}

// Explicit Diag (local natural slab, device): transposed once into the z-pencil layout the
// fused z pass reads (a collective: every rank calls it), then every apply divides by it.
extern "C" int cfp_dist_plan_set_diag(cfp_dist_plan_t p, const double* diag_local, void* stream) {
  if (!p || !diag_local) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  SlabRank& R = p->R;
  if (!R.diag_t) HIPCHK(hipMalloc(&R.diag_t, sizeof(cd) * (size_t)R.L.work));
  const std::vector<Step> st = slab_steps(R.L, R.schedule, 1, L_DIAG_T);
  int rc = dist_run(p, st, (const cd*)diag_local, nullptr, (hipStream_t)stream, nullptr);
  if (rc) return rc;
  R.diag = true;
  return CFP_SUCCESS;
}

// back to the separable symbol (if one was set); the z-pencil Diag stays for cfp_dist_plan_use_diag
extern "C" int cfp_dist_plan_clear_diag(cfp_dist_plan_t p) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  p->R.diag = false;
  return CFP_SUCCESS;
}

// switch between the last Diag given to cfp_dist_plan_set_diag (on) and the separable symbol
extern "C" int cfp_dist_plan_use_diag(cfp_dist_plan_t p, int on) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (on && !p->R.diag_t) return set_error(CFP_ERR_ARG_WRONGSTATE, "no Diag was set (cfp_dist_plan_set_diag)");
  p->R.diag = on != 0;
  return CFP_SUCCESS;
}

// Unnormalised 3-D transforms of the slab in natural order (MatMult / MatMultTranspose of a
// distributed MATFFTW): one piece, 6 steps.
extern "C" int cfp_dist_plan_forward(cfp_dist_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  const std::vector<Step> st = slab_steps(p->R.L, p->R.schedule, 1, L_FORWARD);
  return dist_run(p, st, (const cd*)in, (cd*)out, (hipStream_t)stream, nullptr);
}

extern "C" int cfp_dist_plan_backward(cfp_dist_plan_t p, const double* in, double* out, void* stream) {
  if (!p || !in || !out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  HIPCHK(hipSetDevice(p->R.device));
  const std::vector<Step> st = slab_steps(p->R.L, p->R.schedule, 1, L_BACKWARD);
  return dist_run(p, st, (const cd*)in, (cd*)out, (hipStream_t)stream, nullptr);
}

// ------------------------------------------------------------------ step-by-step (external)
extern "C" int cfp_dist_plan_num_steps(cfp_dist_plan_t p, int* n) {
  if (!p || !n) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *n = (int)apply_list(p).size();
  return CFP_SUCCESS;
}

extern "C" int cfp_dist_plan_step(cfp_dist_plan_t p, int i, int64_t* desc) {
  if (!p || !desc) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  const std::vector<Step>& st = apply_list(p);
  if (i < 0 || i >= (int)st.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "step index");
  double sc;
  describe(p->R.L, st[(size_t)i], desc, &sc);
  return CFP_SUCCESS;
}

// enqueue the kernels of step i (not an exchange: the caller performs those)
extern "C" int cfp_dist_plan_run_step(cfp_dist_plan_t p, int i, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!p->R.sym && !p->R.diag) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  const std::vector<Step>& st = apply_list(p);
  if (i < 0 || i >= (int)st.size()) return set_error(CFP_ERR_ARG_OUTOFRANGE, "step index");
  if (st[(size_t)i].kind == K_EXCH) return set_error(CFP_ERR_ARG_WRONG, "step %d is an exchange", i);
  HIPCHK(hipSetDevice(p->R.device));
  int rc = p->R.prepare(st);
  if (rc) return rc;
  return p->R.launch(st[(size_t)i], (const cd*)b, (cd*)x, (hipStream_t)stream);
}

// segment 0: kernels before the first exchange (which sends work -> receives into x);
// segment 1: between the exchanges (the exchange after it sends x -> receives into work);
// segment 2: kernels after the second exchange.  One piece only (cfp_dist_plan_set_pieces(1)).
extern "C" int cfp_dist_plan_run_segment(cfp_dist_plan_t p, int seg, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (seg < 0 || seg > 2) return set_error(CFP_ERR_ARG_OUTOFRANGE, "segment must be 0, 1 or 2");
  if (!p->R.sym && !p->R.diag) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  const std::vector<Step>& st = apply_list(p);
  int nex = 0;
  for (const Step& s : st) nex += s.kind == K_EXCH;
  if (nex != 2) return set_error(CFP_ERR_ARG_WRONGSTATE, "segments need one piece (cfp_dist_plan_set_pieces(plan, 1))");
  HIPCHK(hipSetDevice(p->R.device));
  for (const Step& s : st) {
    if (s.kind == K_EXCH || s.seg != seg) continue;
    int rc = p->R.launch(s, (const cd*)b, (cd*)x, (hipStream_t)stream);
    if (rc) return rc;
  }
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ profiling
// sampled per-step events inside the caller's own applies (cfp_plan_profile_begin's contract);
// a step's time is measured on the stream it runs on (exchanges on the exchange stream when
// pieces > 1, where they overlap the passes)
extern "C" int cfp_dist_plan_profile_begin(cfp_dist_plan_t p, int max_applies, int every) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (max_applies < 1 || max_applies > 100000 || every < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "bad profile range");
  HIPCHK(hipSetDevice(p->R.device));
  dist_profile_free(p);
  p->prof_stride = 2 * apply_list(p).size();
  p->prof_ev.resize(p->prof_stride * (size_t)max_applies, nullptr);
  for (auto& e : p->prof_ev) {
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (r != hipSuccess) {
      dist_profile_free(p);
      return hip_error(r, "hipEventCreate");
    }
  }
  p->prof_cap = (size_t)max_applies;
  p->prof_every = (size_t)every;
  return CFP_SUCCESS;
}

static void accumulate(const std::vector<hipEvent_t>& ev, size_t applies, size_t np, std::vector<double>& acc) {
  for (size_t a = 0; a < applies; ++a)
    for (size_t i = 0; i < np; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[a * 2 * np + 2 * i], ev[a * 2 * np + 2 * i + 1]);
      acc[i] += ms;
    }
}

extern "C" int cfp_dist_plan_profile_end(cfp_dist_plan_t p, double* ms_out, int* applies) {
  if (!p || !ms_out || !applies) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (!p->prof_cap) return set_error(CFP_ERR_ARG_WRONGSTATE, "profiling was not started");
  HIPCHK(hipSetDevice(p->R.device));
  const size_t np = p->prof_stride / 2, used = p->prof_used;
  std::vector<double> acc(np, 0.0);
  int rc = CFP_SUCCESS;
  if (used > 0) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = hip_error(e, "profile sync");
  }
  if (!rc) accumulate(p->prof_ev, used, np, acc);
  for (size_t i = 0; i < np; ++i) ms_out[i] = used ? acc[i] / (double)used : 0.0;
  *applies = (int)used;
  dist_profile_free(p);
  return rc;
}

extern "C" int cfp_dist_plan_time_phases(cfp_dist_plan_t p, const double* b, double* x, int iters, double* ms_out,
                                         void* stream) {
  if (!p || !b || !x || !ms_out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (iters < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "iters must be >= 1");
  if (!p->R.sym && !p->R.diag) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the slab plan");
  HIPCHK(hipSetDevice(p->R.device));
  const std::vector<Step>& steps = apply_list(p);
  const size_t np = steps.size();
  std::vector<hipEvent_t> ev(2 * np);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  std::vector<double> acc(np, 0.0);
  int rc = CFP_SUCCESS;
  for (int it = 0; it < iters && !rc; ++it) {
    rc = dist_run(p, steps, (const cd*)b, (cd*)x, (hipStream_t)stream, ev.data());
    if (rc) break;
    if (hipDeviceSynchronize() != hipSuccess) { rc = set_error(CFP_ERR_LIB, "device sync"); break; }
    accumulate(ev, 1, np, acc);
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
    hipDeviceSynchronize();
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

// Every rank's steps in list order; an exchange piece is a set of device copies (rank r's
// [q chunk + off, + cnt) -> rank q's [r chunk + off]) after all streams have drained.
extern "C" int cfp_group_apply(cfp_group_t g, const double* const* b, double* const* x) {
  if (!g || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  const int P = (int)g->R.size();
  for (auto& R : g->R) {
    if (!R.sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set on the group");
    HIPCHK(hipSetDevice(R.device));
    int rc = R.prepare(R.steps);
    if (rc) return rc;
  }
  const size_t nsteps = g->R[0].steps.size();
  for (size_t i = 0; i < nsteps; ++i) {
    const Step& st = g->R[0].steps[i];
    if (st.kind != K_EXCH) {
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
      for (int r = 0; r < P; ++r) {
        const SlabRank& S = g->R[r];
        HIPCHK(hipSetDevice(S.device));
        const cd* src = S.buf(st.src, (const cd*)b[r], (cd*)x[r]);
        for (int q = 0; q < P; ++q) {
          const SlabRank& D = g->R[q];
          cd* dst = D.buf(st.dst, (const cd*)b[q], (cd*)x[q]);
          HIPCHK(hipMemcpyAsync(dst + r * D.L.chunk + st.ex_off, src + q * S.L.chunk + st.ex_off,
                                sizeof(cd) * (size_t)st.ex_cnt, hipMemcpyDefault, g->streams[r]));
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
