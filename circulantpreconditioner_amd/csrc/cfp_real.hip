// cfp_real.hip -- real-data circulant apply (include/circulant_fft_real.h, SURVEY.md §8f row
// f4): the reference's real-scalar solve_3D (src/FftLinearSolver_3D.c:6-78, 166-190) as an
// r2c / half-spectrum / c2r schedule.
//
// x pass, forward (k_rx<false>): a real row of nx = 2M values is read as M complex values
// z[j] = (x[2j], x[2j+1]) (no repacking: the same bytes), Z = FFT_M(z) in registers/LDS, then
//     E[k] = (Z[k] + conj Z[M-k]) / 2,  O[k] = (Z[k] - conj Z[M-k]) / 2i,
//     X[k] = E[k] + W_2M^k O[k]  (k < M),   X[M] = E[0] - O[0]  (Nyquist),
// with Z[M-k] taken from the partner lane of the same row (cross-lane shuffle).  X[0..M) goes
// to the half-spectrum grid H (M x ny x nz), X[M] to the Nyquist grid Q (1 x ny x nz).
// y/z: the complex plan's passes on H and on Q (z fused with the symbol, no 1/N).
// x pass, inverse (k_rx<true>): the even/odd merge run backwards, then IFFT_M and 2/N.
#include <hip/hip_runtime.h>

#include <cmath>
#include <memory>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/circulant_fft_real.h"
#include "cfp_fft_device.h"
#include "cfp_host.h"
#include "cfp_three_pass.h"

namespace cfp {

__device__ __forceinline__ cd shfl_cd(cd v, int lane) { return make_cd(__shfl(v.x, lane), __shfl(v.y, lane)); }

// M = nx/2 points per row FFT, PTS points per thread, first radix R0, T rows per workgroup
template <int M, int PTS, int R0, int T, bool INV>
__global__ void __launch_bounds__(T*(M / PTS)) k_rx(const double* in_r, cd* half, cd* nyq, double* out_r,
                                                    const cd* twn, i64 rows, double scale) {
  constexpr int TPC = M / PTS;
  static_assert(64 % TPC == 0, "a row's threads must sit in one wavefront");
  constexpr int NT = T * TPC;
  constexpr int LDS_N = T * (M + M / 16);
  constexpr bool NEED_LDS = Shape<M, PTS, R0>::S > 1;
  constexpr int F = F_SPLIT_LDS;
  __shared__ __attribute__((aligned(16))) double lds[NEED_LDS ? LDS_N : 2];
  __shared__ cd tws[M];  // W_M[k] = W_2M[2k]
  const int tid = threadIdx.x;
  for (int i = tid; i < M; i += NT) tws[i] = twn[2 * i];
  const int tpc = tid % TPC, c = tid / TPC;
  const i64 row = (i64)blockIdx.x * T + c;
  const bool live = row < rows;
  const int lane = tid & 63;
  const int pl = lane - tpc + ((TPC - tpc) & (TPC - 1));  // lane of the mirror partner
  cd v[PTS];
  if (!INV) {
    const cd* in = reinterpret_cast<const cd*>(in_r) + row * M;
#pragma unroll
    for (int t = 0; t < PTS; ++t) v[t] = live ? in[tpc + t * TPC] : make_cd(0.0, 0.0);
    fft_stages<M, PTS, R0, true, T, F>(v, lds, tws, c, tpc, true);  // v[t] = Z[tpc + t TPC]
#pragma unroll
    for (int t = 0; t < PTS; ++t) {
      const int k = tpc + t * TPC;
      const cd za = shfl_cd(v[(PTS - t) % PTS], pl), zb = shfl_cd(v[PTS - 1 - t], pl);
      const cd zm = tpc == 0 ? za : zb;  // Z[M - k]
      const cd e = make_cd(0.5 * (v[t].x + zm.x), 0.5 * (v[t].y - zm.y));
      const cd d = make_cd(v[t].x - zm.x, v[t].y + zm.y);  // Z[k] - conj Z[M-k]
      const cd o = make_cd(0.5 * d.y, -0.5 * d.x);          // d / 2i
      if (live) {
        half[row * M + k] = cadd(e, cmul(twn[k], o));
        if (k == 0) nyq[row] = csub(e, o);
      }
    }
  } else {
    cd X[PTS];
    const cd* h = half + row * M;
#pragma unroll
    for (int t = 0; t < PTS; ++t) X[t] = live ? h[tpc + t * TPC] : make_cd(0.0, 0.0);
    const cd xn = (live && tpc == 0) ? nyq[row] : make_cd(0.0, 0.0);
#pragma unroll
    for (int t = 0; t < PTS; ++t) {
      const int k = tpc + t * TPC;
      const cd xa = shfl_cd(X[(PTS - t) % PTS], pl), xb = shfl_cd(X[PTS - 1 - t], pl);
      const cd xm = tpc == 0 ? (t == 0 ? xn : xa) : xb;  // X[M - k]
      const cd e = make_cd(0.5 * (X[t].x + xm.x), 0.5 * (X[t].y - xm.y));
      const cd d = make_cd(0.5 * (X[t].x - xm.x), 0.5 * (X[t].y + xm.y));
      const cd o = cmul(d, cconj(twn[k]));  // (X[k] - conj X[M-k]) W^-k / 2
      const cd z = make_cd(e.x - o.y, e.y + o.x);  // E + i O
      v[t] = cconj(z);  // inverse FFT by conjugation
    }
    fft_stages<M, PTS, R0, true, T, F>(v, lds, tws, c, tpc, true);
    cd* out = reinterpret_cast<cd*>(out_r) + row * M;
    if (live) {
#pragma unroll
      for (int t = 0; t < PTS; ++t) out[tpc + t * TPC] = make_cd(v[t].x * scale, -v[t].y * scale);
    }
  }
}

// row-pass shapes per M (TPC = M / PTS divides 64)
template <int M> struct RCfg;
template <> struct RCfg<16> { static constexpr int PTS = 4, R0 = 4, T = 64; };
template <> struct RCfg<32> { static constexpr int PTS = 8, R0 = 4, T = 64; };
template <> struct RCfg<64> { static constexpr int PTS = 8, R0 = 8, T = 32; };
template <> struct RCfg<128> { static constexpr int PTS = 8, R0 = 2, T = 16; };
template <> struct RCfg<256> { static constexpr int PTS = 8, R0 = 4, T = 8; };
template <> struct RCfg<512> { static constexpr int PTS = 16, R0 = 2, T = 8; };

template <int M, bool INV>
static hipError_t launch_rx_m(const double* in, cd* half, cd* nyq, double* out, const cd* twn, i64 rows, double sc,
                              hipStream_t s) {
  typedef RCfg<M> C;
  const unsigned blocks = (unsigned)((rows + C::T - 1) / C::T);
  hipLaunchKernelGGL((k_rx<M, C::PTS, C::R0, C::T, INV>), dim3(blocks), dim3(C::T * (M / C::PTS)), 0, s, in, half, nyq,
                     out, twn, rows, sc);
  return hipGetLastError();
}

static hipError_t launch_rx(int M, bool inv, const double* in, cd* half, cd* nyq, double* out, const cd* twn, i64 rows,
                            double sc, hipStream_t s) {
#define CFP_RX(MM)                                                                       \
  case MM:                                                                               \
    return inv ? launch_rx_m<MM, true>(in, half, nyq, out, twn, rows, sc, s)             \
               : launch_rx_m<MM, false>(in, half, nyq, out, twn, rows, sc, s);
  switch (M) {
    CFP_RX(16) CFP_RX(32) CFP_RX(64) CFP_RX(128) CFP_RX(256) CFP_RX(512)
    default: return hipErrorInvalidValue;
  }
#undef CFP_RX
}

}  // namespace cfp

using namespace cfp;

#define HIPCHK(expr)                                        \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return cfp::hip_error(_e, #expr); \
  } while (0)
#define CFPCHK(expr)              \
  do {                            \
    int _r = (expr);              \
    if (_r != CFP_SUCCESS) return _r; \
  } while (0)

struct cfp_rplan_s {
  int device = 0;
  i64 n[3] = {1, 1, 1};
  i64 M = 1;
  cfp_plan_t main = nullptr;  // M x ny x nz half spectrum, y/z passes only
  cfp_plan_t nyq = nullptr;   // 1 x ny x nz Nyquist column kx = nx/2
  cd* H = nullptr;
  cd* Q = nullptr;
  cd* twn = nullptr;  // W_nx
  bool has_sym = false;
  // the Nyquist grid's passes overlap the half-spectrum passes (5-pass schedule only; created on
  // first use: a process holding an extra stream ran the 128^3 apply on the default stream 9 %
  // slower afterwards, 17.1k against 18.8k applies/s in bench.py, r03z)
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // 3-sweep schedule at 128^3 / 256^3 (cfp_three_pass.hip): separable symbol of the half spectrum
  int schedule = CFP_RSCHEDULE_AUTO;
  cd* colsym3 = nullptr;  // [kx + M ky], kx < M
  cd* axsym3 = nullptr;   // [kz]
  cd* colsymq = nullptr;  // [ky] of the Nyquist column kx = M
};

static bool three_ok(const cfp_rplan_s* p) {
  return p->n[0] == p->n[1] && p->n[1] == p->n[2] && (p->n[0] == 128 || p->n[0] == 256);
}
static bool use_three(const cfp_rplan_s* p) { return three_ok(p) && p->schedule != CFP_RSCHEDULE_FIVE; }

namespace {
struct RGuard {
  int prev = -1;
  explicit RGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~RGuard() {
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

void free_rplan(cfp_rplan_s* p) {
  if (p->main) cfp_plan_destroy(p->main);
  if (p->nyq) cfp_plan_destroy(p->nyq);
  if (p->H) hipFree(p->H);
  if (p->Q) hipFree(p->Q);
  if (p->twn) hipFree(p->twn);
  if (p->colsym3) hipFree(p->colsym3);
  if (p->colsymq) hipFree(p->colsymq);
  if (p->axsym3) hipFree(p->axsym3);
  if (p->fork) hipEventDestroy(p->fork);
  if (p->join) hipEventDestroy(p->join);
  if (p->side) hipStreamDestroy(p->side);
  delete p;
}

// 3 sweeps at 128^3 and 256^3: P1r (r2c rows + y1, also of the Nyquist column into Q) | P2 on the
// half spectrum, then on Q's 32 k1 (one small launch) | P3r (y1 inverse + c2r rows).  (Until r04
// the column took its own 3-launch y / z plan between P2 and P3r: 18.4 us at 256^3.)
int run_real_three(cfp_rplan_s* p, const double* b, double* x, hipStream_t s, std::vector<hipEvent_t>* ev) {
  TPArgs a;
  a.tw = p->twn;  // W_n: nx = ny = nz = n
  a.colsym = p->colsym3;
  a.axsym = p->axsym3;
  a.scale = 2.0 / (double)(p->n[0] * p->n[1] * p->n[2]);
  if (ev) HIPCHK(hipEventRecord((*ev)[0], s));
  const bool alt = p->schedule == CFP_RSCHEDULE_THREE_ALT;
  hipError_t e = launch_three_pass_real(0, (int)p->n[0], b, p->H, p->Q, nullptr, a, s, alt);
  if (e != hipSuccess) return hip_error(e, "r2c rows + y1 pass");
  if (ev) HIPCHK(hipEventRecord((*ev)[1], s));
  e = launch_three_pass_real(1, (int)p->n[0], nullptr, p->H, nullptr, nullptr, a, s);
  if (e != hipSuccess) return hip_error(e, "half-spectrum y2/z pass");
  if (ev) HIPCHK(hipEventRecord((*ev)[2], s));
  TPArgs aq = a;
  aq.colsym = p->colsymq;
  e = launch_three_pass_real(3, (int)p->n[0], nullptr, nullptr, p->Q, nullptr, aq, s);
  if (e != hipSuccess) return hip_error(e, "Nyquist column y2/z pass");
  if (ev) HIPCHK(hipEventRecord((*ev)[3], s));
  e = launch_three_pass_real(2, (int)p->n[0], nullptr, p->H, p->Q, x, a, s, alt);
  if (e != hipSuccess) return hip_error(e, "y1 inverse + c2r rows pass");
  if (ev) HIPCHK(hipEventRecord((*ev)[4], s));
  return CFP_SUCCESS;
}

int run_real(cfp_rplan_s* p, const double* b, double* x, hipStream_t s, std::vector<hipEvent_t>* ev) {
  if (!p->has_sym) return set_error(CFP_ERR_ARG_WRONGSTATE, "no symbol set (call cfp_rplan_set_symbol_transport)");
  if (use_three(p)) return run_real_three(p, b, x, s, ev);
  const i64 rows = p->n[1] * p->n[2];
  const double sc = 2.0 / (double)(p->n[0] * p->n[1] * p->n[2]);
  if (ev) HIPCHK(hipEventRecord((*ev)[0], s));
  hipError_t e = launch_rx((int)p->M, false, b, p->H, p->Q, nullptr, p->twn, rows, 1.0, s);
  if (e != hipSuccess) return hip_error(e, "r2c row pass");
  // small grids: the cross-stream handshake costs more than the Nyquist passes it hides
  const bool overlap = p->M * rows >= (i64(1) << 21);
  if (ev || !overlap) {  // timed, or small: the stages one after the other
    if (ev) HIPCHK(hipEventRecord((*ev)[1], s));
    CFPCHK(cfp_plan_apply(p->main, (const double*)p->H, (double*)p->H, s));
    if (ev) HIPCHK(hipEventRecord((*ev)[2], s));
    CFPCHK(cfp_plan_apply(p->nyq, (const double*)p->Q, (double*)p->Q, s));
    if (ev) HIPCHK(hipEventRecord((*ev)[3], s));
  } else {  // Nyquist grid on the side stream, concurrently with the half spectrum
    if (!p->side) {  // created on first use: the 3-sweep grids never need it
      HIPCHK(hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&p->fork, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&p->join, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(p->fork, s));
    HIPCHK(hipStreamWaitEvent(p->side, p->fork, 0));
    CFPCHK(cfp_plan_apply(p->nyq, (const double*)p->Q, (double*)p->Q, p->side));
    HIPCHK(hipEventRecord(p->join, p->side));
    CFPCHK(cfp_plan_apply(p->main, (const double*)p->H, (double*)p->H, s));
    HIPCHK(hipStreamWaitEvent(s, p->join, 0));
  }
  e = launch_rx((int)p->M, true, nullptr, p->H, p->Q, x, p->twn, rows, sc, s);
  if (e != hipSuccess) return hip_error(e, "c2r row pass");
  if (ev) HIPCHK(hipEventRecord((*ev)[4], s));
  return CFP_SUCCESS;
}
}  // namespace

extern "C" int cfp_rplan_create(cfp_rplan_t* plan, int64_t nx, int64_t ny, int64_t nz, int device) {
  if (!plan) return set_error(CFP_ERR_ARG_NULL, "plan is NULL");
  *plan = nullptr;
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const i64 M = nx / 2;
  if (nx % 2 || M < 16 || M > 512 || (M & (M - 1)))
    return set_error(CFP_ERR_SUP, "real plan: nx/2 must be a power of two in [16, 512] (nx = %lld)", (long long)nx);
  if (ny * nz < 2) return set_error(CFP_ERR_SUP, "real plan: needs ny * nz > 1");
  cfp_rplan_s* p = new cfp_rplan_s;
  p->device = device;
  p->n[0] = nx;
  p->n[1] = ny;
  p->n[2] = nz;
  p->M = M;
  int rc = cfp_plan_create(&p->main, M, ny, nz, device);
  if (rc == CFP_SUCCESS) rc = cfp_plan_set_external_x(p->main, 1);
  if (rc == CFP_SUCCESS) rc = cfp_plan_create(&p->nyq, 1, ny, nz, device);
  if (rc == CFP_SUCCESS) rc = cfp_plan_set_external_x(p->nyq, 1);
  if (rc != CFP_SUCCESS) {
    free_rplan(p);
    return rc;
  }
  RGuard g(device);
  std::vector<cd> tw = host_twiddles((int)nx, -1);
  hipError_t e = hipMalloc(&p->H, sizeof(cd) * (size_t)(M * ny * nz));
  if (e == hipSuccess) e = hipMalloc(&p->Q, sizeof(cd) * (size_t)(ny * nz));
  if (e == hipSuccess) e = hipMalloc(&p->twn, sizeof(cd) * (size_t)nx);
  if (e == hipSuccess) e = hipMemcpy(p->twn, tw.data(), sizeof(cd) * (size_t)nx, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_rplan(p);
    return hip_error(e, "real plan buffers");
  }
  *plan = p;
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_destroy(cfp_rplan_t p) {
  if (!p) return CFP_SUCCESS;
  RGuard g(p->device);
  free_rplan(p);
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_set_symbol_transport(cfp_rplan_t p, const double lam[3]) {
  if (!p || !lam) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  const std::vector<cd> hx = host_transport_symbol(p->n[0]), hy = host_transport_symbol(p->n[1]),
                        hz = host_transport_symbol(p->n[2]);
  const double lam6[6] = {lam[0], 0.0, lam[1], 0.0, lam[2], 0.0};
  // half spectrum kx < nx/2, and the Nyquist column kx = nx/2
  CFPCHK(cfp_plan_set_symbol_separable(p->main, (const double*)hx.data(), (const double*)hy.data(),
                                       (const double*)hz.data(), lam6));
  CFPCHK(cfp_plan_set_symbol_separable(p->nyq, (const double*)&hx[(size_t)p->M], (const double*)hy.data(),
                                       (const double*)hz.data(), lam6));
  if (three_ok(p)) {  // the 3-sweep tables: colsym [kx + M ky] = lx hx[kx] + ly hy[ky], axsym = lz hz
    RGuard g(p->device);
    const i64 M = p->M, ny = p->n[1], nz = p->n[2];
    std::vector<cd> col((size_t)(M * ny)), ax((size_t)nz);
    for (i64 ky = 0; ky < ny; ++ky)
      for (i64 kx = 0; kx < M; ++kx)
        col[(size_t)(kx + M * ky)] = make_cd(lam[0] * hx[(size_t)kx].x + lam[1] * hy[(size_t)ky].x,
                                             lam[0] * hx[(size_t)kx].y + lam[1] * hy[(size_t)ky].y);
    for (i64 kz = 0; kz < nz; ++kz) ax[(size_t)kz] = make_cd(lam[2] * hz[(size_t)kz].x, lam[2] * hz[(size_t)kz].y);
    std::vector<cd> colq((size_t)ny);  // the Nyquist column kx = M
    for (i64 ky = 0; ky < ny; ++ky)
      colq[(size_t)ky] = make_cd(lam[0] * hx[(size_t)M].x + lam[1] * hy[(size_t)ky].x,
                                 lam[0] * hx[(size_t)M].y + lam[1] * hy[(size_t)ky].y);
    if (!p->colsym3) HIPCHK(hipMalloc(&p->colsym3, sizeof(cd) * col.size()));
    if (!p->axsym3) HIPCHK(hipMalloc(&p->axsym3, sizeof(cd) * ax.size()));
    if (!p->colsymq) HIPCHK(hipMalloc(&p->colsymq, sizeof(cd) * colq.size()));
    HIPCHK(hipMemcpy(p->colsym3, col.data(), sizeof(cd) * col.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->axsym3, ax.data(), sizeof(cd) * ax.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->colsymq, colq.data(), sizeof(cd) * colq.size(), hipMemcpyHostToDevice));
  }
  p->has_sym = true;
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_set_schedule(cfp_rplan_t p, int schedule) {
  if (!p) return set_error(CFP_ERR_ARG_NULL, "NULL plan");
  if (schedule != CFP_RSCHEDULE_AUTO && schedule != CFP_RSCHEDULE_FIVE && schedule != CFP_RSCHEDULE_THREE &&
      schedule != CFP_RSCHEDULE_THREE_ALT)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "unknown real-plan schedule %d", schedule);
  if ((schedule == CFP_RSCHEDULE_THREE || schedule == CFP_RSCHEDULE_THREE_ALT) && !three_ok(p))
    return set_error(CFP_ERR_SUP, "the 3-sweep real schedule needs a 128^3 or 256^3 grid");
  p->schedule = schedule;
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_schedule(cfp_rplan_t p, int* three) {
  if (!p || !three) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *three = use_three(p) ? 1 : 0;
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_apply(cfp_rplan_t p, const double* b, double* x, void* stream) {
  if (!p || !b || !x) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  RGuard g(p->device);
  return run_real(p, b, x, (hipStream_t)stream, nullptr);
}

extern "C" int cfp_rplan_num_passes(cfp_rplan_t p, int* passes) {
  if (!p || !passes) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *passes = 4;  // r2c rows | half-spectrum y/z plan | Nyquist y/z plan | c2r rows
  return CFP_SUCCESS;
}

extern "C" int cfp_rplan_time_passes(cfp_rplan_t p, const double* b, double* x, int iters, double* ms_out,
                                     void* stream) {
  if (!p || !b || !x || !ms_out) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (iters < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "iters must be >= 1");
  RGuard g(p->device);
  hipStream_t s = (hipStream_t)stream;
  std::vector<hipEvent_t> ev(5);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  double acc[4] = {0, 0, 0, 0};
  int rc = CFP_SUCCESS;
  for (int it = 0; it < iters && rc == CFP_SUCCESS; ++it) {
    rc = run_real(p, b, x, s, &ev);
    if (rc) break;
    if (hipEventSynchronize(ev[4]) != hipSuccess) {
      rc = set_error(CFP_ERR_LIB, "event sync");
      break;
    }
    for (int i = 0; i < 4; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
      acc[i] += ms;
    }
  }
  for (auto& e : ev) hipEventDestroy(e);
  if (rc) return rc;
  for (int i = 0; i < 4; ++i) ms_out[i] = acc[i] / iters;
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ real <-> complex layouts
// Conversions of the real-scalar PETSc boundary (pcshell_fft3d_real.cpp): a real Vec <-> the
// complex plan's data, and FFTW's r2c half spectrum ([nz][ny][nx/2 + 1] complex, what a
// real-scalar MATFFTW MatMult produces) <-> the full spectrum by Hermitian symmetry
// X(-k) = conj X(k) of the transform of real data.  Elementwise, one thread per output value.
namespace {
#define RB_LOOP(i, n) for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)
__global__ void k_rb_promote(const double* __restrict__ x, cd* __restrict__ z, int64_t n) {
  RB_LOOP(i, n) z[i] = make_cd(x[i], 0.0);
}
__global__ void k_rb_real(const cd* __restrict__ z, double* __restrict__ x, int64_t n, double scale) {
  RB_LOOP(i, n) x[i] = z[i].x * scale;
}
__global__ void k_rb_half(const cd* __restrict__ full, cd* __restrict__ half, int64_t nx, int64_t M, int64_t rows) {
  RB_LOOP(i, rows * M) {
    const int64_t row = i / M, kx = i - row * M;
    half[i] = full[row * nx + kx];
  }
}
__global__ void k_rb_extend(const cd* __restrict__ half, cd* __restrict__ full, int64_t nx, int64_t ny, int64_t nz) {
  const int64_t M = nx / 2 + 1;
  RB_LOOP(i, nx * ny * nz) {
    const int64_t kx = i % nx, r = i / nx, ky = r % ny, kz = r / ny;
    if (kx < M) {
      full[i] = half[r * M + kx];
    } else {  // X(kx, ky, kz) = conj X(nx - kx, -ky, -kz)
      const int64_t my = ky ? ny - ky : 0, mz = kz ? nz - kz : 0;
      const cd v = half[(mz * ny + my) * M + (nx - kx)];
      full[i] = make_cd(v.x, -v.y);
    }
  }
}
// Z = the weighted, zero-padded half spectrum over `rows` rows of nx: Z(kx) = w(kx) S(kx) for
// kx <= nx/2 (w = 1 on the self-mirrored columns kx = 0 and, nx even, nx/2; else 2) and 0 above,
// with S = half (its [rows][nx/2 + 1] layout) or, half == NULL, full itself (in place); divided
// by diag (the half-spectrum layout; 0 where diag = 0, PETSc's VecPointwiseDivide) when given.
// For any half spectrum H, Re IDFT(Z) = Re IDFT(Hermitian extension of H) = FFTW's c2r of H, and
// the padding needs no value from another z-plane (the extension's X(-kz) mirror does).
__global__ void k_rb_pad(const cd* __restrict__ half, const cd* __restrict__ diag, cd* full, int64_t nx, int64_t rows) {
  const int64_t M = nx / 2 + 1;
  RB_LOOP(i, nx * rows) {
    const int64_t kx = i % nx, r = i / nx;
    cd v = make_cd(0.0, 0.0);
    if (kx < M) {
      v = half ? half[r * M + kx] : full[i];
      if (diag) {
        const cd d = diag[r * M + kx];
        const double den = d.x * d.x + d.y * d.y;
        v = den != 0.0 ? make_cd((v.x * d.x + v.y * d.y) / den, (v.y * d.x - v.x * d.y) / den) : make_cd(0.0, 0.0);
      }
      const double w = (kx == 0 || 2 * kx == nx) ? 1.0 : 2.0;
      v = make_cd(w * v.x, w * v.y);
    }
    full[i] = v;
  }
}
unsigned rb_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}
}  // namespace

extern "C" int cfp_real_to_complex(const double* x, double* z, int64_t n, void* stream) {
  if (!x || !z) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (n > 0) hipLaunchKernelGGL(k_rb_promote, dim3(rb_grid(n)), dim3(256), 0, (hipStream_t)stream, x, (cd*)z, n);
  HIPCHK(hipGetLastError());
  return CFP_SUCCESS;
}
extern "C" int cfp_complex_real_part(const double* z, double* x, int64_t n, double scale, void* stream) {
  if (!x || !z) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (n > 0) hipLaunchKernelGGL(k_rb_real, dim3(rb_grid(n)), dim3(256), 0, (hipStream_t)stream, (const cd*)z, x, n, scale);
  HIPCHK(hipGetLastError());
  return CFP_SUCCESS;
}
extern "C" int cfp_half_spectrum_extract(const double* full, double* half, int64_t nx, int64_t ny, int64_t nz,
                                         void* stream) {
  if (!full || !half) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const int64_t M = nx / 2 + 1, rows = ny * nz;
  hipLaunchKernelGGL(k_rb_half, dim3(rb_grid(rows * M)), dim3(256), 0, (hipStream_t)stream, (const cd*)full, (cd*)half,
                     nx, M, rows);
  HIPCHK(hipGetLastError());
  return CFP_SUCCESS;
}
extern "C" int cfp_half_spectrum_pad(const double* half, const double* diag, double* full, int64_t nx, int64_t rows,
                                     void* stream) {
  if (!full) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (nx < 1 || rows < 0) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  if (rows > 0)
    hipLaunchKernelGGL(k_rb_pad, dim3(rb_grid(nx * rows)), dim3(256), 0, (hipStream_t)stream, (const cd*)half,
                       (const cd*)diag, (cd*)full, nx, rows);
  HIPCHK(hipGetLastError());
  return CFP_SUCCESS;
}
extern "C" int cfp_half_spectrum_extend(const double* half, double* full, int64_t nx, int64_t ny, int64_t nz,
                                        void* stream) {
  if (!full || !half) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  hipLaunchKernelGGL(k_rb_extend, dim3(rb_grid(nx * ny * nz)), dim3(256), 0, (hipStream_t)stream, (const cd*)half,
                     (cd*)full, nx, ny, nz);
  HIPCHK(hipGetLastError());
  return CFP_SUCCESS;
}
