// cfp_blas.hip -- device vector kernels behind the PETSc-compatible Vec/Mat layer: axpy-family
// updates, PETSc-convention dot / norms, CSR SpMV.  These carry the GMRES harness (SURVEY.md §8f
// row f1), not the FFT hot path.  Every kernel is templated on the scalar: complex double (cd,
// the default stand-in PETSc) and double (the real-scalar build, PetscScalar = double).
#include "cfp_blas.h"

#include <hip/hip_ext.h>

#include <cstdint>

namespace cfp {

// ------------------------------------------------------------------ kernel profile
// (PetscMiniProfileBegin / End): each stamped launch takes two events from the pool and passes
// them to hipExtLaunchKernelGGL, which records the kernel's own start and end (no event packets
// between kernels); copies are bracketed by events.
namespace {
struct KProf {
  bool on = false;
  size_t used = 0;
  std::vector<hipEvent_t> ev;  // 2 per record
  std::vector<int> kind;
};
KProf g_kprof;
}  // namespace

hipError_t kprof_begin(size_t cap) {
  kprof_reset();
  for (size_t i = 0; i < 2 * cap; ++i) {
    hipEvent_t e;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (r != hipSuccess) {
      kprof_reset();
      return r;
    }
    g_kprof.ev.push_back(e);
  }
  g_kprof.kind.assign(cap, 0);
  g_kprof.on = true;
  return hipSuccess;
}
void kprof_reset() {
  for (auto& e : g_kprof.ev) hipEventDestroy(e);
  g_kprof = KProf{};
}
bool kprof_take(int kind, hipEvent_t* e0, hipEvent_t* e1) {
  if (!g_kprof.on || 2 * (g_kprof.used + 1) > g_kprof.ev.size()) return false;
  g_kprof.kind[g_kprof.used] = kind;
  *e0 = g_kprof.ev[2 * g_kprof.used];
  *e1 = g_kprof.ev[2 * g_kprof.used + 1];
  ++g_kprof.used;
  return true;
}
hipError_t kprof_end(double ms[4], long long launches[4]) {
  for (int k = 0; k < 4; ++k) {
    ms[k] = 0.0;
    launches[k] = 0;
  }
  hipError_t r = hipSuccess;
  if (g_kprof.used) r = hipEventSynchronize(g_kprof.ev[2 * g_kprof.used - 1]);
  for (size_t i = 0; r == hipSuccess && i < g_kprof.used; ++i) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_kprof.ev[2 * i], g_kprof.ev[2 * i + 1]) != hipSuccess) continue;
    const int k = g_kprof.kind[i] & 3;
    ms[k] += t;
    launches[k] += 1;
  }
  kprof_reset();
  return r;
}

// a kernel launch that stamps its dispatch while the profile is on
template <typename K, typename... A>
static void blaunch(int kind, K k, dim3 g, dim3 b, unsigned lds, hipStream_t s, A... args) {
  hipEvent_t e0, e1;
  if (kprof_take(kind, &e0, &e1)) hipExtLaunchKernelGGL(k, g, b, lds, s, e0, e1, 0, args...);
  else hipLaunchKernelGGL(k, g, b, lds, s, args...);
}
// an async copy bracketed by events while the profile is on
hipError_t kprof_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  hipEvent_t e0, e1;
  const bool st = kprof_take(3, &e0, &e1);
  if (st) hipEventRecord(e0, s);
  hipError_t r = hipMemcpyAsync(dst, src, bytes, kind, s);
  if (st) hipEventRecord(e1, s);
  return r;
}

// The host's wait for a reduction result (the Krylov loop waits once per iteration): an event
// recorded on the stream and polled, instead of hipStreamSynchronize.  The result itself is
// already in pinned host memory when the event completes; polling returns a few microseconds
// sooner than the blocking wait, and the next launches follow at once.
hipError_t host_wait(hipStream_t s) {
  static thread_local hipEvent_t ev = nullptr;
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    ev = nullptr;
    return hipStreamSynchronize(s);
  }
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) return e;
  for (;;) {
    e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    __builtin_ia32_pause();
  }
}

// Device-to-device copy (VecCopy, cfp_device_copy): 16-byte lanes, four 256-thread workgroups per
// CU striding the vector, non-temporal stores (the copy's destination is not read back soon; the
// source keeps its Infinity Cache lines).  tools/kexp/copy_probe.hip measured this shape at
// 7.14 TB/s on a 268 MB vector (6.16 on 537 MB) against 5.05 for plain stores at 8 per CU
// (profiles/r03u_copy_probe.txt); hipMemcpyAsync D2D runs at about 5.5.
typedef double cpv2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_copy16(const cpv2* __restrict__ in, cpv2* __restrict__ out, i64 n) {
  const i64 stride = (i64)gridDim.x * blockDim.x;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(in[i], out + i);
}

static int blas_cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

hipError_t blas_copy_bytes(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0 || dst == src) return hipSuccess;
  if (bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16)
    return kprof_copy(dst, src, bytes, hipMemcpyDeviceToDevice, s);
  const i64 n = (i64)(bytes / 16);
  i64 g = (n + 255) / 256;
  const i64 cap = 4 * (i64)blas_cu_count();
  if (g > cap) g = cap;
  blaunch(3, k_copy16, dim3((unsigned)g), dim3(256), 0, s, (const cpv2*)src, (cpv2*)dst, n);
  return hipGetLastError();
}

#define BLAS_THREADS 256
// Workgroups of the synchronous reductions (dot / norm), the multi-dot and the MAXPY sweep
// (whose norm rides in it).  r05 A/B inside config 3's GMRES (profiles/r05d_gmres_reduce_ab.txt):
// the dot / norm at 2048 and the multi-dot at 1024 workgroups stream at 5.8 / 5.7 TB/s (from
// 5.1 / 4.4 at 1024 / 512); the MAXPY loses at 2048 (171 against 155 us), so it keeps 1024.
#ifndef RED_BLOCKS
#define RED_BLOCKS 2048
#endif
#ifndef MDOT_BLOCKS
#define MDOT_BLOCKS 1024
#endif
#ifndef MAXPY_BLOCKS
#define MAXPY_BLOCKS 1024
#endif

// Store policy of the Krylov-vector kernels (measured inside config 3's GMRES loop, DESIGN.md
// f1): bit 0 = the SpMV's y, bit 1 = the MAXPY / AXPY results, stored non-temporally.
#ifndef CFP_BLAS_NT
#define CFP_BLAS_NT 0
#endif
typedef double bdv2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void bstore(cd* p, cd v) {
  if constexpr (NT) {
    bdv2 w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<bdv2*>(p));
  } else {
    *p = v;
  }
}
template <bool NT>
__device__ __forceinline__ void bstore(double* p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ cd badd(cd a, cd b) { return make_cd(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd bmul(cd a, cd b) { return make_cd(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ double badd(double a, double b) { return a + b; }
__device__ __forceinline__ double bmul(double a, double b) { return a * b; }
template <class T> __device__ __forceinline__ T bzero();
template <> __device__ __forceinline__ cd bzero<cd>() { return make_cd(0.0, 0.0); }
template <> __device__ __forceinline__ double bzero<double>() { return 0.0; }
// |v|^2, and the dot contribution u conj(v) as (re, im)
__device__ __forceinline__ double babs2(cd v) { return v.x * v.x + v.y * v.y; }
__device__ __forceinline__ double babs2(double v) { return v * v; }
__device__ __forceinline__ double babs1(cd v) { return fabs(v.x) + fabs(v.y); }
__device__ __forceinline__ double babs1(double v) { return fabs(v); }
__device__ __forceinline__ double bmod(cd v) { return hypot(v.x, v.y); }
__device__ __forceinline__ double bmod(double v) { return fabs(v); }
__device__ __forceinline__ void bdot(cd u, cd v, double& a, double& b) {
  a += u.x * v.x + u.y * v.y;
  b += u.y * v.x - u.x * v.y;
}
__device__ __forceinline__ void bdot(double u, double v, double& a, double&) { a += u * v; }

static unsigned nblocks(i64 n) {
  i64 b = (n + BLAS_THREADS - 1) / BLAS_THREADS;
  if (b > 16384) b = 16384;
  return (unsigned)(b < 1 ? 1 : b);
}

#define GRID_LOOP(i, n) for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (i64)gridDim.x * blockDim.x)

template <class T> __global__ void k_set(T* x, T a, i64 n) { GRID_LOOP(i, n) x[i] = a; }
template <class T> __global__ void k_shift(T* x, T a, i64 n) { GRID_LOOP(i, n) x[i] = badd(x[i], a); }
template <class T> __global__ void k_copy(T* y, const T* x, i64 n) { GRID_LOOP(i, n) y[i] = x[i]; }
template <class T> __global__ void k_scal(T* x, T a, i64 n) { GRID_LOOP(i, n) x[i] = bmul(a, x[i]); }
// y = y + a x
template <class T> __global__ void k_axpy(T* y, T a, const T* x, i64 n) {
  GRID_LOOP(i, n) bstore<(CFP_BLAS_NT & 2) != 0>(y + i, badd(y[i], bmul(a, x[i])));
}
// y = x + b y
template <class T> __global__ void k_aypx(T* y, T b, const T* x, i64 n) { GRID_LOOP(i, n) y[i] = badd(x[i], bmul(b, y[i])); }
// w = a x + y
template <class T> __global__ void k_waxpy(T* w, T a, const T* x, const T* y, i64 n) {
  GRID_LOOP(i, n) w[i] = badd(bmul(a, x[i]), y[i]);
}
template <class T> __global__ void k_pmult(T* w, const T* x, const T* y, i64 n) { GRID_LOOP(i, n) w[i] = bmul(x[i], y[i]); }
// real w = x / y with PETSc's rule: a zero divisor gives 0 (VecPointwiseDivide, bvec2.c); the
// complex divide is launch_pointwise_divide (cfp_kernels.hip)
__global__ void k_pdiv_real(double* w, const double* x, const double* y, i64 n) {
  GRID_LOOP(i, n) w[i] = y[i] != 0.0 ? x[i] / y[i] : 0.0;
}

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// y = (OW ? 0 : y) + sum_j a_j x_j (the GMRES basis update, up to MV_MAX vectors per launch),
// with NRM: per-block sums of |y|^2 of the result (one sweep)
template <class T, bool OW, bool NRM>
__global__ void __launch_bounds__(BLAS_THREADS) k_maxpy(T* y, int k, MVCoefT<T> a, MVPtrsT<T> xs, i64 n,
                                                         double* partial) {
  double s2 = 0.0;
  GRID_LOOP(i, n) {
    T acc = OW ? bzero<T>() : y[i];
    for (int j = 0; j < k; ++j) acc = badd(acc, bmul(a.a[j], xs.p[j][i]));
    bstore<(CFP_BLAS_NT & 2) != 0>(y + i, acc);
    if (NRM) s2 += babs2(acc);
  }
  if constexpr (NRM) {
    __shared__ double sm[BLAS_THREADS / 64];
    s2 = wave_sum(s2);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s2;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int q = 0; q < BLAS_THREADS / 64; ++q) t += sm[q];
      partial[blockIdx.x] = t;
    }
  }
}

// kind: 0 = dot y^H x (re, im), 1 = sum |x|^2, 2 = sum |re|+|im|, 3 = max |x|
template <class T>
__global__ void k_reduce(const T* x, const T* y, i64 n, int kind, double* partial) {
  __shared__ double s0[BLAS_THREADS / 64], s1[BLAS_THREADS / 64];
  double a = 0.0, b = 0.0;
  GRID_LOOP(i, n) {
    const T u = x[i];
    if (kind == 0) bdot(u, y[i], a, b);
    else if (kind == 1) a += babs2(u);
    else if (kind == 2) a += babs1(u);
    else a = fmax(a, bmod(u));
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (kind == 3) a = wave_max(a);
  else { a = wave_sum(a); b = wave_sum(b); }
  if (lane == 0) { s0[w] = a; s1[w] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = s0[0], tb = s1[0];
    for (int k = 1; k < BLAS_THREADS / 64; ++k) {
      if (kind == 3) ta = fmax(ta, s0[k]);
      else { ta += s0[k]; tb += s1[k]; }
    }
    partial[2 * blockIdx.x] = ta;
    partial[2 * blockIdx.x + 1] = tb;
  }
}

// several dots against one vector, PETSc VecMDot(x, k, y[], val): val_j = y_j^H x.
// One sweep of x per launch; up to MDOT_K accumulators per thread.
#define MDOT_K 8
template <class T>
__global__ void k_mdot(const T* x, int k, MVPtrsT<T> ys, i64 n, double* partial) {
  __shared__ double sm[2 * MDOT_K][BLAS_THREADS / 64];
  double a[MDOT_K], b[MDOT_K];
#pragma unroll
  for (int j = 0; j < MDOT_K; ++j) { a[j] = 0.0; b[j] = 0.0; }
  GRID_LOOP(i, n) {
    const T u = x[i];
#pragma unroll
    for (int j = 0; j < MDOT_K; ++j)
      if (j < k) bdot(u, ys.p[j][i], a[j], b[j]);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < MDOT_K; ++j) {
    const double ra = wave_sum(a[j]), rb = wave_sum(b[j]);
    if (lane == 0) { sm[2 * j][w] = ra; sm[2 * j + 1][w] = rb; }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * k; t += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q < BLAS_THREADS / 64; ++q) s += sm[t][q];
    partial[(size_t)blockIdx.x * 2 * MDOT_K + t] = s;
  }
}

// The dots of several k_mdot launches (chunks of MDOT_K vectors, partials of chunk c at
// partial + c 2 MDOT_K MDOT_BLOCKS) summed on the device: one wave per output value (re or im
// of dot j), lanes over the nb workgroups' partials, then a wave sum -- deterministic.
__global__ void __launch_bounds__(1024) k_mdot_finish(const double* partial, int nb, int k, double* dots) {
  const int o = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= 2 * k) return;  // whole waves
  const int j = o >> 1, c = j / MDOT_K;
  const double* p = partial + (size_t)c * 2 * MDOT_K * MDOT_BLOCKS + 2 * (j % MDOT_K) + (o & 1);
  double s = 0.0;
  for (int q = lane; q < nb; q += 64) s += p[(size_t)q * 2 * MDOT_K];
  s = wave_sum(s);
  if (lane == 0) dots[o] = s;
}

// y += sum_j scale_j dots_j xs_j with the dots on the device (k_mdot_finish), |y|^2 partials:
// the MAXPY of classical Gram-Schmidt without the host round trip between the dots and the update
__device__ __forceinline__ cd dcoef(const double* dots, double sc, int j, cd) {
  return make_cd(sc * dots[2 * j], sc * dots[2 * j + 1]);
}
__device__ __forceinline__ double dcoef(const double* dots, double sc, int j, double) { return sc * dots[2 * j]; }
template <class T>
__global__ void __launch_bounds__(BLAS_THREADS) k_maxpy_dc(T* y, int k, MVCoefT<double> scale, const double* dots,
                                                            MVPtrsT<T> xs, i64 n, double* partial, double* dots_out) {
  if (blockIdx.x == 0 && threadIdx.x < 2 * k) dots_out[threadIdx.x] = dots[threadIdx.x];  // for the host
  double s2 = 0.0;
  GRID_LOOP(i, n) {
    T acc = y[i];
    for (int j = 0; j < k; ++j) acc = badd(acc, bmul(dcoef(dots, scale.a[j], j, acc), xs.p[j][i]));
    bstore<(CFP_BLAS_NT & 2) != 0>(y + i, acc);
    s2 += babs2(acc);
  }
  __shared__ double sm[BLAS_THREADS / 64];
  s2 = wave_sum(s2);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int q = 0; q < BLAS_THREADS / 64; ++q) t += sm[q];
    partial[blockIdx.x] = t;
  }
}

// CSR y = A x, one thread per row (rows of about one nonzero)
template <class T>
__global__ void k_csr_spmv(i64 m, const i64* rowptr, const i64* col, const T* val, const T* x, T* y) {
  GRID_LOOP(r, m) {
    T acc = bzero<T>();
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p) acc = badd(acc, bmul(val[p], x[col[p]]));
    y[r] = acc;
  }
}

// CSR y = A x, L lanes per row: the lanes of a row read its nonzeros side by side, so a wave's
// loads of val / col are contiguous runs over 64 / L consecutive rows (one thread per row reads
// them at a stride of the row length: 4.5x below bandwidth on the 7-nonzero wave-system rows).
// The L partial sums meet through lane shuffles; lane 0 of the group stores.
__device__ __forceinline__ void spmv_acc(cd a, cd b, double& ax, double& ay) {
  ax = fma(a.x, b.x, fma(-a.y, b.y, ax));
  ay = fma(a.x, b.y, fma(a.y, b.x, ay));
}
__device__ __forceinline__ void spmv_acc(double a, double b, double& ax, double&) { ax = fma(a, b, ax); }
__device__ __forceinline__ void spmv_store(cd* y, double ax, double ay) { bstore<(CFP_BLAS_NT & 1) != 0>(y, make_cd(ax, ay)); }
__device__ __forceinline__ void spmv_store(double* y, double ax, double) { bstore<(CFP_BLAS_NT & 1) != 0>(y, ax); }

template <class T, int L>
__global__ void __launch_bounds__(BLAS_THREADS) k_csr_spmv_vec(i64 m, const i64* rowptr, const i64* col,
                                                               const T* val, const T* x, T* y) {
  const int lane = threadIdx.x & (L - 1);
  const i64 groups = (i64)gridDim.x * (blockDim.x / L);
  for (i64 r = (i64)blockIdx.x * (blockDim.x / L) + threadIdx.x / L; r < m; r += groups) {
    const i64 p0 = rowptr[r], p1 = rowptr[r + 1];
    double ax = 0.0, ay = 0.0;
    for (i64 p = p0 + lane; p < p1; p += L) spmv_acc(val[p], x[col[p]], ax, ay);
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) {
      ax += __shfl_xor(ax, o, L);
      if constexpr (std::is_same<T, cd>::value) ay += __shfl_xor(ay, o, L);
    }
    if (lane == 0) spmv_store(y + r, ax, ay);
  }
}

// halo of a distributed AIJ (petsc_mini.cpp MATMPIAIJ): out[i] = x[idx[i]] (idx < 0: zero
// padding), and y += B g for the off-diagonal block B (CSR over the ghost slots)
template <class T> __global__ void k_gather(T* out, const T* x, const i64* idx, i64 n) {
  GRID_LOOP(i, n) {
    const i64 j = idx[i];
    out[i] = j >= 0 ? x[j] : bzero<T>();
  }
}
template <class T>
__global__ void k_csr_spmv_add(i64 m, const i64* rowptr, const i64* col, const T* val, const T* x, T* y) {
  GRID_LOOP(r, m) {
    const i64 p0 = rowptr[r], p1 = rowptr[r + 1];
    if (p0 == p1) continue;
    T acc = y[r];
    for (i64 p = p0; p < p1; ++p) acc = badd(acc, bmul(val[p], x[col[p]]));
    y[r] = acc;
  }
}

// Row-class diagonal SpMV (r05).  A constant-coefficient stencil on a
// Cartesian grid -- the transport operator of configs 1 and 3 (transport_cartesian.cpp) -- has
// its nonzeros on a few fixed diagonals and only a handful of distinct rows (interior, and the
// borders where faces drop out).  Stored as one class byte per row and a table of the classes'
// diagonal values (staged in LDS), y = A x reads the class bytes and x (the neighbours x[r +
// off] come from the caches) and writes y: 33 N bytes for complex vectors, against CSR's
// 24 B per nonzero + 8 B rowptr + the vectors (the 256^3 CSR SpMV took 271 us per call inside
// GMRES, profiles/r04_gmres256_kernels.txt).  Absent entries are skipped (mask bit clear), so a
// row never loads outside x.
template <class T>
__global__ void __launch_bounds__(BLAS_THREADS) k_dia_spmv(i64 m, DiaDesc d, const unsigned char* cls,
                                                           const unsigned char* masks, const T* tab, const T* x, T* y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dia_lds[];
  T* st = reinterpret_cast<T*>(dia_lds);
  unsigned char* sm = dia_lds + sizeof(T) * (size_t)(d.ncls * d.nd);
  for (int i = threadIdx.x; i < d.ncls * d.nd; i += blockDim.x) st[i] = tab[i];
  for (int i = threadIdx.x; i < d.ncls; i += blockDim.x) sm[i] = masks[i];
  __syncthreads();
  GRID_LOOP(r, m) {
    const int c = cls[r];
    const unsigned mk = sm[c];
    const T* row = st + c * d.nd;
    double ax = 0.0, ay = 0.0;
#pragma unroll
    for (int k = 0; k < DIA_MAX; ++k)
      if (k < d.nd && ((mk >> k) & 1u)) spmv_acc(row[k], x[r + d.off[k]], ax, ay);
    spmv_store(y + r, ax, ay);
  }
}

// Block row-class form (cfp_blas.h): one thread per block row.  The class table sits in LDS; the
// threads of a wave mostly share a class (interior cells), so its reads are broadcasts and the
// per-entry tests below are uniform branches.  Per present block diagonal the thread loads the
// neighbour's values in the columns the block uses and multiplies by the block's nonzeros only
// (the wave operator: 4 of 16 entries in a neighbour block, 2 of 4 columns).  The interleaved wave
// operator on a Cartesian grid: x read once through the caches, y written once, one class byte per
// cell -- against CSR's 24 bytes per nonzero (about 28 nonzeros per 3-D cell).
template <class T, int B>
__global__ void __launch_bounds__(512) k_bdia_spmv(i64 mb, BDiaDesc d, const unsigned char* cls,
                                                            const unsigned short* masks, const unsigned short* cbase,
                                                            const unsigned* bnz, const T* tab, const T* x, T* y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char bdia_lds[];
  T* st = reinterpret_cast<T*>(bdia_lds);
  const int nt = d.nblk * B * B;
  unsigned* sz = reinterpret_cast<unsigned*>(bdia_lds + sizeof(T) * (size_t)nt);
  unsigned short* sm = reinterpret_cast<unsigned short*>(sz + d.nblk);
  unsigned short* sb = sm + d.ncls;
  __shared__ i64 so[BDIA_MAX];
  if (threadIdx.x < BDIA_MAX) so[threadIdx.x] = threadIdx.x < d.nd ? d.off[threadIdx.x] : 0;
  for (int i = threadIdx.x; i < nt; i += blockDim.x) st[i] = tab[i];
  for (int i = threadIdx.x; i < d.nblk; i += blockDim.x) sz[i] = bnz[i];
  for (int i = threadIdx.x; i < d.ncls; i += blockDim.x) {
    sm[i] = masks[i];
    sb[i] = cbase[i];
  }
  __syncthreads();
  const i64 stride = (i64)gridDim.x * blockDim.x;
  i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  int cn = r < mb ? cls[r] : 0;  // the class byte of the next cell is loaded one iteration ahead
  for (; r < mb; r += stride) {
    const int c = cn;
    if (r + stride < mb) cn = cls[r + stride];
    // the present blocks in ascending k, software-pipelined: the next block's neighbour values
    // are loaded before the current block's products, so one load latency per cell instead of
    // one per block (the offsets come from LDS: a per-lane index into the kernel arguments
    // would go through scratch)
    unsigned rem = sm[c];
    int q = sb[c];
    double ax[B], ay[B];
#pragma unroll
    for (int i = 0; i < B; ++i) ax[i] = ay[i] = 0.0;
    T xc[B], xn[B];
    unsigned nzc = 0;
    if (rem) {
      const int k = __builtin_ctz(rem);
      rem &= rem - 1;
      nzc = sz[q];
      const T* xb = x + (r + so[k]) * B;
#pragma unroll
      for (int j = 0; j < B; ++j) xc[j] = ((nzc >> (16 + j)) & 1u) ? xb[j] : T{};
      for (;;) {
        const bool more = rem != 0;
        unsigned nzn = 0;
        if (more) {
          const int k2 = __builtin_ctz(rem);
          rem &= rem - 1;
          nzn = sz[q + 1];
          const T* xb2 = x + (r + so[k2]) * B;
#pragma unroll
          for (int j = 0; j < B; ++j) xn[j] = ((nzn >> (16 + j)) & 1u) ? xb2[j] : T{};
        }
        const T* blk = st + q * B * B;
#pragma unroll
        for (int i = 0; i < B; ++i)
#pragma unroll
          for (int j = 0; j < B; ++j)
            if ((nzc >> (i * B + j)) & 1u) spmv_acc(blk[i * B + j], xc[j], ax[i], ay[i]);
        if (!more) break;
        ++q;
        nzc = nzn;
#pragma unroll
        for (int j = 0; j < B; ++j) xc[j] = xn[j];
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) spmv_store(y + r * B + i, ax[i], ay[i]);
  }
}

// B = 4 (the 3-D wave system's cells): one thread per row, 4 lanes of a quad per cell.  Each lane
// loads only its own column of a neighbour cell -- consecutive lanes read consecutive 16 bytes, so
// a wave instruction reads whole lines -- and takes the other columns from its quad through DPP
// broadcasts (the quad shares a class, so it is active together).  All present blocks' values
// are loaded before the products: one load latency per cell.
template <int J>
__device__ __forceinline__ double quad_bc(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), J * 0x55, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), J * 0x55, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int J>
__device__ __forceinline__ cd quad_bc(cd v) { return make_cd(quad_bc<J>(v.x), quad_bc<J>(v.y)); }

#ifndef CFP_BDIA_XCD
#define CFP_BDIA_XCD 0
#endif
#ifndef CFP_BDIA_RE
#define CFP_BDIA_RE 1
#endif
#ifndef CFP_BDIA_PF
#define CFP_BDIA_PF 0
#endif
// RE (complex fields, d.re): the table's entries are real, so each product is two FMAs on the
// real part instead of a complex multiply-add's four
__device__ __forceinline__ void spmv_acc_re(cd a, cd b, double& ax, double& ay) {
  ax = fma(a.x, b.x, ax);
  ay = fma(a.x, b.y, ay);
}
__device__ __forceinline__ void spmv_acc_re(double a, double b, double& ax, double&) { ax = fma(a, b, ax); }
template <class T, int NDC, bool RE>
__global__ void __launch_bounds__(512) k_bdia4_spmv(i64 m, BDiaDesc d, const unsigned char* cls,
                                                    const unsigned short* masks, const unsigned short* cbase,
                                                    const unsigned* bnz, const T* tab, const T* x, T* y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char bdia_lds[];
  T* st = reinterpret_cast<T*>(bdia_lds);
  const int nt = d.nblk * 16;
  unsigned* sz = reinterpret_cast<unsigned*>(bdia_lds + sizeof(T) * (size_t)nt);
  unsigned short* sm = reinterpret_cast<unsigned short*>(sz + d.nblk);
  unsigned short* sb = sm + d.ncls;
  __shared__ i64 so[BDIA_MAX];
  if (threadIdx.x < BDIA_MAX) so[threadIdx.x] = threadIdx.x < d.nd ? d.off[threadIdx.x] : 0;
  for (int i = threadIdx.x; i < nt; i += blockDim.x) st[i] = tab[i];
  for (int i = threadIdx.x; i < d.nblk; i += blockDim.x) sz[i] = bnz[i];
  for (int i = threadIdx.x; i < d.ncls; i += blockDim.x) {
    sm[i] = masks[i];
    sb[i] = cbase[i];
  }
  __syncthreads();
  // XCD-contiguous cells (-DCFP_BDIA_XCD=1, A/B only): with the grid a multiple of 8, workgroup b
  // runs on XCD b mod 8, and each XCD walks its own eighth of the rows in order, so the y / z
  // neighbours a wave reads were pulled into that XCD's L2 by its own earlier waves.  Measured
  // 2 us slower per MatMult than the plain grid-stride order (profiles/r06z4_wave_spmv_ab.txt).
  i64 r0 = (i64)blockIdx.x * blockDim.x + threadIdx.x, r1 = m, rs = (i64)gridDim.x * blockDim.x;
#if CFP_BDIA_XCD
  if ((gridDim.x & 7) == 0) {
    const i64 xcd = blockIdx.x & 7, mb = m >> 2;
    r0 = ((xcd * mb) >> 3) * 4 + (i64)(blockIdx.x >> 3) * blockDim.x + threadIdx.x;
    r1 = (((xcd + 1) * mb) >> 3) * 4;
    rs = (i64)(gridDim.x >> 3) * blockDim.x;
  }
#endif
  const auto load = [&](i64 rr, int c, T* xk) {
    const i64 R = rr >> 2;
    const int i = (int)(rr & 3);
    const unsigned mk = sm[c];
#pragma unroll
    for (int k = 0; k < NDC; ++k)
      if (k < d.nd && ((mk >> k) & 1u)) xk[k] = x[(R + so[k]) * 4 + i];
  };
  const auto product = [&](i64 rr, int c, const T* xk) {
    const int i = (int)(rr & 3);
    const unsigned mk = sm[c];
    int q = sb[c];
    double ax = 0.0, ay = 0.0;
#pragma unroll
    for (int k = 0; k < NDC; ++k) {
      if (k < d.nd && ((mk >> k) & 1u)) {
        const unsigned nz = sz[q];
        const T* row = st + q * 16 + i * 4;
        if constexpr (RE) {
          if ((nz >> 16) & 1u) spmv_acc_re(row[0], quad_bc<0>(xk[k]), ax, ay);
          if ((nz >> 17) & 1u) spmv_acc_re(row[1], quad_bc<1>(xk[k]), ax, ay);
          if ((nz >> 18) & 1u) spmv_acc_re(row[2], quad_bc<2>(xk[k]), ax, ay);
          if ((nz >> 19) & 1u) spmv_acc_re(row[3], quad_bc<3>(xk[k]), ax, ay);
        } else {
          if ((nz >> 16) & 1u) spmv_acc(row[0], quad_bc<0>(xk[k]), ax, ay);
          if ((nz >> 17) & 1u) spmv_acc(row[1], quad_bc<1>(xk[k]), ax, ay);
          if ((nz >> 18) & 1u) spmv_acc(row[2], quad_bc<2>(xk[k]), ax, ay);
          if ((nz >> 19) & 1u) spmv_acc(row[3], quad_bc<3>(xk[k]), ax, ay);
        }
        ++q;
      }
    }
    spmv_store(y + rr, ax, ay);
  };
#if CFP_BDIA_PF
  // software-pipelined over the grid-stride iterations (-DCFP_BDIA_PF=1, A/B only): the next
  // row's neighbour values are in flight while this row's products run, and the class byte is
  // read two rows ahead.  124 VGPRs against 80, so 2 workgroups per CU instead of 3: 103-107
  // against 91-95 us per MatMult (profiles/r06z6_wave_spmv_pf_ab.txt)
  i64 rr = r0;
  int c = rr < r1 ? cls[rr >> 2] : 0;
  int cn = rr + rs < r1 ? cls[(rr + rs) >> 2] : 0;
  T xk[NDC];
  if (rr < r1) load(rr, c, xk);
  for (; rr < r1; rr += rs) {
    const i64 rn = rr + rs;
    T xn[NDC];
    if (rn < r1) load(rn, cn, xn);
    const int cnn = rn + rs < r1 ? cls[(rn + rs) >> 2] : 0;
    product(rr, c, xk);
#pragma unroll
    for (int k = 0; k < NDC; ++k) xk[k] = xn[k];
    c = cn;
    cn = cnn;
  }
#else
  for (i64 rr = r0; rr < r1; rr += rs) {
    const int c = cls[rr >> 2];
    T xk[NDC];
    load(rr, c, xk);
    product(rr, c, xk);
  }
#endif
}

// ------------------------------------------------------------------ host launchers
#define L1(K, ...) \
  do { if (n > 0) blaunch(2, K, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, __VA_ARGS__); return hipGetLastError(); } while (0)

template <class T> static hipError_t set_t(T* x, T a, i64 n, hipStream_t s) { L1(k_set<T>, x, a, n); }
template <class T> static hipError_t shift_t(T* x, T a, i64 n, hipStream_t s) { L1(k_shift<T>, x, a, n); }
template <class T> static hipError_t copy_t(T* y, const T* x, i64 n, hipStream_t s) { L1(k_copy<T>, y, x, n); }
template <class T> static hipError_t axpy_t(T* y, T a, const T* x, i64 n, hipStream_t s) { L1(k_axpy<T>, y, a, x, n); }
template <class T> static hipError_t aypx_t(T* y, T b, const T* x, i64 n, hipStream_t s) { L1(k_aypx<T>, y, b, x, n); }
template <class T> static hipError_t waxpy_t(T* w, T a, const T* x, const T* y, i64 n, hipStream_t s) {
  L1(k_waxpy<T>, w, a, x, y, n);
}
template <class T> static hipError_t pmult_t(T* w, const T* x, const T* y, i64 n, hipStream_t s) {
  L1(k_pmult<T>, w, x, y, n);
}

hipError_t blas_set(cd* x, cd a, i64 n, hipStream_t s) { return set_t(x, a, n, s); }
hipError_t blas_shift(cd* x, cd a, i64 n, hipStream_t s) { return shift_t(x, a, n, s); }
hipError_t blas_copy(cd* y, const cd* x, i64 n, hipStream_t s) { return copy_t(y, x, n, s); }
hipError_t blas_axpy(cd* y, cd a, const cd* x, i64 n, hipStream_t s) { return axpy_t(y, a, x, n, s); }
hipError_t blas_aypx(cd* y, cd b, const cd* x, i64 n, hipStream_t s) { return aypx_t(y, b, x, n, s); }
hipError_t blas_waxpy(cd* w, cd a, const cd* x, const cd* y, i64 n, hipStream_t s) { return waxpy_t(w, a, x, y, n, s); }
hipError_t blas_pmult(cd* w, const cd* x, const cd* y, i64 n, hipStream_t s) { return pmult_t(w, x, y, n, s); }
hipError_t blas_set(double* x, double a, i64 n, hipStream_t s) { return set_t(x, a, n, s); }
hipError_t blas_shift(double* x, double a, i64 n, hipStream_t s) { return shift_t(x, a, n, s); }
hipError_t blas_copy(double* y, const double* x, i64 n, hipStream_t s) { return copy_t(y, x, n, s); }
hipError_t blas_axpy(double* y, double a, const double* x, i64 n, hipStream_t s) { return axpy_t(y, a, x, n, s); }
hipError_t blas_aypx(double* y, double b, const double* x, i64 n, hipStream_t s) { return aypx_t(y, b, x, n, s); }
hipError_t blas_waxpy(double* w, double a, const double* x, const double* y, i64 n, hipStream_t s) {
  return waxpy_t(w, a, x, y, n, s);
}
hipError_t blas_pmult(double* w, const double* x, const double* y, i64 n, hipStream_t s) { return pmult_t(w, x, y, n, s); }
hipError_t blas_scale(double* x, double a, i64 n, hipStream_t s) { L1(k_scal<double>, x, a, n); }
hipError_t blas_pdivide(double* w, const double* x, const double* y, i64 n, hipStream_t s) { L1(k_pdiv_real, w, x, y, n); }
#undef L1

template <class T>
static hipError_t spmv_t(i64 m, i64 nnz, const i64* rowptr, const i64* col, const T* val, const T* x, T* y,
                         hipStream_t s) {
  if (m <= 0) return hipSuccess;
  // lanes per row: the power of two at or above the mean row length, 1 .. 16
  const double mean = (double)nnz / (double)m;
  const int L = mean <= 1.5 ? 1 : mean <= 2.5 ? 2 : mean <= 4.5 ? 4 : mean <= 8.5 ? 8 : 16;
  const dim3 blk(BLAS_THREADS);
  switch (L) {
    case 1: blaunch(1, k_csr_spmv<T>, dim3(nblocks(m)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 2: blaunch(1, (k_csr_spmv_vec<T, 2>), dim3(nblocks(m * 2)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 4: blaunch(1, (k_csr_spmv_vec<T, 4>), dim3(nblocks(m * 4)), blk, 0, s, m, rowptr, col, val, x, y); break;
    case 8: blaunch(1, (k_csr_spmv_vec<T, 8>), dim3(nblocks(m * 8)), blk, 0, s, m, rowptr, col, val, x, y); break;
    default: blaunch(1, (k_csr_spmv_vec<T, 16>), dim3(nblocks(m * 16)), blk, 0, s, m, rowptr, col, val, x, y);
  }
  return hipGetLastError();
}
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                         hipStream_t s) {
  return spmv_t(m, nnz, rowptr, col, val, x, y, s);
}
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const double* val, const double* x,
                         double* y, hipStream_t s) {
  return spmv_t(m, nnz, rowptr, col, val, x, y, s);
}

template <class T>
static hipError_t gather_t(T* out, const T* x, const i64* idx, i64 n, hipStream_t s) {
  if (n > 0) blaunch(1, k_gather<T>, dim3(nblocks(n)), dim3(BLAS_THREADS), 0, s, out, x, idx, n);
  return hipGetLastError();
}
template <class T>
static hipError_t spmv_add_t(i64 m, const i64* rowptr, const i64* col, const T* val, const T* x, T* y, hipStream_t s) {
  if (m > 0) blaunch(1, k_csr_spmv_add<T>, dim3(nblocks(m)), dim3(BLAS_THREADS), 0, s, m, rowptr, col, val, x, y);
  return hipGetLastError();
}
hipError_t blas_gather(cd* out, const cd* x, const i64* idx, i64 n, hipStream_t s) { return gather_t(out, x, idx, n, s); }
hipError_t blas_gather(double* out, const double* x, const i64* idx, i64 n, hipStream_t s) {
  return gather_t(out, x, idx, n, s);
}
hipError_t blas_csr_spmv_add(i64 m, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                             hipStream_t s) {
  return spmv_add_t(m, rowptr, col, val, x, y, s);
}
hipError_t blas_csr_spmv_add(i64 m, const i64* rowptr, const i64* col, const double* val, const double* x, double* y,
                             hipStream_t s) {
  return spmv_add_t(m, rowptr, col, val, x, y, s);
}

template <class T>
static hipError_t dia_t(i64 m, const DiaDesc& d, const unsigned char* cls, const unsigned char* masks, const T* tab,
                        const T* x, T* y, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  if (d.nd < 1 || d.nd > DIA_MAX || d.ncls < 1 || d.ncls > 256) return hipErrorInvalidValue;
  const size_t lds = sizeof(T) * (size_t)(d.ncls * d.nd) + 256;
  blaunch(1, k_dia_spmv<T>, dim3(nblocks(m)), dim3(BLAS_THREADS), lds, s, m, d, cls, masks, tab, x, y);
  return hipGetLastError();
}
hipError_t blas_dia_spmv(i64 m, const DiaDesc& d, const unsigned char* cls, const unsigned char* masks, const cd* tab,
                         const cd* x, cd* y, hipStream_t s) {
  return dia_t(m, d, cls, masks, tab, x, y, s);
}
hipError_t blas_dia_spmv(i64 m, const DiaDesc& d, const unsigned char* cls, const unsigned char* masks,
                         const double* tab, const double* x, double* y, hipStream_t s) {
  return dia_t(m, d, cls, masks, tab, x, y, s);
}

template <class T>
static hipError_t bdia_t(i64 mb, const BDiaDesc& d, const unsigned char* cls, const unsigned short* masks,
                         const unsigned short* cbase, const unsigned* bnz, const T* tab, const T* x, T* y,
                         hipStream_t s) {
  if (mb <= 0) return hipSuccess;
  if (d.nd < 1 || d.nd > BDIA_MAX || d.ncls < 1 || d.ncls > 256 || d.B < 2 || d.B > 4 || d.nblk < 1)
    return hipErrorInvalidValue;
  const size_t lds = (sizeof(T) * d.B * d.B + sizeof(unsigned)) * (size_t)d.nblk + 2 * sizeof(unsigned short) * 256;
  if (lds > BDIA_LDS_MAX + 2048) return hipErrorInvalidValue;
  // persistent grid: each workgroup stages the class table into LDS once (tens of KB), so a
  // workgroup per 256 cells would re-read it ~8,000 times at 128^3.  512-thread workgroups, as
  // many per CU as the table's LDS allows (at most 3: 24 waves, the kernel's ~70 VGPRs allow 28)
  i64 nb = (mb + 511) / 512;
  const i64 per_cu = lds <= 48 * 1024 ? 3 : (lds <= 75 * 1024 ? 2 : 1);
  const i64 cap = per_cu * (i64)blas_cu_count();
  if (nb > cap) nb = cap;
  const dim3 g((unsigned)(nb < 1 ? 1 : nb)), b(512);
  if (d.B == 4) {  // one thread per row (k_bdia4_spmv): 4 times the threads
    i64 nb4 = (4 * mb + 511) / 512;
    // the pipelined kernel holds two rows' values (~124 VGPRs): 4 waves per SIMD, 2 workgroups per CU
    const i64 cap4 = CFP_BDIA_PF ? (per_cu < 2 ? per_cu : 2) * (i64)blas_cu_count() : cap;
    if (nb4 > cap4) nb4 = cap4;
    const dim3 g4((unsigned)(nb4 < 1 ? 1 : nb4));
    constexpr bool CX = std::is_same<T, cd>::value;
    if (d.nd <= 8 && CX && d.re && CFP_BDIA_RE)
      blaunch(1, (k_bdia4_spmv<T, 8, CX>), g4, b, (unsigned)lds, s, 4 * mb, d, cls, masks, cbase, bnz, tab, x, y);
    else if (d.nd <= 8)
      blaunch(1, (k_bdia4_spmv<T, 8, false>), g4, b, (unsigned)lds, s, 4 * mb, d, cls, masks, cbase, bnz, tab, x, y);
    else
      blaunch(1, (k_bdia4_spmv<T, 16, false>), g4, b, (unsigned)lds, s, 4 * mb, d, cls, masks, cbase, bnz, tab, x, y);
    return hipGetLastError();
  }
  switch (d.B) {
    case 2: blaunch(1, (k_bdia_spmv<T, 2>), g, b, (unsigned)lds, s, mb, d, cls, masks, cbase, bnz, tab, x, y); break;
    case 3: blaunch(1, (k_bdia_spmv<T, 3>), g, b, (unsigned)lds, s, mb, d, cls, masks, cbase, bnz, tab, x, y); break;
    default: blaunch(1, (k_bdia_spmv<T, 4>), g, b, (unsigned)lds, s, mb, d, cls, masks, cbase, bnz, tab, x, y);
  }
  return hipGetLastError();
}
hipError_t blas_bdia_spmv(i64 mb, const BDiaDesc& d, const unsigned char* cls, const unsigned short* masks,
                          const unsigned short* cbase, const unsigned* bnz, const cd* tab, const cd* x, cd* y,
                          hipStream_t s) {
  return bdia_t(mb, d, cls, masks, cbase, bnz, tab, x, y, s);
}
hipError_t blas_bdia_spmv(i64 mb, const BDiaDesc& d, const unsigned char* cls, const unsigned short* masks,
                          const unsigned short* cbase, const unsigned* bnz, const double* tab, const double* x,
                          double* y, hipStream_t s) {
  return bdia_t(mb, d, cls, masks, cbase, bnz, tab, x, y, s);
}

// per-thread device + pinned staging of block partial sums (synchronous reductions).  hd is the
// device address of the pinned host buffer h (coherent, mapped): a kernel whose results only the
// host reads writes them there directly, with vector stores, and the host reads them after the
// stream sync -- no device-to-host copy (each one a copy kernel of ~4-5 us on the device, several
// per GMRES iteration).
struct Partials {
  double* d = nullptr;
  double* h = nullptr;
  double* hd = nullptr;
  hipError_t get(size_t count) {
    if (d) return hipSuccess;
    hipError_t e = hipMalloc(&d, sizeof(double) * count);
    if (e != hipSuccess) return e;
    e = hipHostMalloc(&h, sizeof(double) * count, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    return hipHostGetDevicePointer((void**)&hd, h, 0);
  }
};

template <class T>
static hipError_t maxpy_t(T* y, int k, const T* a, const T* const* xs, i64 n, bool overwrite, double* norm2,
                          hipStream_t s) {
  static thread_local Partials part;
  if (norm2) {
    hipError_t e = part.get(MAXPY_BLOCKS);
    if (e != hipSuccess) return e;
  }
  unsigned nb = nblocks(n);
  if (nb > MAXPY_BLOCKS) nb = MAXPY_BLOCKS;
  if (n > 0) {
    for (int j0 = 0; j0 < (k > 0 ? k : 1); j0 += MV_MAX) {
      const int kk = k - j0 < MV_MAX ? (k - j0 > 0 ? k - j0 : 0) : MV_MAX;
      MVCoefT<T> c;
      MVPtrsT<T> p;
      for (int j = 0; j < kk; ++j) { c.a[j] = a[j0 + j]; p.p[j] = xs[j0 + j]; }
      const bool ow = overwrite && j0 == 0, nrm = norm2 && j0 + MV_MAX >= k;
      const dim3 g(nb), blk(BLAS_THREADS);
      if (ow && nrm) blaunch(2, (k_maxpy<T, true, true>), g, blk, 0, s, y, kk, c, p, n, part.hd);
      else if (ow) blaunch(2, (k_maxpy<T, true, false>), g, blk, 0, s, y, kk, c, p, n, part.hd);
      else if (nrm) blaunch(2, (k_maxpy<T, false, true>), g, blk, 0, s, y, kk, c, p, n, part.hd);
      else blaunch(2, (k_maxpy<T, false, false>), g, blk, 0, s, y, kk, c, p, n, part.hd);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !norm2) return e;
  if (n <= 0) {
    *norm2 = 0.0;
    return hipSuccess;
  }
  e = host_wait(s);  // the partials are in pinned host memory
  if (e != hipSuccess) return e;
  double t = 0.0;
  for (unsigned q = 0; q < nb; ++q) t += part.h[q];
  *norm2 = t;
  return hipSuccess;
}
template <class T>
static hipError_t axpy_partials_t(T* y, T a, const T* x, i64 n, double* partial, unsigned* nb_out, hipStream_t s) {
  static_assert(BLAS_NORM_PARTIALS <= MAXPY_BLOCKS, "partials");
  unsigned nb = nblocks(n);
  if (nb > BLAS_NORM_PARTIALS) nb = BLAS_NORM_PARTIALS;
  *nb_out = n > 0 ? nb : 0;
  if (n <= 0) return hipSuccess;
  MVCoefT<T> c;
  MVPtrsT<T> p;
  c.a[0] = a;
  p.p[0] = x;
  blaunch(2, (k_maxpy<T, false, true>), dim3(nb), dim3(BLAS_THREADS), 0, s, y, 1, c, p, n, partial);
  return hipGetLastError();
}
hipError_t blas_axpy_partials(cd* y, cd a, const cd* x, i64 n, double* partial, unsigned* nb, hipStream_t s) {
  return axpy_partials_t(y, a, x, n, partial, nb, s);
}
hipError_t blas_axpy_partials(double* y, double a, const double* x, i64 n, double* partial, unsigned* nb,
                              hipStream_t s) {
  return axpy_partials_t(y, a, x, n, partial, nb, s);
}
hipError_t blas_maxpy(cd* y, int k, const cd* a, const cd* const* xs, i64 n, hipStream_t s) {
  return maxpy_t(y, k, a, xs, n, false, nullptr, s);
}
hipError_t blas_maxpy(double* y, int k, const double* a, const double* const* xs, i64 n, hipStream_t s) {
  return maxpy_t(y, k, a, xs, n, false, nullptr, s);
}
hipError_t blas_maxpy_norm(cd* y, int k, const cd* a, const cd* const* xs, i64 n, bool overwrite, double* norm2,
                           hipStream_t s) {
  return maxpy_t(y, k, a, xs, n, overwrite, norm2, s);
}
hipError_t blas_maxpy_norm(double* y, int k, const double* a, const double* const* xs, i64 n, bool overwrite,
                           double* norm2, hipStream_t s) {
  return maxpy_t(y, k, a, xs, n, overwrite, norm2, s);
}

// Synchronous reductions (the result is needed on the host, as in PETSc).
template <class T>
static hipError_t reduce(const T* x, const T* y, i64 n, int kind, double out[2], hipStream_t s) {
  static thread_local Partials part;
  hipError_t e = part.get(2 * RED_BLOCKS);
  if (e != hipSuccess) return e;
  unsigned nb = nblocks(n);
  if (nb > RED_BLOCKS) nb = RED_BLOCKS;
  blaunch(2, k_reduce<T>, dim3(nb), dim3(BLAS_THREADS), 0, s, x, y, n, kind, part.hd);
  e = host_wait(s);  // the partials are in pinned host memory
  if (e != hipSuccess) return e;
  double a = 0.0, b = 0.0;
  for (unsigned k = 0; k < nb; ++k) {
    if (kind == 3) a = fmax(a, part.h[2 * k]);
    else { a += part.h[2 * k]; b += part.h[2 * k + 1]; }
  }
  out[0] = a;
  out[1] = b;
  return hipSuccess;
}

hipError_t blas_dot(const cd* x, const cd* y, i64 n, cd* val, hipStream_t s) {
  double o[2];
  hipError_t e = reduce(x, y, n, 0, o, s);
  *val = make_cd(o[0], o[1]);
  return e;
}
hipError_t blas_dot(const double* x, const double* y, i64 n, double* val, hipStream_t s) {
  double o[2];
  hipError_t e = reduce(x, y, n, 0, o, s);
  *val = o[0];
  return e;
}
template <class T>
static hipError_t norm_t(const T* x, i64 n, int type, double* val, hipStream_t s) {
  double o[2];
  const int kind = type == 1 ? 1 : (type == 0 ? 2 : (type == 3 ? 3 : 1));
  hipError_t e = reduce(x, (const T*)nullptr, n, kind, o, s);
  *val = kind == 1 ? sqrt(o[0]) : o[0];
  return e;
}
hipError_t blas_norm(const cd* x, i64 n, int type, double* val, hipStream_t s) { return norm_t(x, n, type, val, s); }
hipError_t blas_norm(const double* x, i64 n, int type, double* val, hipStream_t s) { return norm_t(x, n, type, val, s); }

// vals[j] = (re, im) of ys[j]^H x
template <class T>
static hipError_t mdot_t(const T* x, int k, const T* const* ys, i64 n, double* vals, hipStream_t s) {
  static thread_local Partials part;
  const int NB = MDOT_BLOCKS;
  hipError_t e = part.get(2 * MDOT_K * NB);
  if (e != hipSuccess) return e;
  for (int j0 = 0; j0 < k; j0 += MDOT_K) {
    const int kk = k - j0 < MDOT_K ? k - j0 : MDOT_K;
    MVPtrsT<T> p;
    for (int j = 0; j < kk; ++j) p.p[j] = ys[j0 + j];
    unsigned nb = nblocks(n);
    if (nb > (unsigned)NB) nb = NB;
    blaunch(2, k_mdot<T>, dim3(nb), dim3(BLAS_THREADS), 0, s, x, kk, p, n, part.d);
    e = kprof_copy(part.h, part.d, sizeof(double) * 2 * MDOT_K * nb, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    e = host_wait(s);
    if (e != hipSuccess) return e;
    for (int j = 0; j < kk; ++j) {
      double ra = 0.0, rb = 0.0;
      for (unsigned q = 0; q < nb; ++q) {
        ra += part.h[(size_t)q * 2 * MDOT_K + 2 * j];
        rb += part.h[(size_t)q * 2 * MDOT_K + 2 * j + 1];
      }
      vals[2 * (j0 + j)] = ra;
      vals[2 * (j0 + j) + 1] = rb;
    }
  }
  return hipSuccess;
}
hipError_t blas_mdot(const cd* x, int k, const cd* const* ys, i64 n, cd* vals, hipStream_t s) {
  return mdot_t(x, k, ys, n, (double*)vals, s);
}

// k_mdot partials [chunk][block][2 MDOT_K] -> dots (device), one k_mdot_finish
hipError_t blas_mdot_finish(const double* partial, int nb, int k, double* dots_dev, hipStream_t s) {
  if (k < 1 || nb < 1 || nb > MDOT_BLOCKS) return hipErrorInvalidValue;
  blaunch(2, k_mdot_finish, dim3((2 * k + 15) / 16), dim3(1024), 0, s, partial, nb, k, dots_dev);
  return hipGetLastError();
}

// multi-dot launches into part (chunks of MDOT_K vectors), returns the workgroup count
template <class T>
static unsigned mdot_launch(const T* w, int k, const T* const* ys, i64 n, double* part, hipStream_t s) {
  unsigned nb = nblocks(n);
  if (nb > (unsigned)MDOT_BLOCKS) nb = MDOT_BLOCKS;
  for (int j0 = 0; j0 < k; j0 += MDOT_K) {
    const int kk = k - j0 < MDOT_K ? k - j0 : MDOT_K;
    MVPtrsT<T> p;
    for (int j = 0; j < kk; ++j) p.p[j] = ys[j0 + j] ? ys[j0 + j] : w;
    blaunch(2, k_mdot<T>, dim3(nb), dim3(BLAS_THREADS), 0, s, w, kk, p, n,
                       part + (size_t)(j0 / MDOT_K) * 2 * MDOT_K * MDOT_BLOCKS);
  }
  return nb;
}

// dots_dev[2 j + re/im] = ys_j^H x (ys_j == NULL: x), on the device without a host wait
hipError_t blas_mdot_dev(const cd* x, int k, const cd* const* ys, i64 n, double* dots_dev, hipStream_t s) {
  if (k < 1 || k > MV_MAX || n < 1) return hipErrorInvalidValue;
  static thread_local Partials part;
  const size_t mlen = (size_t)((MV_MAX + MDOT_K - 1) / MDOT_K) * 2 * MDOT_K * MDOT_BLOCKS;
  hipError_t e = part.get(mlen);
  if (e != hipSuccess) return e;
  const unsigned nb = mdot_launch(x, k, ys, n, part.d, s);
  blaunch(2, k_mdot_finish, dim3((2 * k + 15) / 16), dim3(1024), 0, s, part.d, (int)nb, k, dots_dev);
  return hipGetLastError();
}

// w += sum_j scale_j dd_j ys_j on the device dots dd (2 k doubles), |w|^2; copies dd and the norm
// partials back with one host wait
template <class T>
static hipError_t maxpy_dc_norm_t(T* w, int k, const T* const* ys, const double* scale, const double* dd, i64 n,
                                  double* dots, double* norm2, hipStream_t s) {
  if (k < 1 || k > MV_MAX) return hipErrorInvalidValue;
  static thread_local Partials part;  // dots [2 MV_MAX] | norm [MAXPY_BLOCKS]
  const size_t dlen = 2 * MV_MAX;
  hipError_t e = part.get(dlen + MAXPY_BLOCKS);
  if (e != hipSuccess) return e;
  MVCoefT<double> sc;
  MVPtrsT<T> p;
  for (int j = 0; j < k; ++j) { sc.a[j] = scale[j]; p.p[j] = ys[j]; }
  unsigned mb = nblocks(n);
  if (mb > MAXPY_BLOCKS) mb = MAXPY_BLOCKS;
  // the norm partials and (block 0) the dots straight into pinned host memory
  blaunch(2, k_maxpy_dc<T>, dim3(mb), dim3(BLAS_THREADS), 0, s, w, k, sc, dd, p, n, part.hd + dlen, part.hd);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = host_wait(s);
  if (e != hipSuccess) return e;
  for (int o = 0; o < 2 * k; ++o) dots[o] = part.h[o];
  double t = 0.0;
  for (unsigned q = 0; q < mb; ++q) t += part.h[dlen + q];
  *norm2 = t;
  return hipSuccess;
}
hipError_t blas_maxpy_dc_norm(cd* w, int k, const cd* const* ys, const double* scale, const double* dots_dev, i64 n,
                              cd* dots, double* norm2, hipStream_t s) {
  return maxpy_dc_norm_t(w, k, ys, scale, dots_dev, n, (double*)dots, norm2, s);
}

// dots_j = ys_j^H w, w += sum_j scale_j dots_j ys_j, |w|^2: multi-dot launches, the device finish,
// the MAXPY on the device dots, one copy back and one host wait (k <= MV_MAX)
template <class T>
static hipError_t mdot_maxpy_norm_t(T* w, int k, const T* const* ys, const double* scale, i64 n, double* dots,
                                    double* norm2, hipStream_t s) {
  if (k < 1 || k > MV_MAX) return hipErrorInvalidValue;
  static thread_local Partials part;  // [mdot chunks][2 MDOT_K][MDOT_BLOCKS] | dots [2 MV_MAX]
  const int chunks = (MV_MAX + MDOT_K - 1) / MDOT_K;
  const size_t mlen = (size_t)chunks * 2 * MDOT_K * MDOT_BLOCKS, dlen = 2 * MV_MAX;
  hipError_t e = part.get(mlen + dlen);
  if (e != hipSuccess) return e;
  const unsigned nb = mdot_launch((const T*)w, k, ys, n, part.d, s);
  double* dd = part.d + mlen;
  blaunch(2, k_mdot_finish, dim3((2 * k + 15) / 16), dim3(1024), 0, s, part.d, (int)nb, k, dd);
  return maxpy_dc_norm_t(w, k, ys, scale, (const double*)dd, n, dots, norm2, s);
}
hipError_t blas_mdot_maxpy_norm(cd* w, int k, const cd* const* ys, const double* scale, i64 n, cd* dots,
                                double* norm2, hipStream_t s) {
  return mdot_maxpy_norm_t(w, k, ys, scale, n, (double*)dots, norm2, s);
}
hipError_t blas_mdot_maxpy_norm(double* w, int k, const double* const* ys, const double* scale, i64 n, double* dots,
                                double* norm2, hipStream_t s) {
  std::vector<double> v(2 * (size_t)(k > 0 ? k : 1));
  hipError_t e = mdot_maxpy_norm_t(w, k, ys, scale, n, v.data(), norm2, s);
  for (int j = 0; j < k; ++j) dots[j] = v[2 * (size_t)j];
  return e;
}
hipError_t blas_mdot(const double* x, int k, const double* const* ys, i64 n, double* vals, hipStream_t s) {
  std::vector<double> v(2 * (size_t)(k > 0 ? k : 1));
  hipError_t e = mdot_t(x, k, ys, n, v.data(), s);
  for (int j = 0; j < k; ++j) vals[j] = v[2 * (size_t)j];
  return e;
}

}  // namespace cfp
