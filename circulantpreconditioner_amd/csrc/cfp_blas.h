// cfp_blas.h -- device vector kernels of the PETSc-compatible layer (cfp_blas.hip), for complex
// double (the default stand-in PETSc) and double (the real-scalar build, PetscScalar = double).
#pragma once
#include <type_traits>
#include <vector>

#include "cfp_internal.h"

namespace cfp {
#define MV_MAX 32
template <class T> struct MVPtrsT { const T* p[MV_MAX]; };
template <class T> struct MVCoefT { T a[MV_MAX]; };
using MVPtrs = MVPtrsT<cd>;
using MVCoef = MVCoefT<cd>;

hipError_t blas_set(cd* x, cd a, i64 n, hipStream_t s);
hipError_t blas_shift(cd* x, cd a, i64 n, hipStream_t s);
hipError_t blas_copy(cd* y, const cd* x, i64 n, hipStream_t s);
hipError_t blas_axpy(cd* y, cd a, const cd* x, i64 n, hipStream_t s);    // y += a x
hipError_t blas_aypx(cd* y, cd b, const cd* x, i64 n, hipStream_t s);    // y = x + b y
hipError_t blas_waxpy(cd* w, cd a, const cd* x, const cd* y, i64 n, hipStream_t s);  // w = a x + y
hipError_t blas_pmult(cd* w, const cd* x, const cd* y, i64 n, hipStream_t s);
// y += sum_j a[j] xs[j]   (a, xs: host arrays of k coefficients / device pointers)
hipError_t blas_maxpy(cd* y, int k, const cd* a, const cd* const* xs, i64 n, hipStream_t s);
// y = (overwrite ? 0 : y) + sum_j a[j] xs[j]; norm2 != nullptr: also sum |y|^2 of the result,
// accumulated in the same sweep (synchronous then, like the reductions below)
// y += a x with the |y|^2 per-workgroup partials of the result written to partial (a device
// address, e.g. of mapped pinned memory; at most BLAS_NORM_PARTIALS), no wait: *nb = the partial
// count (0 for n = 0).  The stand-in VecAXPY keeps them for a following VecNorm (petsc_mini.cpp).
#define BLAS_NORM_PARTIALS 1024
hipError_t blas_axpy_partials(cd* y, cd a, const cd* x, i64 n, double* partial, unsigned* nb, hipStream_t s);
hipError_t blas_axpy_partials(double* y, double a, const double* x, i64 n, double* partial, unsigned* nb,
                              hipStream_t s);
hipError_t blas_maxpy_norm(cd* y, int k, const cd* a, const cd* const* xs, i64 n, bool overwrite, double* norm2,
                           hipStream_t s);
// y = A x for a CSR matrix of m rows and nnz nonzeros (nnz picks the lanes per row)
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                         hipStream_t s);
// Row-class diagonal form (k_dia_spmv): nonzeros on nd <= DIA_MAX fixed diagonals (column - row =
// off[k], ascending), each row one of ncls <= 256 classes; class c holds tab[c nd + k] on
// diagonal k where bit k of masks[c] is set.  y[r] = sum_k tab[cls[r] nd + k] x[r + off[k]].
#define DIA_MAX 8
struct DiaDesc {
  i64 off[DIA_MAX];
  int nd = 0, ncls = 0;
};
hipError_t blas_dia_spmv(i64 m, const DiaDesc& d, const unsigned char* cls, const unsigned char* masks, const cd* tab,
                         const cd* x, cd* y, hipStream_t s);
hipError_t blas_dia_spmv(i64 m, const DiaDesc& d, const unsigned char* cls, const unsigned char* masks,
                         const double* tab, const double* x, double* y, hipStream_t s);
// Block row-class form (k_bdia_spmv): the matrix in B x B blocks (B = 2..4, e.g. the d + 1
// interleaved unknowns of a wave-system cell), every nonzero in a block on one of nd <= BDIA_MAX
// block diagonals (block column - block row = off[k], ascending), each block row one of
// ncls <= 256 classes; class c has a block on the diagonals whose bit k of masks[c] is set, stored
// densely (row i, column j) in ascending k from block cbase[c] of tab: the q-th present block of
// class c is tab[((cbase[c] + q) B + i) B + j], and bnz[cbase[c] + q] marks its nonzero entries
// (bit i B + j) and, in bits 16.., the columns that have any.
// y[R B + i] = sum_k,j block(k)[i][j] x[(R + off[k]) B + j].
#define BDIA_MAX 16
struct BDiaDesc {
  i64 off[BDIA_MAX];
  int nd = 0, ncls = 0, B = 0, nblk = 0;  // nblk: blocks in tab
  int re = 0;  // 1: every table entry has a zero imaginary part (the wave operator): real x complex products
};
#define BDIA_LDS_MAX (60 * 1024)
hipError_t blas_bdia_spmv(i64 mb, const BDiaDesc& d, const unsigned char* cls, const unsigned short* masks,
                          const unsigned short* cbase, const unsigned* bnz, const cd* tab, const cd* x, cd* y,
                          hipStream_t s);
hipError_t blas_bdia_spmv(i64 mb, const BDiaDesc& d, const unsigned char* cls, const unsigned short* masks,
                          const unsigned short* cbase, const unsigned* bnz, const double* tab, const double* x,
                          double* y, hipStream_t s);
// distributed AIJ halo: out[i] = x[idx[i]] (idx < 0: 0); y += B x for a CSR block B
hipError_t blas_gather(cd* out, const cd* x, const i64* idx, i64 n, hipStream_t s);
hipError_t blas_gather(double* out, const double* x, const i64* idx, i64 n, hipStream_t s);
hipError_t blas_csr_spmv_add(i64 m, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                             hipStream_t s);
hipError_t blas_csr_spmv_add(i64 m, const i64* rowptr, const i64* col, const double* val, const double* x, double* y,
                             hipStream_t s);
// synchronous reductions, PETSc conventions: dot = y^H x; norm type 0 = NORM_1 (sum |re|+|im|),
// 1 = NORM_2, 3 = NORM_INFINITY (max modulus)
hipError_t blas_dot(const cd* x, const cd* y, i64 n, cd* val, hipStream_t s);
hipError_t blas_norm(const cd* x, i64 n, int type, double* val, hipStream_t s);
// vals[j] = ys[j]^H x  (ys: host array of k device pointers)
hipError_t blas_mdot(const cd* x, int k, const cd* const* ys, i64 n, cd* vals, hipStream_t s);
// classical Gram-Schmidt in one host round trip: dots[j] = ys[j]^H w, w += sum_j scale[j] dots[j]
// ys[j] (coefficients formed on the device), norm2 = |w|^2; k <= MV_MAX (scale: host, real)
hipError_t blas_mdot_maxpy_norm(cd* w, int k, const cd* const* ys, const double* scale, i64 n, cd* dots,
                                double* norm2, hipStream_t s);
// the two halves of it, for dots computed elsewhere (a fused PCApply, cfp_plan_apply_ex):
// dots_dev[2 j + re/im] = ys[j]^H x (ys[j] == NULL: x itself), on the device, no host wait
hipError_t blas_mdot_dev(const cd* x, int k, const cd* const* ys, i64 n, double* dots_dev, hipStream_t s);
// workgroup partials in k_mdot's layout ([block][16]: 2 values per vector, k <= 8) -> dots_dev
hipError_t blas_mdot_finish(const double* partial, int nb, int k, double* dots_dev, hipStream_t s);
// w += sum_j scale[j] dots_j ys[j] with the dots on the device, |w|^2; copies the dots back
// (dots, host) with the norm, one host wait
hipError_t blas_maxpy_dc_norm(cd* w, int k, const cd* const* ys, const double* scale, const double* dots_dev, i64 n,
                              cd* dots, double* norm2, hipStream_t s);

// the same on real vectors (PetscScalar = double), plus the scale and the divide that the
// complex build takes from cfp_kernels.hip (launch_scale, launch_pointwise_divide)
hipError_t blas_set(double* x, double a, i64 n, hipStream_t s);
hipError_t blas_shift(double* x, double a, i64 n, hipStream_t s);
hipError_t blas_copy(double* y, const double* x, i64 n, hipStream_t s);
hipError_t blas_axpy(double* y, double a, const double* x, i64 n, hipStream_t s);
hipError_t blas_aypx(double* y, double b, const double* x, i64 n, hipStream_t s);
hipError_t blas_waxpy(double* w, double a, const double* x, const double* y, i64 n, hipStream_t s);
hipError_t blas_pmult(double* w, const double* x, const double* y, i64 n, hipStream_t s);
hipError_t blas_scale(double* x, double a, i64 n, hipStream_t s);
hipError_t blas_pdivide(double* w, const double* x, const double* y, i64 n, hipStream_t s);  // 0 where y = 0
hipError_t blas_maxpy(double* y, int k, const double* a, const double* const* xs, i64 n, hipStream_t s);
hipError_t blas_maxpy_norm(double* y, int k, const double* a, const double* const* xs, i64 n, bool overwrite,
                           double* norm2, hipStream_t s);
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const double* val, const double* x,
                         double* y, hipStream_t s);
hipError_t blas_dot(const double* x, const double* y, i64 n, double* val, hipStream_t s);
hipError_t blas_norm(const double* x, i64 n, int type, double* val, hipStream_t s);
hipError_t blas_mdot(const double* x, int k, const double* const* ys, i64 n, double* vals, hipStream_t s);
hipError_t blas_mdot_maxpy_norm(double* w, int k, const double* const* ys, const double* scale, i64 n, double* dots,
                                double* norm2, hipStream_t s);
// device-time profile of the launches above (petsc_mini PetscMiniProfileBegin / End): kinds
// 1 = MatMult kernels, 2 = vector kernels, 3 = copies (kprof_copy); kprof_take hands out the next
// event pair for a launch of that kind (false: profile off or full)
hipError_t kprof_begin(size_t cap);
hipError_t kprof_end(double ms[4], long long launches[4]);
void kprof_reset();
bool kprof_take(int kind, hipEvent_t* e0, hipEvent_t* e1);
hipError_t kprof_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s);
// device-to-device copy on the library's tuned kernel (16-byte lanes, NT stores; kprof kind 3);
// unaligned or odd sizes go through hipMemcpyAsync
hipError_t blas_copy_bytes(void* dst, const void* src, size_t bytes, hipStream_t s);
// wait on the host for the work queued on s so far (an event polled; see cfp_blas.hip)
hipError_t host_wait(hipStream_t s);
}  // namespace cfp
