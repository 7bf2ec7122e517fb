// cfp_blas.h -- device vector kernels of the PETSc-compatible layer (cfp_blas.hip).
#pragma once
#include "cfp_internal.h"

namespace cfp {
#define MV_MAX 32
struct MVPtrs { const cd* p[MV_MAX]; };
struct MVCoef { cd a[MV_MAX]; };
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
hipError_t blas_maxpy_norm(cd* y, int k, const cd* a, const cd* const* xs, i64 n, bool overwrite, double* norm2,
                           hipStream_t s);
// y = A x for a CSR matrix of m rows and nnz nonzeros (nnz picks the lanes per row)
hipError_t blas_csr_spmv(i64 m, i64 nnz, const i64* rowptr, const i64* col, const cd* val, const cd* x, cd* y,
                         hipStream_t s);
// synchronous reductions, PETSc conventions: dot = y^H x; norm type 0 = NORM_1 (sum |re|+|im|),
// 1 = NORM_2, 3 = NORM_INFINITY (max modulus)
hipError_t blas_dot(const cd* x, const cd* y, i64 n, cd* val, hipStream_t s);
hipError_t blas_norm(const cd* x, i64 n, int type, double* val, hipStream_t s);
// vals[j] = ys[j]^H x  (ys: host array of k device pointers)
hipError_t blas_mdot(const cd* x, int k, const cd* const* ys, i64 n, cd* vals, hipStream_t s);
}  // namespace cfp
