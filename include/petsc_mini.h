/*
 * petsc_mini.h -- the subset of the PETSc C API that the circulant preconditioner boundary
 * uses, implemented by libcirculant_fft.so when real PETSc is absent (it is absent in this
 * image and on the GPU box: SURVEY.md §8c).
 *
 * Names, argument order and semantics follow PETSc >= 3.19 (complex scalars, VECHIP
 * offload model).  Compiling with -DCFP_WITH_PETSC replaces this whole header by the real
 * <petscksp.h>; pcshell_fft3d.cpp only calls functions that exist there.  Deliberate
 * differences of the stand-in:
 *   - PetscInt is 64-bit (as a PETSc built --with-64-bit-indices);
 *   - MPI_Comm is an int handle (no MPI library inside).  PETSC_COMM_SELF has one rank;
 *     PETSC_COMM_WORLD has one rank until PetscMiniSetCommWorld points it at a communicator of
 *     several ranks made by PetscMiniCommCreate (the caller's collectives: all-to-all and
 *     all-reduce callbacks, e.g. torch.distributed) or PetscMiniCommCreateRCCL (an RCCL
 *     communicator, one process per GPU).  Vecs made on such a communicator hold the
 *     PETSC_DECIDE block of rows of their rank; VecDot / VecNorm / VecMDot reduce over it;
 *     VecSetValues applies the calling rank's rows at once and stashes the others, as PETSc
 *     does, until VecAssemblyBegin/End delivers them (see VecAssemblyBegin);
 *   - Vec is either host-only (VECSEQ) or device-resident with a host mirror (VECSEQHIP),
 *     with PETSc's offload mask semantics for the Get/Restore pairs;
 *   - Mat supports MATSHELL (user operations), MATSEQAIJ (CSR, device SpMV) and the FFT
 *     shell made by MatCreateFFT / MatCreateFFTHIP.
 */
#ifndef CFP_PETSC_MINI_H
#define CFP_PETSC_MINI_H

#ifdef CFP_WITH_PETSC
#include <petscksp.h>
#else

#include <stddef.h>
#include <stdint.h>

/* PetscScalar: complex double (PETSC_USE_COMPLEX, the default), or double when built with
 * -DCFP_REAL_SCALAR (a PETSc configured with real scalars, the reference's !PETSC_USE_COMPLEX
 * branches: libcirculant_fft_real.so) */
#ifdef CFP_REAL_SCALAR
typedef double PetscScalar;
#else
#define PETSC_USE_COMPLEX 1
#endif
#ifdef __cplusplus
#include <complex>
#ifndef CFP_REAL_SCALAR
typedef std::complex<double> PetscScalar;
#endif
extern "C" {
#else
#ifndef CFP_REAL_SCALAR
#include <complex.h>
typedef double _Complex PetscScalar;
#endif
#endif

typedef int PetscErrorCode;
typedef int64_t PetscInt;
typedef double PetscReal;
typedef double PetscLogDouble;
typedef int PetscMPIInt;
typedef enum { PETSC_FALSE = 0, PETSC_TRUE = 1 } PetscBool;
typedef int MPI_Comm;
#define PETSC_COMM_WORLD ((MPI_Comm)0)
#define PETSC_COMM_SELF ((MPI_Comm)1)
#define MPI_SUCCESS 0
#define PETSC_DECIDE (-1)
#define PETSC_DETERMINE (-1)
#define PETSC_DEFAULT (-2)

/* error codes (petscerror.h) */
#define PETSC_SUCCESS 0
#define PETSC_ERR_MEM 55
#define PETSC_ERR_SUP 56
#define PETSC_ERR_ARG_SIZ 60
#define PETSC_ERR_ARG_IDN 61
#define PETSC_ERR_ARG_WRONG 62
#define PETSC_ERR_ARG_OUTOFRANGE 63
#define PETSC_ERR_ARG_WRONGSTATE 73
#define PETSC_ERR_LIB 76
#define PETSC_ERR_PLIB 77
#define PETSC_ERR_ARG_NULL 85
#define PETSC_ERR_CONV_FAILED 91

typedef enum { PETSC_MEMTYPE_HOST = 0, PETSC_MEMTYPE_DEVICE = 1, PETSC_MEMTYPE_HIP = 3 } PetscMemType;
typedef enum { NORM_1 = 0, NORM_2 = 1, NORM_FROBENIUS = 2, NORM_INFINITY = 3 } NormType;
typedef enum { INSERT_VALUES = 1, ADD_VALUES = 2 } InsertMode;

typedef struct _p_PetscObject *PetscObject;
typedef int64_t PetscObjectState;
typedef int64_t PetscObjectId;
typedef struct _p_Vec *Vec;
typedef struct _p_Mat *Mat;
typedef struct _p_PC *PC;
typedef const char *MatType;
typedef const char *PCType;
typedef const char *VecType;
#define VECSEQ "seq"
#define VECSEQHIP "seqhip"
#define VECMPI "mpi"
#define VECMPIHIP "mpihip"
#define MATSHELL "shell"
#define MATSEQAIJ "seqaij"
#define MATMPIAIJ "mpiaij"
#define MATAIJ "aij"
#define MATFFTW "fftw"
#define PCSHELL "shell"
#define PCNONE "none"

typedef enum {
  MATOP_MULT = 3,
  MATOP_MULT_TRANSPOSE = 5,
  MATOP_DESTROY = 26
} MatOperation;

/* error reporting (PetscCall/PetscCheck in the PETSc style) */
PetscErrorCode PetscErrorSet(PetscErrorCode code, const char *func, const char *msg);
const char *PetscErrorLastMessage(void);
#define PetscFunctionBeginUser do { } while (0)
#define PetscFunctionReturn(x) return (x)
#define PetscCall(expr)                                   \
  do {                                                    \
    PetscErrorCode ierr__ = (expr);                       \
    if (ierr__) return ierr__;                            \
  } while (0)
#define PetscCheck(cond, comm, code, msg)                  \
  do {                                                    \
    if (!(cond)) return PetscErrorSet((code), __func__, (msg)); \
  } while (0)
PetscErrorCode PetscTime(PetscLogDouble *t);
#define PetscCallMPI(expr)                                                   \
  do {                                                                       \
    int mpierr__ = (expr);                                                   \
    if (mpierr__) return PetscErrorSet(PETSC_ERR_LIB, __func__, "MPI error"); \
  } while (0)

/* ---- communicators (stand-in for the MPI subset the boundary uses) */
int MPI_Comm_size(MPI_Comm comm, int *size);
int MPI_Comm_rank(MPI_Comm comm, int *rank);
/* the caller's collectives for a communicator of `size` ranks (host buffers):
 *   alltoall: sendbuf holds `size` blocks of bytes_per_rank bytes, block q goes to rank q;
 *             recvbuf block q is what rank q sent to this rank
 *   allreduce: in place over `count` doubles, op PETSCMINI_OP_SUM or PETSCMINI_OP_MAX
 * each returns 0 on success */
#define PETSCMINI_OP_SUM 0
#define PETSCMINI_OP_MAX 1
typedef struct {
  int (*alltoall)(void *user, const void *sendbuf, void *recvbuf, int64_t bytes_per_rank);
  int (*allreduce)(void *user, double *buf, int64_t count, int op);
  void *user;
} PetscMiniCommOps;
PetscErrorCode PetscMiniCommCreate(int size, int rank, const PetscMiniCommOps *ops, MPI_Comm *comm);
/* an RCCL communicator on the current HIP device (unique_id = the 128 bytes of
 * cfp_dist_get_unique_id, created on rank 0 and broadcast by the caller).  It is created
 * NON-BLOCKING (ncclCommInitRankConfig, blocking = 0), polled against a 300 s deadline; a rank
 * that never joins is an error, not a hang.  CFP_RCCL_BLOCKING=1 in the environment selects
 * ncclCommInitRank (blocking, no deadline) instead; cfp_rccl_blocking reports which. */
PetscErrorCode PetscMiniCommCreateRCCL(int size, int rank, const char *unique_id, MPI_Comm *comm);
/* refused (PETSC_ERR_ARG_WRONGSTATE) while FFT matrices built on the communicator still exist */
PetscErrorCode PetscMiniCommDestroy(MPI_Comm *comm);
/* reference count of the objects that use a communicator (FFT matrices of several ranks) */
PetscErrorCode PetscMiniCommRetain(MPI_Comm comm);
PetscErrorCode PetscMiniCommRelease(MPI_Comm comm);
/* PETSC_COMM_WORLD resolves to comm from now on (PETSC_COMM_SELF: back to one rank) */
PetscErrorCode PetscMiniSetCommWorld(MPI_Comm comm);
/* the communicator PETSC_COMM_WORLD currently stands for (others: themselves) */
PetscErrorCode PetscMiniCommResolve(MPI_Comm comm, MPI_Comm *resolved);
PetscErrorCode PetscMiniAllreduce(MPI_Comm comm, double *buf, int64_t count, int op);
/* Device storage the stand-in AIJ picked at its first device MatMult: 1 = row-class diagonal
 * form (k_dia_spmv: nonzeros on <= 8 fixed diagonals, <= 256 distinct rows -- Cartesian
 * stencils), 2 = block row-class form (k_bdia_spmv: B x B blocks, B = 2..4, on <= 8 block
 * diagonals, <= 256 distinct block rows -- the interleaved wave operator), 0 = CSR, -1 = not
 * uploaded yet (MatShift resets it). */
PetscErrorCode PetscMiniMatAIJGetFormat(Mat A, int *format);
/* The device row-class form of an AIJ (above; uploaded now if it has not been): its class bytes,
 * class masks and coefficient table as device arrays, in the layout of cfp_stencil_t
 * (include/circulant_fft.h).  *has = PETSC_FALSE when the matrix is not representable (CSR only).
 * *x_local = PETSC_TRUE when no entry leaves its row's run of `rowlen` consecutive indices (an
 * operator coupling cells along x only, on an x-fastest grid with n_x = rowlen). */
typedef struct {
  const unsigned char *cls;
  const unsigned char *mask;
  const PetscScalar *tab;
  int64_t off[8];
  int nd, ncls;
  const unsigned char *cls_x; /* [rowlen] device when cls[r] = cls_x[r mod rowlen] for all rows, else NULL */
} PetscMiniDia;
PetscErrorCode PetscMiniMatAIJGetDia(Mat A, PetscInt rowlen, PetscBool *has, PetscBool *x_local, PetscMiniDia *dia);
/* the ncclComm_t behind an RCCL communicator (NULL for a callback communicator).  Unless
 * CFP_RCCL_BLOCKING is set it is a non-blocking communicator: an RCCL call the caller makes on it
 * (ncclGroupEnd, a collective, ncclCommFinalize) may return ncclInProgress, and the caller must
 * poll ncclCommGetAsyncError until the state leaves ncclInProgress before relying on it.  The
 * communicator stays the library's: do not destroy it. */
PetscErrorCode PetscMiniCommGetNCCL(MPI_Comm comm, void **nccl_comm);
/* One exchange piece of a slab plan over a communicator (the cfp_dist_exchange_fn contract of
 * include/circulant_fft_dist.h; user = (void *)(intptr_t)comm): device buffers, staged through
 * pinned host memory for a callback communicator, grouped ncclSend/ncclRecv for RCCL. */
int PetscMiniCommExchange(void *user, const double *src_dev, double *dst_dev, int64_t chunk, int64_t off,
                          int64_t count, void *stream);

/* Object state and id, as PETSc's: the state of a Vec increases on every write access (write
 * Get/RestoreArray, VecSet, VecScale, VecCopy into it, ...); the id is unique per object.
 * Vecs only in this stand-in (PETSC_ERR_ARG_WRONG for other objects). */
PetscErrorCode PetscObjectStateGet(PetscObject obj, PetscObjectState *state);
PetscErrorCode PetscObjectGetId(PetscObject obj, PetscObjectId *id);

/* ---- Vec */
PetscErrorCode VecCreateSeq(MPI_Comm comm, PetscInt n, Vec *v);
PetscErrorCode VecCreateSeqHIP(MPI_Comm comm, PetscInt n, Vec *v);
PetscErrorCode VecCreateSeqHIPWithArray(MPI_Comm comm, PetscInt bs, PetscInt n, const PetscScalar *gpuarray, Vec *v);
/* distributed: nlocal or N may be PETSC_DECIDE (N / size rows, the first N % size ranks one
 * more); VECMPI lives in host memory, VECMPIHIP on the device */
PetscErrorCode VecCreateMPI(MPI_Comm comm, PetscInt nlocal, PetscInt N, Vec *v);
PetscErrorCode VecCreateMPIHIP(MPI_Comm comm, PetscInt nlocal, PetscInt N, Vec *v);
PetscErrorCode VecCreateMPIHIPWithArray(MPI_Comm comm, PetscInt bs, PetscInt nlocal, PetscInt N,
                                        const PetscScalar *gpuarray, Vec *v);
PetscErrorCode VecGetComm(Vec v, MPI_Comm *comm); /* not in PETSc (PetscObjectGetComm) */
PetscErrorCode VecDuplicate(Vec v, Vec *newv);
PetscErrorCode VecDestroy(Vec *v);
PetscErrorCode VecGetType(Vec v, VecType *type);
PetscErrorCode VecGetSize(Vec v, PetscInt *n);
PetscErrorCode VecGetLocalSize(Vec v, PetscInt *n);
PetscErrorCode VecGetOwnershipRange(Vec v, PetscInt *lo, PetscInt *hi);
PetscErrorCode VecGetArray(Vec v, PetscScalar **a);
PetscErrorCode VecRestoreArray(Vec v, PetscScalar **a);
PetscErrorCode VecGetArrayRead(Vec v, const PetscScalar **a);
PetscErrorCode VecRestoreArrayRead(Vec v, const PetscScalar **a);
PetscErrorCode VecGetArrayWrite(Vec v, PetscScalar **a);
PetscErrorCode VecRestoreArrayWrite(Vec v, PetscScalar **a);
PetscErrorCode VecGetArrayReadAndMemType(Vec v, const PetscScalar **a, PetscMemType *mtype);
PetscErrorCode VecRestoreArrayReadAndMemType(Vec v, const PetscScalar **a);
PetscErrorCode VecGetArrayWriteAndMemType(Vec v, PetscScalar **a, PetscMemType *mtype);
PetscErrorCode VecRestoreArrayWriteAndMemType(Vec v, PetscScalar **a);
PetscErrorCode VecGetArrayAndMemType(Vec v, PetscScalar **a, PetscMemType *mtype);
PetscErrorCode VecRestoreArrayAndMemType(Vec v, PetscScalar **a);
PetscErrorCode VecHIPGetArray(Vec v, PetscScalar **a);
PetscErrorCode VecHIPRestoreArray(Vec v, PetscScalar **a);
PetscErrorCode VecHIPGetArrayRead(Vec v, const PetscScalar **a);
PetscErrorCode VecHIPRestoreArrayRead(Vec v, const PetscScalar **a);
PetscErrorCode VecHIPGetArrayWrite(Vec v, PetscScalar **a);
PetscErrorCode VecHIPRestoreArrayWrite(Vec v, PetscScalar **a);
PetscErrorCode VecSet(Vec v, PetscScalar alpha);
PetscErrorCode VecSetValue(Vec v, PetscInt i, PetscScalar value, InsertMode mode);
PetscErrorCode VecSetValues(Vec v, PetscInt n, const PetscInt *idx, const PetscScalar *y, InsertMode mode);
PetscErrorCode VecGetValues(Vec v, PetscInt n, const PetscInt *idx, PetscScalar *y);
/* VecSetValues on a Vec of several ranks: rows of other ranks go to a per-Vec stash (no size
 * limit below PETSC_ERR_MEM at 2^27 entries) that only VecAssemblyBegin empties.
 * VecAssemblyBegin is COLLECTIVE on the Vec's communicator, as in PETSc: every rank must call it
 * (two all-reduces and one all-to-all), stash or no stash; a call on some ranks only blocks in
 * the first collective (with torch.distributed callbacks: until the process group's timeout).
 * VecAssemblyEnd completes the pair and communicates nothing.  On one rank both only clear the
 * stash. */
PetscErrorCode VecAssemblyBegin(Vec v);
PetscErrorCode VecAssemblyEnd(Vec v);
PetscErrorCode VecCopy(Vec x, Vec y);
PetscErrorCode VecScale(Vec x, PetscScalar alpha);
PetscErrorCode VecShift(Vec x, PetscScalar alpha);
PetscErrorCode VecAXPY(Vec y, PetscScalar alpha, Vec x);
PetscErrorCode VecAYPX(Vec y, PetscScalar beta, Vec x);
PetscErrorCode VecWAXPY(Vec w, PetscScalar alpha, Vec x, Vec y);
PetscErrorCode VecPointwiseDivide(Vec w, Vec x, Vec y);
PetscErrorCode VecPointwiseMult(Vec w, Vec x, Vec y);
PetscErrorCode VecDot(Vec x, Vec y, PetscScalar *val);
PetscErrorCode VecNorm(Vec x, NormType type, PetscReal *val);
PetscErrorCode VecMDot(Vec x, PetscInt nv, const Vec y[], PetscScalar val[]); /* val_i = y_i^H x */
PetscErrorCode VecMAXPY(Vec y, PetscInt nv, const PetscScalar alpha[], Vec x[]); /* y += sum alpha_i x_i */
PetscErrorCode VecDuplicateVecs(Vec v, PetscInt m, Vec *V[]);
PetscErrorCode VecDestroyVecs(PetscInt m, Vec *V[]);
/* stream the Vec kernels are enqueued on (hipStream_t, NULL = default); not in PETSc.  Like
 * PETSc's VECHIP operations on its default device stream, work on device Vecs is stream-ordered
 * on it and returns before completion; host reads (VecGetArray...) synchronise. */
PetscErrorCode VecMiniSetStream(void *stream);
PetscErrorCode VecMiniGetStream(void **stream);
/* wait for the work queued on that stream if v is a device vector; not in PETSc */
PetscErrorCode VecMiniSynchronize(Vec v);
/* y = (overwrite ? 0 : y) + sum alpha_i x_i and, if norm != NULL, ||y||_2 over the Vec's ranks,
 * in one sweep of y (the stand-in GMRES's orthogonalisation + norm, and its solution update
 * into a zero x without a VecSet); not in PETSc */
/* Classical Gram-Schmidt step of the stand-in GMRES: dots[j] = V[j]^H w (PETSc's VecMDot), then
 * w += sum_j scale[j] dots[j] V[j] and *norm = |w| -- on one rank's device Vecs (nv <= 32) with the
 * coefficients formed on the device, one host wait per call. */
PetscErrorCode VecMiniMDotMAXPYNorm(Vec w, PetscInt nv, const PetscReal scale[], Vec V[], PetscScalar dots[],
                                    PetscReal *norm);
PetscErrorCode VecMiniMAXPYNorm(Vec y, PetscInt nv, const PetscScalar alpha[], Vec x[], PetscBool overwrite,
                                PetscReal *norm);
/* The second half of VecMiniMDotMAXPYNorm for dots already on the device (dots_dev[2 j + re/im] =
 * V[j]^H w, e.g. from a fused PCApply, PCMiniApplyDots): w += sum_j scale[j] dots_j V[j], *norm =
 * |w|, the dots copied back into dots[]; one host wait.  Device Vecs of one rank, nv <= 32. */
PetscErrorCode VecMiniMAXPYNormDeviceDots(Vec w, PetscInt nv, const PetscReal scale[], Vec V[], const double *dots_dev,
                                          PetscScalar dots[], PetscReal *norm);
/* Device-time profile of the stand-in's own kernels (not in PETSc; what rocprofv3 --kernel-trace
 * would sum, from inside the process): between Begin and End every MatMult / vector kernel launch
 * stamps its own dispatch (hipExtLaunchKernelGGL start / stop events) and every device copy is
 * bracketed by events.  End waits, then writes the summed ms and launch counts per kind: [0]
 * unused here (PCApply: KSPMiniGetPCApplyStats), [1] MatMult, [2] vector kernels, [3] copies.
 * At most max_records launches are stamped (later ones run unstamped). */
PetscErrorCode PetscMiniProfileBegin(PetscInt max_records);
PetscErrorCode PetscMiniProfileEnd(double ms[4], int64_t launches[4]);
/* host copy of n doubles of device memory, ordered on the Vec stream (waits) */
PetscErrorCode PetscMiniDeviceRead(const double *dev, PetscInt n, double *host);

/* ---- Mat */
PetscErrorCode MatCreateShell(MPI_Comm comm, PetscInt m, PetscInt n, PetscInt M, PetscInt N, void *ctx, Mat *A);
PetscErrorCode MatShellSetOperation(Mat A, MatOperation op, void (*f)(void));
PetscErrorCode MatShellGetContext(Mat A, void *ctx);
PetscErrorCode MatCreateSeqAIJWithArrays(MPI_Comm comm, PetscInt m, PetscInt n, PetscInt *i, PetscInt *j,
                                         PetscScalar *a, Mat *A);
PetscErrorCode MatGetType(Mat A, MatType *type);
PetscErrorCode MatGetSize(Mat A, PetscInt *m, PetscInt *n);
PetscErrorCode MatGetLocalSize(Mat A, PetscInt *m, PetscInt *n);
/* MatCreateAIJ (the reference's transport / wave drivers, tests/TransportEquation_SphericalExplosion_
 * impl_mpi.cxx:82-84): m, n local sizes or PETSC_DECIDE (PETSc's row blocks, as VecCreateMPI), M, N
 * global; the preallocation hints are accepted and not needed.  Entries go in with MatSetValue(s)
 * -- another rank's rows are stashed and delivered by MatAssemblyBegin/End, which are collective on
 * the communicator -- and the matrix is usable after MatAssemblyEnd(A, MAT_FINAL_ASSEMBLY).  One
 * rank: a MATSEQAIJ.  Several (MATMPIAIJ): this rank's rows, split as PETSc does into the diagonal
 * block (its own columns: row-class form / CSR, device SpMV) and the off-diagonal block over the
 * ghost columns, whose values MatMult fetches from their owners (one all-to-all per MatMult; none
 * when no rank has ghosts -- an operator that couples cells inside z-slabs only).  Square
 * matrices always store their diagonal (MatShift). */
typedef enum { MAT_FINAL_ASSEMBLY = 0, MAT_FLUSH_ASSEMBLY = 1 } MatAssemblyType;
PetscErrorCode MatCreateAIJ(MPI_Comm comm, PetscInt m, PetscInt n, PetscInt M, PetscInt N, PetscInt d_nz,
                            const PetscInt d_nnz[], PetscInt o_nz, const PetscInt o_nnz[], Mat *A);
PetscErrorCode MatSetValue(Mat A, PetscInt i, PetscInt j, PetscScalar v, InsertMode mode);
PetscErrorCode MatSetValues(Mat A, PetscInt m, const PetscInt idxm[], PetscInt n, const PetscInt idxn[],
                            const PetscScalar v[], InsertMode mode);
PetscErrorCode MatAssemblyBegin(Mat A, MatAssemblyType type);
PetscErrorCode MatAssemblyEnd(Mat A, MatAssemblyType type);
PetscErrorCode MatGetOwnershipRange(Mat A, PetscInt *lo, PetscInt *hi);
/* not in PETSc: ghost columns of this rank's rows and the largest per-peer halo of any rank (0:
 * MatMult exchanges nothing) -- MATMPIAIJ after assembly; 0, 0 otherwise */
PetscErrorCode PetscMiniMatMPIAIJGetHalo(Mat A, PetscInt *ghosts, PetscInt *max_per_peer);
PetscErrorCode MatGetComm(Mat A, MPI_Comm *comm); /* not in PETSc (PetscObjectGetComm) */
PetscErrorCode MatMult(Mat A, Vec x, Vec y);
PetscErrorCode MatMultTranspose(Mat A, Vec x, Vec y);
PetscErrorCode MatShift(Mat A, PetscScalar a);
PetscErrorCode MatDestroy(Mat *A);
/* the FFT matrix: a MATSHELL around a cfp plan; dims = {n_z, n_y, n_x} for ndim = 3
 * (row-major, x fastest), {n_y, n_x} for 2, {n_x} for 1.  MatCreateFFT accepts only
 * MATFFTW as type and returns the HIP implementation.  On a communicator of several ranks the
 * matrix is z-slab distributed (FFTW-MPI's local_n0 = PETSC_DECIDE rows) and
 * MatCreateVecsFFTW gives VECMPIHIP vectors of the local slab. */
PetscErrorCode MatCreateFFT(MPI_Comm comm, PetscInt ndim, const PetscInt dims[], MatType type, Mat *A);
PetscErrorCode MatCreateVecsFFTW(Mat A, Vec *x, Vec *y, Vec *z);

/* ---- PC */
PetscErrorCode PCCreate(MPI_Comm comm, PC *pc);
PetscErrorCode PCSetType(PC pc, PCType type);
PetscErrorCode PCGetType(PC pc, PCType *type);
PetscErrorCode PCShellSetContext(PC pc, void *ctx);
PetscErrorCode PCShellGetContext(PC pc, void *ctx); /* ctx is a pointer to the user's pointer */
PetscErrorCode PCShellSetApply(PC pc, PetscErrorCode (*apply)(PC, Vec, Vec));
PetscErrorCode PCShellSetSetUp(PC pc, PetscErrorCode (*setup)(PC));
PetscErrorCode PCShellSetDestroy(PC pc, PetscErrorCode (*destroy)(PC));
PetscErrorCode PCShellSetName(PC pc, const char *name);
PetscErrorCode PCSetUp(PC pc);
PetscErrorCode PCApply(PC pc, Vec x, Vec y);
PetscErrorCode PCDestroy(PC *pc);
/* the operators the PC was given (KSPSetOperators passes them on, as PETSc's KSP does) */
typedef enum { PC_LEFT = 0, PC_RIGHT = 1, PC_SYMMETRIC = 2 } PCSide;
PetscErrorCode PCSetOperators(PC pc, Mat Amat, Mat Pmat);
PetscErrorCode PCGetOperators(PC pc, Mat *Amat, Mat *Pmat);
/* y = B A x (left) or A B x (right), work a scratch Vec: the shell's applyBA callback when set
 * (PCShellSetApplyBA), else MatMult and PCApply with pc's Amat (PETSc's PCApplyBAorAB) */
PetscErrorCode PCShellSetApplyBA(PC pc, PetscErrorCode (*applyBA)(PC, PCSide, Vec, Vec, Vec));
PetscErrorCode PCApplyBAorAB(PC pc, PCSide side, Vec x, Vec y, Vec work);
/* not in PETSc: the stand-in KSP asks the next PCApply / PCApplyBAorAB of a shell for the dots
 * of its output y with device vectors, out[2 j + re/im] = v[j]^H y (v[j] == NULL: y itself), out a
 * device array; a shell that computed them (fused into its apply) sets done = PETSC_TRUE.
 * PCMiniSetApplyDots(pc, NULL) withdraws the request. */
typedef struct {
  PetscInt nv;
  const PetscScalar *v[8];
  double *out;
  PetscBool done;
} PCMiniApplyDots;
PetscErrorCode PCMiniSetApplyDots(PC pc, PCMiniApplyDots *req);
PetscErrorCode PCMiniGetApplyDots(PC pc, PCMiniApplyDots **req);

/* ---- KSP: GMRES(restart) with PETSc's defaults (restart 30, left preconditioning,
 * classical Gram-Schmidt without refinement, preconditioned residual norm, convergence when
 * ||r_k|| <= max(rtol ||r_0||, abstol), divergence when ||r_k|| > dtol ||r_0||) */
typedef struct _p_KSP *KSP;
typedef const char *KSPType;
#define KSPGMRES "gmres"
#define KSPPREONLY "preonly"
typedef enum {
  KSP_CONVERGED_ITERATING = 0,
  KSP_CONVERGED_RTOL = 2,
  KSP_CONVERGED_ATOL = 3,
  KSP_CONVERGED_ITS = 4,
  KSP_CONVERGED_HAPPY_BREAKDOWN = 7,
  KSP_DIVERGED_ITS = -3,
  KSP_DIVERGED_DTOL = -4,
  KSP_DIVERGED_BREAKDOWN = -5
} KSPConvergedReason;
PetscErrorCode KSPCreate(MPI_Comm comm, KSP *ksp);
PetscErrorCode KSPSetType(KSP ksp, KSPType type);
PetscErrorCode KSPSetTolerances(KSP ksp, PetscReal rtol, PetscReal abstol, PetscReal dtol, PetscInt maxits);
PetscErrorCode KSPGMRESSetRestart(KSP ksp, PetscInt restart);
PetscErrorCode KSPSetPCSide(KSP ksp, PCSide side);
PetscErrorCode KSPSetInitialGuessNonzero(KSP ksp, PetscBool flg);
PetscErrorCode KSPGetPC(KSP ksp, PC *pc);
PetscErrorCode KSPSetOperators(KSP ksp, Mat A, Mat P);
PetscErrorCode KSPSetUp(KSP ksp);
/* GMRES with a zero initial guess does not zero x first (the first update overwrites it); an
 * error return before that update leaves x = 0, as PETSc's zeroed x would be. */
PetscErrorCode KSPSolve(KSP ksp, Vec b, Vec x);
PetscErrorCode KSPGetConvergedReason(KSP ksp, KSPConvergedReason *reason);
PetscErrorCode KSPGetIterationNumber(KSP ksp, PetscInt *its);
PetscErrorCode KSPGetResidualNorm(KSP ksp, PetscReal *rnorm);
PetscErrorCode KSPDestroy(KSP *ksp);
/* not in PETSc: the device time of the PCApply calls of the last KSPSolve (HIP events around
 * each call on the Vec stream; a device-Vec PCApply is stream-ordered there), and their count */
PetscErrorCode KSPMiniGetPCApplyStats(KSP ksp, PetscInt *calls, PetscLogDouble *seconds);
/* not in PETSc: whether the solver asks a shell PC for the Gram-Schmidt dots and residual norms
 * of its output (PCMiniApplyDots; default PETSC_TRUE) */
PetscErrorCode KSPMiniSetFusion(KSP ksp, PetscBool on);
/* not in PETSc: in the last KSPSolve, how many Gram-Schmidt steps took their dots, and how many
 * restarts their residual norm, from the shell's apply (PCMiniApplyDots) */
PetscErrorCode KSPMiniGetFusedCounts(KSP ksp, PetscInt *dots, PetscInt *norms);
/* not in PETSc: allocate the GMRES work vectors now (duplicates of v) instead of in the first
 * KSPSolve, so a timed solve does not include their allocation */
PetscErrorCode KSPMiniSetUpWork(KSP ksp, Vec v);

#ifdef __cplusplus
}
#endif
#endif /* CFP_WITH_PETSC */
#endif /* CFP_PETSC_MINI_H */
