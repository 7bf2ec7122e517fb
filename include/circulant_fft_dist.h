/*
 * circulant_fft_dist.h -- slab-decomposed circulant FFT preconditioner over several GPUs.
 *
 * Layout: rank r of P owns the z-planes [r*nz/P, (r+1)*nz/P) of the
 * x-fastest grid, i.e. the contiguous rows [r*N/P, (r+1)*N/P) -- exactly PETSc's
 * PETSC_DECIDE distribution of VecCreateMPI (tests/TransportEquationFFT_..._mpi.cxx:66) and
 * FFTW-MPI's local_n0 slabs of MATFFTW (src/PCSHELLFft_3D.cxx:34-35).  Requires P | nz; ny
 * is split into blocks of ceil(ny / P) rows for the z pass, as FFTW-MPI splits its transposed
 * dimension (cfp_slab_layout), so P need not divide ny.
 *
 * One apply = x-fwd, y-fwd (written straight into per-peer send chunks), all-to-all,
 * z: DFT ./Diag IDFT, all-to-all back, y-inv (read straight from the received chunks),
 * x-inv * 1/N.  Two all-to-alls per apply (FFTW-MPI's non-transposed plans need four).
 * Diag is generated per rank from lambda and global frequency indices (no communication).
 *
 * Pipelining ("pieces", cfp_dist_plan_set_pieces): with K > 1 each all-to-all is cut into K
 * pieces along the local z-planes (block k of every per-peer chunk is contiguous); piece k of
 * the forward exchange leaves as soon as block k's x and y passes are done, and block k's
 * inverse passes start as soon as piece k of the backward exchange is in.  The exchanges run on
 * a second stream, ordered by events.  Every executor runs the same step list.
 *
 * Executors:
 *   cfp_dist_plan_*   one process per GPU: RCCL (ncclSend/ncclRecv in a group) over xGMI, or
 *                     the caller's exchange callback, or step by step (the caller runs the
 *                     exchanges between cfp_dist_plan_run_step calls);
 *   cfp_group_*       one process driving P slabs (on one or several GPUs) with device
 *                     copies as the exchange -- a single-process multi-GPU mode and the way
 *                     the slab layouts are exercised on a one-GPU machine.
 */
#ifndef CIRCULANT_FFT_DIST_H
#define CIRCULANT_FFT_DIST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfp_dist_plan_s *cfp_dist_plan_t;
typedef struct cfp_group_s *cfp_group_t;

/* host-only layout query: out[0..8) = {nz_local, ny_local, z0, y0, local_size,
 * chunk (elements per peer message), local_offset (global index of the first local element),
 * nranks}.  nranks must divide nz (whole z-planes: PETSC_DECIDE rows); ny is split as FFTW-MPI
 * splits its transposed dimension, in blocks of ceil(ny / nranks) rows: rank r transforms the
 * z-pencil rows [y0, y0 + ny_local) with y0 = r ceil(ny / nranks), and the last ranks may hold
 * fewer rows (or none).  chunk = nz_local * ceil(ny / nranks) * nx (padded rows included). */
int cfp_slab_layout(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int64_t *out);
/* elements of one work buffer of the slab plan: max(local_size, nranks * chunk) (they differ
 * when nranks does not divide ny); cfp_dist_plan_set_work_buffers takes buffers of this size */
int cfp_slab_work_size(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int64_t *n);

/* Host-only description of rank `rank`'s step list (no GPU needed; tests replay it on the CPU
 * across processes).  schedule: CFP_SCHEDULE_AUTO / _FIVE_PASS / _THREE_PASS (AUTO resolves as
 * the plan does); pieces: 0 = AUTO (as the plan), else K | nz/nranks; list: what the steps
 * compute.  desc[0..CFP_SLAB_DESC_LEN):
 *   [0] kind: 0 axis pass, 1 exchange piece, 2 3-sweep stage, 3 repack (natural <-> chunks)
 *   [1] source buffer, [2] destination buffer (0 = b, 1 = x, 2 = work W, 3 = work W2,
 *       4 = the z-pencil Diag)
 *   [3] axis (pass) | stage (3-sweep) | to_chunks (repack), [4] length n, [5] mode (PASS_*:
 *       0 fwd, 1 inv, 2 fused with the separable symbol, 3 fused with the explicit Diag, 5-7
 *       the 3-sweep stages), [6] columns (pass) | local z-planes (3-sweep P1/P3, repack),
 *   [7] inner_n, then for the source and the destination side: inner_stride, outer_stride,
 *       pt_stride, seg_len, seg_stride ([8..13), [13..18)),
 *   [18] source offset, [19] destination offset (elements: the step's base in its buffers),
 *   [20] piece offset, [21] piece count (exchange: peer q gets src[q*chunk + off, + count) and
 *        stores it at dst[rank*chunk + off]), [22] chunk (elements per peer per exchange),
 *   [23] the step (on the other stream) this one waits for, or -1,
 *   [24] log2 rows per chunk, [25] first global k1 (3-sweep P2), [26] segment (0 before the
 *        first exchange, 1 between, 2 after), [27] symbol (1 separable, 2 explicit Diag).
 * Element (column g, point k) of a pass side sits at base + (g % inner_n) * inner_stride
 *   + (g / inner_n) * outer_stride + (k / seg_len) * seg_stride + (k % seg_len) * pt_stride.
 * *scale = the factor the step applies to its output (1/N on the last launch of each block). */
#define CFP_SLAB_DESC_LEN 28
#define CFP_SLAB_LIST_APPLY 0      /* the apply with the separable symbol */
#define CFP_SLAB_LIST_APPLY_DIAG 1 /* the apply with an explicit Diag */
#define CFP_SLAB_LIST_FORWARD 2    /* unnormalised forward 3-D DFT, natural order out */
#define CFP_SLAB_LIST_BACKWARD 3   /* unnormalised backward 3-D DFT */
#define CFP_SLAB_LIST_DIAG 4       /* Diag slab -> z-pencil copy (cfp_dist_plan_set_diag) */
int cfp_slab_steps_count(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int schedule, int pieces,
                         int list, int *nsteps);
int cfp_slab_steps_get(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int schedule, int pieces, int list,
                       int step, int64_t *desc, double *scale);
/* Round-2 form: the FIVE_PASS apply list with one piece, desc[0..18) as above. */
int cfp_slab_num_steps(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int *nsteps);
int cfp_slab_step_info(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int step, int64_t *desc,
                       double *scale);

/* RCCL unique id (128 bytes): created on rank 0, broadcast by the caller, passed to every rank */
int cfp_dist_unique_id_bytes(void);
int cfp_dist_get_unique_id(char *id_out);

/* The plan's own communicator is created non-blocking (ncclCommInitRankConfig, blocking = 0) and
 * polled against a deadline (unless CFP_RCCL_BLOCKING is set, see cfp_rccl_blocking): a rank that never joins returns CFP_ERR_LIB ("timed out") instead
 * of hanging.  cfp_dist_plan_create uses 300 s; _timeout takes the deadline in seconds.  The
 * same deadline bounds each exchange's enqueue and the finalize in cfp_dist_plan_destroy.
 * Replaces FFTW-MPI's plan creation inside MatCreateFFT(PETSC_COMM_WORLD, ...)
 * (src/PCSHELLFft_3D.cxx:34-35). */
int cfp_dist_plan_create(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                         const char *unique_id, int device);
int cfp_dist_plan_create_timeout(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                                 const char *unique_id, int device, double timeout_s);
/* What RCCL the plan talks through: ncclCommCount / ncclCommUserRank of its communicator (0 / -1
 * for a plan without one), ncclGetVersion, the communicator's creation time (ms), and the path
 * of the shared object that defines the RCCL entry points the library binds (any output may be
 * NULL; lib_path gets at most path_len bytes). */
int cfp_dist_plan_rccl_info(cfp_dist_plan_t plan, int *nranks, int *rank, int *version, double *init_ms,
                            char *lib_path, int path_len);
/* Host-only, no GPU: 1 when CFP_RCCL_BLOCKING (environment, read once per process) selects the
 * blocking protocol for the library's communicators (ncclCommInitRank with no deadline,
 * ncclCommDestroy), 0 for the default non-blocking creation polled against the deadline. */
int cfp_rccl_blocking(int *blocking);
/* Host-only, no GPU: the RCCL version and library this process resolved. */
int cfp_rccl_version(int *version, char *lib_path, int path_len);
/* Same on the caller's RCCL communicator (an ncclComm_t of nranks ranks; it stays the caller's). */
int cfp_dist_plan_create_with_comm(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                                   void *nccl_comm, int device);
int cfp_dist_plan_destroy(cfp_dist_plan_t plan);
/* Same plan without a communicator.  The caller performs the exchanges itself, either
 *   - inside cfp_dist_plan_apply, through a callback (cfp_dist_plan_set_exchange), or
 *   - step by step: for i < cfp_dist_plan_num_steps, cfp_dist_plan_step(i) describes step i
 *     (desc as cfp_slab_steps_get); a kernel step is enqueued by cfp_dist_plan_run_step, an
 *     exchange piece is the caller's all-to-all between the named buffers, or
 *   - (one piece only) run_segment(0); alltoall(work -> x); run_segment(1);
 *     alltoall(x -> work); run_segment(2) (equal splits of `chunk` values per peer). */
int cfp_dist_plan_create_external(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                                  int device);
/* The caller's exchange of one piece: for every peer q (q = rank included), send
 * src_dev[q*chunk + off, + count) to rank q, which stores it at dst_dev[rank*chunk + off]
 * (complex values; device pointers), stream-ordered on `stream`.  Returns 0 on success. */
typedef int (*cfp_dist_exchange_fn)(void *user, const double *src_dev, double *dst_dev, int64_t chunk, int64_t off,
                                    int64_t count, void *stream);
int cfp_dist_plan_set_exchange(cfp_dist_plan_t plan, cfp_dist_exchange_fn fn, void *user);
int cfp_dist_plan_work_buffer(cfp_dist_plan_t plan, double **work_dev);
int cfp_dist_plan_set_work_buffer(cfp_dist_plan_t plan, double *work_dev); /* caller-owned, cfp_slab_work_size values */
/* both work buffers (W, W2: the second is used by pieces > 1, padded layouts and the transforms;
 * NULL keeps the plan's own, allocated on first use), cfp_slab_work_size complex values each */
int cfp_dist_plan_set_work_buffers(cfp_dist_plan_t plan, double *work_dev, double *work2_dev);
int cfp_dist_plan_run_segment(cfp_dist_plan_t plan, int segment, const double *b_dev, double *x_dev, void *stream);
int cfp_dist_plan_num_steps(cfp_dist_plan_t plan, int *nsteps);
int cfp_dist_plan_step(cfp_dist_plan_t plan, int step, int64_t *desc);
int cfp_dist_plan_run_step(cfp_dist_plan_t plan, int step, const double *b_dev, double *x_dev, void *stream);
int cfp_dist_plan_set_symbol_transport(cfp_dist_plan_t plan, const double lam[6]);
/* Explicit Diag: this rank's natural slab of it (local_size values, device).  A collective
 * (every rank calls it): the Diag is moved once into the z-pencil layout of the fused z pass,
 * and later applies divide by it until cfp_dist_plan_clear_diag.  (solve_3D with a Diag Vec.) */
int cfp_dist_plan_set_diag(cfp_dist_plan_t plan, const double *diag_local_dev, void *stream);
int cfp_dist_plan_clear_diag(cfp_dist_plan_t plan);
/* on != 0: divide by the last Diag given to cfp_dist_plan_set_diag again (no transpose);
 * 0: the separable symbol (as cfp_dist_plan_clear_diag) */
int cfp_dist_plan_use_diag(cfp_dist_plan_t plan, int on);
/* b_dev, x_dev: this rank's slab (local_size complex values); b may alias x */
int cfp_dist_plan_apply(cfp_dist_plan_t plan, const double *b_dev, double *x_dev, void *stream);
/* Unnormalised 3-D DFT of the distributed grid, this rank's natural slab in and out (MatMult /
 * MatMultTranspose of a distributed MATFFTW; FFTW-MPI's non-transposed layout).  in may not
 * alias out. */
int cfp_dist_plan_forward(cfp_dist_plan_t plan, const double *in_dev, double *out_dev, void *stream);
int cfp_dist_plan_backward(cfp_dist_plan_t plan, const double *in_dev, double *out_dev, void *stream);
int cfp_dist_plan_local_size(cfp_dist_plan_t plan, int64_t *local_size);
int cfp_dist_plan_num_phases(cfp_dist_plan_t plan, int *phases);
/* phase i: *is_exchange = 1 for an all-to-all piece, else 0 (axis pass); *axis, *n, *mode of a pass */
int cfp_dist_plan_phase_info(cfp_dist_plan_t plan, int phase, int *is_exchange, int *axis, int *n, int *mode);
/* mean ms of each phase (kernels and exchange pieces, in order, each on its own stream) over
 * `iters` applies */
int cfp_dist_plan_time_phases(cfp_dist_plan_t plan, const double *b_dev, double *x_dev, int iters, double *ms_out,
                              void *stream);
/* sampled per-phase HIP events inside the caller's own applies (cfp_plan_profile_begin's
 * contract: every `every`-th apply, at most max_applies; _end writes the mean ms per phase) */
int cfp_dist_plan_profile_begin(cfp_dist_plan_t plan, int max_applies, int every);
int cfp_dist_plan_profile_end(cfp_dist_plan_t plan, double *ms_out, int *applies);
/* local passes of each rank: CFP_SCHEDULE_AUTO (3 sweeps -- x + y1 | y2 + z + symbol + inverses |
 * inverse, cfp_three_pass.hip -- for a 256^3 or 512^3 grid with nranks | 32, nranks <= 16; else
 * 5 axis passes),
 * CFP_SCHEDULE_FIVE_PASS, or CFP_SCHEDULE_THREE_PASS (CFP_ERR_SUP where unsupported).  The
 * exchanges and the per-peer chunk layout are the same for both. */
int cfp_dist_plan_set_schedule(cfp_dist_plan_t plan, int schedule);
/* pipeline depth: 0 = AUTO (1 on one rank or under 64 MiB per rank, else 4, or 2 where 4 does
 * not divide the local planes), else K | nz / nranks */
int cfp_dist_plan_set_pieces(cfp_dist_plan_t plan, int pieces);
int cfp_dist_plan_pieces(cfp_dist_plan_t plan, int *pieces);

/* single-process group of P slabs; devices[r] = HIP device of slab r (may repeat) */
int cfp_group_create(cfp_group_t *group, int64_t nx, int64_t ny, int64_t nz, int nranks, const int *devices);
int cfp_group_destroy(cfp_group_t group);
int cfp_group_set_symbol_transport(cfp_group_t group, const double lam[6]);
/* b_devs[r], x_devs[r]: slab r on devices[r]; synchronous */
int cfp_group_apply(cfp_group_t group, const double *const *b_devs, double *const *x_devs);
int cfp_group_set_schedule(cfp_group_t group, int schedule); /* as cfp_dist_plan_set_schedule */
int cfp_group_set_pieces(cfp_group_t group, int pieces);     /* as cfp_dist_plan_set_pieces */

#ifdef __cplusplus
}
#endif
#endif /* CIRCULANT_FFT_DIST_H */
