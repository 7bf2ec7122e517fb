/*
 * circulant_fft_dist.h -- slab-decomposed circulant FFT preconditioner over several GPUs.
 *
 * Layout: rank r of P owns the z-planes [r*nz/P, (r+1)*nz/P) of the
 * x-fastest grid, i.e. the contiguous rows [r*N/P, (r+1)*N/P) -- exactly PETSc's
 * PETSC_DECIDE distribution of VecCreateMPI (tests/TransportEquationFFT_..._mpi.cxx:66) and
 * FFTW-MPI's local_n0 slabs of MATFFTW (src/PCSHELLFft_3D.cxx:34-35).  Requires P | nz and
 * P | ny.
 *
 * One apply = x-fwd, y-fwd (written straight into per-peer send chunks), all-to-all,
 * z: DFT ./Diag IDFT, all-to-all back, y-inv (read straight from the received chunks),
 * x-inv * 1/N.  Two all-to-alls per apply (FFTW-MPI's non-transposed plans need four).
 * Diag is generated per rank from lambda and global frequency indices (no communication).
 *
 * Two executors share the same pass schedule:
 *   cfp_dist_plan_*   one process per GPU, RCCL (ncclSend/ncclRecv in a group) over xGMI;
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
 * nranks} */
int cfp_slab_layout(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int64_t *out);

/* Host-only description of rank `rank`'s apply: the steps cfp_dist_plan_apply runs, in order
 * (no GPU needed; tests replay them on the CPU across processes).  desc[0..18):
 *   [0] kind (0 axis pass, 1 all-to-all), [1] source buffer, [2] destination buffer
 *   (0 = b, 1 = x, 2 = the plan's work buffer), [3] axis, [4] length n, [5] mode (PASS_*: 0 fwd,
 *   1 inv, 2 fused with the separable symbol), [6] columns, [7] inner_n, then for the source and
 *   the destination side: inner_stride, outer_stride, pt_stride, seg_len, seg_stride.
 * Element (column g, point k) of a side sits at
 *   (g % inner_n) * inner_stride + (g / inner_n) * outer_stride
 *   + (k / seg_len) * seg_stride + (k % seg_len) * pt_stride.
 * *scale = the factor the step applies to its output (1/N on the last pass).  An all-to-all
 * sends chunk q (elements [q*chunk, (q+1)*chunk)) of the source to rank q, which stores it as
 * chunk `rank` of its destination. */
int cfp_slab_num_steps(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int *nsteps);
int cfp_slab_step_info(int64_t nx, int64_t ny, int64_t nz, int nranks, int rank, int step, int64_t *desc,
                       double *scale);

/* RCCL unique id (128 bytes): created on rank 0, broadcast by the caller, passed to every rank */
int cfp_dist_unique_id_bytes(void);
int cfp_dist_get_unique_id(char *id_out);

int cfp_dist_plan_create(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                         const char *unique_id, int device);
int cfp_dist_plan_destroy(cfp_dist_plan_t plan);
/* Same plan without a communicator: the caller runs the three kernel segments and performs
 * the two all-to-alls in between with its own collective library:
 *   run_segment(0); alltoall(work -> x); run_segment(1); alltoall(x -> work); run_segment(2)
 * (equal splits of `chunk` complex values per peer, peer order = rank order). */
int cfp_dist_plan_create_external(cfp_dist_plan_t *plan, int64_t nx, int64_t ny, int64_t nz, int nranks, int rank,
                                  int device);
int cfp_dist_plan_work_buffer(cfp_dist_plan_t plan, double **work_dev);
int cfp_dist_plan_set_work_buffer(cfp_dist_plan_t plan, double *work_dev); /* caller-owned, local_size values */
int cfp_dist_plan_run_segment(cfp_dist_plan_t plan, int segment, const double *b_dev, double *x_dev, void *stream);
int cfp_dist_plan_set_symbol_transport(cfp_dist_plan_t plan, const double lam[6]);
/* b_dev, x_dev: this rank's slab (local_size complex values); b may alias x */
int cfp_dist_plan_apply(cfp_dist_plan_t plan, const double *b_dev, double *x_dev, void *stream);
int cfp_dist_plan_local_size(cfp_dist_plan_t plan, int64_t *local_size);
int cfp_dist_plan_num_phases(cfp_dist_plan_t plan, int *phases);
/* phase i: *is_exchange = 1 for an all-to-all, else 0 (axis pass); *axis, *n, *mode of a pass */
int cfp_dist_plan_phase_info(cfp_dist_plan_t plan, int phase, int *is_exchange, int *axis, int *n, int *mode);
/* mean ms of each phase (kernels and exchanges, in order) over `iters` applies */
int cfp_dist_plan_time_phases(cfp_dist_plan_t plan, const double *b_dev, double *x_dev, int iters, double *ms_out,
                              void *stream);
/* sampled per-phase HIP events inside the caller's own applies (cfp_plan_profile_begin's
 * contract: every `every`-th apply, at most max_applies; _end writes the mean ms per phase) */
int cfp_dist_plan_profile_begin(cfp_dist_plan_t plan, int max_applies, int every);
int cfp_dist_plan_profile_end(cfp_dist_plan_t plan, double *ms_out, int *applies);
/* local passes of each rank: CFP_SCHEDULE_AUTO (3 sweeps -- x + y1 | y2 + z + symbol + inverses |
 * inverse, cfp_three_pass.hip -- for a 256^3 grid with nranks <= 4, else 5 axis passes; 3 sweeps
 * are available up to nranks = 16, nranks | 32),
 * CFP_SCHEDULE_FIVE_PASS, or CFP_SCHEDULE_THREE_PASS (CFP_ERR_SUP where unsupported).  The
 * exchanges and the per-peer chunk layout are the same for both. */
int cfp_dist_plan_set_schedule(cfp_dist_plan_t plan, int schedule);

/* single-process group of P slabs; devices[r] = HIP device of slab r (may repeat) */
int cfp_group_create(cfp_group_t *group, int64_t nx, int64_t ny, int64_t nz, int nranks, const int *devices);
int cfp_group_destroy(cfp_group_t group);
int cfp_group_set_symbol_transport(cfp_group_t group, const double lam[6]);
/* b_devs[r], x_devs[r]: slab r on devices[r]; synchronous */
int cfp_group_apply(cfp_group_t group, const double *const *b_devs, double *const *x_devs);
int cfp_group_set_schedule(cfp_group_t group, int schedule); /* as cfp_dist_plan_set_schedule */

#ifdef __cplusplus
}
#endif
#endif /* CIRCULANT_FFT_DIST_H */
