// wave_system.cpp -- the wave-system operator on a Cartesian grid, the block-circulant PCSHELL
// and the implicit GMRES time loop (include/wave_system.h).
//
//   cfp_wave_csr                    computeDivergenceMatrix + jacobianMatrices,
//                                   src/WaveSystem.cxx:92-176
//   initial_conditions_shock_wave   src/WaveSystem.cxx:25-76
//   WaveSystemGMRES                 WaveSystem_impl_seq, tests/WaveSystem_SphericalExplosion_
//                                   impl_seq.cxx:11-150 (GMRES rtol = abstol = 1e-5, 1000 its),
//                                   with the block-circulant PCSHELL in place of PCILU
#ifndef CFP_WITH_PETSC
#include <sys/time.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/circulant_fft_dist.h"
#include "../../include/transport_equation.h"
#include "../../include/wave_system.h"
#include "cfp_fft_device.h"
#include "pcshell_common.h"

using namespace cfp_pc;

namespace {
const int kC = 4;  // most unknowns per cell (3-D: pressure, 3 momentum components)

double wall() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

// jacobianMatrices(normal = s e_d, coeff = kappa): (A(n) - |A(n)|) kappa / 2,
// A(n) = [[0, c0^2 n^T], [n, 0]], |A(n)| = diag(c0, c0 n n^T)   (src/WaveSystem.cxx:92-107)
void jacobian_minus(int d, int s, double kappa, double c0, double Am[kC][kC]) {
  for (int r = 0; r < kC; ++r)
    for (int c = 0; c < kC; ++c) Am[r][c] = 0.0;
  const double h = 0.5 * kappa;
  Am[0][0] = -h * c0;
  Am[0][1 + d] = h * c0 * c0 * s;
  Am[1 + d][0] = h * s;
  Am[1 + d][1 + d] = -h * c0;
}

struct Entry {
  int64_t col;
  double val;
};
}  // namespace

extern "C" int cfp_wave_csr_dim(int64_t nx, int64_t ny, int64_t nz, int dim, const double h[3], double dt, double c0,
                                int bc, double shift, int64_t* rowptr, int64_t* col, double* val, int64_t* nnz) {
  if (!h || !rowptr || !col || !val || !nnz) return CFP_ERR_ARG_NULL;
  if (nx < 1 || ny < 1 || nz < 1 || h[0] <= 0 || h[1] <= 0 || h[2] <= 0 || !(c0 > 0)) return CFP_ERR_ARG_OUTOFRANGE;
  if (bc != CFP_WAVE_BC_WALL && bc != CFP_WAVE_BC_PERIODIC && bc != CFP_WAVE_BC_NEUMANN) return CFP_ERR_ARG_OUTOFRANGE;
  if (dim < 1 || dim > 3) return CFP_ERR_ARG_OUTOFRANGE;
  if ((dim < 3 && nz != 1) || (dim < 2 && ny != 1)) return CFP_ERR_ARG_SIZ;
  const int C = dim + 1;  // nbComp (src/WaveSystem.cxx:113)
  const int64_t n[3] = {nx, ny, nz};
  int64_t p = 0;
  rowptr[0] = 0;
  // one cell at a time: its (at most 2 dim + 1) coupled cells and their C x C blocks
  std::vector<Entry> row[kC];
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j)
      for (int64_t i = 0; i < nx; ++i) {
        const int64_t cell = i + nx * (j + ny * k);
        const int64_t idx[3] = {i, j, k};
        double self[kC][kC];
        for (int r = 0; r < kC; ++r)
          for (int c = 0; c < kC; ++c) self[r][c] = r == c ? shift : 0.0;
        for (int r = 0; r < kC; ++r) row[r].clear();
        for (int d = 0; d < dim; ++d) {  // a dim-D mesh has faces along its dim axes only
          const double kappa = dt / h[d];  // dt |F| / |C|
          for (int s = -1; s <= 1; s += 2) {
            double Am[kC][kC];
            jacobian_minus(d, s, kappa, c0, Am);
            const bool border = s < 0 ? idx[d] == 0 : idx[d] == n[d] - 1;
            int64_t other = -1;
            if (!border) {
              other = cell + s * (d == 0 ? 1 : (d == 1 ? nx : nx * ny));
            } else if (bc == CFP_WAVE_BC_PERIODIC) {
              const int64_t wrap = s < 0 ? n[d] - 1 : 0;
              int64_t o[3] = {i, j, k};
              o[d] = wrap;
              other = o[0] + nx * (o[1] + ny * o[2]);
            } else if (bc == CFP_WAVE_BC_WALL) {
              // -Am (2 v v^T), v = (0, n): only column 1+d is hit (src/WaveSystem.cxx:148-155)
              for (int r = 0; r < C; ++r) self[r][1 + d] -= 2.0 * Am[r][1 + d];
              continue;
            } else {
              continue;  // Neumann: nothing
            }
            for (int r = 0; r < C; ++r)
              for (int c = 0; c < C; ++c) {
                if (Am[r][c] == 0.0) continue;
                row[r].push_back({other * C + c, Am[r][c]});  // addValue(j, other, Am)
                self[r][c] -= Am[r][c];                         // addValue(j, j, -Am)
              }
          }
        }
        for (int r = 0; r < C; ++r) {
          for (int c = 0; c < C; ++c)
            if (self[r][c] != 0.0 || c == r) row[r].push_back({cell * C + c, self[r][c]});
          std::vector<Entry>& e = row[r];
          std::sort(e.begin(), e.end(), [](const Entry& a, const Entry& b) { return a.col < b.col; });
          // merge duplicates (periodic wrap on a 1- or 2-cell axis), keep the diagonal
          int64_t start = p;
          for (size_t q = 0; q < e.size(); ++q) {
            if (p > start && col[p - 1] == e[q].col) {
              val[2 * (p - 1)] += e[q].val;
            } else {
              col[p] = e[q].col;
              val[2 * p] = e[q].val;
              val[2 * p + 1] = 0.0;
              ++p;
            }
          }
          // drop exact zeros except the diagonal
          int64_t w = start;
          for (int64_t q = start; q < p; ++q) {
            if (val[2 * q] != 0.0 || col[q] == cell * C + r) {
              col[w] = col[q];
              val[2 * w] = val[2 * q];
              val[2 * w + 1] = 0.0;
              ++w;
            }
          }
          p = w;
          rowptr[cell * C + r + 1] = p;
        }
      }
  *nnz = p;
  return CFP_SUCCESS;
}

extern "C" int cfp_wave_csr(int64_t nx, int64_t ny, int64_t nz, const double h[3], double dt, double c0, int bc,
                            double shift, int64_t* rowptr, int64_t* col, double* val, int64_t* nnz) {
  return cfp_wave_csr_dim(nx, ny, nz, 3, h, dt, c0, bc, shift, rowptr, col, val, nnz);
}

extern "C" PetscErrorCode computeDivergenceMatrixWaveCartesianDim(PetscInt nx, PetscInt ny, PetscInt nz, PetscInt dim,
                                                                  const PetscReal h[3], PetscReal dt, PetscReal c0,
                                                                  PetscInt bc, Mat* A) {
  PetscFunctionBeginUser;
  PetscCheck(A && h, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "computeDivergenceMatrixWaveCartesian: NULL argument");
  PetscCheck(nx >= 1 && ny >= 1 && nz >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  PetscCheck(dim >= 1 && dim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  const int C = (int)dim + 1;
  const int64_t M = C * nx * ny * nz;
  const int64_t room = (int64_t)C * C * (2 * dim + 1);
  std::vector<int64_t> rowptr((size_t)M + 1), col((size_t)(nx * ny * nz * room));
  std::vector<PetscScalar> val((size_t)(nx * ny * nz * room));
  int64_t nnz = 0;
  const int rc = cfp_wave_csr_dim(nx, ny, nz, (int)dim, h, dt, c0, (int)bc, 0.0, rowptr.data(), col.data(),
                                  reinterpret_cast<double*>(val.data()), &nnz);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, "computeDivergenceMatrixWaveCartesian: bad arguments");
  PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, M, M, rowptr.data(), col.data(), val.data(), A));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// the same on a communicator (MatCreateAIJ on PETSC_COMM_WORLD as the reference's MPI wave driver,
// tests/WaveSystem_SphericalExplosion_impl_mpi.cxx:83-85): every rank sets its own rows
extern "C" PetscErrorCode computeDivergenceMatrixWaveCartesianAIJ(MPI_Comm comm, PetscInt nx, PetscInt ny, PetscInt nz,
                                                                  PetscInt dim, const PetscReal h[3], PetscReal dt,
                                                                  PetscReal c0, PetscInt bc, Mat* A) {
  PetscFunctionBeginUser;
  PetscCheck(A && h, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "computeDivergenceMatrixWaveCartesianAIJ: NULL argument");
  PetscCheck(dim >= 1 && dim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  const int C = (int)dim + 1;
  const int64_t M = C * nx * ny * nz;
  const int64_t room = (int64_t)C * C * (2 * dim + 1);
  std::vector<int64_t> rowptr((size_t)M + 1), col((size_t)(nx * ny * nz * room));
  std::vector<PetscScalar> val((size_t)(nx * ny * nz * room));
  int64_t nnz = 0;
  const int rc = cfp_wave_csr_dim(nx, ny, nz, (int)dim, h, dt, c0, (int)bc, 0.0, rowptr.data(), col.data(),
                                  reinterpret_cast<double*>(val.data()), &nnz);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, "computeDivergenceMatrixWaveCartesianAIJ: bad arguments");
  PetscCall(MatCreateAIJ(comm, PETSC_DECIDE, PETSC_DECIDE, M, M, (PetscInt)room, NULL, (PetscInt)room, NULL, A));
  PetscInt lo, hi;
  PetscCall(MatGetOwnershipRange(*A, &lo, &hi));
  for (PetscInt r = lo; r < hi; ++r)
    PetscCall(MatSetValues(*A, 1, &r, rowptr[(size_t)r + 1] - rowptr[(size_t)r], col.data() + rowptr[(size_t)r],
                           val.data() + rowptr[(size_t)r], ADD_VALUES));
  PetscCall(MatAssemblyBegin(*A, MAT_FINAL_ASSEMBLY));
  PetscCall(MatAssemblyEnd(*A, MAT_FINAL_ASSEMBLY));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode computeDivergenceMatrixWaveCartesian(PetscInt nx, PetscInt ny, PetscInt nz,
                                                               const PetscReal h[3], PetscReal dt, PetscReal c0,
                                                               PetscInt bc, Mat* A) {
  return computeDivergenceMatrixWaveCartesianDim(nx, ny, nz, 3, h, dt, c0, bc, A);
}

extern "C" PetscErrorCode initial_conditions_shock_wave(PetscInt nx, PetscInt ny, PetscInt nz, const PetscReal xmin[3],
                                                        const PetscReal xmax[3], Vec U) {
  PetscFunctionBeginUser;
  PetscCheck(xmin && xmax, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL domain bounds");
  PetscInt n, ng, lo;
  PetscCall(VecGetSize(U, &ng));
  PetscCall(VecGetLocalSize(U, &n));
  PetscCall(VecGetOwnershipRange(U, &lo, NULL));
  const PetscInt N = nx * ny * nz;
  PetscCheck(N >= 1 && ng % N == 0 && ng / N >= 2 && ng / N <= kC, PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ,
             "U size is not (dim+1)*nx*ny*nz with dim = 1, 2 or 3");
  const int C = (int)(ng / N), dim = C - 1;  // nbComp = dim + 1
  const double hx = (xmax[0] - xmin[0]) / (double)nx, hy = (xmax[1] - xmin[1]) / (double)ny,
               hz = (xmax[2] - xmin[2]) / (double)nz;
  const double cx = (xmin[0] + xmax[0]) / 2, cy = (xmin[1] + xmax[1]) / 2, cz = (xmin[2] + xmax[2]) / 2;
  PetscScalar* u;
  PetscCall(VecGetArrayWrite(U, &u));
  // this rank's rows; PETSC_DECIDE may split a cell's d+1 unknowns between two ranks
  for (PetscInt cell = lo / C; cell * C < lo + n; ++cell) {
    const PetscInt i = cell % nx, j = (cell / nx) % ny, k = cell / (nx * ny);
    const double x = xmin[0] + (i + 0.5) * hx, y = xmin[1] + (j + 0.5) * hy, z = xmin[2] + (k + 0.5) * hz;
    // src/WaveSystem.cxx:48-61: y enters r for dim > 1, z for dim == 3 (a single cell
    // layer's centre is the domain centre, so a 3-D grid with n = 1 adds 0)
    double r2 = (x - cx) * (x - cx);
    if (dim > 1 && ny > 1) r2 += (y - cy) * (y - cy);
    if (dim == 3 && nz > 1) r2 += (z - cz) * (z - cz);
    for (int d = 0; d < C; ++d) {  // pressure, then rho0 * velocity (velocity = 0)
      const int64_t row = C * cell + d;
      if (row >= lo && row < lo + n) u[row - lo] = d == 0 ? (std::sqrt(r2) < 0.3 ? 155e5 : 70e5) : 0.0;
    }
  }
  PetscCall(VecRestoreArrayWrite(U, &u));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// ------------------------------------------------------------------ PCSHELL
// Several ranks (the reference's MPI wave driver, tests/WaveSystem_SphericalExplosion_impl_mpi.cxx:
// 63,83-85,130: Vecs of PETSC_DECIDE rows on PETSC_COMM_WORLD, (d+1) N rows, i.e. whole z-planes of
// cells when P | n_z; whole rows of cells of a 2-D grid when P | n_y): the block-circulant inverse
// on the z-slab plan of pcshell_common.h.  Per apply: the interleaved cells split into d+1
// component slabs, each one's distributed DFT (the slab plan's forward transform, two all-to-alls
// through the communicator), the (d+1)x(d+1) solve per frequency on the local slab of the
// spectrum (global frequency from the rank's first plane), each component's backward transform,
// and the components interleaved again x 1/N.  A 2-D grid (n_x, n_y) runs as the plan grid
// (1, n_x, n_y): the same memory order, its rows split over the ranks.
struct WaveDist {
  SlabBacking slab;
  int ncomp = 4;               // d + 1 interleaved unknowns per cell
  int64_t pd[3] = {0, 0, 0};   // the slab plan's grid: (n_x, n_y, n_z), or (1, n_x, n_y) for d = 2
  int64_t nloc = 0, z0 = 0;    // local cells, first global plane of the plan's slowest axis
  cfp::cd* buf = nullptr;      // 2 x (d + 1) component slabs of nloc values
  double2* tab = nullptr;      // (p, q) per physical axis: [n_x | n_y | n_z]
  double c0sq = 0.0;
};
std::mutex g_wave_mu;
std::unordered_map<const void*, WaveDist*> g_wave_dist;

WaveDist* wave_dist(const FFTPrecWaveContext* ctx) {
  std::lock_guard<std::mutex> g(g_wave_mu);
  auto it = g_wave_dist.find(ctx);
  return it == g_wave_dist.end() ? nullptr : it->second;
}
void wave_dist_free(const FFTPrecWaveContext* ctx) {
  WaveDist* w = nullptr;
  {
    std::lock_guard<std::mutex> g(g_wave_mu);
    auto it = g_wave_dist.find(ctx);
    if (it == g_wave_dist.end()) return;
    w = it->second;
    g_wave_dist.erase(it);
  }
  slab_destroy(&w->slab);
  if (w->buf) hipFree(w->buf);
  if (w->tab) hipFree(w->tab);
  delete w;
}

template <int C>
__global__ void k_wave_split(const cfp::cd* b, cfp::cd* u, int64_t n) {  // u[c n + i] = b[C i + c]
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#pragma unroll
    for (int c = 0; c < C; ++c) u[c * n + i] = b[C * i + c];
}
template <int C>
__global__ void k_wave_join(const cfp::cd* u, cfp::cd* x, int64_t n, double sc) {  // x[C i + c] = sc u[c n + i]
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#pragma unroll
    for (int c = 0; c < C; ++c) x[C * i + c] = cfp::make_cd(sc * u[c * n + i].x, sc * u[c * n + i].y);
}
// v <- S(k)^-1 v on the local slab of the spectrum.  Point i of the slab is (i0, i1, z0 + i2) on
// the plan's grid pd; its physical frequency is that for d = 3, and (i1, z0 + i2, 0) for d = 2
// (the 2-D grid runs as the plan grid (1, n_x, n_y), the same memory order).  A 2-D cell has no
// z velocity: r[3] = 0 and n_z = 1 gives (p, q) = (0, 0) on that axis, so wave_solve's 4x4 algebra
// reduces to the 3x3 block.
template <int C>
__global__ void k_wave_slab_solve(cfp::cd* v, int64_t n, int64_t pd0, int64_t pd1, int64_t z0, int64_t nx,
                                  int64_t ny, const double2* tab, double c0sq) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = i % pd0, i1 = (i / pd0) % pd1, i2 = z0 + i / (pd0 * pd1);
    const int64_t kx = C == 4 ? i0 : i1, ky = C == 4 ? i1 : i2, kz = C == 4 ? i2 : 0;
    const double2 pq[3] = {tab[kx], tab[nx + ky], tab[nx + ny + kz]};
    cfp::cd r[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = c < C ? v[c * n + i] : cfp::make_cd(0.0, 0.0);
#pragma unroll
    for (int c = 0; c < C; ++c) v[c * n + i] = cfp::wave_solve(r, c, pq, c0sq);
  }
}
unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

PetscErrorCode wave_dist_setup(FFTPrecWaveContext* ctx, int P, int dev) {
  const int dim = ctx->dim ? (int)ctx->dim : 3;
  // PETSC_DECIDE rows are whole planes of cells of the slowest axis when P divides it; the slab
  // plan splits that axis the same way, so no redistribution is needed
  PetscCheck((dim == 3 && ctx->n_z % P == 0) || (dim == 2 && ctx->n_z == 1 && ctx->n_y % P == 0), PETSC_COMM_SELF,
             PETSC_ERR_SUP,
             "setupFFTPrec3DWave on several ranks: a 3-D grid with the rank count dividing n_z, or a 2-D grid "
             "with it dividing n_y");
  int rank = 0;
  PetscCallMPI(MPI_Comm_rank(PETSC_COMM_WORLD, &rank));
  wave_dist_free(ctx);
  WaveDist* w = new WaveDist;
  w->ncomp = dim + 1;
  if (dim == 3) {
    w->pd[0] = ctx->n_x, w->pd[1] = ctx->n_y, w->pd[2] = ctx->n_z;
  } else {
    w->pd[0] = 1, w->pd[1] = ctx->n_x, w->pd[2] = ctx->n_y;
  }
  const PetscInt dims[3] = {w->pd[0], w->pd[1], w->pd[2]};
  PetscErrorCode e = slab_create(PETSC_COMM_WORLD, P, rank, dims, dev, &w->slab);
  int64_t lay[8] = {0};
  if (!e) e = cfp_err(cfp_slab_layout(w->pd[0], w->pd[1], w->pd[2], P, rank, lay), "setupFFTPrec3DWave");
  w->nloc = lay[4];
  w->z0 = lay[2];
  // the symbol's per-axis (p, q) = (kappa c0 (1 - cos theta), kappa sin theta), as cfp_wave_plan_set_symbol
  const int64_t n3[3] = {ctx->n_x, ctx->n_y, ctx->n_z};
  const double kap[3] = {ctx->kappa_x, ctx->kappa_y, ctx->kappa_z};
  std::vector<double2> t;
  for (int a = 0; a < 3; ++a)
    for (int64_t k = 0; k < n3[a]; ++k) {
      const long double th = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n3[a];
      t.push_back(make_double2((double)((long double)kap[a] * ctx->c0 * (1.0L - cosl(th))),
                               (double)((long double)kap[a] * sinl(th))));
    }
  if (!e && (hipMalloc(&w->tab, sizeof(double2) * t.size()) != hipSuccess ||
             hipMemcpy(w->tab, t.data(), sizeof(double2) * t.size(), hipMemcpyHostToDevice) != hipSuccess ||
             hipMalloc(&w->buf, sizeof(cfp::cd) * 2 * w->ncomp * (size_t)(w->nloc > 0 ? w->nloc : 1)) != hipSuccess))
    e = PetscErrorSet(PETSC_ERR_MEM, "setupFFTPrec3DWave", "slab buffers");
  w->c0sq = ctx->c0 * ctx->c0;
  if (e) {
    slab_destroy(&w->slab);
    if (w->tab) hipFree(w->tab);
    if (w->buf) hipFree(w->buf);
    delete w;
    return e;
  }
  std::lock_guard<std::mutex> g(g_wave_mu);
  g_wave_dist[ctx] = w;
  return PETSC_SUCCESS;
}

template <int C>
int wave_dist_run(const FFTPrecWaveContext* ctx, const WaveDist* w, const cfp::cd* b, cfp::cd* x, void* vst) {
  const int64_t n = w->nloc;
  hipStream_t st = (hipStream_t)vst;
  cfp::cd *u = w->buf, *v = w->buf + C * n;
  const unsigned g = grid_for(n);
  int rc = CFP_SUCCESS;
  hipLaunchKernelGGL(k_wave_split<C>, dim3(g), dim3(256), 0, st, b, u, n);
  if (hipGetLastError() != hipSuccess) rc = CFP_ERR_LIB;
  for (int c = 0; c < C && !rc; ++c)
    rc = cfp_dist_plan_forward(w->slab.plan, (const double*)(u + c * n), (double*)(v + c * n), vst);
  if (!rc) {
    hipLaunchKernelGGL(k_wave_slab_solve<C>, dim3(g), dim3(256), 0, st, v, n, w->pd[0], w->pd[1], w->z0,
                       (int64_t)ctx->n_x, (int64_t)ctx->n_y, (const double2*)w->tab, w->c0sq);
    if (hipGetLastError() != hipSuccess) rc = CFP_ERR_LIB;
  }
  for (int c = 0; c < C && !rc; ++c)
    rc = cfp_dist_plan_backward(w->slab.plan, (const double*)(v + c * n), (double*)(u + c * n), vst);
  if (!rc) {
    const double sc = 1.0 / (double)(ctx->n_x * ctx->n_y * ctx->n_z);
    hipLaunchKernelGGL(k_wave_join<C>, dim3(g), dim3(256), 0, st, (const cfp::cd*)u, x, n, sc);
    if (hipGetLastError() != hipSuccess) rc = CFP_ERR_LIB;
  }
  if (!rc) rc = cfp_stream_sync(vst);  // the slab applies are host-driven: complete on return
  return rc;
}

PetscErrorCode wave_dist_apply(FFTPrecWaveContext* ctx, WaveDist* w, Vec b, Vec x) {
  const int64_t M = w->ncomp * w->nloc;
  PetscCall(check_size(b, M, "applyFFT3DPrecWave: b has the wrong size for this rank's slab"));
  PetscCall(check_size(x, M, "applyFFT3DPrecWave: x has the wrong size for this rank's slab"));
  DevIn in;
  DevOut out;
  PetscCall(in.get(b, M));
  PetscCall(out.get(x, M));
  void* vst = nullptr;
  bool wait = true;
  device_stream(&vst, &wait);
  const cfp::cd* bp = (const cfp::cd*)in.ptr();
  cfp::cd* xp = (cfp::cd*)out.ptr();
  const int rc = w->ncomp == 4 ? wave_dist_run<4>(ctx, w, bp, xp, vst) : wave_dist_run<3>(ctx, w, bp, xp, vst);
  PetscCall(out.put());
  PetscCall(in.put());
  CFPCALL(rc);
  return PETSC_SUCCESS;
}

extern "C" PetscErrorCode setupFFTPrec3DWave(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  PetscCheck(ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "setupFFTPrec3DWave: no context attached to the PC");
  PetscCheck(ctx->n_x >= 1 && ctx->n_y >= 1 && ctx->n_z >= 1, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE,
             "setupFFTPrec3DWave: n_x, n_y, n_z must be >= 1");
  int dev = 0;
  PetscCheck(hipGetDevice(&dev) == hipSuccess, PETSC_COMM_SELF, PETSC_ERR_LIB, "no HIP device");
  if (ctx->plan) CFPCALL(cfp_wave_plan_destroy(ctx->plan));
  ctx->plan = nullptr;
  int P = 1;
  PetscCallMPI(MPI_Comm_size(PETSC_COMM_WORLD, &P));
  if (P > 1) {
    PetscCall(wave_dist_setup(ctx, P, dev));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  const int dim = ctx->dim ? (int)ctx->dim : 3;
  CFPCALL(cfp_wave_plan_create_dim(&ctx->plan, ctx->n_x, ctx->n_y, ctx->n_z, dim, dev));
  const double kappa[3] = {ctx->kappa_x, ctx->kappa_y, ctx->kappa_z};
  CFPCALL(cfp_wave_plan_set_symbol(ctx->plan, kappa, ctx->c0));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode applyFFT3DPrecWave(PC pc, Vec b, Vec x) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  if (WaveDist* w = ctx ? wave_dist(ctx) : nullptr) {  // several ranks: the slab-backed apply
    PetscCall(wave_dist_apply(ctx, w, b, x));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  PetscCheck(ctx && ctx->plan, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONGSTATE, "applyFFT3DPrecWave: setup has not run");
  const PetscInt M = ((ctx->dim ? ctx->dim : 3) + 1) * ctx->n_x * ctx->n_y * ctx->n_z;
  PetscCall(check_size(b, M, "applyFFT3DPrecWave: b has the wrong size"));
  PetscCall(check_size(x, M, "applyFFT3DPrecWave: x has the wrong size"));
  DevIn in;
  DevOut out;
  PetscCall(in.get(b, M));
  PetscCall(out.get(x, M));
  // device Vecs: ordered on the Vec stream without a host round trip (cfp_pc::device_stream);
  // a staged host Vec is waited for (its buffers are copied back / freed below)
  void* st = nullptr;
  bool wait = true;
  if (!in.tmp && !out.tmp) device_stream(&st, &wait);
  // the stand-in KSP may ask for dots of x with its basis (PCMiniApplyDots): on the 3-sweep
  // schedule they ride in the last sweep's stores (cfp_wave_plan_apply_dots); otherwise the
  // request stays open and the KSP runs its own multi-dot
  PCMiniApplyDots* req = nullptr;
  int npass = 0;
  if (!in.tmp && !out.tmp && PCMiniGetApplyDots(pc, &req) == PETSC_SUCCESS && req && !req->done && req->nv >= 1 &&
      req->nv <= 4 && cfp_wave_plan_num_passes(ctx->plan, &npass) == CFP_SUCCESS && npass == 3) {
    int fused = 0;
    int rc = cfp_wave_plan_apply_dots(ctx->plan, in.ptr(), out.ptr(), st, (int)req->nv,
                                      reinterpret_cast<const double* const*>(req->v), req->out, &fused);
    if (rc == CFP_SUCCESS && fused) req->done = PETSC_TRUE;
    if (rc == CFP_SUCCESS && wait) rc = cfp_stream_sync(st);
    PetscCall(out.put());
    PetscCall(in.put());
    CFPCALL(rc);
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  int rc = cfp_wave_plan_apply(ctx->plan, in.ptr(), out.ptr(), st);
  if (rc == CFP_SUCCESS && (wait || in.tmp || out.tmp)) rc = cfp_stream_sync(st);
  PetscCall(out.put());
  PetscCall(in.put());
  CFPCALL(rc);
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode destroyFFTPrec3DWave(PC pc) {
  PetscFunctionBeginUser;
  FFTPrecWaveContext* ctx = nullptr;
  PetscCall(PCShellGetContext(pc, &ctx));
  if (ctx) wave_dist_free(ctx);
  if (ctx && ctx->plan) {
    CFPCALL(cfp_wave_plan_destroy(ctx->plan));
    ctx->plan = nullptr;
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

// ------------------------------------------------------------------ time loop
extern "C" void cfp_wave_config_default(cfp_wave_config* cfg, int64_t n) {
  if (!cfg) return;
  std::memset((void*)cfg, 0, sizeof(*cfg));
  cfg->nx = cfg->ny = cfg->nz = n;
  for (int d = 0; d < 3; ++d) {
    cfg->xmin[d] = -0.5;
    cfg->xmax[d] = 0.5;
  }
  cfg->c0 = 700.0;
  cfg->cfl = 1.0e3 / 3.0;
  cfg->tmax = 0.05;
  cfg->ntmax = 2000000;
  cfg->precision = 1e-5;
  cfg->max_its = 1000;
  cfg->restart = 30;
  cfg->pc = CFP_WAVE_PC_FFT;
  cfg->bc = CFP_WAVE_BC_WALL;
  cfg->pc_side = PC_LEFT;
  cfg->on_device = 1;
  cfg->dim = 3;
  cfg->fuse = 1;
}

extern "C" void cfp_wave_config_default_dim(cfp_wave_config* cfg, int64_t n, int dim) {
  if (!cfg) return;
  cfp_wave_config_default(cfg, n);
  if (dim < 1 || dim > 3) return;
  cfg->dim = dim;
  if (dim < 3) cfg->nz = 1;
  if (dim < 2) cfg->ny = 1;
  cfg->cfl = 1.0e3 / (double)dim;  // main: cfl = 1e3 / getSpaceDimension()
}

extern "C" PetscErrorCode WaveSystemGMRES(const cfp_wave_config* cfg, cfp_wave_result* res, double* U_out) {
  PetscFunctionBeginUser;
  PetscCheck(cfg && res, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "WaveSystemGMRES: NULL argument");
  PetscCheck(cfg->pc == CFP_WAVE_PC_NONE || cfg->on_device, PETSC_COMM_SELF, PETSC_ERR_SUP,
             "the block-circulant preconditioner runs on HIP vectors only");
  std::memset((void*)res, 0, sizeof(*res));
  const double t_setup = wall();
  const int dim = cfg->dim ? cfg->dim : 3;
  PetscCheck(dim >= 1 && dim <= 3, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3");
  const PetscInt nx = cfg->nx, ny = cfg->ny, nz = cfg->nz, M = (dim + 1) * nx * ny * nz;
  const double h[3] = {(cfg->xmax[0] - cfg->xmin[0]) / (double)nx, (cfg->xmax[1] - cfg->xmin[1]) / (double)ny,
                       (cfg->xmax[2] - cfg->xmin[2]) / (double)nz};
  // dt = cfl * minRatioVolSurf / c0 (impl_seq.cxx:18,73): cell measure over its faces' measure
  const double dt = cfg->cfl * cfp_cartesian_min_ratio_vol_surf(dim, h) / cfg->c0;
  res->dt = dt;
  for (int d = 0; d < 3; ++d) res->kappa[d] = d < dim ? dt / h[d] : 0.0;

  // several ranks (PETSC_COMM_WORLD of PetscMiniSetCommWorld): VecCreateMPI / MatCreateAIJ on
  // PETSC_COMM_WORLD with PETSC_DECIDE rows, as the reference's MPI driver (:63,83-85)
  int P = 1;
  PetscCallMPI(MPI_Comm_size(PETSC_COMM_WORLD, &P));
  Vec Un, dUn;
  if (P > 1 && cfg->on_device) PetscCall(VecCreateMPIHIP(PETSC_COMM_WORLD, PETSC_DECIDE, M, &Un));
  else if (P > 1) PetscCall(VecCreateMPI(PETSC_COMM_WORLD, PETSC_DECIDE, M, &Un));
  else if (cfg->on_device) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, M, &Un));
  else PetscCall(VecCreateSeq(PETSC_COMM_SELF, M, &Un));
  PetscCall(VecDuplicate(Un, &dUn));
  PetscCall(initial_conditions_shock_wave(nx, ny, nz, cfg->xmin, cfg->xmax, Un));
  PetscInt lo, nloc;
  PetscCall(VecGetOwnershipRange(Un, &lo, NULL));
  PetscCall(VecGetLocalSize(Un, &nloc));
  res->rstart = lo;
  res->nlocal = nloc;
  Mat A;
  if (P > 1)
    PetscCall(computeDivergenceMatrixWaveCartesianAIJ(PETSC_COMM_WORLD, nx, ny, nz, dim, h, dt, cfg->c0, cfg->bc, &A));
  else
    PetscCall(computeDivergenceMatrixWaveCartesianDim(nx, ny, nz, dim, h, dt, cfg->c0, cfg->bc, &A));
  PetscCall(MatShift(A, 1.0));  // :86

  KSP ksp;
  PC pc;
  PetscCall(KSPCreate(PETSC_COMM_WORLD, &ksp));
  PetscCall(KSPSetType(ksp, KSPGMRES));
  PetscCall(KSPSetTolerances(ksp, cfg->precision, cfg->precision, PETSC_DEFAULT, cfg->max_its));
  PetscCall(KSPGMRESSetRestart(ksp, cfg->restart > 0 ? cfg->restart : 30));
  PetscCall(KSPSetPCSide(ksp, (PCSide)cfg->pc_side));
  PetscCall(KSPMiniSetFusion(ksp, cfg->fuse ? PETSC_TRUE : PETSC_FALSE));
  PetscCall(KSPGetPC(ksp, &pc));
  FFTPrecWaveContext ctx;
  std::memset((void*)&ctx, 0, sizeof(ctx));
  if (cfg->pc == CFP_WAVE_PC_FFT) {
    ctx.n_x = nx;
    ctx.n_y = ny;
    ctx.n_z = nz;
    ctx.kappa_x = res->kappa[0];
    ctx.kappa_y = res->kappa[1];
    ctx.kappa_z = res->kappa[2];
    ctx.c0 = cfg->c0;
    ctx.dim = dim;
    PetscCall(PCSetType(pc, PCSHELL));
    PetscCall(PCShellSetContext(pc, &ctx));
    PetscCall(PCShellSetSetUp(pc, setupFFTPrec3DWave));
    PetscCall(PCShellSetApply(pc, applyFFT3DPrecWave));
    PetscCall(PCShellSetDestroy(pc, destroyFFTPrec3DWave));
    PetscCall(PCShellSetName(pc, "block-circulant FFT (HIP)"));
  } else {
    PetscCall(PCSetType(pc, PCNONE));
  }
  PetscCall(KSPSetOperators(ksp, A, A));
  PetscCall(KSPSetUp(ksp));
  PetscCall(KSPMiniSetUpWork(ksp, Un));
  PetscCall(MatMult(A, Un, dUn));  // device copy of A made outside the timed solves
  if (cfg->on_device)
    PetscCheck(cfp_stream_sync(nullptr) == CFP_SUCCESS, PETSC_COMM_SELF, PETSC_ERR_LIB, "stream sync failed");
  res->setup_seconds = wall() - t_setup;

  int64_t it = 0;
  double time = 0.0;
  bool stationary = false;
  res->all_converged = 1;
  res->min_step_its = -1;
  if (cfg->profile) PetscCall(PetscMiniProfileBegin(1 << 16));
  const double t_loop = wall();
  while (it < cfg->ntmax && time <= cfg->tmax && !stationary) {  // :95
    PetscCall(VecCopy(Un, dUn));
    const double v = wall();
    PetscCall(KSPSolve(ksp, Un, Un));
    const double w = wall();
    PetscCall(VecAXPY(dUn, -1.0, Un));
    time += dt;
    it += 1;
    PetscReal norm;
    PetscCall(VecNorm(dUn, NORM_2, &norm));
    stationary = norm < cfg->precision;
    KSPConvergedReason reason;
    PetscInt its;
    PetscReal residu;
    PetscCall(KSPGetConvergedReason(ksp, &reason));
    PetscCall(KSPGetIterationNumber(ksp, &its));
    PetscCall(KSPGetResidualNorm(ksp, &residu));
    PetscInt calls;
    PetscLogDouble pcs;
    PetscCall(KSPMiniGetPCApplyStats(ksp, &calls, &pcs));
    res->solve_seconds += w - v;
    res->pc_seconds += pcs;
    res->pc_calls += calls;
    res->total_its += its;
    res->max_step_its = std::max<int64_t>(res->max_step_its, its);
    res->min_step_its = res->min_step_its < 0 ? its : std::min<int64_t>(res->min_step_its, its);
    res->last_reason = (int)reason;
    res->last_residual = residu;
    res->last_norm_dU = norm;
    if (reason != KSP_CONVERGED_RTOL && reason != KSP_CONVERGED_ATOL) res->all_converged = 0;
    PetscInt fd, fn;
    PetscCall(KSPMiniGetFusedCounts(ksp, &fd, &fn));
    res->fused_dots += fd;
    res->fused_norms += fn;
  }
  res->loop_seconds = wall() - t_loop;
  if (cfg->profile) {
    PetscCall(PetscMiniProfileEnd(res->dev_ms, res->dev_launches));
    res->dev_ms[0] = 1e3 * res->pc_seconds;
    res->dev_launches[0] = res->pc_calls;
  }
  res->steps = it;
  res->time = time;
  if (U_out) {  // this rank's rows (all of them on one rank)
    const PetscScalar* u;
    PetscCall(VecGetArrayRead(Un, &u));
    std::memcpy(U_out, (const void*)u, sizeof(double) * 2 * (size_t)nloc);
    PetscCall(VecRestoreArrayRead(Un, &u));
  }
  PetscCall(KSPDestroy(&ksp));
  PetscCall(MatDestroy(&A));
  PetscCall(VecDestroy(&Un));
  PetscCall(VecDestroy(&dUn));
  PetscFunctionReturn(PETSC_SUCCESS);
}
#endif  // CFP_WITH_PETSC
