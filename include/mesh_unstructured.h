/*
 * mesh_unstructured.h -- unstructured 3-D meshes (tetrahedra, hexahedra), the mesh ->
 * Cartesian intersection matrix of the PCSHELL, and the upwind transport operator on such a
 * mesh.
 *
 * Reference interface each entry point replaces:
 *   src/PCSHELLFft_3D.hxx:17, src/PCSHELLFft_3D.cxx:17-18
 *       FFTPrecTransportContext::intersectionMatrix and the MatMult that moves b from the
 *       mesh onto the Cartesian FFT grid.  The reference declares it but never builds it
 *       (SURVEY App. A item 2); ToDo.md:12 asks for MEDCoupling's getCrudeMatrix (P0->P0
 *       intersection volumes, one map<source cell, volume> per target cell) as a PETSc Mat.
 *   src/PCSHELLFft_3D.cxx:101-151 getFFTPrec3DContext(..., Mesh srcMesh): n_d and the bounds
 *       come from the mesh.
 *   src/TransportEquation.cxx:25-73, :75-133 initial_conditions_shock / computeDivergenceMatrix
 *       over the faces of a general mesh (SOLVERLAB Mesh/Cell/Face).
 *   SOLVERLAB Mesh(filename), Mesh::minRatioVolSurf (tests/...impl_mpi.cxx:51-52, :248-250).
 * SOLVERLAB and MEDCoupling are absent in this image; the meshes are read from the Gmsh 2.2
 * ASCII files that sit beside the reference's MED files (meshes/<family>/<name>.msh), or passed as
 * arrays.  Node ordering of the cells is Gmsh's (tet: 4 nodes; hex: 0-3 bottom, 4-7 top).
 *
 * Everything here is host-side set-up (assembly), as MatSetValue and MEDCoupling are in the
 * reference; the per-apply work (the remap SpMV) runs on the GPU through the AIJ Mat.
 */
#ifndef CFP_MESH_UNSTRUCTURED_H
#define CFP_MESH_UNSTRUCTURED_H

#include <stdint.h>

#include "petsc_mini.h"
#include "pcshell_fft3d.h"
#include "transport_equation.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfp_mesh_s *cfp_mesh_t;

/* Gmsh 2.2 ASCII: keeps the 3-D cells (element types 4 = tet4, 5 = hex8), drops the rest. */
int cfp_mesh_read_gmsh(const char *path, cfp_mesh_t *mesh);
/* From arrays: xyz[3*nnodes]; cell c has cell_ptr[c+1]-cell_ptr[c] (4 or 8) nodes
 * cell_nodes[cell_ptr[c] ...] (0-based). */
int cfp_mesh_create(int64_t nnodes, const double *xyz, int64_t ncells, const int64_t *cell_ptr,
                    const int64_t *cell_nodes, cfp_mesh_t *mesh);
int cfp_mesh_destroy(cfp_mesh_t mesh);
/* sizes and bounding box {xmin, xmax, ymin, ymax, zmin, zmax} */
int cfp_mesh_info(cfp_mesh_t mesh, int64_t *nnodes, int64_t *ncells, int64_t *nfaces, double bbox[6]);
/* cell measures and barycentres (3 per cell); either pointer may be NULL */
int cfp_mesh_cell_geometry(cfp_mesh_t mesh, double *volumes, double *centers);
/* SOLVERLAB Mesh::minRatioVolSurf: min over cells of |C| / sum of |F| over its faces */
int cfp_mesh_min_ratio_vol_surf(cfp_mesh_t mesh, double *ratio);
/* faces: per face its two cells (second = -1 on the border), measure, and unit normal
 * oriented out of the first cell; arrays of nfaces entries (normal: 3 per face) */
int cfp_mesh_faces(cfp_mesh_t mesh, int64_t *cell0, int64_t *cell1, double *measure, double *normal);

/* MEDCoupling getCrudeMatrix for P0->P0 from the mesh (source) to the Cartesian grid
 * nx*ny*nz over bbox (target, cell i = ix + nx (iy + ny iz)): entry (i, c) = volume of
 * (Cartesian cell i) ∩ (mesh cell c), computed exactly by clipping the cell's tetrahedra
 * against the grid's slabs.  Two calls: with rowptr/col/val NULL it only returns *nnz;
 * then rowptr (nx*ny*nz+1), col and val (*nnz) are filled, columns ascending per row. */
int cfp_mesh_crude_matrix_cartesian(cfp_mesh_t mesh, int64_t nx, int64_t ny, int64_t nz, const double bbox[6],
                                    int64_t *nnz, int64_t *rowptr, int64_t *col, double *val);

/* computeDivergenceMatrix on the mesh (+ shift I): row j sums over the faces of cell j with
 * outward unit normal n, un = n . a; an interior face with un > 0 adds dt |F|/|C| un to
 * (j, j), otherwise (j, neighbour) gets -dt |F|/|C| un (CFP_UPWIND_REFERENCE) or
 * +dt |F|/|C| un (CFP_UPWIND_FIXED); border faces add nothing.  Every row stores its
 * diagonal, columns ascend.  Two calls as above (val: interleaved re, im). */
int cfp_mesh_transport_csr(cfp_mesh_t mesh, double dt, const double a[3], int sign_mode, double shift,
                           int64_t *nnz, int64_t *rowptr, int64_t *col, double *val);

/* ---- PETSc-level (stand-in) entry points */
/* The PCSHELL's two remap matrices from the crude matrix V (Cartesian x mesh):
 *   *toCart = diag(1 / row sums) V         (mesh -> Cartesian, intensive: a cell average)
 *   *toMesh = diag(1 / column sums) V^T    (Cartesian -> mesh)
 * Cartesian cells that no mesh cell touches get an empty row.  Either output may be NULL. */
PetscErrorCode MatCreateMeshCartesianRemap(cfp_mesh_t mesh, PetscInt nx, PetscInt ny, PetscInt nz,
                                           const PetscReal bbox[6], Mat *toCart, Mat *toMesh);
/* getFFTPrec3DContext with the Mesh argument of the reference (src/PCSHELLFft_3D.cxx:101-151):
 * nbCells and the bounds come from the mesh, lambda_d = a_d dt (max_d - min_d) / n_d as the
 * reference, and the context gets intersectionMatrix (mesh -> Cartesian) and remapBack
 * (Cartesian -> mesh) unless the mesh is the Cartesian grid itself (then both stay NULL:
 * identity).  The caller owns both matrices (destroyFFTPrec3D leaves them, as the reference's
 * destroy leaves intersectionMatrix); FFTPrec3DContextDestroyRemap frees them. */
PetscErrorCode getFFTPrec3DContextMesh(PetscInt ndim, PetscScalar dt, PetscScalar a_x, PetscScalar a_y,
                                       PetscScalar a_z, cfp_mesh_t srcMesh, FFTPrecTransportContext *ctx);
PetscErrorCode FFTPrec3DContextDestroyRemap(FFTPrecTransportContext *ctx);
/* initial_conditions_shock on the mesh: 650 where |barycentre - bbox centre| < 0.3, else 600 */
PetscErrorCode initial_conditions_shock_mesh(cfp_mesh_t mesh, Vec U);

/* ---- the implicit transport time loop with GMRES on the mesh (TransportEquation_impl_mpi
 * with Mesh(filename), tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:13-189, :248).
 * cfg: the Cartesian config's solver fields are used (a, cfl, tmax, ntmax, precision,
 * max_its, restart, pc, sign_mode, lambda_mode, pc_side, on_device); nx/ny/nz/xmin/xmax are
 * ignored (the mesh gives them).  lambda_mode MATCHED uses lambda_d = a_d dt / h_d with
 * h_d = (max_d - min_d) / n_d of the PCSHELL's Cartesian grid. */
PetscErrorCode TransportEquationGMRESMesh(cfp_mesh_t mesh, const cfp_transport_config *cfg,
                                          cfp_transport_result *res, double *U_out);

#ifdef __cplusplus
}
#endif
#endif /* CFP_MESH_UNSTRUCTURED_H */
