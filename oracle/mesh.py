"""CPU oracle for unstructured meshes and the mesh <-> Cartesian remap -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  Independent restatements
(different algorithms from csrc/mesh_unstructured.cpp wherever one exists):

* ``read_gmsh``: Gmsh 2.2 ASCII reader (the format of the reference's
  ``meshes/<family>/*.msh``, which hold the same FVCA6 meshes as the ``.med`` files the
  reference's ctests load, tests/CMakeLists.txt:30-36).
* ``geometry``: tetrahedron volumes from the determinant; hexahedron volumes and barycentres
  from the divergence theorem over its (planar) faces -- not from a tetrahedral split.
* ``crude_matrix``: MEDCoupling getCrudeMatrix semantics for P0->P0 (ToDo.md:12): entry
  (Cartesian cell i, mesh cell c) = volume of their intersection, here computed as the volume
  of the convex polytope {cell half-spaces} ∩ {box half-spaces} by vertex enumeration and a
  facet-pyramid sum -- not by clipping.
* ``transport_csr``: computeDivergenceMatrix (src/TransportEquation.cxx:75-133) as a face loop
  over the cells, with SOLVERLAB's outward unit normals and measures.
* ``min_ratio_vol_surf``: SOLVERLAB Mesh::minRatioVolSurf (tests/...impl_mpi.cxx:51).
* ``pc_apply``: the PCSHELL apply on a mesh: remap to the Cartesian grid (row-normalised crude
  matrix), the circulant solve (oracle.np_solve_3d), remap back (column-normalised transpose).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

TET_FACES = [(0, 1, 2), (0, 1, 3), (0, 2, 3), (1, 2, 3)]
HEX_FACES = [(0, 3, 2, 1), (0, 1, 5, 4), (0, 4, 7, 3), (1, 2, 6, 5), (2, 3, 7, 6), (4, 5, 6, 7)]


def read_gmsh(path: str):
    """(xyz[nn, 3], cells: list of node-index tuples) of the tet4 (type 4) / hex8 (type 5)
    elements of a Gmsh ASCII 2.x or 4.1 file, coincident nodes merged."""
    nverts = {1: 2, 2: 3, 3: 4, 4: 4, 5: 8, 6: 6, 7: 5, 15: 1}
    with open(path) as f:
        tok = f.read().split()
    pos = 0
    ver = None
    ids, xyz, cells = {}, [], []

    def nxt(k=1):
        nonlocal pos
        v = tok[pos:pos + k]
        pos += k
        return v

    while pos < len(tok):
        t = nxt()[0]
        if t == "$MeshFormat":
            ver = float(nxt()[0])
            nxt(2)
        elif t == "$Nodes" and ver >= 4:
            nblocks = int(nxt(4)[0])
            for _ in range(nblocks):
                _dim, _tag, _par, n = (int(v) for v in nxt(4))
                tags = [int(v) for v in nxt(n)]
                for tg in tags:
                    ids[tg] = len(xyz)
                    xyz.append([float(v) for v in nxt(3)])
        elif t == "$Nodes":
            n = int(nxt()[0])
            for _ in range(n):
                p = nxt(4)
                ids[int(p[0])] = len(xyz)
                xyz.append([float(v) for v in p[1:]])
        elif t == "$Elements" and ver >= 4:
            nblocks = int(nxt(4)[0])
            for _ in range(nblocks):
                _dim, _tag, etype, n = (int(v) for v in nxt(4))
                for _ in range(n):
                    p = [int(v) for v in nxt(1 + nverts[etype])]
                    if etype in (4, 5):
                        cells.append(tuple(ids[v] for v in p[1:]))
        elif t == "$Elements":
            n = int(nxt()[0])
            for _ in range(n):
                _id, etype, ntags = (int(v) for v in nxt(3))
                nxt(ntags)
                p = [int(v) for v in nxt(nverts[etype])]
                if etype in (4, 5):
                    cells.append(tuple(ids[v] for v in p))
    xyz = np.array(xyz, dtype=np.float64)
    # nodes with identical coordinates are one node (the Kershaw files repeat internal-surface nodes)
    uniq, inv = np.unique(xyz, axis=0, return_inverse=True)
    if len(uniq) != len(xyz):
        inv = inv.reshape(-1)
        xyz, cells = uniq, [tuple(int(inv[v]) for v in c) for c in cells]
    return xyz, cells


def _faces_of(cell):
    return [tuple(cell[j] for j in f) for f in (TET_FACES if len(cell) == 4 else HEX_FACES)]


def _area_vector(P):
    """Vector area of a planar polygon (sum of the fan's cross products / 2)."""
    a = np.zeros(3)
    for k in range(1, len(P) - 1):
        a += np.cross(P[k] - P[0], P[k + 1] - P[0])
    return 0.5 * a


def geometry(xyz, cells):
    """(volumes, barycentres) -- tets by determinant, hexes by the divergence theorem."""
    vol = np.empty(len(cells))
    ctr = np.empty((len(cells), 3))
    for c, cell in enumerate(cells):
        P = xyz[list(cell)]
        if len(cell) == 4:
            vol[c] = abs(np.linalg.det(np.array([P[1] - P[0], P[2] - P[0], P[3] - P[0]]))) / 6.0
            ctr[c] = P.mean(axis=0)
            continue
        # V = 1/3 oint x.n dS;  int_V x_i dV = 1/2 oint x_i^2 n_i dS, on a fan of triangles of
        # each (planar) face with int_T x_i^2 dS = |T|/6 (a_i^2 + b_i^2 + d_i^2 + a_i b_i +
        # b_i d_i + d_i a_i).
        centre = P.mean(axis=0)
        V = 0.0
        M = np.zeros(3)
        for f in HEX_FACES:
            Q = P[list(f)]
            A = _area_vector(Q)
            if np.dot(A, Q.mean(axis=0) - centre) < 0:
                Q = Q[::-1]
            for k in range(1, len(Q) - 1):
                a, b, d = Q[0], Q[k], Q[k + 1]
                n2 = np.cross(b - a, d - a)  # 2 * area * unit normal
                V += np.dot(a, n2) / 6.0
                s = a * a + b * b + d * d + a * b + b * d + d * a
                M += n2 * s / 12.0  # int_T x_i^2 n_i dS (n2 = 2 |T| n)
        vol[c] = V
        ctr[c] = M / (2.0 * V)
    return vol, ctr


def faces(xyz, cells):
    """dict sorted-node-key -> [cell0, cell1 or -1, measure, unit normal out of cell0]."""
    _, ctr = geometry(xyz, cells)
    F = {}
    for c, cell in enumerate(cells):
        for fv in _faces_of(cell):
            key = tuple(sorted(fv))
            if key in F:
                F[key][1] = c
                continue
            Q = xyz[list(fv)]
            A = _area_vector(Q) if len(fv) == 3 else 0.5 * np.cross(Q[2] - Q[0], Q[3] - Q[1])
            if np.dot(A, Q.mean(axis=0) - ctr[c]) < 0:
                A = -A
            m = np.linalg.norm(A)
            F[key] = [c, -1, m, A / m]
    return F


def min_ratio_vol_surf(xyz, cells):
    vol, _ = geometry(xyz, cells)
    F = faces(xyz, cells)
    surf = np.zeros(len(cells))
    for c0, c1, m, _n in F.values():
        surf[c0] += m
        if c1 >= 0:
            surf[c1] += m
    return float(np.min(vol / surf))


def transport_csr(xyz, cells, dt, a, sign="reference", shift=0.0):
    """computeDivergenceMatrix + shift I as a scipy CSR (complex)."""
    vol, _ = geometry(xyz, cells)
    F = faces(xyz, cells)
    n = len(cells)
    A = sp.lil_matrix((n, n), dtype=np.complex128)
    for c in range(n):
        A[c, c] += shift
    sgn = -1.0 if sign == "reference" else 1.0
    a = np.asarray(a, dtype=np.float64)
    for c0, c1, m, nrm in F.values():
        if c1 < 0:
            continue  # border: Neumann
        for j, other, s in ((c0, c1, 1.0), (c1, c0, -1.0)):
            un = s * float(np.dot(nrm, a))
            coef = dt * m / vol[j]
            if un > 0:
                A[j, j] += coef * un
            else:
                A[j, other] += sgn * coef * un
    return A.tocsr()


def _cell_halfspaces(P, cell):
    """A x + b <= 0 for the cell's faces (outward normals)."""
    centre = P.mean(axis=0)
    rows = []
    for f in (TET_FACES if len(cell) == 4 else HEX_FACES):
        Q = P[list(f)]
        nrm = _area_vector(Q)
        if np.dot(nrm, Q.mean(axis=0) - centre) < 0:
            nrm = -nrm
        nrm = nrm / np.linalg.norm(nrm)
        rows.append(np.concatenate([nrm, [-np.dot(nrm, Q.mean(axis=0))]]))
    return rows


def _polytope_volume(H, tol=1e-12):
    """Volume of the convex polytope {x : H[:, :3] x + H[:, 3] <= 0} (unit normals, bounded):
    vertex enumeration over every triple of planes, then V = sum over facets of
    (1/3) (distance from an interior point to the facet's plane) x (facet polygon area)."""
    keep = []  # drop repeated planes (a cell face lying on a box plane)
    for i in range(len(H)):
        if not any(np.allclose(H[i], H[j], atol=1e-13) for j in keep):
            keep.append(i)
    H = H[keep]
    A, b = H[:, :3], H[:, 3]
    m = len(H)
    verts = []
    for i in range(m):
        for j in range(i + 1, m):
            for k in range(j + 1, m):
                M3 = A[[i, j, k]]
                if abs(np.linalg.det(M3)) < 1e-12:
                    continue
                x = np.linalg.solve(M3, -b[[i, j, k]])
                if np.all(A @ x + b <= tol):
                    verts.append(x)
    if len(verts) < 4:
        return 0.0
    V = np.array(verts)
    # merge coincident vertices (several plane triples meet at one point)
    uniq = []
    for v in V:
        if not any(np.linalg.norm(v - u) < 1e-11 for u in uniq):
            uniq.append(v)
    V = np.array(uniq)
    if len(V) < 4:
        return 0.0
    c = V.mean(axis=0)
    vol = 0.0
    for f in range(m):
        on = V[np.abs(A[f] @ V.T + b[f]) <= 1e-11]
        if len(on) < 3:
            continue
        g = on.mean(axis=0)
        # order the facet's vertices by angle in its plane
        u = on[0] - g
        if np.linalg.norm(u) == 0:
            u = on[1] - g
        u = u / np.linalg.norm(u)
        w = np.cross(A[f], u)
        ang = np.arctan2((on - g) @ w, (on - g) @ u)
        P = on[np.argsort(ang)]
        area = 0.5 * np.linalg.norm(sum(np.cross(P[q] - g, P[(q + 1) % len(P)] - g) for q in range(len(P))))
        h = -(A[f] @ c + b[f])
        vol += h * area / 3.0
    return float(vol)


def crude_matrix(xyz, cells, dims, bbox=None, only=None):
    """Intersection volumes, scipy CSR of shape (nx ny nz, ncells); `only`: the mesh cells whose
    columns are computed (the others stay empty)."""
    nx, ny, nz = dims
    if bbox is None:
        lo, hi = xyz.min(axis=0), xyz.max(axis=0)
        bbox = [lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]]
    x0, y0, z0 = bbox[0], bbox[2], bbox[4]
    h = np.array([(bbox[1] - bbox[0]) / nx, (bbox[3] - bbox[2]) / ny, (bbox[5] - bbox[4]) / nz])
    rows, cols, vals = [], [], []
    vol, _ = geometry(xyz, cells)
    for c in (range(len(cells)) if only is None else only):
        cell = cells[c]
        P = xyz[list(cell)]
        ch = _cell_halfspaces(P, cell)
        lo = np.floor((P.min(axis=0) - [x0, y0, z0]) / h).astype(int)
        hi = np.floor((P.max(axis=0) - [x0, y0, z0]) / h).astype(int)
        lo = np.maximum(lo, 0)
        hi = np.minimum(hi, [nx - 1, ny - 1, nz - 1])
        for iz in range(lo[2], hi[2] + 1):
            for iy in range(lo[1], hi[1] + 1):
                for ix in range(lo[0], hi[0] + 1):
                    bx = [x0 + ix * h[0], x0 + (ix + 1) * h[0], y0 + iy * h[1], y0 + (iy + 1) * h[1],
                          z0 + iz * h[2], z0 + (iz + 1) * h[2]]
                    H = np.array(ch + [[1, 0, 0, -bx[1]], [-1, 0, 0, bx[0]], [0, 1, 0, -bx[3]], [0, -1, 0, bx[2]],
                                       [0, 0, 1, -bx[5]], [0, 0, -1, bx[4]]], dtype=np.float64)
                    v = _polytope_volume(H)
                    if v > 1e-14 * vol[c]:
                        rows.append(ix + nx * (iy + ny * iz))
                        cols.append(c)
                        vals.append(v)
    return sp.csr_matrix((vals, (rows, cols)), shape=(nx * ny * nz, len(cells)))


def remap_matrices(V):
    """(toCart, toMesh) from the crude matrix V: row-normalised V and column-normalised V^T."""
    rs = np.asarray(V.sum(axis=1)).ravel()
    cs = np.asarray(V.sum(axis=0)).ravel()
    rinv = np.where(rs > 0, 1.0 / np.where(rs > 0, rs, 1.0), 0.0)
    return sp.diags(rinv) @ V, sp.diags(1.0 / cs) @ V.T.tocsr()


def pc_apply(V, dims, lam, b):
    """x = toMesh ( C^{-1} ( toCart b ) ) with the circulant solve of the oracle."""
    from . import oracle as O
    toCart, toMesh = remap_matrices(V)
    bc = toCart @ b
    xc = O.np_solve_3d(O.np_diag_closed_form(dims, lam), bc, dims)
    return toMesh @ xc
