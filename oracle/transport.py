"""CPU oracle for the transport operator and the GMRES solve -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  Restatements:

* ``divergence_matrix``: ``computeDivergenceMatrix`` (``src/TransportEquation.cxx:75-133``)
  as the reference writes it -- a loop over cells and their faces, outward normal ``n``,
  ``un = n . a``, ``dt |F| / |C| un`` added to the diagonal when ``un > 0`` (:109-110), else
  ``-dt |F| / |C| un`` to the neighbour column (:111-112, the reference sign) or
  ``+dt |F| / |C| un`` (the fixed sign); border faces skipped (:114-129).  |F| and |C| are
  the face area and cell volume of the Cartesian cell.
* ``initial_conditions_shock``: ``src/TransportEquation.cxx:25-73``.
* ``gmres``: PETSc's KSPGMRES as the reference's KSP runs it with default options
  (``tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:120-126``): restart 30, left
  preconditioning, classical Gram-Schmidt, the complex Givens update of
  KSPGMRESUpdateHessenberg, KSPConvergedDefault on the preconditioned residual norm.
  PETSc itself is absent (no vendored copy, no pinned version; CMakeLists.txt:47 asks
  for >= 3.4), so this restates its published algorithm.

Parity status: the operator has no reference-held fixture (it needs SOLVERLAB, absent);
it is pinned indirectly -- the fixed-sign operator's interior rows must equal the
golden-pinned circulant of ``oracle.np_dense_C`` (tests/test_transport.py).  GMRES is
"parity unpinned" against PETSc itself; it is checked against scipy's direct solve.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def divergence_matrix(dims, h, dt, a, sign: str = "reference", shift: float = 0.0) -> sp.csr_matrix:
    nx, ny, nz = (int(v) for v in dims)
    hx, hy, hz = (float(v) for v in h)
    vol = hx * hy * hz
    area = (hy * hz, hx * hz, hx * hy)
    n = nx * ny * nz
    rows, cols, vals = [], [], []
    sgn = -1.0 if sign in ("reference", "faithful") else 1.0
    for k in range(nz):
        for j in range(ny):
            for i in range(nx):
                c = i + nx * (j + ny * k)
                rows.append(c)
                cols.append(c)
                vals.append(shift)
                idx = (i, j, k)
                size = (nx, ny, nz)
                stride = (1, nx, nx * ny)
                for d in range(3):
                    for s in (-1, 1):  # face with outward normal s e_d
                        if (s < 0 and idx[d] == 0) or (s > 0 and idx[d] == size[d] - 1):
                            continue  # border: Neumann, nothing added
                        un = s * float(a[d])
                        coef = dt * area[d] / vol
                        if un > 0:
                            rows.append(c)
                            cols.append(c)
                            vals.append(coef * un)
                        else:
                            rows.append(c)
                            cols.append(c + s * stride[d])
                            vals.append(sgn * coef * un)
    A = sp.coo_matrix((np.array(vals, dtype=np.complex128), (rows, cols)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.eliminate_zeros()
    return A


def min_ratio_vol_surf(h) -> float:
    hx, hy, hz = (float(v) for v in h)
    return hx * hy * hz / (2.0 * (hx * hy + hy * hz + hz * hx))


def initial_conditions_shock(dims, xmin=(-0.5,) * 3, xmax=(0.5,) * 3) -> np.ndarray:
    nx, ny, nz = (int(v) for v in dims)
    h = [(xmax[d] - xmin[d]) / (nx, ny, nz)[d] for d in range(3)]
    c = [(xmin[d] + xmax[d]) / 2 for d in range(3)]
    x = xmin[0] + (np.arange(nx) + 0.5) * h[0]
    y = xmin[1] + (np.arange(ny) + 0.5) * h[1]
    z = xmin[2] + (np.arange(nz) + 0.5) * h[2]
    Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
    r2 = (X - c[0]) ** 2
    if ny > 1:
        r2 = r2 + (Y - c[1]) ** 2
    if nz > 1:
        r2 = r2 + (Z - c[2]) ** 2
    return np.where(np.sqrt(r2) < 0.3, 650.0, 600.0).astype(np.complex128).reshape(-1)


def gmres(A, b, M=None, x0=None, rtol=1e-5, abstol=1e-50, dtol=1e5, maxits=10000, restart=30, side="left"):
    """PETSc-default GMRES.  A, M: callables or matrices (M applies the preconditioner).
    Returns (x, its, reason, rnorm, history) with PETSc's KSPConvergedReason codes."""
    mv = A if callable(A) else (lambda v: A @ v)
    pc = (lambda v: v.copy()) if M is None else (M if callable(M) else (lambda v: M @ v))
    b = np.asarray(b, dtype=np.complex128)
    x = np.zeros_like(b) if x0 is None else np.array(x0, dtype=np.complex128)
    x_zero = x0 is None
    its, rnorm0, hist = 0, None, []
    reason = 0

    def conv(rn):
        if np.isnan(rn) or np.isnan(rnorm0):
            return -5
        if rn <= max(rtol * rnorm0, abstol):
            return 3 if rn < abstol else 2
        if its > 0 and rn >= dtol * rnorm0:
            return -4
        return 0

    while True:
        r = b.copy() if x_zero else b - mv(x)
        x_zero = False
        z = pc(r) if side == "left" else r
        beta = np.linalg.norm(z)
        if rnorm0 is None:
            rnorm0 = beta
        rn = beta
        hist.append(rn)
        reason = conv(rn)
        if reason != 0:
            break
        if its >= maxits:
            reason = -3
            break
        V = [z / beta]
        H = np.zeros((restart + 1, restart), dtype=np.complex128)
        cs = np.zeros(restart, dtype=np.complex128)
        sn = np.zeros(restart, dtype=np.complex128)
        rs = np.zeros(restart + 1, dtype=np.complex128)
        rs[0] = beta
        j = 0
        while j < restart and reason == 0 and its < maxits:
            w = pc(mv(V[j])) if side == "left" else mv(pc(V[j]))
            hcol = np.array([np.vdot(V[i], w) for i in range(j + 1)])
            w = w - sum(hcol[i] * V[i] for i in range(j + 1))
            hn = np.linalg.norm(w)
            H[: j + 1, j] = hcol
            H[j + 1, j] = hn
            happy = hn < min(hn / abs(rs[j]), 1e-30)  # KSPGMRESCycle, haptol 1e-30
            V.append(w / hn if not happy else w)
            for i in range(j):
                tt = H[i, j]
                H[i, j] = np.conj(cs[i]) * tt + sn[i] * H[i + 1, j]
                H[i + 1, j] = cs[i] * H[i + 1, j] - sn[i] * tt
            if not happy:
                tt = np.sqrt(abs(H[j, j]) ** 2 + abs(H[j + 1, j]) ** 2)
                if tt == 0.0:
                    reason = -5
                    break
                cs[j] = H[j, j] / tt
                sn[j] = H[j + 1, j] / tt
                rs[j + 1] = -(sn[j] * rs[j])
                rs[j] = np.conj(cs[j]) * rs[j]
                H[j, j] = np.conj(cs[j]) * H[j, j] + sn[j] * H[j + 1, j]
                rn = abs(rs[j + 1])
            else:
                rs[j + 1] = 0.0
                rn = 0.0
            its += 1
            hist.append(rn)
            reason = conv(rn)
            if happy and reason == 0:
                reason = -5
            if reason == 0 and its >= maxits:
                reason = -3
            j += 1
            if reason != 0 or happy:
                break
        kk = j
        y = np.zeros(kk, dtype=np.complex128)
        for i in range(kk - 1, -1, -1):
            y[i] = (rs[i] - H[i, i + 1:kk] @ y[i + 1:kk]) / H[i, i]
        if kk:
            upd = sum(y[i] * V[i] for i in range(kk))
            x = x + (upd if side == "left" else pc(upd))
        if reason != 0:
            break
    return x, its, reason, rn, hist


def fft_preconditioner(dims, lam):
    """x = IDFT3(DFT3(b) ./ Diag) / N with Diag from build_diag_mat_vec_3D: the PCSHELL apply."""
    from .oracle import np_build_diag_3d, np_solve_3d
    n = tuple(int(v) for v in dims)
    diag = np_build_diag_3d(n, tuple(float(v) for v in lam))
    return lambda v: np_solve_3d(diag, v, n)
