"""CPU oracle for the wave-system block-circulant preconditioner -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  Restatements:

* ``jacobian_minus``: ``jacobianMatrices`` (``src/WaveSystem.cxx:92-107``) for a general
  normal: ``(A(n) - |A(n)|) coeff / 2`` with ``A(n) = [[0, c0^2 n^T], [n, 0]]`` and
  ``|A(n)| = diag(c0, c0 n n^T)``.
* ``wave_matrix``: ``computeDivergenceMatrix`` (``src/WaveSystem.cxx:109-176``) as a loop over
  cells and faces: interior/periodic faces ``addValue(j, other, Am)`` and ``addValue(j, j, -Am)``;
  wall faces ``addValue(j, j, -Am (2 v v^T))`` with ``v = (0, n)``; Neumann faces nothing.
* ``block_symbol`` / ``block_solve``: the periodic operator's (dim+1)x(dim+1) symbol built explicitly from
  the same Jacobians, ``S(k) = I + sum_d sum_s Am(s e_d) (exp(i s theta_d) - 1)``, and the exact
  block-circulant inverse ``IDFT(S^-1 DFT(b))`` with ``numpy.linalg.solve`` per frequency.
* ``initial_conditions_shock_wave``: ``src/WaveSystem.cxx:25-76`` (pressure 155e5 inside
  r < 0.3, else 70e5; momentum rho0 * 0).

Parity status: the reference's wave system has no fixture (SOLVERLAB, PETSc absent) and no
FFT preconditioner at all (ToDo.md:10), so this is "parity unpinned" against reference
outputs; ``block_solve`` is pinned to the reference's own assembly instead: the periodic
``wave_matrix`` applied to ``block_solve(b)`` returns ``b`` (tests/test_wave.py).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

C0 = 700.0


def jacobian_minus(normal, coeff, c0=C0) -> np.ndarray:
    n = np.asarray(normal, dtype=float)
    dim = n.size
    A = np.zeros((dim + 1, dim + 1))
    absA = np.zeros((dim + 1, dim + 1))
    absA[0, 0] = c0 * coeff
    for i in range(dim):
        A[i + 1, 0] = n[i] * coeff
        A[0, i + 1] = c0 * c0 * n[i] * coeff
        for j in range(dim):
            absA[i + 1, j + 1] = c0 * n[i] * n[j] * coeff
    return (A - absA) * 0.5


def _dims3(dims):
    d = tuple(int(v) for v in dims)
    return d + (1,) * (3 - len(d))


def wave_matrix(dims, h, dt, c0=C0, bc="wall", shift=0.0, dim=3) -> sp.csr_matrix:
    """computeDivergenceMatrix on a dim-D Cartesian mesh: nbComp = dim + 1 unknowns per cell,
    faces along the first dim axes only (src/WaveSystem.cxx:111-113)."""
    nx, ny, nz = _dims3(dims)
    n = (nx, ny, nz)
    C = dim + 1
    rows, cols, vals = [], [], []

    def add(i, j, M):
        for k in range(C):
            for l in range(C):
                rows.append(i + k)
                cols.append(j + l)
                vals.append(M[k, l])

    for kz in range(nz):
        for jy in range(ny):
            for ix in range(nx):
                cell = ix + nx * (jy + ny * kz)
                add(cell * C, cell * C, shift * np.eye(C))
                idx = [ix, jy, kz]
                for d in range(dim):
                    coeff = dt / h[d]  # dt |F| / |C| on the Cartesian cell
                    for s in (-1, 1):
                        normal = np.zeros(dim)
                        normal[d] = s
                        Am = jacobian_minus(normal, coeff, c0)
                        border = idx[d] == 0 if s < 0 else idx[d] == n[d] - 1
                        if not border:
                            o = list(idx)
                            o[d] += s
                        elif bc == "periodic":
                            o = list(idx)
                            o[d] = n[d] - 1 if s < 0 else 0
                        elif bc == "wall":
                            v = np.zeros(C)
                            v[1:] = normal
                            add(cell * C, cell * C, Am * (-1.0) @ (np.outer(v, v) * 2))
                            continue
                        else:
                            continue
                        other = o[0] + nx * (o[1] + ny * o[2])
                        add(cell * C, other * C, Am)
                        add(cell * C, cell * C, -Am)
    m = C * nx * ny * nz
    A = sp.coo_matrix((np.array(vals, dtype=np.complex128), (rows, cols)), shape=(m, m)).tocsr()
    A.sum_duplicates()
    A.eliminate_zeros()
    return A


def block_symbol(dims, kappa, c0=C0, dim=3) -> np.ndarray:
    """S[kz, ky, kx] ((dim+1) x (dim+1)) of the periodic operator I + A."""
    nx, ny, nz = _dims3(dims)
    C = dim + 1
    kz, ky, kx = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    theta = (2 * np.pi * kx / nx, 2 * np.pi * ky / ny, 2 * np.pi * kz / nz)
    S = np.zeros((nz, ny, nx, C, C), dtype=np.complex128)
    S[...] = np.eye(C)
    for d in range(dim):
        for s in (-1, 1):
            normal = np.zeros(dim)
            normal[d] = s
            Am = jacobian_minus(normal, kappa[d], c0)
            S += Am[None, None, None] * (np.exp(1j * s * theta[d]) - 1)[..., None, None]
    return S


def block_solve(dims, kappa, b, c0=C0, dim=3) -> np.ndarray:
    nx, ny, nz = _dims3(dims)
    B = np.fft.fftn(np.asarray(b, dtype=np.complex128).reshape(nz, ny, nx, dim + 1), axes=(0, 1, 2))
    S = block_symbol(dims, kappa, c0, dim)
    X = np.linalg.solve(S, B[..., None])[..., 0]
    return np.fft.ifftn(X, axes=(0, 1, 2)).reshape(-1)


def initial_conditions_shock_wave(dims, xmin=(-0.5,) * 3, xmax=(0.5,) * 3, dim=3) -> np.ndarray:
    nx, ny, nz = _dims3(dims)
    h = [(xmax[d] - xmin[d]) / (nx, ny, nz)[d] for d in range(3)]
    c = [(xmin[d] + xmax[d]) / 2 for d in range(3)]
    x = xmin[0] + (np.arange(nx) + 0.5) * h[0]
    y = xmin[1] + (np.arange(ny) + 0.5) * h[1]
    z = xmin[2] + (np.arange(nz) + 0.5) * h[2]
    Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
    # src/WaveSystem.cxx:48-61: y enters for dim > 1, z for dim == 3
    r2 = (X - c[0]) ** 2 + ((Y - c[1]) ** 2 if dim > 1 else 0) + ((Z - c[2]) ** 2 if dim == 3 else 0)
    U = np.zeros((nz, ny, nx, dim + 1), dtype=np.complex128)
    U[..., 0] = np.where(np.sqrt(r2) < 0.3, 155e5, 70e5)
    return U.reshape(-1)


def dt_and_kappa(dims, cfl=None, c0=C0, xmin=(-0.5,) * 3, xmax=(0.5,) * 3, dim=3):
    """dt = cfl * minRatioVolSurf / c0 (impl_seq.cxx:18,73; cfl = 1e3/dim by default, :212):
    a cell's measure over the measure of its faces (1-D: two unit-measure end points)."""
    dims = _dims3(dims)
    cfl = 1e3 / dim if cfl is None else cfl
    h = [(xmax[d] - xmin[d]) / dims[d] for d in range(3)]
    if dim == 1:
        ratio = h[0] / 2
    elif dim == 2:
        ratio = h[0] * h[1] / (2 * (h[0] + h[1]))
    else:
        ratio = h[0] * h[1] * h[2] / (2 * (h[0] * h[1] + h[1] * h[2] + h[2] * h[0]))
    dt = cfl * ratio / c0
    return dt, [dt / h[d] if d < dim else 0.0 for d in range(3)], h
