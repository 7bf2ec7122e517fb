"""CPU oracle for the circulant FFT preconditioner -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module; the product package
(``circulantpreconditioner_amd``) never does.

Two restatements of the reference arithmetic live here:

* ``libcfp_oracle.so`` (``oracle/cfp_oracle.c``): the C restatement of
  ``src/FftLinearSolver_3D.c:80-190`` (Diag build via Kronecker tiling,
  ``solve_3D``) plus FFTW's unnormalised DFT semantics.  Used for large sizes
  and as the CPU baseline.
* numpy functions below that restate the reference's own Python oracle
  ``tests/FFTDirectSolver/testFftSolver_3D.py:6-52`` with ``numpy.fft``.

Both are pinned by the golden fixtures in ``tests/golden/`` that were
generated from the reference's Python functions (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcfp_oracle.so")
_lib = None


def build() -> str:
    """Compile the C restatement (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, dp, c_int = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
        L.oracle_set_threads.argtypes = [c_int]
        L.oracle_get_max_threads.restype = c_int
        L.oracle_dft1d.argtypes = [i64, c_int, dp, dp]
        L.oracle_fft3d.argtypes = [i64, i64, i64, c_int, dp, dp]
        L.oracle_build_transport_col.argtypes = [i64, dp]
        L.oracle_kron_left.argtypes = [dp, dp, i64, i64, ctypes.c_double, ctypes.c_double]
        L.oracle_kron_right.argtypes = [dp, dp, i64, i64, ctypes.c_double, ctypes.c_double]
        L.oracle_build_diag_3d.argtypes = [dp, dp, dp, dp, i64, i64, i64, dp]
        L.oracle_build_diag_transport.argtypes = [i64, i64, i64, dp, dp]
        L.oracle_solve_3d.argtypes = [i64, i64, i64, dp, dp, dp]
        L.oracle_apply_circulant.argtypes = [i64, i64, i64, dp, dp, dp]
        L.oracle_fill_uniform.argtypes = [i64, ctypes.c_uint64, i64, dp]
        _lib = L
    return _lib


def _c128(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.complex128)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _lam6(lam) -> np.ndarray:
    lam = [complex(v) for v in lam]
    return np.array([lam[0].real, lam[0].imag, lam[1].real, lam[1].imag, lam[2].real, lam[2].imag],
                    dtype=np.float64)


def set_threads(n: int) -> None:
    lib().oracle_set_threads(int(n))


# ---------------------------------------------------------------- C oracle
def c_dft1d(x, sign=-1) -> np.ndarray:
    x = _c128(x)
    out = np.empty_like(x)
    lib().oracle_dft1d(x.size, sign, _ptr(x), _ptr(out))
    return out


def c_fft3d(b, n, sign=-1) -> np.ndarray:
    """MatMult (sign=-1) / MatMultTranspose (sign=+1) on a MATFFTW of dims {nz,ny,nx}."""
    nx, ny, nz = n
    b = _c128(b).reshape(-1)
    out = np.empty_like(b)
    lib().oracle_fft3d(nx, ny, nz, sign, _ptr(b), _ptr(out))
    return out


def c_build_diag_transport(n, lam) -> np.ndarray:
    nx, ny, nz = n
    d = np.empty(nx * ny * nz, dtype=np.complex128)
    l6 = _lam6(lam)
    lib().oracle_build_diag_transport(nx, ny, nz, _ptr(l6), _ptr(d))
    return d


def c_build_diag_3d(cx_hat, cy_hat, cz_hat, n, lam) -> np.ndarray:
    nx, ny, nz = n
    cx, cy, cz = _c128(cx_hat), _c128(cy_hat), _c128(cz_hat)
    d = np.empty(nx * ny * nz, dtype=np.complex128)
    l6 = _lam6(lam)
    lib().oracle_build_diag_3d(_ptr(d), _ptr(cx), _ptr(cy), _ptr(cz), nx, ny, nz, _ptr(l6))
    return d


def c_solve_3d(diag, b, n) -> np.ndarray:
    nx, ny, nz = n
    d, bb = _c128(diag).reshape(-1), _c128(b).reshape(-1)
    x = np.empty_like(bb)
    lib().oracle_solve_3d(nx, ny, nz, _ptr(d), _ptr(bb), _ptr(x))
    return x


def c_apply_circulant(x, n, lam) -> np.ndarray:
    nx, ny, nz = n
    xx = _c128(x).reshape(-1)
    y = np.empty_like(xx)
    l6 = _lam6(lam)
    lib().oracle_apply_circulant(nx, ny, nz, _ptr(l6), _ptr(xx), _ptr(y))
    return y


def c_fill_uniform(count: int, seed: int, offset: int = 0) -> np.ndarray:
    out = np.empty(count, dtype=np.complex128)
    lib().oracle_fill_uniform(count, seed, offset, _ptr(out))
    return out


# ------------------------------------------------------------ numpy oracle
def np_transport_col(size: int) -> np.ndarray:
    """build_circulant_col, testFftSolver_3D.py:6-10 (size-1 axis -> zero column,
    as build_transport_col src/FftLinearSolver_3D.c:80-90)."""
    col = np.zeros(size, dtype=np.complex128)
    if size > 1:
        col[0], col[1] = 1, -1
    return col


def np_build_diag_3d(n, lam) -> np.ndarray:
    """build_diag_mat_vec_3D, testFftSolver_3D.py:26-36."""
    nx, ny, nz = n
    lx, ly, lz = lam
    cx, cy, cz = (np.fft.fft(np_transport_col(k)) for k in (nx, ny, nz))
    return 1 + lx * np.tile(cx, ny * nz) + ly * np.repeat(np.tile(cy, nz), nx) + lz * np.repeat(cz, nx * ny)


def np_diag_closed_form(n, lam) -> np.ndarray:
    """Diag[k] = 1 + sum_d lambda_d (1 - exp(-2 pi i k_d / n_d))  (SURVEY App. B)."""
    nx, ny, nz = n
    kz, ky, kx = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    d = np.ones((nz, ny, nx), dtype=np.complex128)
    for lam_d, k, nd in ((lam[0], kx, nx), (lam[1], ky, ny), (lam[2], kz, nz)):
        if nd > 1:
            d = d + lam_d * (1 - np.exp(-2j * np.pi * k / nd))
    return d.reshape(-1)


def np_solve_3d(diag, b, n) -> np.ndarray:
    """solve_circulant_system_3D, testFftSolver_3D.py:48-52 == solve_3D (x fastest)."""
    nx, ny, nz = n
    bh = np.fft.fftn(np.asarray(b, dtype=np.complex128).reshape(nz, ny, nx))
    d = np.asarray(diag).reshape(nz, ny, nx)
    with np.errstate(divide="ignore", invalid="ignore"):  # PETSc VecPointwiseDivide: y = 0 -> 0
        q = np.where(d != 0, bh / np.where(d != 0, d, 1), 0)
    return np.fft.ifftn(q).reshape(-1)


def np_dense_C(n, lam) -> np.ndarray:
    """build_C_3D, testFftSolver_3D.py:12-24, dense (small sizes only)."""
    from scipy.linalg import circulant
    nx, ny, nz = n
    lx, ly, lz = lam
    Cx = np.kron(np.eye(ny * nz), circulant(np_transport_col(nx)))
    Cy = np.kron(np.eye(nz), np.kron(circulant(np_transport_col(ny)), np.eye(nx)))
    Cz = np.kron(circulant(np_transport_col(nz)), np.eye(nx * ny))
    return np.eye(nx * ny * nz) + lx * Cx + ly * Cy + lz * Cz


def rel_l2(a, b) -> float:
    a = np.asarray(a).reshape(-1)
    b = np.asarray(b).reshape(-1)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))
