"""Implicit upwind transport on a Cartesian grid, solved by the stand-in KSPGMRES with the
circulant FFT PCSHELL (include/transport_equation.h, csrc/transport_cartesian.cpp).

SURVEY.md §8f row f1: the operator of src/TransportEquation.cxx:75-133 and the time loop of
tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:13-189, with the PCSHELL registered
in the KSP as ToDo.md:1 asks.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from ._lib import check, lib
from ._lib_ext import TransportConfig, TransportResult
from .petsc import PetscCall

UPWIND_REFERENCE, UPWIND_FIXED = 0, 1
PC_NONE, PC_FFT = 0, 1
LAMBDA_REFERENCE, LAMBDA_MATCHED = 0, 1

_SIGN = {"reference": UPWIND_REFERENCE, "faithful": UPWIND_REFERENCE, "fixed": UPWIND_FIXED}
_PC = {"none": PC_NONE, "fft": PC_FFT}
_LAM = {"reference": LAMBDA_REFERENCE, "matched": LAMBDA_MATCHED}


def _d3(v) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def transport_csr(dims: Sequence[int], h: Sequence[float], dt: float, a: Sequence[float],
                  sign: str | int = "reference", shift: float = 0.0):
    """(rowptr, col, val) of shift*I + computeDivergenceMatrix on the grid (host only)."""
    nx, ny, nz = (int(v) for v in dims)
    n = nx * ny * nz
    sm = _SIGN[sign] if isinstance(sign, str) else int(sign)
    rowptr = np.empty(n + 1, dtype=np.int64)
    col = np.empty(7 * n, dtype=np.int64)
    val = np.empty(7 * n, dtype=np.complex128)
    nnz = ctypes.c_int64()
    P64 = ctypes.POINTER(ctypes.c_int64)
    check(lib().cfp_transport_csr(nx, ny, nz, _d3(h), float(dt), _d3(a), sm, float(shift),
                                  rowptr.ctypes.data_as(P64), col.ctypes.data_as(P64),
                                  val.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(nnz)))
    k = nnz.value
    return rowptr, col[:k].copy(), val[:k].copy()


def min_ratio_vol_surf(dim: int, h: Sequence[float]) -> float:
    return float(lib().cfp_cartesian_min_ratio_vol_surf(int(dim), _d3(h)))


def config(n: int | Sequence[int] = 32, **kw) -> TransportConfig:
    """The reference main's defaults (cube [-0.5,0.5]^3, a=(1,0,0), cfl=1e3/3, tmax=0.05,
    precision 1e-5, 1000 KSP iterations) with keyword overrides:
    pc='none'|'fft', sign='reference'|'fixed', lam='reference'|'matched', steps=ntmax,
    device=True/False, plus any TransportConfig field."""
    cfg = TransportConfig()
    dims = (int(n),) * 3 if np.isscalar(n) else tuple(int(v) for v in n)
    lib().cfp_transport_config_default(ctypes.byref(cfg), dims[0])
    cfg.nx, cfg.ny, cfg.nz = dims
    for k, v in kw.items():
        if k == "pc":
            cfg.pc = _PC[v] if isinstance(v, str) else int(v)
        elif k == "sign":
            cfg.sign_mode = _SIGN[v] if isinstance(v, str) else int(v)
        elif k == "lam":
            cfg.lambda_mode = _LAM[v] if isinstance(v, str) else int(v)
        elif k == "steps":
            cfg.ntmax = int(v)
            cfg.tmax = 1e300
        elif k == "device":
            cfg.on_device = 1 if v else 0
        elif k in ("xmin", "xmax", "a"):
            setattr(cfg, k, _d3(v))
        else:
            if not hasattr(cfg, k):
                raise KeyError(k)
            setattr(cfg, k, v)
    return cfg


def run(cfg: TransportConfig, return_field: bool = False):
    """TransportEquationGMRES: the implicit time loop; returns the result dict (and the final
    field as a complex128 array when asked: this rank's rows res['rstart'] .. + res['nlocal'] when
    PETSC_COMM_WORLD has several ranks, the whole field on one)."""
    res = TransportResult()
    n = int(cfg.nx * cfg.ny * cfg.nz)
    out = np.empty(n, dtype=np.complex128) if return_field else None
    ptr = out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if out is not None else None
    PetscCall(lib().TransportEquationGMRES(ctypes.byref(cfg), ctypes.byref(res), ptr))
    d = res.as_dict()
    if out is not None:
        out = out[:d["nlocal"]].copy()
    return (d, out) if return_field else d


def run_direct(cfg: TransportConfig, return_field: bool = False):
    """TransportEquationFFTDirect: the reference's direct-solver time loop
    (tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:20-150), one
    PetscFft3DTransportSolver(ctx, Un, Un) per implicit step."""
    res = TransportResult()
    n = int(cfg.nx * cfg.ny * cfg.nz)
    out = np.empty(n, dtype=np.complex128) if return_field else None
    ptr = out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if out is not None else None
    PetscCall(lib().TransportEquationFFTDirect(ctypes.byref(cfg), ctypes.byref(res), ptr))
    d = res.as_dict()
    return (d, out) if return_field else d
