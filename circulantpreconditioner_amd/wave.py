"""Wave-system block-circulant preconditioner and implicit GMRES loop (include/wave_system.h,
SURVEY.md §8f row f2, BASELINE config 4).

``WavePlan``: x = S^{-1} b for the periodic wave-system operator with dim + 1 interleaved
unknowns per cell (pressure, dim momentum components; idx = cell*(dim+1) + comp as the
reference's Un, tests/WaveSystem_SphericalExplosion_impl_seq.cxx:19,57-68), one HIP plan,
at most 5 HBM sweeps.  dim = 3 by default; the reference mains' own default is 2-D (50 x 50).
``wave_csr``: the reference operator (src/WaveSystem.cxx:92-176) on a Cartesian grid.
``config``/``run``: WaveSystem_impl_seq's time loop with the block-circulant PCSHELL.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from ._lib import check, lib
from ._lib_ext import WaveConfig, WaveResult
from .petsc import PetscCall
from .plan import _dev_ptr, _stream_handle

C0 = 700.0  # src/WaveSystem.hxx:17
BC_WALL, BC_PERIODIC, BC_NEUMANN = 0, 1, 2
_BC = {"wall": BC_WALL, "periodic": BC_PERIODIC, "neumann": BC_NEUMANN}
PC_NONE, PC_FFT = 0, 1


def _d3(v) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def _dims3(dims: Sequence[int]) -> tuple:
    d = tuple(int(v) for v in dims)
    return d + (1,) * (3 - len(d))


class WavePlan:
    """Block-circulant inverse on an nx*ny*nz grid with dim + 1 interleaved components."""

    def __init__(self, dims: Sequence[int], device: int | None = None, dim: int = 3):
        nx, ny, nz = _dims3(dims)
        self.dims = (nx, ny, nz)
        self.dim = int(dim)
        self.ncomp = self.dim + 1
        self.size = self.ncomp * nx * ny * nz
        self.device = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        check(lib().cfp_wave_plan_create_dim(ctypes.byref(h), nx, ny, nz, self.dim, self.device))
        self._h = h

    def set_symbol(self, kappa: Sequence[float], c0: float = C0) -> "WavePlan":
        check(lib().cfp_wave_plan_set_symbol(self._h, _d3(kappa), float(c0)))
        return self

    SCHEDULES = {"auto": 0, "five": 1, "three": 2}

    def set_schedule(self, schedule: str | int = "auto") -> "WavePlan":
        """'auto' (3 sweeps on a 3-D 128^3 grid, else 5), 'five', or 'three' (3-D 128^3 only)."""
        v = self.SCHEDULES[schedule] if isinstance(schedule, str) else int(schedule)
        check(lib().cfp_wave_plan_set_schedule(self._h, v))
        return self

    def apply(self, b: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(b)
        check(lib().cfp_wave_plan_apply(self._h, _dev_ptr(b, self.size, "b"), _dev_ptr(out, self.size, "out"),
                                        _stream_handle(stream)))
        return out

    def apply_dots(self, b: torch.Tensor, out: torch.Tensor | None = None, dots_with=(), stream=None):
        """x = S^{-1} b and the dots v^H x for each v in dots_with (None: x itself), at most 8,
        computed inside the last sweep on the 3-sweep schedule (cfp_wave_plan_apply_dots).
        Returns (x, dots as a complex128 tensor on the device, fused)."""
        if out is None:
            out = torch.empty_like(b)
        nv = len(dots_with)
        dots = torch.zeros(max(1, nv), dtype=torch.complex128, device=b.device)
        ptrs = (ctypes.c_void_p * max(1, nv))(*[None if v is None else _dev_ptr(v, self.size, "v") for v in dots_with])
        fused = ctypes.c_int()
        check(lib().cfp_wave_plan_apply_dots(self._h, _dev_ptr(b, self.size, "b"), _dev_ptr(out, self.size, "out"),
                                             _stream_handle(stream), nv, ptrs, dots.data_ptr(), ctypes.byref(fused)))
        return out, dots[:nv], fused.value

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(x)
        check(lib().cfp_wave_plan_forward(self._h, _dev_ptr(x, self.size, "x"), _dev_ptr(out, self.size, "out"),
                                          _stream_handle(stream)))
        return out

    def backward(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(x)
        check(lib().cfp_wave_plan_backward(self._h, _dev_ptr(x, self.size, "x"), _dev_ptr(out, self.size, "out"),
                                           _stream_handle(stream)))
        return out

    def num_passes(self) -> int:
        n = ctypes.c_int()
        check(lib().cfp_wave_plan_num_passes(self._h, ctypes.byref(n)))
        return n.value

    def time_passes(self, b: torch.Tensor, x: torch.Tensor, iters: int = 10, stream=None) -> list:
        np_ = self.num_passes()
        ms = (ctypes.c_double * np_)()
        check(lib().cfp_wave_plan_time_passes(self._h, _dev_ptr(b, self.size, "b"), _dev_ptr(x, self.size, "x"),
                                              int(iters), ms, _stream_handle(stream)))
        return list(ms)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cfp_wave_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def wave_csr(dims: Sequence[int], h: Sequence[float], dt: float, c0: float = C0, bc: str | int = "wall",
             shift: float = 0.0, dim: int = 3):
    """(rowptr, col, val) of shift*I + computeDivergenceMatrix of the wave system (host)."""
    nx, ny, nz = _dims3(dims)
    C = int(dim) + 1
    m = C * nx * ny * nz
    room = C * (2 * int(dim) + 1) * m
    rowptr = np.empty(m + 1, dtype=np.int64)
    col = np.empty(room, dtype=np.int64)
    val = np.empty(room, dtype=np.complex128)
    nnz = ctypes.c_int64()
    P64 = ctypes.POINTER(ctypes.c_int64)
    b = _BC[bc] if isinstance(bc, str) else int(bc)
    hh = list(h) + [1.0] * (3 - len(h))
    check(lib().cfp_wave_csr_dim(nx, ny, nz, int(dim), _d3(hh), float(dt), float(c0), b, float(shift),
                                 rowptr.ctypes.data_as(P64), col.ctypes.data_as(P64),
                                 val.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(nnz)))
    k = nnz.value
    return rowptr, col[:k].copy(), val[:k].copy()


def config(n: int | Sequence[int] = 32, dim: int = 3, **kw) -> WaveConfig:
    """WaveSystem_impl_seq's defaults (c0 = 700, cfl = 1e3/dim, tmax = 0.05, precision 1e-5,
    1000 iterations, wall boundaries) on a dim-D grid of n cells a side (or the given dims),
    with overrides: pc='none'|'fft', bc='wall'|'periodic'|'neumann', steps=ntmax,
    device=True/False, or any WaveConfig field.  The reference main's default is
    ``config(50, dim=2)``."""
    cfg = WaveConfig()
    dim = int(dim)
    dims = (int(n),) * dim + (1,) * (3 - dim) if np.isscalar(n) else _dims3(n)
    lib().cfp_wave_config_default_dim(ctypes.byref(cfg), dims[0], dim)
    cfg.nx, cfg.ny, cfg.nz = dims
    for k, v in kw.items():
        if k == "pc":
            cfg.pc = {"none": PC_NONE, "fft": PC_FFT}[v] if isinstance(v, str) else int(v)
        elif k == "bc":
            cfg.bc = _BC[v] if isinstance(v, str) else int(v)
        elif k == "steps":
            cfg.ntmax = int(v)
            cfg.tmax = 1e300
        elif k == "device":
            cfg.on_device = 1 if v else 0
        elif k in ("xmin", "xmax"):
            setattr(cfg, k, _d3(v))
        else:
            if not hasattr(cfg, k):
                raise KeyError(k)
            setattr(cfg, k, v)
    return cfg


def run(cfg: WaveConfig, return_field: bool = False):
    """WaveSystemGMRES: the implicit time loop; result dict (and the final (dim+1)N field: this
    rank's rows res['rstart'] .. + res['nlocal'] when PETSC_COMM_WORLD has several ranks)."""
    res = WaveResult()
    m = int(((cfg.dim or 3) + 1) * cfg.nx * cfg.ny * cfg.nz)
    out = np.empty(m, dtype=np.complex128) if return_field else None
    ptr = out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if out is not None else None
    PetscCall(lib().WaveSystemGMRES(ctypes.byref(cfg), ctypes.byref(res), ptr))
    d = res.as_dict()
    if out is not None:  # this rank's rows when PETSC_COMM_WORLD has several ranks
        out = out[:d["nlocal"]].copy()
    return (d, out) if return_field else d
