"""Python host API over the HIP plan (``include/circulant_fft.h``).

PyTorch only supplies device memory and streams here; every computation is a
launch of the gfx950 kernels in ``libcirculant_fft.so``.

    plan = CirculantPlan((nx, ny, nz), device=0)
    plan.set_transport_symbol((lx, ly, lz))      # setupFFTPrec3D (src/PCSHELLFft_3D.cxx:26-84)
    x = plan.apply(b)                            # solve_3D       (src/FftLinearSolver_3D.c:166-190)
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def _stream_handle(stream=None) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def _dev_ptr(t: torch.Tensor, n: int, name: str, device: int | None = None) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != torch.complex128:
        raise TypeError(f"{name} must be complex128, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor")
    if device is not None and t.device.index != device:
        raise ValueError(f"{name} is on cuda:{t.device.index}, the plan on cuda:{device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.numel() != n:
        raise ValueError(f"{name} has {t.numel()} elements, expected {n}")
    return t.data_ptr()


def _lam6(lam: Sequence) -> ctypes.Array:
    vals = []
    for v in lam:
        c = complex(v)
        vals += [c.real, c.imag]
    if len(vals) != 6:
        raise ValueError("lambda must have three entries (x, y, z)")
    return (ctypes.c_double * 6)(*vals)


class StencilT(ctypes.Structure):
    """cfp_stencil_t (include/circulant_fft.h): a row-class diagonal operator on device arrays."""
    _fields_ = [("cls", ctypes.c_void_p), ("mask", ctypes.c_void_p), ("tab", ctypes.c_void_p),
                ("off", ctypes.c_int64 * 8), ("nd", ctypes.c_int), ("ncls", ctypes.c_int), ("x_local", ctypes.c_int),
                ("cls_x", ctypes.c_void_p)]


class ApplyExT(ctypes.Structure):
    """cfp_apply_ex_t (include/circulant_fft.h)."""
    _fields_ = [("pre", ctypes.POINTER(StencilT)), ("post_nv", ctypes.c_int), ("post_v", ctypes.c_void_p * 8),
                ("post_out", ctypes.c_void_p), ("fused", ctypes.c_int)]


def row_class_form(indptr, indices, data, rowlen: int):
    """Row-class diagonal form of a CSR matrix (numpy arrays), as the stand-in AIJ builds it
    (petsc_mini.cpp aij_build_dia): (cls uint8 [n], mask uint8 [ncls], tab complex [ncls, nd],
    offsets [nd], x_local).  Raises ValueError when the matrix has more than 8 diagonals or 256
    distinct rows."""
    n = len(indptr) - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    off_all = indices.astype(np.int64) - rows
    offs = np.unique(off_all)
    if len(offs) > 8:
        raise ValueError("more than 8 diagonals")
    k = np.searchsorted(offs, off_all)
    vals = np.zeros((n, len(offs)), dtype=np.complex128)
    vals[rows, k] = data
    present = np.zeros((n, len(offs)), dtype=bool)
    present[rows, k] = True
    mask_rows = (present * (1 << np.arange(len(offs)))).sum(1).astype(np.uint8)
    key = np.concatenate([vals.view(np.float64), mask_rows[:, None].astype(np.float64)], axis=1)
    uniq, first, cls = np.unique(key, axis=0, return_index=True, return_inverse=True)
    if len(uniq) > 256:
        raise ValueError("more than 256 distinct rows")
    cols = rows + offs[k]
    x_local = bool(n % rowlen == 0 and np.all(cols // rowlen == rows // rowlen))
    return (cls.reshape(-1).astype(np.uint8), mask_rows[first], vals[first], offs, x_local)


PASS_MODES = {0: "fwd", 1: "inv", 2: "fused_sep", 3: "fused_diag", 4: "fused_wave", 5: "rows_fwd", 6: "mid_fused",
              7: "rows_inv", 8: "sym_divide", 9: "plane_fwd", 10: "plane_inv"}
PASS_AXES = {-1: "-", 0: "x", 1: "y", 2: "z", 3: "xy", 4: "yz"}


class CirculantPlan:
    """One (n_x, n_y, n_z) grid on one GPU: the reference's FFT_MAT + Diag (+ b_hat)."""

    def __init__(self, dims: Sequence[int], device: int | None = None):
        nx, ny, nz = (int(d) for d in dims)
        if device is None:
            device = torch.cuda.current_device()
        self.dims = (nx, ny, nz)
        self.N = nx * ny * nz
        self.device = int(device)
        h = ctypes.c_void_p()
        check(lib().cfp_plan_create(ctypes.byref(h), nx, ny, nz, self.device))
        self._h = h

    # ---------------------------------------------------------------- symbol
    def set_transport_symbol(self, lam: Sequence) -> "CirculantPlan":
        """Diag = 1 + sum_d lambda_d (1 - e^{-2 pi i k_d/n_d}) (closed form)."""
        check(lib().cfp_plan_set_symbol_transport(self._h, _lam6(lam)))
        return self

    def set_separable_symbol(self, cx_hat, cy_hat, cz_hat, lam: Sequence) -> "CirculantPlan":
        """Diag = 1 + lx*tile(cx_hat) + ly*repeat(tile(cy_hat)) + lz*repeat(cz_hat)."""
        arrs = [np.ascontiguousarray(np.asarray(a, dtype=np.complex128).reshape(-1)) for a in (cx_hat, cy_hat, cz_hat)]
        for a, n in zip(arrs, self.dims):
            if a.size != n:
                raise ValueError("1-D symbol vector length does not match the grid")
        check(lib().cfp_plan_set_symbol_separable(self._h, arrs[0].ctypes.data, arrs[1].ctypes.data,
                                                  arrs[2].ctypes.data, _lam6(lam)))
        return self

    def set_diag(self, diag) -> "CirculantPlan":
        """General symbol: explicit Diag vector (device tensor or host array)."""
        if isinstance(diag, torch.Tensor) and diag.is_cuda:
            check(lib().cfp_plan_set_diag(self._h, _dev_ptr(diag, self.N, "diag", self.device), 1))
            torch.cuda.synchronize(diag.device)
        else:
            d = np.ascontiguousarray(np.asarray(diag.cpu() if isinstance(diag, torch.Tensor) else diag,
                                                dtype=np.complex128).reshape(-1))
            if d.size != self.N:
                raise ValueError("diag size mismatch")
            check(lib().cfp_plan_set_diag(self._h, d.ctypes.data, 0))
        return self

    def get_diag(self) -> torch.Tensor:
        out = torch.empty(self.N, dtype=torch.complex128, device=f"cuda:{self.device}")
        check(lib().cfp_plan_get_diag(self._h, out.data_ptr(), _stream_handle()))
        return out

    # ---------------------------------------------------------------- apply
    def apply(self, b: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """x = (1/N) IDFT(DFT(b) ./ Diag).  `out` may be `b` (in place)."""
        bp = _dev_ptr(b, self.N, "b", self.device)
        if out is None:
            out = torch.empty_like(b)
        xp = _dev_ptr(out, self.N, "out", self.device)
        check(lib().cfp_plan_apply(self._h, bp, xp, _stream_handle(stream)))
        return out

    def apply_ex(self, b: torch.Tensor, out: torch.Tensor, stencil=None, dots_with=(), stream=None):
        """The Krylov step around one apply (cfp_plan_apply_ex): x = apply(A b) when `stencil` =
        (cls, mask, tab, offsets, x_local[, cls_x]) on the device (uint8, uint8, complex128 tensors;
        cls_x: the [n_x] classes when they depend on x alone), then
        dots[j] = v_j^H x for v_j in `dots_with` (None: x itself).  Returns (dots (complex128
        device tensor or None), fused flag)."""
        ex = ApplyExT()
        keep = []
        if stencil is not None:
            cls, mask, tab, offs, xl = stencil[:5]
            st = StencilT()
            st.cls, st.mask, st.tab = cls.data_ptr(), mask.data_ptr(), tab.data_ptr()
            if len(stencil) > 5 and stencil[5] is not None:  # classes by x alone: [n_x] bytes
                st.cls_x = stencil[5].data_ptr()
            for i, o in enumerate(offs):
                st.off[i] = int(o)
            st.nd, st.ncls, st.x_local = len(offs), int(mask.numel()), 1 if xl else 0
            keep.append(st)
            ex.pre = ctypes.pointer(st)
        dots = None
        if dots_with:
            dots = torch.zeros(len(dots_with), dtype=torch.complex128, device=out.device)
            ex.post_nv = len(dots_with)
            for j, v in enumerate(dots_with[:8]):  # more than 8: refused by the library
                ex.post_v[j] = None if v is None else _dev_ptr(v, self.N, "dots_with", self.device)
            ex.post_out = dots.data_ptr()
        check(lib().cfp_plan_apply_ex(self._h, _dev_ptr(b, self.N, "b", self.device),
                                      _dev_ptr(out, self.N, "out", self.device), _stream_handle(stream),
                                      ctypes.byref(ex)))
        return dots, int(ex.fused)

    def apply_with_diag(self, diag: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                        stream=None) -> torch.Tensor:
        bp = _dev_ptr(b, self.N, "b", self.device)
        dp = _dev_ptr(diag, self.N, "diag", self.device)
        if out is None:
            out = torch.empty_like(b)
        check(lib().cfp_plan_apply_with_diag(self._h, dp, bp, _dev_ptr(out, self.N, "out", self.device),
                                             _stream_handle(stream)))
        return out

    def apply_host(self, b) -> np.ndarray:
        """PCIe-inclusive variant: host numpy in, host numpy out (synchronous)."""
        bb = np.ascontiguousarray(np.asarray(b, dtype=np.complex128).reshape(-1))
        if bb.size != self.N:
            raise ValueError("b size mismatch")
        x = np.empty_like(bb)
        check(lib().cfp_plan_apply_host(self._h, bb.ctypes.data, x.ctypes.data))
        return x

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Unnormalised 3-D DFT (MatMult on MATFFTW)."""
        if out is None:
            out = torch.empty_like(x)
        check(lib().cfp_plan_forward(self._h, _dev_ptr(x, self.N, "x", self.device),
                                     _dev_ptr(out, self.N, "out", self.device),
                                     _stream_handle(stream)))
        return out

    def backward(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Unnormalised inverse 3-D DFT (MatMultTranspose on MATFFTW)."""
        if out is None:
            out = torch.empty_like(x)
        check(lib().cfp_plan_backward(self._h, _dev_ptr(x, self.N, "x", self.device),
                                      _dev_ptr(out, self.N, "out", self.device),
                                      _stream_handle(stream)))
        return out

    def set_chunking(self, chunk_planes: int) -> "CirculantPlan":
        """x/y passes alternate over blocks of `chunk_planes` z-planes (0 = off)."""
        check(lib().cfp_plan_set_chunking(self._h, int(chunk_planes)))
        return self

    def set_graph(self, on: bool = True) -> "CirculantPlan":
        """HIP-graph replay of apply(): the launches of each (b, out) pair are captured once and
        replayed as one graph launch (cfp_plan_set_graph)."""
        check(lib().cfp_plan_set_graph(self._h, int(bool(on))))
        return self

    SCHEDULES = {"auto": 0, "five": 1, "three": 2, "five_y": 3, "plane": 4}

    def set_schedule(self, schedule: str | int) -> "CirculantPlan":
        """'auto'/'five' (z fused), 'five_y' (y fused), 'three' (256^3: 3 sweeps) or 'plane'
        (n_x = n_y in {32, 64, 100, 128}: x + y DFTs of whole z-planes | fused z | inverse planes)."""
        v = self.SCHEDULES[schedule] if isinstance(schedule, str) else int(schedule)
        check(lib().cfp_plan_set_schedule(self._h, v))
        return self

    TP_MIDS = {"default": 0, "lane64": 1, "lane32": 2, "swap64": 3, "swap64pf": 4, "blocked": 5, "blocked32": 6,
               "swap32x": 7, "rowsalt": 8}

    def set_three_pass_shape(self, n1: int = 0, mid: str | int = "default") -> "CirculantPlan":
        """Kernel shape of the 256^3 3-sweep schedule (tests / measurements): the y split n1
        (0 = default, 32 or 64) and the middle kernel ('default' = 'swap64pf', 'lane64', 'lane32',
        'swap64': the y2 DFT on permlane register transposes, 64-column tile; 'swap64pf': the
        same with an LDS-DMA prefetch of half the next unit; 'blocked': 'swap64pf' with the
        blocked intermediate layout, 1 KiB P2 runs; 'blocked32': blocks of 4 x and the permlane
        P2 on 32 columns, two workgroups per CU; n1 = 32 only; 'swap32x': the permlane P2 on 32
        natural-layout columns in XCD order; 'rowsalt': the default with P1 / P3's row-FFT
        exchanges the other way, wave-local or workgroup-wide, n1 = 0 only).  At 100^3 (cfp_three_pass_sq.hip)
        mid picks the middle kernel's x tile: 'default' 4 x, 'lane64' 2 x, 'lane32' 5 x.  At 512^3
        'blocked' / 'blocked32' are blocks of 2 / 8 x (profiles/r05i_p2_512_layouts.md)."""
        m = self.TP_MIDS[mid] if isinstance(mid, str) else int(mid)
        check(lib().cfp_plan_set_three_pass_shape(self._h, int(n1), m))
        return self

    # ---------------------------------------------------------------- introspection
    def passes(self) -> list:
        n = ctypes.c_int()
        check(lib().cfp_plan_num_passes(self._h, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            ax, nn, mode, fast = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            nc = ctypes.c_int64()
            check(lib().cfp_plan_pass_info(self._h, i, ctypes.byref(ax), ctypes.byref(nn), ctypes.byref(nc),
                                           ctypes.byref(mode), ctypes.byref(fast)))
            out.append({"axis": PASS_AXES[ax.value], "n": nn.value, "ncols": nc.value,
                        "mode": PASS_MODES[mode.value], "fast": bool(fast.value)})
        return out

    def time_passes(self, b: torch.Tensor, x: torch.Tensor, iters: int = 20, stream=None) -> list:
        """Mean device time (ms) of each launch of one apply, HIP events on `stream`."""
        npass = len(self.passes())
        ms = (ctypes.c_double * npass)()
        check(lib().cfp_plan_time_passes(self._h, _dev_ptr(b, self.N, "b", self.device),
                                         _dev_ptr(x, self.N, "x", self.device), int(iters),
                                         ms, _stream_handle(stream)))
        return list(ms)

    def profile_begin(self, max_applies: int, every: int = 1) -> "CirculantPlan":
        """Record one HIP event per launch in every `every`-th following apply (at most
        `max_applies` of them)."""
        check(lib().cfp_plan_profile_begin(self._h, int(max_applies), int(every)))
        return self

    def profile_end(self) -> tuple:
        """(mean ms of each launch over the recorded applies, number of applies recorded)."""
        npass = len(self.passes())
        ms = (ctypes.c_double * npass)()
        n = ctypes.c_int()
        check(lib().cfp_plan_profile_end(self._h, ms, ctypes.byref(n)))
        return list(ms), n.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cfp_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def fill_uniform(t: torch.Tensor, seed: int, offset: int = 0, stream=None) -> torch.Tensor:
    """Counter-based synthetic input generated on the GPU."""
    check(lib().cfp_fill_uniform(_dev_ptr(t, t.numel(), "t"), t.numel(), int(seed), int(offset),
                                 _stream_handle(stream)))
    return t


def transport_symbol_1d(n: int) -> np.ndarray:
    out = np.empty(int(n), dtype=np.complex128)
    check(lib().cfp_transport_symbol_1d(int(n), out.ctypes.data))
    return out


def pointwise_divide(w: torch.Tensor, x: torch.Tensor, y: torch.Tensor, stream=None) -> torch.Tensor:
    n = w.numel()
    check(lib().cfp_pointwise_divide(_dev_ptr(w, n, "w"), _dev_ptr(x, n, "x"), _dev_ptr(y, n, "y"), n,
                                     _stream_handle(stream)))
    return w


def scale(x: torch.Tensor, alpha: complex, stream=None) -> torch.Tensor:
    a = complex(alpha)
    check(lib().cfp_scale(_dev_ptr(x, x.numel(), "x"), a.real, a.imag, x.numel(), _stream_handle(stream)))
    return x


def build_diag_3d(diag: torch.Tensor, cx_hat: torch.Tensor, cy_hat: torch.Tensor, cz_hat: torch.Tensor,
                  dims: Sequence[int], lam: Sequence, stream=None) -> torch.Tensor:
    nx, ny, nz = (int(d) for d in dims)
    check(lib().cfp_build_diag_3d(_dev_ptr(diag, nx * ny * nz, "diag"), _dev_ptr(cx_hat, nx, "cx_hat"),
                                  _dev_ptr(cy_hat, ny, "cy_hat"), _dev_ptr(cz_hat, nz, "cz_hat"), nx, ny, nz,
                                  _lam6(lam), _stream_handle(stream)))
    return diag


class RealPlan:
    """Real-data apply (include/circulant_fft_real.h): x = C^{-1} b for a
    real float64 b and a real transport symbol, r2c / half spectrum / c2r, ~80 N bytes per
    apply.  The reference's real-scalar solve_3D (src/FftLinearSolver_3D.c:6-78, 166-190)."""

    def __init__(self, dims: Sequence[int], device: int | None = None):
        nx, ny, nz = (int(d) for d in dims)
        self.dims = (nx, ny, nz)
        self.N = nx * ny * nz
        self.device = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        check(lib().cfp_rplan_create(ctypes.byref(h), nx, ny, nz, self.device))
        self._h = h

    def set_transport_symbol(self, lam: Sequence[float]) -> "RealPlan":
        vals = [float(v) for v in lam]
        if len(vals) != 3:
            raise ValueError("lambda must have three real entries")
        check(lib().cfp_rplan_set_symbol_transport(self._h, (ctypes.c_double * 3)(*vals)))
        return self

    SCHEDULES = {"auto": 0, "five": 1, "three": 2, "three_alt": 3}

    def set_schedule(self, schedule: str | int) -> "RealPlan":
        """'auto' (3 sweeps at 128^3 and 256^3), 'five' (r2c + 3 half-spectrum passes + c2r), 'three'
        (128^3 and 256^3 only) or 'three_alt' (the 3 sweeps with the row sweeps' FFT exchanges
        behind workgroup barriers instead of wave-local, for A/B)."""
        v = self.SCHEDULES[schedule] if isinstance(schedule, str) else int(schedule)
        check(lib().cfp_rplan_set_schedule(self._h, v))
        return self

    @property
    def three_sweep(self) -> bool:
        """True when the next apply runs the 3-sweep schedule."""
        t = ctypes.c_int()
        check(lib().cfp_rplan_schedule(self._h, ctypes.byref(t)))
        return bool(t.value)

    def _ptr(self, t: torch.Tensor, name: str) -> int:
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.N:
            raise ValueError(f"{name} must be a contiguous float64 device tensor of {self.N} elements")
        if t.device.index != self.device:
            raise ValueError(f"{name} is on cuda:{t.device.index}, the plan on cuda:{self.device}")
        return t.data_ptr()

    def apply(self, b: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(b)
        check(lib().cfp_rplan_apply(self._h, self._ptr(b, "b"), self._ptr(out, "out"), _stream_handle(stream)))
        return out

    def time_passes(self, b: torch.Tensor, x: torch.Tensor, iters: int = 20, stream=None) -> list:
        """Mean ms of the 4 stages: r2c rows (+ y1 in the 3-sweep schedule), half-spectrum y/z
        (y2/z), Nyquist y/z, (y1 inverse +) c2r rows."""
        ms = (ctypes.c_double * 4)()
        check(lib().cfp_rplan_time_passes(self._h, self._ptr(b, "b"), self._ptr(x, "x"), int(iters), ms,
                                          _stream_handle(stream)))
        return list(ms)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cfp_rplan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
