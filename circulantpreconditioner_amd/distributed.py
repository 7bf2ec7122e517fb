"""Slab-decomposed circulant apply over several GPUs (include/circulant_fft_dist.h).

``SlabPlan``: one process per GPU (torch.distributed.run), RCCL all-to-all over
xGMI between the y and z passes.  The 128-byte RCCL unique id is created by the
library on rank 0 and broadcast through the caller's torch.distributed group.

``SlabGroup``: one process driving P slabs (on one or several GPUs) with device
copies as the exchange -- the same pass schedule, usable on a one-GPU machine.

Layout: rank r holds z-planes [r nz/P, (r+1) nz/P), i.e. the
contiguous elements [r N/P, (r+1) N/P) -- PETSc's PETSC_DECIDE Vec layout.
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Sequence

import torch

from ._lib import check, lib
from .plan import PASS_MODES, _dev_ptr, _lam6, _stream_handle


def _slab_schedule(schedule) -> int:
    """'auto' | 'five' | 'three' (CFP_SCHEDULE_AUTO / _FIVE_PASS / _THREE_PASS)"""
    return {"auto": 0, "five": 1, "three": 2}[schedule] if isinstance(schedule, str) else int(schedule)


def slab_layout(dims: Sequence[int], nranks: int, rank: int) -> dict:
    """Host-only layout query (no GPU needed)."""
    nx, ny, nz = (int(d) for d in dims)
    out = (ctypes.c_int64 * 8)()
    check(lib().cfp_slab_layout(nx, ny, nz, int(nranks), int(rank), out))
    keys = ("nz_local", "ny_local", "z0", "y0", "local_size", "chunk", "local_offset", "nranks")
    return dict(zip(keys, list(out)))


STEP_KEYS = ("kind", "src", "dst", "axis", "n", "mode", "ncols", "inner_n",
             "in_inner", "in_outer", "in_pt", "in_seg_len", "in_seg_stride",
             "out_inner", "out_outer", "out_pt", "out_seg_len", "out_seg_stride")


def slab_steps(dims: Sequence[int], nranks: int, rank: int) -> list:
    """Host-only: the steps rank `rank`'s cfp_dist_plan_apply runs, as dicts (STEP_KEYS + scale);
    buffers 0 = b, 1 = x, 2 = work (include/circulant_fft_dist.h)."""
    nx, ny, nz = (int(d) for d in dims)
    n = ctypes.c_int()
    check(lib().cfp_slab_num_steps(nx, ny, nz, int(nranks), int(rank), ctypes.byref(n)))
    out = []
    for i in range(n.value):
        desc = (ctypes.c_int64 * 18)()
        sc = ctypes.c_double()
        check(lib().cfp_slab_step_info(nx, ny, nz, int(nranks), int(rank), i, desc, ctypes.byref(sc)))
        d = dict(zip(STEP_KEYS, list(desc)))
        d["scale"] = sc.value
        out.append(d)
    return out


class SlabPlan:
    """This rank's part of a slab-distributed plan.

    exchange="rccl": the library's own RCCL communicator does both all-to-alls inside
    cfp_dist_plan_apply.  exchange="torch": the library runs the three kernel segments and
    the two all-to-alls go through torch.distributed.all_to_all_single on `group` (RCCL
    under torch's "nccl" backend; under "gloo" the chunks are staged through host memory,
    which lets several ranks share one GPU in tests).  Both are one stream-ordered apply:
    the exchanges are issued on the apply's stream.
    """

    def __init__(self, dims: Sequence[int], rank: int, world: int, device: int | None = None, group=None,
                 exchange: str = "rccl"):
        import torch.distributed as dist
        nx, ny, nz = (int(d) for d in dims)
        self.dims = (nx, ny, nz)
        self.rank, self.world = int(rank), int(world)
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.group = group
        self.exchange = exchange
        self.layout = slab_layout(self.dims, self.world, self.rank)
        h = ctypes.c_void_p()
        if exchange == "rccl":
            nbytes = lib().cfp_dist_unique_id_bytes()
            uid = ctypes.create_string_buffer(nbytes)
            if self.rank == 0:
                check(lib().cfp_dist_get_unique_id(uid))
            on_dev = dist.get_backend(group) == "nccl"
            t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8)
            t = t.to(f"cuda:{self.device}") if on_dev else t.clone()
            dist.broadcast(t, src=0, group=group)
            uid = ctypes.create_string_buffer(bytes(t.cpu().numpy().tobytes()), nbytes)
            check(lib().cfp_dist_plan_create(ctypes.byref(h), nx, ny, nz, self.world, self.rank, uid, self.device))
        elif exchange == "torch":
            check(lib().cfp_dist_plan_create_external(ctypes.byref(h), nx, ny, nz, self.world, self.rank,
                                                      self.device))
            self.work = torch.empty(self.local_size, dtype=torch.complex128, device=f"cuda:{self.device}")
            check(lib().cfp_dist_plan_set_work_buffer(h, self.work.data_ptr()))
        else:
            raise ValueError("exchange must be 'rccl' or 'torch'")
        self._h = h

    @property
    def local_size(self) -> int:
        return self.layout["local_size"]

    @property
    def local_offset(self) -> int:
        return self.layout["local_offset"]

    def set_transport_symbol(self, lam) -> "SlabPlan":
        check(lib().cfp_dist_plan_set_symbol_transport(self._h, _lam6(lam)))
        return self

    def set_schedule(self, schedule: str | int) -> "SlabPlan":
        """Local passes: 'auto' (3 sweeps at 256^3 with world | 32), 'five' or 'three'."""
        check(lib().cfp_dist_plan_set_schedule(self._h, _slab_schedule(schedule)))
        return self

    def _all_to_all(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        import torch.distributed as dist
        if dist.get_backend(self.group) == "gloo":  # gloo exchanges host tensors only
            h = torch.empty(dst.numel(), dtype=dst.dtype)
            dist.all_to_all_single(h, src.cpu(), group=self.group)
            dst.copy_(h)
        else:
            dist.all_to_all_single(dst, src, group=self.group)

    def apply(self, b: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(b)
        n = self.local_size
        bp, xp = _dev_ptr(b, n, "b", self.device), _dev_ptr(out, n, "out", self.device)
        sh = _stream_handle(stream)
        if self.exchange == "rccl":
            check(lib().cfp_dist_plan_apply(self._h, bp, xp, sh))
            return out
        # the segments run on `stream`; the collectives are ordered on torch's current stream,
        # so make that the same stream for the whole apply
        with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
            check(lib().cfp_dist_plan_run_segment(self._h, 0, bp, xp, sh))
            self._all_to_all(out, self.work)  # work chunks -> x chunks
            check(lib().cfp_dist_plan_run_segment(self._h, 1, bp, xp, sh))
            self._all_to_all(self.work, out)  # x chunks -> work chunks
            check(lib().cfp_dist_plan_run_segment(self._h, 2, bp, xp, sh))
        return out

    def phases(self) -> list:
        """The apply's steps: axis passes and all-to-all exchanges, in order."""
        nph = ctypes.c_int()
        check(lib().cfp_dist_plan_num_phases(self._h, ctypes.byref(nph)))
        out = []
        for i in range(nph.value):
            ex, ax, n, mode = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            check(lib().cfp_dist_plan_phase_info(self._h, i, ctypes.byref(ex), ctypes.byref(ax), ctypes.byref(n),
                                                 ctypes.byref(mode)))
            if ex.value:
                out.append({"kind": "all-to-all"})
            else:
                out.append({"kind": "pass", "axis": "xyz"[ax.value], "n": n.value, "mode": PASS_MODES[mode.value]})
        return out

    def profile_begin(self, max_applies: int, every: int = 1) -> bool:
        """Sampled per-phase events inside the following applies (RCCL exchange only; returns
        False for the torch-exchange path, whose exchanges are outside the library)."""
        if self.exchange != "rccl":
            return False
        check(lib().cfp_dist_plan_profile_begin(self._h, int(max_applies), int(every)))
        return True

    def profile_end(self) -> tuple:
        nph = ctypes.c_int()
        check(lib().cfp_dist_plan_num_phases(self._h, ctypes.byref(nph)))
        ms = (ctypes.c_double * nph.value)()
        n = ctypes.c_int()
        check(lib().cfp_dist_plan_profile_end(self._h, ms, ctypes.byref(n)))
        return list(ms), n.value

    def time_phases(self, b: torch.Tensor, x: torch.Tensor, iters: int = 10, stream=None) -> list:
        """Mean ms of each phase (passes and exchanges, in order) over `iters` applies."""
        if self.exchange == "torch":
            return self._time_phases_torch(b, x, iters)
        nph = ctypes.c_int()
        check(lib().cfp_dist_plan_num_phases(self._h, ctypes.byref(nph)))
        ms = (ctypes.c_double * nph.value)()
        n = self.local_size
        check(lib().cfp_dist_plan_time_phases(self._h, _dev_ptr(b, n, "b", self.device),
                                              _dev_ptr(x, n, "x", self.device), int(iters), ms,
                                              _stream_handle(stream)))
        return list(ms)

    def _time_phases_torch(self, b, x, iters):
        ph = self.phases()
        n = self.local_size
        bp, xp = _dev_ptr(b, n, "b", self.device), _dev_ptr(x, n, "x", self.device)
        sh = _stream_handle()
        acc = [0.0] * len(ph)
        for _ in range(iters):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(ph) + 1)]
            seg = 0
            for i, p in enumerate(ph):
                ev[i].record()
                if p["kind"] == "all-to-all":
                    if seg == 1:
                        self._all_to_all(x, self.work)
                    else:
                        self._all_to_all(self.work, x)
                    continue
                # run this single pass: segments hold consecutive passes, so time per segment
                # once (the first pass of a segment carries the whole segment)
                first_of_seg = i == 0 or ph[i - 1]["kind"] == "all-to-all"
                if first_of_seg:
                    check(lib().cfp_dist_plan_run_segment(self._h, seg, bp, xp, sh))
                    seg += 1
            ev[-1].record()
            torch.cuda.synchronize()
            for i in range(len(ph)):
                acc[i] += ev[i].elapsed_time(ev[i + 1])
        return [a / iters for a in acc]

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cfp_dist_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SlabGroup:
    """P slabs driven from one process (exchange = device copies)."""

    def __init__(self, dims: Sequence[int], nranks: int, devices: Sequence[int] | None = None):
        nx, ny, nz = (int(d) for d in dims)
        self.dims = (nx, ny, nz)
        self.P = int(nranks)
        devs = list(devices) if devices is not None else [torch.cuda.current_device()] * self.P
        if len(devs) != self.P:
            raise ValueError("one device per slab")
        self.devices = devs
        arr = (ctypes.c_int * self.P)(*devs)
        h = ctypes.c_void_p()
        check(lib().cfp_group_create(ctypes.byref(h), nx, ny, nz, self.P, arr))
        self._h = h
        self.layouts = [slab_layout(self.dims, self.P, r) for r in range(self.P)]

    def set_transport_symbol(self, lam) -> "SlabGroup":
        check(lib().cfp_group_set_symbol_transport(self._h, _lam6(lam)))
        return self

    def set_schedule(self, schedule: str | int) -> "SlabGroup":
        """Local passes per slab: 'auto' (3 sweeps at 256^3 with P | 32), 'five' or 'three'."""
        check(lib().cfp_group_set_schedule(self._h, _slab_schedule(schedule)))
        return self

    def scatter(self, full: torch.Tensor) -> list:
        out = []
        for r, L in enumerate(self.layouts):
            o, n = L["local_offset"], L["local_size"]
            out.append(full[o:o + n].to(f"cuda:{self.devices[r]}").contiguous())
        return out

    def apply(self, bs: Sequence[torch.Tensor], xs: Sequence[torch.Tensor] | None = None) -> list:
        if xs is None:
            xs = [torch.empty_like(b) for b in bs]
        bp = (ctypes.c_void_p * self.P)(*[_dev_ptr(b, L["local_size"], "b", d)
                                          for b, L, d in zip(bs, self.layouts, self.devices)])
        xp = (ctypes.c_void_p * self.P)(*[_dev_ptr(x, L["local_size"], "x", d)
                                          for x, L, d in zip(xs, self.layouts, self.devices)])
        check(lib().cfp_group_apply(self._h, bp, xp))
        return list(xs)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cfp_group_destroy(self._h)
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
