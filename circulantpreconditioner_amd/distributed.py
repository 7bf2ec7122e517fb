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
    """Host-only layout query (no GPU needed).  ny_local: this rank's z-pencil rows (blocks of
    ny_chunk = ceil(ny / nranks), FFTW-MPI's split; the last ranks may hold fewer);
    work_size: elements of one work buffer (max(local_size, nranks * chunk))."""
    nx, ny, nz = (int(d) for d in dims)
    out = (ctypes.c_int64 * 8)()
    check(lib().cfp_slab_layout(nx, ny, nz, int(nranks), int(rank), out))
    keys = ("nz_local", "ny_local", "z0", "y0", "local_size", "chunk", "local_offset", "nranks")
    d = dict(zip(keys, list(out)))
    w = ctypes.c_int64()
    check(lib().cfp_slab_work_size(nx, ny, nz, int(nranks), int(rank), ctypes.byref(w)))
    d["work_size"] = w.value
    d["ny_chunk"] = d["chunk"] // (d["nz_local"] * nx)
    return d


STEP_KEYS = ("kind", "src", "dst", "axis", "n", "mode", "ncols", "inner_n",
             "in_inner", "in_outer", "in_pt", "in_seg_len", "in_seg_stride",
             "out_inner", "out_outer", "out_pt", "out_seg_len", "out_seg_stride",
             "src_off", "dst_off", "ex_off", "ex_cnt", "chunk", "wait", "lnyl", "k1_off", "seg", "fused")
STEP_KINDS = {0: "pass", 1: "exchange", 2: "three_sweep", 3: "repack"}
STEP_LISTS = {"apply": 0, "apply_diag": 1, "forward": 2, "backward": 3, "diag": 4}


def slab_steps(dims: Sequence[int], nranks: int, rank: int, schedule="five", pieces: int = 1,
               list_: str = "apply") -> list:
    """Host-only: the steps of rank `rank`'s slab plan as dicts (STEP_KEYS + scale): `schedule`
    'auto' | 'five' | 'three', `pieces` 0 (AUTO) or K, `list_` 'apply' | 'apply_diag' | 'forward'
    | 'backward' | 'diag' (cfp_slab_steps_get; buffers 0 = b, 1 = x, 2 = W, 3 = W2, 4 = the
    z-pencil Diag).  The defaults are the round-2 list: five passes, one piece."""
    nx, ny, nz = (int(d) for d in dims)
    sch, lst = _slab_schedule(schedule), STEP_LISTS[list_]
    n = ctypes.c_int()
    check(lib().cfp_slab_steps_count(nx, ny, nz, int(nranks), int(rank), sch, int(pieces), lst, ctypes.byref(n)))
    out = []
    for i in range(n.value):
        desc = (ctypes.c_int64 * len(STEP_KEYS))()
        sc = ctypes.c_double()
        check(lib().cfp_slab_steps_get(nx, ny, nz, int(nranks), int(rank), sch, int(pieces), lst, i, desc,
                                       ctypes.byref(sc)))
        d = dict(zip(STEP_KEYS, list(desc)))
        d["scale"] = sc.value
        out.append(d)
    return out


def rccl_version() -> dict:
    """Host-only: the RCCL version (ncclGetVersion) and the shared object the library's RCCL
    calls resolve to in this process (torch bundles its own librccl.so.1)."""
    v = ctypes.c_int()
    path = ctypes.create_string_buffer(512)
    check(lib().cfp_rccl_version(ctypes.byref(v), path, 512))
    return {"version": v.value, "lib": path.value.decode(errors="replace"), "mode": rccl_mode()}


def rccl_mode() -> str:
    """Host-only: 'blocking' when CFP_RCCL_BLOCKING selects ncclCommInitRank / ncclCommDestroy for
    the library's communicators, else 'non-blocking' (creation polled against a deadline)."""
    b = ctypes.c_int()
    check(lib().cfp_rccl_blocking(ctypes.byref(b)))
    return "blocking" if b.value else "non-blocking"


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
                 exchange: str = "rccl", timeout_s: float = 300.0):
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
            # non-blocking communicator creation polled against timeout_s (a rank that never
            # joins raises instead of hanging, csrc/cfp_rccl.h)
            check(lib().cfp_dist_plan_create_timeout(ctypes.byref(h), nx, ny, nz, self.world, self.rank, uid,
                                                     self.device, float(timeout_s)))
        elif exchange == "torch":
            check(lib().cfp_dist_plan_create_external(ctypes.byref(h), nx, ny, nz, self.world, self.rank,
                                                      self.device))
            self.work = torch.empty(self.layout["work_size"], dtype=torch.complex128, device=f"cuda:{self.device}")
            self.work2 = torch.empty_like(self.work)
            check(lib().cfp_dist_plan_set_work_buffers(h, self.work.data_ptr(), self.work2.data_ptr()))
        else:
            raise ValueError("exchange must be 'rccl' or 'torch'")
        self._h = h

    def rccl_info(self) -> dict:
        """What RCCL this plan talks through: the communicator's rank count and rank
        (ncclCommCount / ncclCommUserRank; 0 / -1 without one), ncclGetVersion, the creation
        time and the shared object the library's RCCL calls bind to."""
        n, r, v = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ms = ctypes.c_double()
        path = ctypes.create_string_buffer(512)
        check(lib().cfp_dist_plan_rccl_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(v),
                                            ctypes.byref(ms), path, 512))
        return {"ranks": n.value, "rank": r.value, "version": v.value, "init_ms": round(ms.value, 1),
                "lib": path.value.decode(errors="replace"), "mode": rccl_mode()}

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
        """Local passes: 'auto' (3 sweeps at 256^3 and 512^3 with world | 32, world <= 16), 'five' or 'three'."""
        check(lib().cfp_dist_plan_set_schedule(self._h, _slab_schedule(schedule)))
        return self

    def set_pieces(self, pieces: int) -> "SlabPlan":
        """Pipeline depth: 0 = AUTO, K = each all-to-all in K pieces overlapped with the x/y passes."""
        check(lib().cfp_dist_plan_set_pieces(self._h, int(pieces)))
        return self

    @property
    def pieces(self) -> int:
        k = ctypes.c_int()
        check(lib().cfp_dist_plan_pieces(self._h, ctypes.byref(k)))
        return k.value

    def set_diag(self, diag: torch.Tensor, stream=None) -> "SlabPlan":
        """Explicit Diag: this rank's natural slab (a collective; rccl exchange only)."""
        if self.exchange != "rccl":
            raise NotImplementedError("set_diag runs its exchange inside the library (exchange='rccl')")
        check(lib().cfp_dist_plan_set_diag(self._h, _dev_ptr(diag, self.local_size, "diag", self.device),
                                           _stream_handle(stream)))
        return self

    def steps(self) -> list:
        """The apply's step list (dicts of STEP_KEYS)."""
        n = ctypes.c_int()
        check(lib().cfp_dist_plan_num_steps(self._h, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            desc = (ctypes.c_int64 * len(STEP_KEYS))()
            check(lib().cfp_dist_plan_step(self._h, i, desc))
            out.append(dict(zip(STEP_KEYS, list(desc))))
        return out

    def _buffers(self, b, x):
        return {0: b, 1: x, 2: self.work, 3: self.work2}

    def _exchange_piece(self, st: dict, bufs: dict) -> None:
        """One all-to-all piece through torch.distributed: peer q gets src[q chunk + off, + cnt)
        and stores it at dst[rank chunk + off] (gloo: staged through host memory)."""
        import torch.distributed as dist
        c, off, cnt = st["chunk"], st["ex_off"], st["ex_cnt"]
        src, dst = bufs[st["src"]], bufs[st["dst"]]
        send = torch.cat([src[q * c + off:q * c + off + cnt] for q in range(self.world)])
        gloo = dist.get_backend(self.group) == "gloo"
        if gloo:
            send = send.cpu()
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        for q in range(self.world):
            dst[q * c + off:q * c + off + cnt].copy_(recv[q * cnt:(q + 1) * cnt])

    def apply(self, b: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(b)
        n = self.local_size
        bp, xp = _dev_ptr(b, n, "b", self.device), _dev_ptr(out, n, "out", self.device)
        sh = _stream_handle(stream)
        if self.exchange == "rccl":
            check(lib().cfp_dist_plan_apply(self._h, bp, xp, sh))
            return out
        # the library's step list, one stream: kernel steps through cfp_dist_plan_run_step, the
        # exchange pieces through torch.distributed (ordered on torch's current stream, so
        # make that the apply's stream)
        bufs = self._buffers(b, out)
        with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
            for i, st in enumerate(self.steps()):
                if st["kind"] == 1:
                    self._exchange_piece(st, bufs)
                else:
                    check(lib().cfp_dist_plan_run_step(self._h, i, bp, xp, sh))
        return out

    def phases(self) -> list:
        """The apply's steps: axis passes (with the number of grid elements they sweep) and
        all-to-all pieces (with the bytes each leaves this GPU with), in order."""
        out = []
        nx, ny, nz = self.dims
        for st in self.steps():
            if st["kind"] == 1:
                out.append({"kind": "all-to-all", "elements": st["ex_cnt"] * self.world,
                            "bytes_out": 16 * st["ex_cnt"] * (self.world - 1)})
                continue
            if st["kind"] == 2:  # 3-sweep stage: P1/P3 over `ncols` local planes, P2 over the slab
                el = self.local_size if st["axis"] == 1 else st["ncols"] * ny * nx
                ax = {0: "xy", 1: "yz", 2: "xy"}[st["axis"]]
            elif st["kind"] == 3:
                el, ax = st["ncols"] * ny * nx, "-"
            else:
                el, ax = st["ncols"] * st["n"], "xyz"[st["axis"]]
            out.append({"kind": "pass", "axis": ax, "n": st["n"], "mode": PASS_MODES.get(st["mode"], "repack"),
                        "elements": el})
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
        steps = self.steps()
        n = self.local_size
        bp, xp = _dev_ptr(b, n, "b", self.device), _dev_ptr(x, n, "x", self.device)
        sh = _stream_handle()
        bufs = self._buffers(b, x)
        acc = [0.0] * len(steps)
        for _ in range(iters):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(steps) + 1)]
            for i, st in enumerate(steps):
                ev[i].record()
                if st["kind"] == 1:
                    self._exchange_piece(st, bufs)
                else:
                    check(lib().cfp_dist_plan_run_step(self._h, i, bp, xp, sh))
            ev[-1].record()
            torch.cuda.synchronize()
            for i in range(len(steps)):
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
        """Local passes per slab: 'auto' (3 sweeps at 256^3 and 512^3 with P | 32, P <= 16), 'five' or 'three'."""
        check(lib().cfp_group_set_schedule(self._h, _slab_schedule(schedule)))
        return self

    def set_pieces(self, pieces: int) -> "SlabGroup":
        """Exchange pieces (0 = AUTO): the pipelined step list, run here in list order."""
        check(lib().cfp_group_set_pieces(self._h, int(pieces)))
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
