#!/usr/bin/env python3
"""PCApply throughput of the MI355X circulant FFT preconditioner.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 256]

One "step" = one PCApply x = (1/N) IDFT3(DFT3(b) ./ Diag) over one synthetic
256^3 complex-double grid (BASELINE.json metric "PCApply/s on 256^3 complex
grid").  Inputs are generated on the device (SplitMix64
U[-1,1) complex, seed 20251017) and are resident in HBM before timing starts.

N = 1: the single-GPU plan (3 kernel launches per apply at 256^3).  N > 1 (launched by
torch.distributed.run, one rank per GPU): the same grid slab-decomposed along
z over N GPUs with two RCCL all-to-all transposes per apply (strong scaling;
value = whole-job PCApply/s).

Also reported: the roofline of the dominant kernel (algorithmic
bytes / its mean duration from HIP events on the launch stream, vs 8 TB/s), the
apply-level roofline on the bytes the schedule moves (frac_moved; SURVEY's
B_alg = 208 N figure beside it as a speedup, not a fraction), and a CPU
baseline timed on rank 0 on a bounded sample: the fastest of scipy's pocketfft
(kind "library"), FFTW when present ("reference") and the oracle's C
restatement ("port"), each with its 1-thread and all-core legs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
LAM = (0.6, 0.15, 0.02)  # lambda set A, testFftSolver_3D.py:85-91
SEED = 20251017
RES_TOL = 1e-10  # north_star's parity bar, applied to the residual of the timed applies



def transport_residual(b, x, g, lam, rank: int = 0, world: int = 1, dev=None) -> float:
    """Output check of the timed applies, on the device holding x, without the oracle:
    ||C x - b|| / ||b|| with C the transport circulant the plan inverts,
    C x = x + sum_d lam_d (x - roll_d(x, 1))
    (Diag[k] = 1 + sum_d lam_d (1 - e^{-2 pi i k_d / n_d}), src/FftLinearSolver_3D.c:80-164).
    With world > 1, b and x are this rank's z-slab ([nz/world][ny][nx], PETSC_DECIDE rows) and
    the z-roll takes the plane below from the previous rank (periodic)."""
    import torch
    import torch.distributed as dist

    gx, gy, gz = g
    lx, ly, lz = lam
    nzl = gz // world
    X = x.view(nzl, gy, gx)
    B = b.view(nzl, gy, gx)
    on_gpu = world > 1 and dist.get_backend() == "nccl"
    if world == 1:
        Xz = torch.roll(X, 1, 0)
    else:
        # every rank's last plane through one all_gather on the default communicator (a
        # collective like the all_reduce below: no extra point-to-point communicator)
        last = X[-1].contiguous() if on_gpu else X[-1].cpu()
        planes = [torch.empty_like(last) for _ in range(world)]
        dist.all_gather(planes, last)
        prev = planes[(rank - 1) % world]
        Xz = torch.cat([prev.to(X.device).unsqueeze(0), X[:-1]], 0)
        del planes
    r = X * (1.0 + lx + ly + lz) - lx * torch.roll(X, 1, 2) - ly * torch.roll(X, 1, 1) - lz * Xz - B
    nd = torch.stack([r.abs().pow(2).sum(), B.abs().pow(2).sum()])
    del r, Xz
    if world > 1:
        nd = nd.to(dev) if on_gpu else nd.cpu()
        dist.all_reduce(nd)
    return float((nd[0] / nd[1]).sqrt())

def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Per-phase deadlines (seconds).  "timed" and "scaling_512" grow with the step count.
DEADLINES = {"import": 900.0, "init": 300.0, "plan": 360.0, "first_apply": 120.0, "settle": 120.0,
             "timed": 120.0, "check": 120.0, "real": 180.0, "configs": 300.0, "scaling_512": 420.0,
             "cpu_baseline": 300.0, "report": 60.0, "teardown": 120.0}


class Watchdog:
    """Deadline on each phase of the run, so that a hang -- a rank that never joins the RCCL
    communicator, a collective with a missing peer, a kernel that never drains -- ends the
    process with evidence instead of being killed silently at the driver's limit.

    phase(name) re-arms one timer with that phase's deadline.  On expiry the timer thread dumps
    every thread's Python stack (faulthandler) to stderr, prints one JSON line naming the phase
    ({"status": "timeout", ...}: rank 0 on stdout, the other ranks on stderr) and ends the
    process with os._exit(3), skipping any teardown that could block on the hung work."""

    def __init__(self, deadlines: dict, rank: int = 0, world: int = 1, metric: str = ""):
        import threading
        self.deadlines = dict(deadlines)
        self.rank, self.world, self.metric = rank, world, metric
        self.name = None
        self.t_phase = time.monotonic()
        self._lock = threading.Lock()
        self._timer = None
        self.history = []

    def phase(self, name: str, seconds: float | None = None) -> None:
        import threading
        with self._lock:
            if self._timer is not None:
                self._timer.cancel()
            now = time.monotonic()
            if self.name is not None:
                self.history.append((self.name, round(now - self.t_phase, 3)))
            self.name, self.t_phase = name, now
            limit = float(seconds if seconds is not None else self.deadlines.get(name, 300.0))
            self._timer = threading.Timer(limit, self._expire, args=(name, limit))
            self._timer.daemon = True
            self._timer.start()

    def stop(self) -> None:
        with self._lock:
            if self._timer is not None:
                self._timer.cancel()
                self._timer = None

    def _expire(self, name: str, limit: float) -> None:
        import faulthandler
        try:
            log(f"bench watchdog: rank {self.rank} phase '{name}' exceeded {limit:.0f} s; stacks follow")
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            line = json.dumps({"metric": self.metric, "value": None, "status": "timeout", "phase": name,
                               "deadline_s": limit, "rank": self.rank, "n_gpus": self.world,
                               "phases_done": self.history})
            print(line, file=sys.stdout if self.rank == 0 else sys.stderr, flush=True)
        finally:
            os._exit(3)


def phase_extension(steps: int, scaling_steps: int) -> float:
    """Seconds the ranks add to the 'timed' (steps) and 'scaling_512' (scaling_steps) deadlines;
    the self-launcher's kill limit adds the same."""
    return 0.05 * max(0, steps) + 0.2 * max(0, scaling_steps)


def parse_deadlines(items) -> dict:
    """--deadline PHASE=SECONDS (repeatable) over DEADLINES."""
    out = dict(DEADLINES)
    for it in items or []:
        k, _, v = it.partition("=")
        if k not in DEADLINES or not v:
            raise SystemExit(f"--deadline takes PHASE=SECONDS with PHASE in {sorted(DEADLINES)}")
        out[k] = float(v)
    return out


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(nproc: int, argv, deadlines: dict, extra_s: float = 0.0) -> int:
    """--gpus N > 1 without a launcher: start N ranks under torch.distributed.run as a child
    process group (this process has made no GPU call and makes none) and return their exit
    status.  The ranks inherit stdout, so rank 0's JSON line is this run's line.  The whole group
    is killed if it outlives the sum of the phase deadlines plus the ranks' own step-count
    extensions of them (extra_s), so their watchdogs always fire first."""
    import signal
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env["CFP_BENCH_SELF_LAUNCHED"] = "1"
    log(f"bench: --gpus {nproc} without a launcher: starting {nproc} ranks under torch.distributed.run")
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    limit = sum(deadlines.values()) + extra_s + 60.0
    try:
        return proc.wait(timeout=limit)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait()
        print(json.dumps({"metric": "PCApply/s", "value": None, "status": "timeout", "phase": "launcher",
                          "deadline_s": limit, "rank": -1, "n_gpus": nproc}), flush=True)
        return 3


def kernel_alg_bytes(mode: str, N: int, n_axis: int) -> int:
    """Algorithmic HBM bytes of one axis-pass launch (SURVEY.md §8d per-unit figure x units)."""
    b = 32 * N  # read N c128 + write N c128
    if mode == "fused_diag":
        b += 16 * N  # + read Diag
    elif mode in ("fused_sep", "mid_fused"):
        b += 16 * (N // n_axis + n_axis)  # per-column + per-point symbol tables
    return b


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


FFTW_LIBS = ("libfftw3.so.3", "libfftw3.so")
FFTW_OMP_LIBS = ("libfftw3_omp.so.3", "libfftw3_omp.so")


def fftw_leg(grid, b, d, threads: int, budget_s: float):
    """BASELINE.md §4 / SURVEY §8d(i): the reference's own arithmetic on FFTW when the box has
    it -- fftw_plan_dft_3d(nz, ny, nx, FFTW_FORWARD / FFTW_BACKWARD, FFTW_ESTIMATE) (what PETSc's
    MATFFTW uses, src/FftLinearSolver_3D.c:170-184), pointwise divide, 1/N -- on 1 thread and,
    with libfftw3_omp, on `threads`.  Returns {"fftw": "not found", "probed": [...]} otherwise."""
    import ctypes
    import numpy as np
    lib = None
    for name in FFTW_LIBS:
        try:
            lib = ctypes.CDLL(name)
            break
        except OSError:
            continue
    if lib is None:
        return {"fftw": "not found", "probed": list(FFTW_LIBS)}
    omp = None
    for name in FFTW_OMP_LIBS:
        try:
            omp = ctypes.CDLL(name)
            break
        except OSError:
            continue
    nx, ny, nz = grid
    N = nx * ny * nz
    vp = ctypes.c_void_p
    lib.fftw_plan_dft_3d.restype = vp
    lib.fftw_plan_dft_3d.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_uint]
    lib.fftw_execute.argtypes = [vp]
    lib.fftw_destroy_plan.argtypes = [vp]
    FORWARD, BACKWARD, ESTIMATE = -1, 1, 1 << 6
    x = np.empty(N, dtype=np.complex128)
    bh = np.empty(N, dtype=np.complex128)

    def legs_for(nthreads):
        if omp is not None:
            omp.fftw_init_threads()
            omp.fftw_plan_with_nthreads(ctypes.c_int(nthreads))
        fwd = lib.fftw_plan_dft_3d(nz, ny, nx, b.ctypes.data, bh.ctypes.data, FORWARD, ESTIMATE)
        bwd = lib.fftw_plan_dft_3d(nz, ny, nx, bh.ctypes.data, x.ctypes.data, BACKWARD, ESTIMATE)

        def apply():
            lib.fftw_execute(fwd)
            np.divide(bh, d, out=bh)
            lib.fftw_execute(bwd)
            np.multiply(x, 1.0 / N, out=x)

        t0 = time.perf_counter()
        apply()
        first = time.perf_counter() - t0
        reps = max(1, min(5, int(budget_s / max(first, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            apply()
        dt = (time.perf_counter() - t0) / reps
        lib.fftw_destroy_plan(fwd)
        lib.fftw_destroy_plan(bwd)
        return {"threads": nthreads, "value": round(1.0 / dt, 4), "ms_per_apply": round(dt * 1e3, 1),
                "sample": f"{reps} timed applies (+1 warm-up) of the full {nx}x{ny}x{nz} grid"}

    legs = [legs_for(1)]
    if omp is not None and threads > 1:
        legs.append(legs_for(threads))
    return {"fftw": "found", "kind": "reference", "legs": legs, "value": legs[-1]["value"], "unit": "PCApply/s",
            "cores": legs[-1]["threads"], "omp": omp is not None}


def cpu_baseline(grid, budget_s: float = 20.0):
    """The oracle's C restatement (test infrastructure; the checker, never the product), timed
    on 1 thread and on all of this process's host cores."""
    import numpy as np
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    n = tuple(grid)
    N = int(np.prod(n))
    b = O.c_fill_uniform(N, SEED)
    d = O.c_build_diag_transport(n, LAM)

    def leg(nthreads, budget):
        O.set_threads(nthreads)
        t0 = time.perf_counter()
        O.c_solve_3d(d, b, n)  # warm-up (page faults, thread pool); also sizes the sample
        first = time.perf_counter() - t0
        reps = max(1, min(5, int(budget / max(first, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            O.c_solve_3d(d, b, n)
        dt = (time.perf_counter() - t0) / reps
        return {"threads": nthreads, "value": round(1.0 / dt, 4), "ms_per_apply": round(dt * 1e3, 1),
                "sample": f"{reps} timed applies (+1 warm-up) of the full {n[0]}x{n[1]}x{n[2]} grid"}

    port = [leg(1, budget_s * 0.4), leg(threads, budget_s * 0.3)] if threads > 1 else [leg(1, budget_s * 0.7)]
    out = {"unit": "PCApply/s", "cpu_model": cpu_model(),
           "cores_affinity": len(os.sched_getaffinity(0)), "cores_box": os.cpu_count(),
           "port": {"legs": port, "what": "oracle/cfp_oracle.c restatement of solve_3D (recursive mixed-radix "
                                          "FFT, long-double twiddles, OpenMP): the parity checker"}}
    try:
        out["fftw"] = fftw_leg(n, b, d, threads, budget_s * 0.5)
    except Exception as e:  # report, never fake
        out["fftw"] = {"fftw": "error", "error": str(e)}
    # the optimised library beside the port (FFTW is absent here and on the
    # box): scipy's pocketfft on the same grid and symbol -- fftn, divide, ifftn (= x 1/N), the
    # reference arithmetic of solve_3D; 1 worker and all of this process's cores
    lib_legs = []
    try:
        import scipy.fft as sf
        bz = b.reshape(n[2], n[1], n[0])
        dz = d.reshape(n[2], n[1], n[0])
        # 1 worker, the inherited thread budget (OMP_NUM_THREADS: 16 on the GPU box), and every
        # core this process may run on (len(sched_getaffinity(0)): the box's 256), whatever
        # OMP_NUM_THREADS says -- north_star's "same box's host cores"
        aff = len(os.sched_getaffinity(0))
        for w in sorted({1, threads, aff}):
            t0 = time.perf_counter()
            sf.ifftn(sf.fftn(bz, workers=w) / dz, workers=w)  # warm-up; sizes the sample
            first = time.perf_counter() - t0
            reps = max(1, min(5, int(budget_s * 0.15 / max(first, 1e-3))))
            t0 = time.perf_counter()
            for _ in range(reps):
                sf.ifftn(sf.fftn(bz, workers=w) / dz, workers=w)
            dl = (time.perf_counter() - t0) / reps
            lib_legs.append({"threads": w, "value": round(1.0 / dl, 4), "ms_per_apply": round(dl * 1e3, 1),
                             "sample": f"{reps} timed applies (+1 warm-up) of scipy.fft (pocketfft) fftn / Diag / "
                                       f"ifftn, workers={w}, full {n[0]}x{n[1]}x{n[2]} grid"})
        out["library"] = {"legs": lib_legs, "what": "scipy.fft (pocketfft): an optimised FFT library running the "
                                                    "reference arithmetic (FFTW, the reference's own, is absent)"}
    except Exception as e:  # report, never fake
        out["library"] = {"error": str(e)}
    # value: the fastest CPU implementation of the reference arithmetic measured here
    cands = [("port", l) for l in port] + [("library", l) for l in lib_legs]
    if out["fftw"].get("fftw") == "found":
        cands += [("reference", l) for l in out["fftw"]["legs"]]
    kind, top = max(cands, key=lambda c: c[1]["value"])
    out.update({"value": top["value"], "cores": top["threads"], "kind": kind,
                "sample": f"{top['sample']}, {top['ms_per_apply']:.0f} ms/apply (fastest of the legs below)"})
    return out


def moved_bytes(passes, N: int) -> int:
    """Bytes one apply's launches move by design (sum of their algorithmic bytes): 96 N for the
    3-sweep schedule, 160 N for five axis passes (+ the small symbol tables)."""
    return int(sum(kernel_alg_bytes(p["mode"], N, p["n"]) for p in passes))


def copy_rate(dev, nbytes: int = 256 << 20) -> dict:
    """This box's copy rate in the same run: out-of-place device copies of a
    256 MiB buffer, read + write bytes over the HIP-event mean of 50 copies, with the library's
    copy kernel (cfp_device_copy: 16-byte lanes, non-temporal stores) and with torch's.  The
    faster one is the bar: the 3-sweep passes move the same 2 x 268 MB per launch, so
    frac_of_copy says how far the dominant pass sits from a plain copy of its bytes."""
    import torch
    from circulantpreconditioner_amd._lib import check, lib
    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
    a.fill_(1.0)
    c = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    ms_t = event_ms(lambda: c.copy_(a), 50, settle_ms=100.0)
    ms_l = event_ms(lambda: check(lib().cfp_device_copy(c.data_ptr(), a.data_ptr(), nbytes, s)), 50, settle_ms=100.0)
    ok = bool(torch.equal(a, c))
    del a, c
    gb = lambda ms: round(2 * nbytes / (ms * 1e-3) / 1e9, 1)  # noqa: E731
    return {"GBps": max(gb(ms_l), gb(ms_t)), "library_GBps": gb(ms_l), "torch_GBps": gb(ms_t),
            "library_ms": round(ms_l, 5), "torch_ms": round(ms_t, 5), "bytes": nbytes, "library_copy_ok": ok,
            "what": "256 MiB out-of-place device copy, (read + write) / HIP-event mean of 50; GBps = the "
                    "faster of the library's copy kernel and torch's"}


def event_ms(fn, iters: int, settle_ms: float = 150.0) -> float:
    """Mean ms of fn() over iters back-to-back calls (HIP events on the current stream) after
    settle_ms of untimed ones (the clocks ramp between legs, as before the headline's region)."""
    import torch
    t0 = time.perf_counter()
    while True:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
        if (time.perf_counter() - t0) * 1e3 >= settle_ms:
            break
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def gmres_leg(n: int, steps: int) -> dict:
    """BASELINE config 3 (n = 256) / config 1 (n = 32): the implicit upwind transport step of the
    reference's GMRES driver (a = (1,0,0), cfl 1e3/3, rtol = abstol = 1e-5, restart 30, fixed
    inflow sign so the circulant matches the operator) with the FFT PCSHELL on one GPU, `steps`
    back-to-back implicit steps after a 2-step warm-up run.  Device time per step from the
    library's own dispatch stamps (PetscMiniProfile*: every MatMult / vector kernel and copy, plus
    the KSP's PCApply stamps), split by kind; the same run with the fusion off (MatMult + PCApply
    + VecMDot as separate sweeps) beside it."""
    from circulantpreconditioner_amd import transport as T

    def one(fuse: int) -> dict:
        T.run(T.config(n, pc="fft", sign="fixed", device=True, steps=2, fuse=fuse))  # warm-up
        r = T.run(T.config(n, pc="fft", sign="fixed", device=True, steps=steps, fuse=fuse, profile=1))
        k = max(1, r["steps"])
        dev = r["dev_ms"]
        return {"steps": r["steps"], "gmres_its": r["total_its"], "its_per_step": r["total_its"] / k,
                "converged": bool(r["all_converged"]),
                "device_us_per_step": round(1e3 * sum(dev.values()) / k, 1),
                "split_us_per_step": {key: round(1e3 * v / k, 1) for key, v in dev.items()},
                "launches_per_step": {key: round(v / k, 2) for key, v in r["dev_launches"].items()},
                "pcapply_us": round(1e6 * r["pc_seconds"] / max(1, r["pc_calls"]), 1),
                "pc_calls_per_step": r["pc_calls"] / k,
                "wall_ms_per_step": round(1e3 * r["loop_seconds"] / k, 4),
                "wall_ms_per_solve": round(1e3 * r["solve_seconds"] / k, 4),
                "fused_dots": r["fused_dots"], "fused_norms": r["fused_norms"]}

    fused, unfused = one(1), one(0)
    ok = fused["converged"] and unfused["converged"] and fused["gmres_its"] == unfused["gmres_its"]
    return {"value": round(1e3 / fused["wall_ms_per_step"], 2), "unit": "implicit steps/s (GMRES + FFT PCSHELL)",
            "grid": [n] * 3, **fused, "unfused": unfused,
            "note": "device_us_per_step = the step's kernels and copies (pcapply: KSP stamps of each PCApply, "
                    "which with the fused applyBA include the MatMult; matmult / vector / copy: the stand-in's "
                    "stamped launches); wall_ms_per_step includes host waits and the loop's VecCopy / "
                    "VecAXPY / VecNorm",
            "check": {"what": "every solve converged (KSP reason 2/3); fused and unfused take the same iterations",
                      "ok": bool(ok)}}


def wave_gmres_leg(n: int, steps: int) -> dict:
    """BASELINE config 4: the implicit step of the reference's wave-system driver
    (tests/WaveSystem_SphericalExplosion_impl_seq.cxx: wall boundaries, cfl 1e3/3, GMRES with
    rtol = abstol = 1e-5, restart 30) on an n^3 grid, with the (d+1)-block-circulant PCSHELL
    (applyFFT3DPrecWave) on one GPU, `steps` implicit steps after a 1-step warm-up run.  Device time
    per step from the library's dispatch stamps, split by kind (the MatMult runs the block
    row-class SpMV of the interleaved operator; the Gram-Schmidt dot and the residual norm ride
    in the block apply's last sweep, fused_dots / fused_norms)."""
    from circulantpreconditioner_amd import wave as W
    W.run(W.config(n, pc="fft", steps=1))  # warm-up (plan, operator upload)
    r = W.run(W.config(n, pc="fft", steps=steps, profile=1))
    k = max(1, r["steps"])
    dev = r["dev_ms"]
    ok = bool(r["all_converged"])
    return {"value": round(1e3 * k / (1e3 * r["loop_seconds"]), 2), "unit": "implicit steps/s (GMRES + block PCSHELL)",
            "grid": [n] * 3, "steps": r["steps"], "gmres_its": r["total_its"], "its_per_step": r["total_its"] / k,
            "converged": ok, "device_us_per_step": round(1e3 * sum(dev.values()) / k, 1),
            "split_us_per_step": {key: round(1e3 * v / k, 1) for key, v in dev.items()},
            "launches_per_step": {key: round(v / k, 2) for key, v in r["dev_launches"].items()},
            "pcapply_us": round(1e6 * r["pc_seconds"] / max(1, r["pc_calls"]), 1),
            "wall_ms_per_step": round(1e3 * r["loop_seconds"] / k, 4),
            "wall_ms_per_solve": round(1e3 * r["solve_seconds"] / k, 4),
            "fused_dots": r["fused_dots"], "fused_norms": r["fused_norms"],
            "check": {"what": "every solve converged (KSP reason 2/3)", "ok": ok}}


def choose_slab_plan(create, requested, agree, warn=None):
    """Pick the N > 1 exchange.  create(exchange) builds this rank's SlabPlan (raises on
    failure); agree(ok) -> True when every rank's creation succeeded.  RCCL unless the
    environment asks otherwise.  When the library's RCCL communicator fails on any rank: an
    explicit CFP_EXCHANGE=rccl request exits non-zero; the default falls back to
    torch.distributed collectives and says so in the label ("torch-fallback"), which bench.py
    prints as the top-level "exchange" field.  Returns (plan, label)."""
    exchange = requested or "rccl"
    plan, err = None, None
    try:
        plan = create(exchange)
    except Exception as e:  # the library's own communicator failed on this rank
        err = e
    if agree(plan is not None):
        return plan, exchange
    if plan is not None:
        plan.close()
    if requested == "rccl" or exchange != "rccl":
        raise SystemExit(f"{exchange} exchange requested but unavailable on some rank ({err})")
    if warn:
        warn(f"rccl exchange unavailable ({err}); falling back to torch.distributed all_to_all_single")
    return create("torch"), "torch-fallback"


def load_traffic(grid, kernel_name: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        data = json.load(open(path))
    except Exception:
        return None, None
    key = f"{grid[0]}x{grid[1]}x{grid[2]}"
    ent = data.get(key, {}).get(kernel_name)
    if not ent:
        return None, None
    return ent.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--grid", type=int, nargs="+", default=[256])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--schedule", default="auto", choices=["auto", "five", "five_y", "three", "plane"],
                    help="apply schedule: 5 axis passes fused on z or y, 3 sweeps (256^3), or plane "
                         "(n_x = n_y in {64, 100, 128}); auto = the plan's default")
    ap.add_argument("--tp-shape", default=None, metavar="N1,MID",
                    help="3-sweep kernel shape (measurements): y split n1 (0/32/64) and middle kernel "
                         "(default, lane64, lane32, swap64); default: the plan's")
    ap.add_argument("--chunk", type=int, default=None,
                    help="z-planes per chunk of the Infinity-Cache-resident x/y schedule (0 = off; default: plan's)")
    ap.add_argument("--graph", action="store_true",
                    help="single GPU: replay each apply as one captured HIP graph (cfp_plan_set_graph)")
    ap.add_argument("--pieces", type=int, default=0,
                    help="N > 1: exchange pieces per all-to-all (0 = the plan's AUTO: 4 on slabs of 64 MiB and more)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed applies for this long after the warm-up (clock ramp-up; 0 = off)")
    ap.add_argument("--no-real", action="store_true", help="skip the real-data variant line item")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs' line items (128^3, the wave system, 100^3)")
    ap.add_argument("--scaling-grid", type=int, nargs="+", default=[512],
                    help="grid of the scaling_512 line item (BASELINE config 5; 0 = skip)")
    ap.add_argument("--scaling-steps", type=int, default=20)
    ap.add_argument("--gmres-steps", type=int, default=20,
                    help="implicit steps of the config 1 / config 3 GMRES legs (other_configs)")
    ap.add_argument("--event-every", type=int, default=10,
                    help="record per-launch events in every n-th timed apply")
    ap.add_argument("--no-live-events", action="store_true",
                    help="time the passes in separate applies instead of inside the timed region")
    ap.add_argument("--rccl-blocking", action="store_true",
                    help="N > 1: the library's RCCL communicator uses the blocking protocol "
                         "(CFP_RCCL_BLOCKING=1: ncclCommInitRank / ncclCommDestroy, no deadline); "
                         "the line's rccl.mode says which ran")
    ap.add_argument("--deadline", action="append", default=[], metavar="PHASE=SECONDS",
                    help=f"override a phase deadline of the watchdog (phases: {', '.join(DEADLINES)})")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="CPU rehearsal of the launch / rendezvous / phase / report control flow with a host "
                         "stand-in step and a gloo group: no GPU call, no measurement (value null)")
    ap.add_argument("--selftest-stall", default=None, metavar="PHASE",
                    help="--selftest-cpu: block forever in PHASE (exercises the watchdog)")
    ap.add_argument("--selftest-stall-rank", type=int, default=-1, help="rank that stalls (-1 = all)")
    args = ap.parse_args()
    grid = args.grid * 3 if len(args.grid) == 1 else args.grid
    if len(grid) != 3:
        raise SystemExit("--grid takes 1 or 3 integers")
    deadlines = parse_deadlines(args.deadline)
    if args.rccl_blocking:  # before the library loads; self-launched ranks inherit it
        os.environ["CFP_RCCL_BLOCKING"] = "1"

    # N > 1 without a launcher: start the N ranks before anything touches the GPU; a run never
    # silently measures a different GPU count than --gpus asks for
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return self_launch(args.gpus, sys.argv[1:], deadlines, phase_extension(args.steps, args.scaling_steps))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to measure a different GPU count")
        return 2
    launcher = ("none" if world == 1 else
                "self (torch.distributed.run)" if os.environ.get("CFP_BENCH_SELF_LAUNCHED") else "external")
    metric_name = ("PCApply/s on 256^3 complex grid" if grid == [256, 256, 256] else
                   f"PCApply/s on {grid[0]}x{grid[1]}x{grid[2]} complex grid")
    wd = Watchdog(deadlines, rank, world, metric_name)
    wd.phase("import")

    import torch
    import torch.distributed as dist

    if args.selftest_cpu:
        return selftest_cpu(args, wd, rank, world, launcher, metric_name)

    wd.phase("init")
    if os.environ.get("CFP_BENCH_SHARE_DEVICE"):  # rehearsal of N > 1 on a one-GPU box
        local_rank = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        backend = os.environ.get("CFP_BENCH_BACKEND", "nccl")  # "gloo": one-GPU rehearsal of N > 1
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import circulantpreconditioner_amd as cp
    from circulantpreconditioner_amd.distributed import rccl_version

    nx, ny, nz = grid
    N = nx * ny * nz
    roof = None
    roof_apply = None
    passes_info = None

    exchange_used = ["none"]  # N > 1: "rccl", "torch" or "torch-fallback"

    def make(g):
        """(plan, b, x, run, parallelism) of the apply on grid g: one GPU, or this rank's slab."""
        if world == 1:
            b = torch.empty(int(g[0] * g[1] * g[2]), dtype=torch.complex128, device=dev)
            x = torch.empty_like(b)
            cp.fill_uniform(b, SEED)
            plan = cp.CirculantPlan(g, device=local_rank)
            plan.set_transport_symbol(LAM)
            if args.chunk is not None:
                plan.set_chunking(args.chunk)
            plan.set_schedule(args.schedule)
            if args.tp_shape:
                n1, mid = args.tp_shape.split(",")
                plan.set_three_pass_shape(int(n1), int(mid) if mid.isdigit() else mid)
            if args.graph:
                plan.set_graph(True)
            return plan, b, x, (lambda: plan.apply(b, out=x)), "single GPU"
        from circulantpreconditioner_amd.distributed import SlabPlan

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                             device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t.item()) == 1

        # the library's RCCL communicator gives up well inside the watchdog's "plan" deadline,
        # so a rank that never joins becomes a labelled fallback (or a loud failure) first
        plan, exchange = choose_slab_plan(
            lambda ex: SlabPlan(g, rank=rank, world=world, device=local_rank, exchange=ex,
                                timeout_s=0.4 * deadlines["plan"]),
            os.environ.get("CFP_EXCHANGE"), agree, warn=lambda m: log(f"rank {rank}: {m}"))
        exchange_used[0] = exchange
        plan.set_transport_symbol(LAM)
        if args.pieces:
            plan.set_pieces(args.pieces)
        b = torch.empty(plan.local_size, dtype=torch.complex128, device=dev)
        x = torch.empty_like(b)
        cp.fill_uniform(b, SEED, offset=plan.local_offset)
        return plan, b, x, (lambda: plan.apply(b, out=x)), f"z-slab x{world}, all-to-all over xGMI ({exchange})"

    def residual(b, x, g):
        return transport_residual(b, x, g, LAM, rank, world, dev)

    def settle(run, ms):
        """Untimed applies until `ms` of wall time have passed: the GPU leaves its idle clocks
        (sclk reads ~100 MHz idle); without this a 20-step run measures ramp-up, ~10 % low
        (profiles/r02a_settle.txt).  Returns (applies, ms spent)."""
        if ms <= 0:
            return 0, 0.0
        t0 = time.perf_counter()
        k = 0
        while True:
            for _ in range(4):
                run()
            k += 4
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) * 1e3
            done = el >= ms
            if world > 1:  # every rank must run the same applies (they hold collectives)
                f = torch.tensor([1 if done else 0], dtype=torch.int32,
                                 device=dev if dist.get_backend() == "nccl" else "cpu")
                dist.all_reduce(f, op=dist.ReduceOp.MAX)
                done = int(f.item()) == 1
            if done:
                return k, el

    def timed(run, steps, warmup):
        """W untimed + K timed applies between barriers and device syncs; max over ranks (s)."""
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed

    wd.phase("plan")
    plan, b, x, run, parallelism = make(grid)
    rccl = {"ranks": None, **rccl_version()}
    if world > 1 and plan.exchange == "rccl":
        # what RCCL saw: every rank's communicator size and creation time, agreed over the ranks
        rccl = plan.rccl_info()
        t = torch.tensor([rccl["ranks"], -rccl["ranks"], rccl["init_ms"]], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rccl.update({"ranks_max_over_ranks": int(t[0].item()), "ranks_min_over_ranks": int(-t[1].item()),
                     "init_ms_max_over_ranks": round(float(t[2].item()), 1)})
    wd.phase("first_apply")
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    wd.phase("settle")
    settle_n, settle_ms = settle(run, args.settle_ms)
    wd.phase("timed", deadlines["timed"] + phase_extension(args.steps, 0))
    timed_region_ms = None
    live_applies = 0
    every = max(1, args.event_every)
    if world > 1 and not args.no_live_events and plan.exchange == "rccl":
        # the slab plan's phases (passes and RCCL exchanges) timed inside the timed applies
        plan.profile_begin((args.steps + every - 1) // every, every)
        elapsed = timed(run, args.steps, 0)
        timed_region_ms, live_applies = plan.profile_end()
    elif world == 1 and not args.no_live_events:
        # per-launch HIP events recorded by the plan inside the timed applies themselves (on
        # the launch stream), in every EVERY-th apply: the roofline's kernel time comes from
        # the timed region, and the events' own cost (~3 us each) stays out of `value`
        plan.profile_begin((args.steps + every - 1) // every, every)
        elapsed = timed(run, args.steps, 0)
        timed_region_ms, n_rec = plan.profile_end()
        live_applies = n_rec
    else:
        elapsed = timed(run, args.steps, 0)
    ms_per_step = elapsed / args.steps * 1e3
    value = args.steps / elapsed  # whole-job PCApply/s (one grid per step)
    torch.cuda.synchronize()
    wd.phase("check")
    res = residual(b, x, grid)
    check = {"residual": res, "tol": RES_TOL, "ok": res < RES_TOL,
             "what": "||C x - b|| / ||b|| of the last timed apply (transport circulant C, on the GPU)"}

    # per-launch timing of the dominant kernel (HIP events on the launch stream)
    if world == 1:
        passes_info = plan.passes()
        if timed_region_ms is not None:
            ms = timed_region_ms
            timing_src = (f"start / stop HIP events of every launch in {live_applies} of the {args.steps} timed "
                          f"applies (every {max(1, args.event_every)}th; the 3-sweep kernels stamp their own "
                          f"dispatch, hipExtLaunchKernelGGL; launch stream)")
        else:
            ms = plan.time_passes(b, x, iters=max(10, min(50, args.steps)))
            timing_src = "HIP events, separate applies after the timed region (launch stream)"
        for p, m in zip(passes_info, ms):
            p["ms"] = round(m, 5)
        k = max(range(len(ms)), key=lambda i: ms[i])
        dom = passes_info[k]
        alg = kernel_alg_bytes(dom["mode"], N, dom["n"])
        achieved = alg / (ms[k] * 1e-3) / 1e9
        kname = f"pass{k}_{dom['axis']}_{dom['mode']}"
        traffic, tsrc = load_traffic(grid, kname)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kname, "alg_bytes_per_launch": alg, "mean_ms": round(ms[k], 5),
                "timing": timing_src}
        if tsrc:
            roof["traffic_source"] = tsrc
        try:
            cr = copy_rate(dev)
            roof.update(copy_GBps=cr["GBps"], frac_of_copy=round(achieved / cr["GBps"], 4), copy=cr)
        except Exception as e:  # report, never fake
            roof.update(copy_GBps=None, frac_of_copy=None, copy={"error": str(e)})
        b_alg = 208 * N
        ach_apply = b_alg / (ms_per_step * 1e-3) / 1e9
        moved = moved_bytes(passes_info, N)
        ach_moved = moved / (ms_per_step * 1e-3) / 1e9
        pmc = [load_traffic(grid, f"pass{i}_{p['axis']}_{p['mode']}")[0] for i, p in enumerate(passes_info)]
        roof_apply = {"moved_bytes": moved, "moved_per_N": round(moved / N, 2),
                      "achieved_moved": round(ach_moved, 1), "frac_moved": round(ach_moved / HBM_PEAK_GBS, 4),
                      "pmc_bytes": int(sum(pmc)) if all(v is not None for v in pmc) else None,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "B_alg_bytes": b_alg, "B_alg_rate": round(ach_apply, 1),
                      "B_alg_speedup_vs_unfused_roofline": round(ach_apply / HBM_PEAK_GBS, 4),
                      "note": "frac_moved: the bytes this schedule's launches move (sum of their algorithmic "
                              "bytes; pmc_bytes = the committed rocprofv3 FETCH+WRITE of the same launches) / wall "
                              "time per apply / peak: the apply's roofline fraction.  B_alg_*: SURVEY §8d's "
                              "convention, B_alg = 208 N (13 c128 sweeps of an unfused apply); the speedup is "
                              "the time an unfused apply at peak HBM would take over this apply's time, not a "
                              "roofline fraction"}
    else:
        # every rank takes part (the exchanges are collectives); rank 0 reports its own phases
        passes_info = plan.phases()
        if timed_region_ms is not None:
            ms = timed_region_ms
            timing_src = (f"HIP events around every phase of {live_applies} of the {args.steps} timed applies "
                          f"(every {every}th, launch stream)")
        else:
            ms = plan.time_phases(b, x, iters=max(5, min(20, args.steps)))
            timing_src = "HIP events, separate applies after the timed region (launch stream)"
        for p, m in zip(passes_info, ms):
            p["ms"] = round(m, 5)
        nloc = plan.local_size
        kern = [i for i, p in enumerate(passes_info) if p["kind"] == "pass"]
        k = max(kern, key=lambda i: ms[i])
        dom = passes_info[k]
        alg = kernel_alg_bytes(dom["mode"], dom["elements"], dom["n"])
        achieved = alg / (ms[k] * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": f"phase{k}_{dom['axis']}_{dom['mode']} (rank 0 slab)", "alg_bytes_per_launch": alg,
                "mean_ms": round(ms[k], 5), "timing": timing_src}
        # exchange pieces (pieces > 1: on the exchange stream, overlapped with the passes), per
        # direction: summed piece time and bytes leaving this GPU
        exi = [i for i, p in enumerate(passes_info) if p["kind"] == "all-to-all"]
        half = len(exi) // 2
        ex = [sum(ms[i] for i in exi[:half]), sum(ms[i] for i in exi[half:])]
        sent = sum(passes_info[i]["bytes_out"] for i in exi[:half])  # bytes leaving this GPU per all-to-all
        moved = sum(kernel_alg_bytes(p["mode"], p["elements"], p["n"]) for p in passes_info if p["kind"] == "pass")
        roof_apply = {"moved_bytes_per_gpu": moved,
                      "frac_moved": round(moved / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "B_alg_bytes_per_gpu": 208 * nloc,
                      "B_alg_rate_per_gpu": round(208 * nloc / (ms_per_step * 1e-3) / 1e9, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "B_alg_speedup_vs_unfused_roofline": round(208 * nloc / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "alltoall_ms": [round(e, 5) for e in ex],
                      "alltoall_GBps_out_per_gpu": [round(sent / (e * 1e-3) / 1e9, 1) if e > 0 else None for e in ex],
                      "pieces": plan.pieces,
                      "note": "alltoall_ms: summed piece times per direction, each piece timed on the "
                              "stream it runs on (overlapped with the passes when pieces > 1)"}

    # row f4: the real-data variant on the same grid (real b, the same real lambda), reported
    # beside the headline; the headline stays the complex apply
    real_variant = None
    wd.phase("real")
    if world == 1 and not args.no_real:
        try:
            rp = cp.RealPlan(grid, device=local_rank).set_transport_symbol([float(v) for v in LAM])
            br = b.real.contiguous()
            xr = torch.empty_like(br)
            # 200 applies after a 150 ms settle whatever --steps is: with the driver's 20 steps the
            # leg measured the clock ramp (4,576 against 4,930 PCApply/s, profiles/r03z_final_bench*.json)
            rms = event_ms(lambda: rp.apply(br, out=xr), 200)
            real_variant = {"value": round(1e3 / rms, 3), "unit": "PCApply/s", "ms_per_apply": round(rms, 5),
                            "dtype": "f64 real b and x (r2c / half spectrum / c2r)",
                            "stage_ms": [round(v, 5) for v in rp.time_passes(br, xr, iters=10)],
                            "schedule": "3 sweeps" if rp.three_sweep else "r2c + 3 half-spectrum passes + c2r",
                            "stages": (["r2c rows + y1", "half-spectrum y2/z", "Nyquist y/z", "y1 inverse + c2r rows"]
                                       if rp.three_sweep else
                                       ["r2c rows", "half-spectrum y/z", "Nyquist y/z", "c2r rows"])}
            rp.close()
            del br, xr
        except Exception as e:  # unsupported grid or failure: report, never fake
            real_variant = {"error": str(e)}

    # the other single-GPU BASELINE configs, measured after the headline on the same box: config 2
    # (128^3 complex apply), config 4's block preconditioner (wave system 128^3) and the
    # reference's default mesh (100^3); each with its own output check
    other_configs = None
    wd.phase("configs")
    if world == 1 and not args.no_configs:
        other_configs = {}
        for key, g3 in (("config2_128", [128, 128, 128]), ("reference_mesh_100", [100, 100, 100])):
            try:
                with cp.CirculantPlan(g3, device=local_rank) as p3:
                    p3.set_transport_symbol(LAM)
                    b3 = torch.empty(g3[0] * g3[1] * g3[2], dtype=torch.complex128, device=dev)
                    cp.fill_uniform(b3, SEED)
                    x3 = torch.empty_like(b3)
                    ms3 = event_ms(lambda: p3.apply(b3, out=x3), 2000)
                    r3 = transport_residual(b3, x3, g3, LAM, 0, 1, dev)
                    n3 = g3[0] * g3[1] * g3[2]
                    mv3 = moved_bytes(p3.passes(), n3)
                    other_configs[key] = {"value": round(1e3 / ms3, 1), "unit": "PCApply/s",
                                          "ms_per_apply": round(ms3, 5),
                                          "moved_bytes": mv3, "moved_GBps": round(mv3 / (ms3 * 1e-3) / 1e9, 1),
                                          "B_alg_GBps": round(208 * n3 / (ms3 * 1e-3) / 1e9, 1),
                                          "schedule": " | ".join(f"{q['axis']}:{q['mode']}" for q in p3.passes()),
                                          "check": {"residual": r3, "tol": RES_TOL, "ok": r3 < RES_TOL}}
                    if not r3 < RES_TOL:
                        check["ok"] = False
                    del b3, x3
            except Exception as e:  # report, never fake
                other_configs[key] = {"error": str(e)}
        try:
            from circulantpreconditioner_amd import wave as W
            wg = (128, 128, 128)
            wp = W.WavePlan(wg, device=local_rank).set_symbol((0.079, 0.079, 0.079))
            bw = torch.empty(4 * 128 ** 3, dtype=torch.complex128, device=dev)
            cp.fill_uniform(bw, SEED)
            xw = torch.empty_like(bw)
            msw = event_ms(lambda: wp.apply(bw, out=xw), 1000)
            sweeps = wp.num_passes()
            wp.set_schedule("five")
            x5 = wp.apply(bw)
            dw = float(torch.linalg.vector_norm(x5 - xw) / torch.linalg.vector_norm(x5))
            nw = 128 ** 3
            mvw = (2 * sweeps) * 64 * nw  # each sweep reads and writes the 4-component field
            other_configs["config4_wave128"] = {
                "value": round(1e3 / msw, 1), "unit": "block PCApply/s", "ms_per_apply": round(msw, 5),
                "sweeps": sweeps, "dtype": "c128, 4 interleaved unknowns per cell",
                "moved_bytes": mvw, "moved_GBps": round(mvw / (msw * 1e-3) / 1e9, 1),
                "B_alg_GBps": round(1024 * nw / (msw * 1e-3) / 1e9, 1),
                "note": "moved = 2 x 64 B per cell per sweep; B_alg = SURVEY 8(d)'s 1024 N for the block config",
                "check": {"what": "rel. difference to the 5-sweep schedule", "value": dw, "ok": dw < 1e-12}}
            if not dw < 1e-12:
                check["ok"] = False
            wp.close()
            del bw, xw, x5
        except Exception as e:  # report, never fake
            other_configs["config4_wave128"] = {"error": str(e)}
        torch.cuda.empty_cache()
        # BASELINE configs 1 and 3: the PCApply inside the reference caller's GMRES step
        # (tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:117-136, fixed inflow sign)
        for key, n in (("config3_gmres256", 256), ("config1_gmres32", 32)):
            try:
                other_configs[key] = gmres_leg(n, args.gmres_steps)
                if not other_configs[key]["check"]["ok"]:
                    check["ok"] = False
            except Exception as e:  # report, never fake
                other_configs[key] = {"error": str(e)}
        # BASELINE config 4 proper: the wave system's implicit step with the block PCSHELL
        try:
            other_configs["config4_gmres128"] = wave_gmres_leg(128, max(1, args.gmres_steps // 2))
            if not other_configs["config4_gmres128"]["check"]["ok"]:
                check["ok"] = False
        except Exception as e:  # report, never fake
            other_configs["config4_gmres128"] = {"error": str(e)}
        torch.cuda.empty_cache()

    # north_star's scaling curve: the same apply on the 512^3 grid (BASELINE config 5), at every
    # N the driver launches, reported beside the 256^3 headline (strong scaling, whole job)
    scaling = None
    sg = [int(v) for v in args.scaling_grid]
    sg = sg * 3 if len(sg) == 1 else sg
    if len(sg) == 3 and min(sg) > 0 and sg != grid:
        wd.phase("scaling_512", deadlines["scaling_512"] + phase_extension(0, args.scaling_steps))
        if world > 1:
            plan.close()  # one library RCCL communicator at a time
            dist.barrier()
        del plan, b, x, run
        torch.cuda.empty_cache()
        try:
            plan, b, x, run, par2 = make(sg)
            k = max(1, args.scaling_steps)
            for _ in range(max(1, min(args.warmup, 3))):
                run()
            settle(run, min(args.settle_ms, 200.0))
            el = timed(run, k, 0)
            torch.cuda.synchronize()
            res2 = residual(b, x, sg)
            nl = sg[0] * sg[1] * sg[2] // world
            if world == 1:
                mv = moved_bytes(plan.passes(), nl)
            else:
                mv = sum(kernel_alg_bytes(p["mode"], p["elements"], p["n"]) for p in plan.phases()
                         if p["kind"] == "pass")
            scaling = {"grid": sg, "value": round(k / el, 4), "unit": "PCApply/s", "n_gpus": world,
                       "pieces": plan.pieces if world > 1 else 1,
                       "steps": k, "ms_per_step": round(el / k * 1e3, 4), "scaling": "strong",
                       "parallelism": par2,
                       "moved_bytes_per_gpu": mv,
                       "moved_GBps_per_gpu": round(mv / (el / k) / 1e9, 1),
                       "frac_moved": round(mv / (el / k) / 1e9 / HBM_PEAK_GBS, 4),
                       "B_alg_GBps_per_gpu": round(208 * nl / (el / k) / 1e9, 1),
                       "note": "moved = the schedule's launches (exchanges excluded); B_alg = SURVEY's 208 N convention",
                       "check": {"residual": res2, "tol": RES_TOL, "ok": res2 < RES_TOL}}
            if not res2 < RES_TOL:
                check["ok"] = False
                check["scaling_512_failed"] = True
        except Exception as e:  # report, never fake
            scaling = {"grid": sg, "error": str(e)}
            plan = None

    cpu = None
    wd.phase("cpu_baseline")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(grid, args.cpu_budget)
        except Exception as e:  # report, never fake
            log(f"cpu baseline failed: {e}")

    wd.phase("report")
    if rank == 0:
        out = {
            "metric": metric_name,
            "value": round(value, 3),
            "unit": "PCApply/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "c128 (f64 complex)",
            "data": f"synthetic: SplitMix64 U[-1,1) complex b, seed {SEED}, generated in HBM",
            "config": {"workload": f"{nx}x{ny}x{nz} c128 circulant PCApply, transport symbol lambda={LAM}",
                       "grid": grid, "global_batch": 1, "parallelism": parallelism},
            "status": "ok",
            "launcher": launcher,
            "exchange": exchange_used[0],
            "rccl": rccl,
            "settle": {"ms": round(settle_ms, 1), "applies": settle_n,
                       "note": "untimed applies after the W warm-up steps, before the timed region"},
            "check": check,
            "roofline": roof,
            "roofline_apply": roof_apply,
            "cpu_baseline": cpu,
        }
        if real_variant is not None:
            out["real_variant"] = real_variant
        if other_configs is not None:
            out["other_configs"] = other_configs
        if scaling is not None:
            out["scaling_512"] = scaling
        if passes_info is not None:
            out["passes"] = passes_info
        out["phases_s"] = wd.history
        print(json.dumps(out), flush=True)
    wd.phase("teardown")
    if world > 1:
        # tear down the library's RCCL communicator on every rank together, before torch's
        torch.cuda.synchronize()
        dist.barrier()
        if plan is not None:
            plan.close()
        dist.barrier()
        dist.destroy_process_group()
    wd.stop()
    if not check["ok"]:
        log(f"bench: output check FAILED: {check}")
        return 3
    return 0


def selftest_cpu(args, wd, rank: int, world: int, launcher: str, metric: str) -> int:
    """CPU rehearsal of bench.py's control flow: launch (self-launched or external), a gloo
    rendezvous, the phases under the watchdog, barriers around the K steps, the max over ranks
    and one JSON line with n_gpus = WORLD_SIZE.  The step is a host stand-in (a 16^3 numpy FFT
    round trip plus one all_reduce); no GPU call is made and nothing is measured ("value" null,
    "status" "selftest").  --selftest-stall PHASE blocks forever in PHASE to exercise the watchdog."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def stall(name):
        if args.selftest_stall == name and args.selftest_stall_rank in (-1, rank):
            log(f"selftest: rank {rank} stalls in phase '{name}'")
            while True:
                time.sleep(3600)

    wd.phase("init")
    stall("init")
    if world > 1:
        dist.init_process_group("gloo")
    wd.phase("plan")
    stall("plan")
    a = np.random.default_rng(rank).standard_normal((16, 16, 16)) + 0j
    tok = torch.zeros(1, dtype=torch.float64)

    def run():
        np.fft.ifftn(np.fft.fftn(a))
        if world > 1:
            dist.all_reduce(tok)
    wd.phase("first_apply")
    stall("first_apply")
    for _ in range(args.warmup):
        run()
    wd.phase("timed", wd.deadlines["timed"] + phase_extension(args.steps, 0))
    stall("timed")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    wd.phase("report")
    stall("report")
    if rank == 0:
        print(json.dumps({"metric": metric, "value": None, "unit": "PCApply/s", "status": "selftest",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(float(el.item()) / max(1, args.steps) * 1e3, 5),
                          "launcher": launcher, "phases_s": wd.history,
                          "note": "CPU rehearsal of bench.py's launch and control flow: host stand-in step, "
                                  "no GPU work, no measurement"}), flush=True)
    wd.phase("teardown")
    stall("teardown")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    wd.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
