"""bench.py host logic on CPU: the N > 1 exchange choice cannot hide an RCCL failure, and
the moved-bytes accounting of the schedules."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


class _Plan:
    def __init__(self, ex):
        self.exchange = ex
        self.closed = False

    def close(self):
        self.closed = True


def _creator(fail_rccl):
    def create(ex):
        if ex == "rccl" and fail_rccl:
            raise RuntimeError("ncclCommInitRank: invalid unique id")
        return _Plan(ex)
    return create


def test_rccl_ok_is_used():
    plan, label = bench.choose_slab_plan(_creator(False), None, lambda ok: ok)
    assert label == "rccl" and plan.exchange == "rccl"


def test_default_fallback_is_labelled():
    msgs = []
    plan, label = bench.choose_slab_plan(_creator(True), None, lambda ok: ok, warn=msgs.append)
    assert label == "torch-fallback" and plan.exchange == "torch" and msgs


def test_explicit_rccl_request_fails_loudly():
    with pytest.raises(SystemExit):
        bench.choose_slab_plan(_creator(True), "rccl", lambda ok: ok)


def test_other_rank_failure_is_agreed():
    """This rank's communicator is fine, another rank's is not: the rank closes its plan and
    falls back with everyone else."""
    made = []

    def create(ex):
        made.append(_Plan(ex))
        return made[-1]
    plan, label = bench.choose_slab_plan(create, None, lambda ok: False)
    assert label == "torch-fallback" and made[0].closed and plan.exchange == "torch"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        import sys
        import torch
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench as B

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t.item()) == 1
        # rank 1 gets a bad unique id: its RCCL communicator fails, rank 0's would not
        _, label = B.choose_slab_plan(_creator(rank == 1), None, agree)
        try:
            B.choose_slab_plan(_creator(rank == 1), "rccl", agree)
            strict = "no-exit"
        except SystemExit:
            strict = "exit"
        q.put((rank, label, strict))
    finally:
        dist.destroy_process_group()


def test_forced_rccl_failure_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, "torch-fallback", "exit"), (1, "torch-fallback", "exit")]


def test_moved_bytes_of_the_schedules():
    N = 256 ** 3
    three = [{"mode": "rows_fwd", "n": 256}, {"mode": "mid_fused", "n": 256}, {"mode": "rows_inv", "n": 256}]
    five = [{"mode": "fwd", "n": 256}, {"mode": "fwd", "n": 256}, {"mode": "fused_sep", "n": 256},
            {"mode": "inv", "n": 256}, {"mode": "inv", "n": 256}]
    assert 96 * N <= bench.moved_bytes(three, N) < 96.1 * N
    assert 160 * N <= bench.moved_bytes(five, N) < 160.1 * N


def _residual_case(n, lam, seed, wrong=False):
    import numpy as np
    import torch
    from oracle import oracle as O

    N = int(np.prod(n))
    b = O.c_fill_uniform(N, seed)
    x = O.c_solve_3d(O.c_build_diag_transport(n, lam), b, n)
    if wrong:
        x = x * (1 + 1e-6)
    return torch.from_numpy(b), torch.from_numpy(x)


def test_transport_residual_one_rank():
    """bench.py's output check: ~1e-16 on the oracle's solve, far above 1e-10 on a perturbed one."""
    n, lam = (12, 10, 8), (0.6, 0.15, 0.02)
    b, x = _residual_case(n, lam, 5)
    assert bench.transport_residual(b, x, n, lam) < 1e-14
    b, x = _residual_case(n, lam, 5, wrong=True)
    assert bench.transport_residual(b, x, n, lam) > bench.RES_TOL


def _residual_rank(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench as B

        n, lam = (12, 10, 8), (0.6, 0.15, 0.02)
        b, x = _residual_case(n, lam, 5)
        loc = 12 * 10 * 4  # this rank's z-slab (PETSC_DECIDE rows)
        sl = slice(rank * loc, (rank + 1) * loc)
        q.put((rank, B.transport_residual(b[sl].clone(), x[sl].clone(), n, lam, rank, 2)))
    finally:
        dist.destroy_process_group()


def test_transport_residual_two_slabs_gloo():
    """The slab form of the check (z-roll across ranks through all_gather) equals the one-rank value."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_residual_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, lam = (12, 10, 8), (0.6, 0.15, 0.02)
    b, x = _residual_case(n, lam, 5)
    one = bench.transport_residual(b, x, n, lam)
    assert res[0][1] == pytest.approx(one, rel=1e-6) and res[1][1] == pytest.approx(one, rel=1e-6)
    assert one < 1e-14


# ---------------------------------------------------------------- launch and watchdog
import json
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, extra_env=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "CFP_BENCH_SELF_LAUNCHED")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus_2_without_launcher_self_launches():
    """bench.py --gpus 2 with no launcher starts its 2 ranks itself (torch.distributed.run child,
    gloo here) and rank 0 prints one line with n_gpus 2 -- it never runs one GPU silently."""
    rc, lines, err = _bench(["--gpus", "2", "--selftest-cpu", "--steps", "5", "--warmup", "2"],
                            {"CFP_BENCH_SHARE_DEVICE": "1", "CFP_BENCH_BACKEND": "gloo"})
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["status"] == "selftest" and ln["value"] is None
    assert ln["launcher"] == "self (torch.distributed.run)"
    assert [p[0] for p in ln["phases_s"]][:4] == ["import", "init", "plan", "first_apply"]


def test_watchdog_names_the_stalled_phase():
    """A rank that blocks in the timed region: every rank's watchdog fires, rank 0 prints the
    timeout line naming the phase, and the run exits non-zero."""
    rc, lines, err = _bench(["--gpus", "2", "--selftest-cpu", "--steps", "5", "--warmup", "1",
                             "--selftest-stall", "timed", "--selftest-stall-rank", "1", "--deadline", "timed=3"])
    assert rc != 0
    assert len(lines) == 1, (lines, err[-2000:])
    assert lines[0]["status"] == "timeout" and lines[0]["phase"] == "timed" and lines[0]["rank"] == 0
    assert "phase 'timed' exceeded" in err and "Thread 0x" in err  # faulthandler stacks


def test_watchdog_single_rank_init_stall():
    rc, lines, err = _bench(["--gpus", "1", "--selftest-cpu", "--selftest-stall", "init", "--deadline", "init=2"])
    assert rc == 3 and lines and lines[0]["status"] == "timeout" and lines[0]["phase"] == "init"


def test_world_size_mismatch_is_refused():
    rc, lines, err = _bench(["--gpus", "2", "--selftest-cpu"], {"WORLD_SIZE": "1"})
    assert rc == 2 and not lines and "refusing" in err


def test_deadline_override_parsing():
    d = bench.parse_deadlines(["timed=7", "init=1.5"])
    assert d["timed"] == 7.0 and d["init"] == 1.5 and d["plan"] == bench.DEADLINES["plan"]
    with pytest.raises(SystemExit):
        bench.parse_deadlines(["nosuchphase=3"])


def test_rccl_library_is_reported_host_only():
    """The library reports which librccl its RCCL calls bind to (torch bundles one with the same
    soname as /opt/rocm's), without a GPU."""
    from circulantpreconditioner_amd.distributed import rccl_version
    v = rccl_version()
    assert v["version"] >= 21400 and "rccl" in v["lib"]


def test_rccl_blocking_switch_is_reported():
    """CFP_RCCL_BLOCKING=1 (bench.py --rccl-blocking) selects the blocking RCCL protocol
    for the library's communicators, read once per process; rccl_version() / rccl_info() say which."""
    code = "from circulantpreconditioner_amd.distributed import rccl_mode; print(rccl_mode())"
    for env, want in (({"CFP_RCCL_BLOCKING": "1"}, "blocking"), ({"CFP_RCCL_BLOCKING": "0"}, "non-blocking"),
                      ({}, "non-blocking")):
        e = {k: v for k, v in os.environ.items() if k != "CFP_RCCL_BLOCKING"}
        e.update(env)
        out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120,
                             cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert out.returncode == 0, out.stderr
        assert out.stdout.strip() == want
