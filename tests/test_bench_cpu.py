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
