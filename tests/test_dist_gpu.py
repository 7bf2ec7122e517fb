"""GPU parity of the slab-decomposed pass schedule (cfp_dist.hip) on one device.

* The single-process group executor runs P slabs with device copies as the exchange, so the
  split y layouts, the per-rank symbol and the chunk bookkeeping are checked on real
  kernels, up to BASELINE config 5's grid (512^3 in 8 slabs).
* SlabPlan runs in fresh child processes, one per rank, sharing cuda:0: each rank runs the
  library's kernel segments and the two all-to-alls go through torch.distributed (gloo,
  staged through host memory), so the per-rank plan is exercised across processes.
* The RCCL executor with world = 1 only.  With more ranks it runs only in the driver's
  multi-GPU bench (bench.py --gpus N on an 8-GPU node); this suite never starts it.  The
  per-rank plan it drives is the one the gloo multi-process tests check.
* At 256^3 and 512^3 (AUTO for every P | 32 up to 16 since r05)
  every rank runs the 3-sweep schedule (x + y1 into the per-peer chunks | y2 + z + symbol +
  inverses on its k1 rows | inverse), checked against the oracle and against the 5-pass slab
  schedule.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.mark.parametrize("dims,P", [((64, 64, 64), 2), ((64, 64, 64), 4), ((64, 64, 64), 8),
                                    ((128, 32, 16), 4), ((20, 12, 8), 4), ((256, 256, 256), 8),
                                    ((1, 8, 8), 2), ((32, 16, 8), 1), ((100, 100, 100), 4),
                                    ((200, 20, 10), 2),
                                    # VERDICT r03 item 7's layouts, and P not dividing ny (FFTW-MPI's
                                    # ceil(ny / P) row blocks: the last ranks hold fewer rows, or none)
                                    ((64, 40, 32), 4), ((256, 120, 256), 8), ((64, 30, 32), 4),
                                    ((256, 100, 256), 8), ((16, 3, 8), 4), ((100, 50, 30), 3)])
def test_group_vs_oracle(dims, P, oracle):
    from circulantpreconditioner_amd.distributed import SlabGroup
    lam = (0.6, 0.15 - 0.1j, 0.02)
    N = int(np.prod(dims))
    b = oracle.c_fill_uniform(N, 13)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    full = torch.from_numpy(b).cuda()
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        xs = g.apply(g.scatter(full))
        got = torch.cat([x.cpu() for x in xs]).numpy()
    assert oracle.rel_l2(got, ref) < TOL


def test_group_config5_512_in_8_slabs(oracle, case512):
    """BASELINE config 5's decomposition (512^3, z slabs of 64 planes, 8 ranks) on one device,
    against the oracle's full-grid solve (AUTO pieces: 4 per all-to-all at this size)."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, lam, b, ref = case512
    P = 8
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        bs = g.scatter(torch.from_numpy(b).cuda())
        xs = g.apply(bs)
        got = torch.cat([x.cpu() for x in xs]).numpy()
        del bs, xs
    assert oracle.rel_l2(got, ref) < TOL


@pytest.fixture(scope="module")
def case256(oracle):
    dims, lam = (256, 256, 256), (0.6, 0.15 - 0.1j, 0.02)
    b = oracle.c_fill_uniform(256 ** 3, 17)
    return dims, lam, b, oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)


@pytest.mark.parametrize("P", [1, 2, 4, 8, 16])
def test_group_three_sweep_256(P, case256, oracle):
    """The 3-sweep slab schedule (AUTO at 256^3, P | 32) against the oracle and against the
    5-pass slab schedule; P = 4 also in place."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, lam, b, ref = case256
    full = torch.from_numpy(b).cuda()
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam).set_schedule("three")  # AUTO picks it too (r05)
        bs = g.scatter(full)
        x3 = torch.cat(g.apply(bs))
        assert oracle.rel_l2(x3.cpu().numpy(), ref) < TOL
        g.set_schedule("five")
        x5 = torch.cat(g.apply(bs))
        assert float(torch.linalg.vector_norm(x5 - x3) / torch.linalg.vector_norm(x3)) < 1e-13
        g.set_schedule("three")
        if P == 4:
            g.apply(bs, bs)  # in place, as the direct solver's (Un, Un)
            assert torch.equal(torch.cat(bs), x3)
        del bs


def test_slab_schedule_rules():
    from circulantpreconditioner_amd import CirculantError
    from circulantpreconditioner_amd.distributed import SlabGroup
    with SlabGroup((64, 64, 64), 2) as g:
        with pytest.raises(CirculantError):
            g.set_schedule("three")  # 256^3 and 512^3 only
        g.set_schedule("five").set_schedule("auto")
    with SlabGroup((256, 256, 256), 32) as g:  # 8 rows per chunk: below the 16 the 3-sweep P3 reads
        with pytest.raises(CirculantError):
            g.set_schedule("three")
        with pytest.raises(CirculantError):
            g.set_schedule(9)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def case512(oracle):
    dims, lam = (512, 512, 512), (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(512 ** 3, 512)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    return dims, lam, b, ref


def test_single_gpu_512_auto_vs_oracle(case512):
    """the single-GPU 512^3 AUTO path (3 sweeps, N1 = 32 x N2 = 16, its own
    z-fused symbol tables) against the oracle's full-grid solve, not only by residual; in place too."""
    import circulantpreconditioner_amd as cp
    dims, lam, b, ref = case512
    rd = torch.from_numpy(ref).cuda()
    tb = torch.from_numpy(b).cuda()
    with cp.CirculantPlan(dims) as p:
        p.set_transport_symbol(lam)
        assert [q["mode"] for q in p.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
        x = p.apply(tb)
        err = float(torch.linalg.vector_norm(x - rd) / torch.linalg.vector_norm(rd))
        assert err < TOL, err
        p.apply(tb, out=tb)  # in place (the direct solver's Un, Un)
        assert torch.equal(tb, x)
    del rd, tb, x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("P", [1, 8, 16])
def test_group_three_sweep_512(P, case512):
    """Config 5's grid on the 3-sweep slab schedule (AUTO at 512^3 for P | 32 since r05: N1 = 32 x
    N2 = 16, P2 on the rank's nyl / 16 k1 values with the global k1 offset) against the oracle,
    and against the 5-pass slab schedule (compared on the device)."""
    from circulantpreconditioner_amd.distributed import SlabGroup, slab_steps
    dims, lam, b, ref = case512
    assert [s["kind"] for s in slab_steps(dims, P, 0, schedule="auto")].count(2) == 3
    full = torch.from_numpy(b).cuda()
    rd = torch.from_numpy(ref).cuda()
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam).set_pieces(1)
        bs = g.scatter(full)
        del full
        x3 = torch.cat(g.apply(bs))
        err = float(torch.linalg.vector_norm(x3 - rd) / torch.linalg.vector_norm(rd))
        assert err < TOL, (P, err)
        del rd
        if P == 8:
            g.set_schedule("five")
            x5 = torch.cat(g.apply(bs))
            assert float(torch.linalg.vector_norm(x5 - x3) / torch.linalg.vector_norm(x3)) < 1e-13
            del x5
        del bs, x3
    torch.cuda.empty_cache()


@pytest.mark.parametrize("P", [2, 4, 8])
def test_group_pieces_512(P, case512):
    """Config 5's grid with the pipelined exchange: the pieced step list (K = 1, 4, 8 pieces per
    all-to-all) through the group executor, against the oracle (compared on the device)."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, lam, b, ref = case512
    full = torch.from_numpy(b).cuda()
    rd = torch.from_numpy(ref).cuda()
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        bs = g.scatter(full)
        del full
        for K in (1, 4, 8):
            g.set_pieces(K)
            xs = g.apply(bs)
            got = torch.cat(xs)
            del xs
            err = float(torch.linalg.vector_norm(got - rd) / torch.linalg.vector_norm(rd))
            del got
            assert err < TOL, (P, K, err)
        del bs
    del rd
    torch.cuda.empty_cache()


@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_group_pieces_256(P, case256):
    """256^3 with pieces (K = 1, 4, 8 where K | 256 / P): the 3-sweep slab schedule (AUTO) and
    the five-pass one, in place at K = 4."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, lam, b, ref = case256
    rd = torch.from_numpy(ref).cuda()
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        bs = g.scatter(torch.from_numpy(b).cuda())
        for sched in ("three", "five"):
            g.set_schedule(sched)
            for K in [k for k in (1, 4, 8) if (256 // P) % k == 0]:
                g.set_pieces(K)
                got = torch.cat(g.apply(bs))
                err = float(torch.linalg.vector_norm(got - rd) / torch.linalg.vector_norm(rd))
                assert err < TOL, (P, sched, K, err)
        g.set_schedule("auto").set_pieces(4)
        g.apply(bs, bs)  # in place, as the direct solver's (Un, Un)
        got = torch.cat(bs)
        assert float(torch.linalg.vector_norm(got - rd) / torch.linalg.vector_norm(rd)) < TOL
        del bs


@pytest.mark.parametrize("dims,P,pieces", [((64, 30, 32), 4, (1, 2, 4, 8)), ((256, 100, 256), 8, (1, 4))])
def test_group_padded_pieces(dims, P, pieces, oracle):
    """P not dividing ny with the pipelined exchanges (K pieces) and in place."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    lam = (0.6, 0.15 - 0.1j, 0.02)
    N = int(np.prod(dims))
    b = oracle.c_fill_uniform(N, 17)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        bs = g.scatter(torch.from_numpy(b).cuda())
        for K in pieces:
            g.set_pieces(K)
            got = torch.cat([x.cpu() for x in g.apply(bs)]).numpy()
            assert oracle.rel_l2(got, ref) < TOL, K
        g.apply(bs, bs)
        got = torch.cat([x.cpu() for x in bs]).numpy()
        assert oracle.rel_l2(got, ref) < TOL


def _slab_rank(rank, world, port, dims, lam, seed, q, pieces=1):
    """One rank of a SlabPlan in its own process (exchange through torch.distributed / gloo)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import circulantpreconditioner_amd as cp
        from circulantpreconditioner_amd.distributed import SlabPlan
        torch.cuda.set_device(0)
        plan = SlabPlan(dims, rank=rank, world=world, device=0, exchange="torch")
        plan.set_transport_symbol(lam).set_pieces(pieces)
        b = torch.empty(plan.local_size, dtype=torch.complex128, device="cuda:0")
        cp.fill_uniform(b, seed, offset=plan.local_offset)
        x = plan.apply(b)
        t = b.clone()
        plan.apply(t, out=t)  # in place, as the direct solver's (Un, Un)
        torch.cuda.synchronize()
        q.put((rank, plan.local_offset, x.cpu().numpy(), bool(torch.equal(t, x))))
        plan.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dims,world,pieces", [((64, 32, 16), 2, 1), ((128, 128, 128), 2, 1), ((64, 64, 64), 4, 1),
                                               ((100, 20, 10), 2, 1), ((256, 256, 256), 2, 1),
                                               ((64, 32, 16), 2, 4), ((128, 128, 128), 2, 4),
                                               ((256, 256, 256), 2, 4), ((64, 64, 64), 4, 2),
                                               ((64, 40, 32), 4, 1), ((64, 30, 32), 4, 2), ((32, 9, 16), 2, 1)])
def test_slab_plan_processes_vs_oracle(dims, world, pieces, oracle):
    """`world` fresh processes, one SlabPlan rank each, on cuda:0; gathered x vs the oracle.
    pieces > 1: the pipelined step list, every piece through torch.distributed."""
    import torch.multiprocessing as mp
    lam, seed = (0.6, 0.15 - 0.1j, 0.02), 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_rank, args=(r, world, port, dims, lam, seed, q, pieces))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    N = int(np.prod(dims))
    x = np.empty(N, dtype=np.complex128)
    for _, off, part, inplace_ok in parts:
        assert inplace_ok
        x[off:off + part.size] = part
    b = oracle.c_fill_uniform(N, seed)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    assert oracle.rel_l2(x, ref) < TOL


def test_group_inplace(oracle):
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, P, lam = (32, 32, 32), 4, (0.3, 0.3, 0.3)
    b = oracle.c_fill_uniform(32 ** 3, 1)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    with SlabGroup(dims, P) as g:
        g.set_transport_symbol(lam)
        bs = g.scatter(torch.from_numpy(b).cuda())
        g.apply(bs, bs)
        got = torch.cat([x.cpu() for x in bs]).numpy()
    assert oracle.rel_l2(got, ref) < TOL


def test_rccl_single_rank(oracle):
    """The RCCL executor with world = 1 (self exchange) in a one-process group."""
    import os
    import torch.distributed as dist
    from circulantpreconditioner_amd.distributed import SlabPlan
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    created = False
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
        created = True
    try:
        dims, lam = (64, 32, 16), (0.6, 0.15, 0.02)
        b = oracle.c_fill_uniform(int(np.prod(dims)), 21)
        ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
        plan = SlabPlan(dims, rank=0, world=1, device=0, timeout_s=60.0)
        # the non-blocking communicator (ncclCommInitRankConfig, polled) reports what it saw
        info = plan.rccl_info()
        assert info["ranks"] == 1 and info["rank"] == 0 and info["version"] >= 21400
        assert "rccl" in info["lib"] and 0.0 <= info["init_ms"] < 60e3
        plan.set_transport_symbol(lam)
        x = plan.apply(torch.from_numpy(b).cuda())
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        # sampled phase events inside ordinary applies (bench.py's N > 1 kernel times)
        assert plan.profile_begin(10, every=2)
        tb = torch.from_numpy(b).cuda()
        for _ in range(5):
            plan.apply(tb, out=x)
        ms, napp = plan.profile_end()
        assert napp == 3 and len(ms) == len(plan.phases()) and all(m >= 0.0 for m in ms)
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        plan.close()
        # 256^3: the 3-sweep slab schedule through the RCCL executor
        dims = (256, 256, 256)
        b = oracle.c_fill_uniform(256 ** 3, 23)
        ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
        plan = SlabPlan(dims, rank=0, world=1, device=0)
        plan.set_transport_symbol(lam)
        assert [p.get("mode") for p in plan.phases()] == ["rows_fwd", None, "mid_fused", None, "rows_inv"]
        x = plan.apply(torch.from_numpy(b).cuda())
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        # the pipelined apply: 4 pieces per exchange on the plan's exchange stream, ordered by
        # events against the passes on the caller's stream (world 1: the pieces are self copies)
        plan.set_pieces(4)
        assert plan.pieces == 4 and sum(p["kind"] == "all-to-all" for p in plan.phases()) == 8
        tb = torch.from_numpy(b).cuda()
        for _ in range(3):
            x = plan.apply(tb, out=x)
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        plan.apply(tb, out=tb)  # in place
        assert oracle.rel_l2(tb.cpu().numpy(), ref) < TOL
        assert plan.profile_begin(4, every=1)
        for _ in range(2):
            plan.apply(torch.from_numpy(b).cuda(), out=x)
        ms, napp = plan.profile_end()
        assert napp == 2 and len(ms) == len(plan.phases()) and all(m >= 0.0 for m in ms)
        plan.set_schedule("five")
        x = plan.apply(torch.from_numpy(b).cuda())
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        plan.close()
    finally:
        if created:
            dist.destroy_process_group()


_MISSING_PEER = r"""
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
from circulantpreconditioner_amd._lib import lib
L = lib()
uid = ctypes.create_string_buffer(L.cfp_dist_unique_id_bytes())
assert L.cfp_dist_get_unique_id(uid) == 0
h = ctypes.c_void_p()
t0 = time.perf_counter()
rc = L.cfp_dist_plan_create_timeout(ctypes.byref(h), 32, 16, 8, 2, 0, uid, 0, 3.0)
print(rc, bool(h.value), round(time.perf_counter() - t0, 2), L.cfp_last_error().decode(), flush=True)
"""


def test_rccl_missing_peer_times_out():
    """the plan's communicator is created non-blocking and polled against a
    deadline, so a rank whose peer never joins gets an error (CFP_ERR_LIB = 76, "timed out")
    instead of hanging -- here rank 0 of 2 in a process whose rank 1 does not exist.  Run in a
    child process with its own time limit, so a hang would fail the test, not the session."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _MISSING_PEER, root], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    rc, made, secs, msg = p.stdout.strip().splitlines()[-1].split(" ", 3)  # (RCCL prints a banner first)
    assert rc == "76" and made == "False" and "timed out" in msg, p.stdout
    assert float(secs) < 60.0


def test_rccl_single_rank_transforms_and_diag(oracle):
    """World 1 through the RCCL executor: the distributed MatMult / MatMultTranspose step lists
    (natural slab in and out) against torch.fft, and the explicit-Diag apply (Diag moved into the
    z-pencil layout once) against the oracle."""
    import torch.distributed as dist
    from circulantpreconditioner_amd._lib import check, lib
    from circulantpreconditioner_amd.distributed import SlabPlan
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29532")
    created = False
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
        created = True
    try:
        dims = (64, 32, 16)
        N = int(np.prod(dims))
        b = oracle.c_fill_uniform(N, 41)
        tb = torch.from_numpy(b).cuda()
        plan = SlabPlan(dims, rank=0, world=1, device=0)
        out = torch.empty_like(tb)
        check(lib().cfp_dist_plan_forward(plan._h, tb.data_ptr(), out.data_ptr(), None))
        torch.cuda.synchronize()
        f = torch.fft.fftn(tb.view(16, 32, 64)).reshape(-1)
        assert float(torch.linalg.vector_norm(out - f) / torch.linalg.vector_norm(f)) < 1e-13
        check(lib().cfp_dist_plan_backward(plan._h, tb.data_ptr(), out.data_ptr(), None))
        torch.cuda.synchronize()
        g = torch.fft.ifftn(tb.view(16, 32, 64)).reshape(-1) * N
        assert float(torch.linalg.vector_norm(out - g) / torch.linalg.vector_norm(g)) < 1e-13
        rng = np.random.default_rng(3)
        d = 1.5 + rng.random(N) + 1j * rng.standard_normal(N)
        ref = oracle.c_solve_3d(d, b, dims)
        plan.set_diag(torch.from_numpy(d).cuda())
        x = plan.apply(tb)
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        plan.set_pieces(2)
        x = plan.apply(tb)
        assert oracle.rel_l2(x.cpu().numpy(), ref) < TOL
        plan.close()
    finally:
        if created:
            dist.destroy_process_group()


_BLOCKING_CHILD = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.getcwd())
import torch
import torch.distributed as dist
from circulantpreconditioner_amd.distributed import SlabPlan, rccl_mode
dist.init_process_group("gloo", rank=0, world_size=1, init_method="tcp://127.0.0.1:%s" % sys.argv[1])
dims, lam = (32, 16, 8), (0.6, 0.15, 0.02)
b = torch.randn(int(np.prod(dims)), dtype=torch.complex128).cuda()
plan = SlabPlan(dims, rank=0, world=1, device=0, timeout_s=60.0)
plan.set_transport_symbol(lam)
x = plan.apply(b)
ref = SlabPlan(dims, rank=0, world=1, device=0, exchange="torch").set_transport_symbol(lam).apply(b)
print(json.dumps({"mode": rccl_mode(), "ranks": plan.rccl_info()["ranks"],
                  "rel": float(torch.linalg.vector_norm(x - ref) / torch.linalg.vector_norm(ref))}))
plan.close()
dist.destroy_process_group()
"""


def test_rccl_blocking_protocol_single_rank():
    """CFP_RCCL_BLOCKING=1 (bench.py --rccl-blocking): the plan's communicator is made
    by ncclCommInitRank and destroyed by ncclCommDestroy; world = 1 through RCCL equals the torch
    exchange.  In a child process: the switch is read once per process."""
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CFP_RCCL_BLOCKING="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _BLOCKING_CHILD, str(port)], env=env, cwd=root, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["mode"] == "blocking" and r["ranks"] == 1
    assert r["rel"] < 1e-14
