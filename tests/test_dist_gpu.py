"""GPU parity of the slab-decomposed pass schedule (cfp_dist.hip) on one device.

* The single-process group executor runs P slabs with device copies as the exchange, so the
  split y layouts, the per-rank symbol and the chunk bookkeeping are checked on real
  kernels, up to BASELINE config 5's grid (512^3 in 8 slabs).
* SlabPlan runs in fresh child processes, one per rank, sharing cuda:0: each rank runs the
  library's kernel segments and the two all-to-alls go through torch.distributed (gloo,
  staged through host memory), so the per-rank plan is exercised across processes.
* The RCCL executor with world = 1; with more ranks it is exercised by bench.py --gpus N.
* At 256^3 (AUTO for P <= 4, on request up to P = 16) every rank runs the 3-sweep schedule
  (x + y1 into the per-peer chunks | y2 + z + symbol + inverses on its k1 rows | inverse),
  checked against the oracle and against the 5-pass slab schedule.
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
                                    ((200, 20, 10), 2)])
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


def test_group_config5_512_in_8_slabs(oracle):
    """BASELINE config 5's decomposition (512^3, z slabs of 64 planes, 8 ranks) on one device,
    against the oracle's full-grid solve."""
    from circulantpreconditioner_amd.distributed import SlabGroup
    dims, P, lam = (512, 512, 512), 8, (0.6, 0.15, 0.02)
    N = int(np.prod(dims))
    b = oracle.c_fill_uniform(N, 512)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
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
        g.set_transport_symbol(lam).set_schedule("three")  # AUTO picks it for P <= 4
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
            g.set_schedule("three")  # 256^3 only
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


def _slab_rank(rank, world, port, dims, lam, seed, q):
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
        plan.set_transport_symbol(lam)
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


@pytest.mark.parametrize("dims,world", [((64, 32, 16), 2), ((128, 128, 128), 2), ((64, 64, 64), 4),
                                        ((100, 20, 10), 2), ((256, 256, 256), 2)])
def test_slab_plan_processes_vs_oracle(dims, world, oracle):
    """`world` fresh processes, one SlabPlan rank each, on cuda:0; gathered x vs the oracle."""
    import torch.multiprocessing as mp
    lam, seed = (0.6, 0.15 - 0.1j, 0.02), 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_rank, args=(r, world, port, dims, lam, seed, q)) for r in range(world)]
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
        plan = SlabPlan(dims, rank=0, world=1, device=0)
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
        plan.close()
    finally:
        if created:
            dist.destroy_process_group()
