"""GPU parity of the slab-decomposed pass schedule (cfp_dist.hip) on one device: the
single-process group executor runs P slabs with device copies as the exchange, so the
split y layouts, the per-rank symbol and the chunk bookkeeping are checked on real
kernels.  The RCCL executor shares the schedule; it is exercised by bench.py --gpus N."""
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
    finally:
        if created:
            dist.destroy_process_group()
