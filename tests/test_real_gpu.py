"""Row f4: the real-data (r2c / half spectrum / c2r) apply against the oracle's
complex solve of the same real right-hand side (whose solution is real for real lambda)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-10


@pytest.fixture(scope="module")
def cp():
    import circulantpreconditioner_amd as cp
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return cp


@pytest.mark.parametrize("n", [(32, 16, 8), (64, 32, 48), (256, 256, 256), (32, 1, 16), (128, 64, 1), (1024, 4, 4),
                               (32, 6, 5), (32, 2, 1), (512, 8, 8)],
                         ids=lambda n: "x".join(map(str, n)))
@pytest.mark.parametrize("lam", [(0.6, 0.15, 0.02), (55.6, 0.0, 0.0), (0.0, 0.0, 0.0)], ids=["bench", "transport", "zero"])
def test_real_plan_vs_oracle(cp, oracle, n, lam):
    N = int(np.prod(n))
    rng = np.random.default_rng(7)
    b = rng.standard_normal(N)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b.astype(np.complex128), n)
    assert np.abs(ref.imag).max() <= 1e-12 * np.abs(ref).max()  # real lambda, real b -> real x
    with cp.RealPlan(n) as plan:
        plan.set_transport_symbol(lam)
        x = plan.apply(torch.from_numpy(b).cuda()).cpu().numpy()
        assert np.linalg.norm(x - ref.real) <= TOL * np.linalg.norm(ref.real)
        t = torch.from_numpy(b).cuda()
        plan.apply(t, out=t)  # in place
        assert np.array_equal(t.cpu().numpy(), x)


def test_real_plan_matches_complex_plan_256(cp):
    n = (256, 256, 256)
    N = 256 ** 3
    lam = (0.6, 0.15, 0.02)
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 5)
    br = b.real.contiguous()
    with cp.CirculantPlan(n) as pc, cp.RealPlan(n) as pr:
        xc = pc.set_transport_symbol(lam).apply(br.to(torch.complex128))
        xr = pr.set_transport_symbol(lam).apply(br)
        assert float(torch.linalg.vector_norm(xr - xc.real) / torch.linalg.vector_norm(xc.real)) < 1e-12
        ms = pr.time_passes(br, torch.empty_like(br), iters=3)
        assert len(ms) == 4 and all(m > 0 for m in ms)


@pytest.mark.parametrize("side", [256, 128])
@pytest.mark.parametrize("lam", [(0.6, 0.15, 0.02), (55.6, 0.0, 0.0), (1.3, 0.0, 2.5)], ids=["bench", "transport", "xz"])
def test_real_three_sweep_256_vs_oracle(cp, oracle, lam, side):
    """The 3-sweep real schedule (r2c rows + y1 | half-spectrum y2/z | y1 inverse + c2r rows) at
    256^3 and 128^3 against the oracle, in place, and against the r2c + 3 half-spectrum passes
    schedule."""
    n = (side, side, side)
    N = side ** 3
    b = oracle.c_fill_uniform(N, 41).real.copy()
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b.astype(np.complex128), n).real
    with cp.RealPlan(n) as plan:
        plan.set_transport_symbol(lam)
        assert plan.three_sweep  # AUTO at 128^3 and 256^3
        x = plan.apply(torch.from_numpy(b).cuda())
        assert np.linalg.norm(x.cpu().numpy() - ref) <= TOL * np.linalg.norm(ref)
        t = torch.from_numpy(b).cuda()
        plan.apply(t, out=t)
        assert torch.equal(t, x)
        plan.set_schedule("three_alt")  # row sweeps with workgroup-barrier exchanges (A/B)
        assert plan.three_sweep
        xa = plan.apply(torch.from_numpy(b).cuda())
        assert float(torch.linalg.vector_norm(xa - x) / torch.linalg.vector_norm(x)) < 1e-13
        t = torch.from_numpy(b).cuda()
        plan.apply(t, out=t)
        assert torch.equal(t, xa)
        plan.set_schedule("five")
        assert not plan.three_sweep
        x5 = plan.apply(torch.from_numpy(b).cuda())
        assert float(torch.linalg.vector_norm(x5 - x) / torch.linalg.vector_norm(x)) < 1e-13


def test_real_plan_errors(cp):
    with pytest.raises(cp.CirculantError):
        cp.RealPlan((30, 4, 4))  # nx/2 not a power of two
    with pytest.raises(cp.CirculantError):
        cp.RealPlan((2048, 4, 4))  # nx/2 above 512
    with pytest.raises(cp.CirculantError):
        cp.RealPlan((64, 1, 1))  # ny * nz == 1
    with cp.RealPlan((32, 4, 4)) as plan:
        with pytest.raises(cp.CirculantError):
            plan.set_schedule("three")  # 128^3 and 256^3 only
        with pytest.raises(cp.CirculantError):
            plan.set_schedule(7)
        assert not plan.three_sweep
        b = torch.zeros(512, dtype=torch.float64, device="cuda")
        with pytest.raises(cp.CirculantError):
            plan.apply(b)  # no symbol
        plan.set_transport_symbol((1.0, 1.0, 1.0))
        with pytest.raises(ValueError):
            plan.apply(torch.zeros(511, dtype=torch.float64, device="cuda"))
