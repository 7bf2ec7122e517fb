"""GPU parity: the HIP path (through the C ABI) vs the golden vectors and the CPU oracle.

Tolerance (north_star): relative L2 error <= 1e-10 on the preconditioned vector.
Full-size cases (256^3, 512^3) are checked through size-independent properties:
the residual ||C x - b|| / ||b|| of the circulant operator, and the round trip
backward(forward(b)) = N b.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _lam(case):
    return tuple(complex(re, im) for re, im in case["lam"])


@pytest.fixture(scope="module")
def cp():
    import circulantpreconditioner_amd as cp
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return cp


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.complex128)).cuda()


def _rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def apply_C_torch(x, n, lam):
    """y = C x on the device with torch.roll (test-side checker, not the product)."""
    nx, ny, nz = n
    u = x.reshape(nz, ny, nx)
    y = u.clone()
    for l, dim, nd in ((lam[0], 2, nx), (lam[1], 1, ny), (lam[2], 0, nz)):
        if nd > 1 and l != 0:
            y = y + l * (u - torch.roll(u, shifts=1, dims=dim))
    return y.reshape(-1)


GOLDEN = ["kat3d_4x3x2", "py3d_10x25x40", "kat1d_4", "py1d_8", "py2d_12x10", "py2d_50x200",
          "rand16_A", "rand16_B", "odd6x5x7"]


@pytest.mark.parametrize("name", GOLDEN)
def test_golden_transport_symbol(cp, golden, name):
    c = golden[name]
    n = tuple(c["n"])
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(_lam(c))
        x = plan.apply(_dev(c["b"]))
        torch.cuda.synchronize()
        assert _rel(x, c["x"]) < TOL
        assert _rel(plan.get_diag(), c["diag"]) < 1e-14


@pytest.mark.parametrize("name", GOLDEN)
def test_golden_explicit_diag(cp, golden, name):
    c = golden[name]
    n = tuple(c["n"])
    with cp.CirculantPlan(n) as plan:
        plan.set_diag(_dev(c["diag"]))
        x = plan.apply(_dev(c["b"]))
        assert _rel(x, c["x"]) < TOL
        # solve_3D with a caller-owned Diag vector
        y = plan.apply_with_diag(_dev(c["diag"]), _dev(c["b"]))
        assert _rel(y, c["x"]) < TOL


def test_golden_rand32(cp, golden):
    c = golden["rand32_A"]
    n = tuple(c["n"])
    b = torch.empty(32 ** 3, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, c["b_generator"]["seed"])
    import hashlib
    assert hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest() == c["b_sha256"]
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(_lam(c))
        assert _rel(plan.apply(b), c["x"]) < TOL


def test_kat1d_published(cp, golden):
    c = golden["kat1d_4"]
    with cp.CirculantPlan((4, 1, 1)) as plan:
        plan.set_transport_symbol((0.5, 0, 0))
        x = plan.apply(_dev(c["b"])).cpu().numpy()
    np.testing.assert_allclose(x.real, [6.7, 2.9, 6.3, 20.1], atol=1e-12)
    assert np.abs(x.imag).max() < 1e-12


SIZES = [(16, 16, 16), (32, 32, 32), (64, 64, 64), (128, 128, 128), (32, 64, 128), (256, 16, 8),
         (8, 256, 16), (512, 4, 16), (16, 32, 512), (1024, 16, 16), (7, 9, 11), (20, 30, 40),
         (64, 1, 1), (1, 64, 1), (1, 1, 64), (100, 1, 1), (1, 1, 1), (48, 64, 1), (2, 2, 2),
         (1000, 3, 2), (3, 243, 5)]


@pytest.mark.parametrize("n", SIZES, ids=lambda n: "x".join(map(str, n)))
@pytest.mark.parametrize("lam", [(0.6, 0.15, 0.02), (55.6, 0.0, 0.0), (0.3 + 0.2j, -0.1j, 1.7)],
                         ids=["bench", "transport", "complex"])
def test_vs_oracle(cp, oracle, n, lam):
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 20251017)
    d = oracle.c_build_diag_transport(n, lam)
    ref = oracle.c_solve_3d(d, b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL, plan.passes()


# radix-10 register passes (n = 10, 20, 50, 100, 200: the reference's ctest sizes 10, 10^2,
# 10^3, 100^3 and its 100^3 default mesh), including partial last tiles (ncols not a multiple
# of the tile) and mixes with the LDS mixed-radix and power-of-two passes
RADIX10 = [(10, 10, 10), (100, 100, 100), (20, 50, 200), (200, 20, 10), (50, 100, 20), (10, 1, 1), (20, 1, 1),
           (1, 50, 1), (1, 1, 200), (100, 7, 3), (13, 100, 1), (100, 64, 9), (3, 5, 100)]


@pytest.mark.parametrize("n", RADIX10, ids=lambda n: "x".join(map(str, n)))
def test_radix10_vs_oracle(cp, oracle, n):
    N = int(np.prod(n))
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(N, 10)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        assert _rel(plan.apply(_dev(b)), ref) < TOL, plan.passes()
        t = _dev(b)
        plan.apply(t, out=t)  # in place
        assert _rel(t, ref) < TOL


@pytest.mark.parametrize("n", [(32, 32, 32), (64, 32, 16), (20, 30, 40), (128, 1, 1), (100, 20, 50), (10, 200, 7)])
def test_forward_backward_vs_oracle(cp, oracle, n):
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 3)
    with cp.CirculantPlan(n) as plan:
        f = plan.forward(_dev(b))
        assert _rel(f, oracle.c_fft3d(b, n, -1)) < 1e-13
        g = plan.backward(_dev(b))
        assert _rel(g, oracle.c_fft3d(b, n, +1)) < 1e-13


def test_alias_in_place(cp, oracle):
    n = (64, 64, 64)
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(int(np.prod(n)), 9)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        t = _dev(b)
        plan.apply(t, out=t)  # PetscFft3DTransportSolver(ctx, Un, Un)
        assert _rel(t, ref) < TOL


def test_b_not_modified(cp, oracle):
    n = (64, 32, 128)
    b = oracle.c_fill_uniform(int(np.prod(n)), 4)
    tb = _dev(b)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol((0.6, 0.15, 0.02))
        plan.apply(tb)
    np.testing.assert_array_equal(tb.cpu().numpy(), b)


def test_separable_symbol_custom_columns(cp, oracle):
    # arbitrary 1-D circulant columns -> separable symbol (build_diag_mat_vec_3D with any c_hat)
    n = (32, 16, 8)
    rng = np.random.default_rng(5)
    cols = [rng.standard_normal(k) * 0.1 for k in n]
    hats = [np.fft.fft(c) for c in cols]
    lam = (1.0, 0.5, 2.0)
    d = oracle.c_build_diag_3d(*hats, n, lam)
    b = oracle.c_fill_uniform(int(np.prod(n)), 8)
    ref = oracle.c_solve_3d(d, b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_separable_symbol(*hats, lam)
        assert _rel(plan.apply(_dev(b)), ref) < TOL
        assert _rel(plan.get_diag(), d) < 1e-14


@pytest.mark.parametrize("n", [(32, 16, 8), (10, 20, 7), (256, 4, 2)], ids=lambda n: "x".join(map(str, n)))
def test_zero_divisor_rule(cp, oracle, n):
    """A singular symbol (PETSc's VecPointwiseDivide: a zero divisor gives 0): the explicit-Diag
    pass, the separable pass (a symbol that vanishes at k = 0) and the standalone divide all
    drop the null frequencies, as the oracle does."""
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 12)
    d = oracle.c_build_diag_transport(n, (0.6, 0.15, 0.02))
    d[[0, 3, N - 1]] = 0
    ref = oracle.c_solve_3d(d, b, n)
    assert np.all(np.isfinite(ref))
    with cp.CirculantPlan(n) as plan:
        plan.set_diag(_dev(d))
        x = plan.apply(_dev(b))
        assert bool(torch.isfinite(x).all()) and _rel(x, ref) < TOL
    # separable: c_x_hat = 1 - exp(-2 pi i k / n) with lam_x = -1/(1 - e^0) ... use a column whose
    # DFT is -1 at k = 0 so that Diag[0] = 1 + (-1) + 0 + 0 = 0 exactly
    hats = [np.fft.fft(oracle.np_transport_col(k)) for k in n]
    hats[0] = hats[0].copy()
    hats[0][0] = -1.0
    lam = (1.0, 0.5, 0.25)
    ds = oracle.c_build_diag_3d(*hats, n, lam)
    assert ds[0] == 0
    ref = oracle.c_solve_3d(ds, b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_separable_symbol(*hats, lam)
        x = plan.apply(_dev(b))
        assert bool(torch.isfinite(x).all()) and _rel(x, ref) < TOL
    y = torch.randn(100, dtype=torch.complex128, device="cuda") + 2
    y[[4, 50]] = 0
    xx = torch.randn(100, dtype=torch.complex128, device="cuda")
    w = torch.empty_like(xx)
    cp.pointwise_divide(w, xx, y)
    expect = torch.where(y != 0, xx / torch.where(y != 0, y, torch.ones_like(y)), torch.zeros_like(xx))
    assert _rel(w, expect) < 1e-15


def test_build_diag_kernel(cp, oracle):
    n = (12, 10, 6)
    lam = (0.6, 0.15 + 0.1j, 0.02)
    hats = [np.fft.fft(oracle.np_transport_col(k)) for k in n]
    d = torch.empty(int(np.prod(n)), dtype=torch.complex128, device="cuda")
    cp.build_diag_3d(d, *[_dev(h) for h in hats], n, lam)
    assert _rel(d, oracle.c_build_diag_3d(*hats, n, lam)) < 1e-15


def test_vector_kernels(cp):
    x = torch.randn(1000, dtype=torch.complex128, device="cuda")
    y = torch.randn(1000, dtype=torch.complex128, device="cuda") + 2
    w = torch.empty_like(x)
    cp.pointwise_divide(w, x, y)
    assert _rel(w, x / y) < 1e-15
    z = x.clone()
    cp.scale(z, 0.25 - 0.5j)
    assert _rel(z, x * (0.25 - 0.5j)) < 1e-15


def test_fill_uniform_matches_oracle(cp, oracle):
    t = torch.empty(12345, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(t, 42, offset=777)
    np.testing.assert_array_equal(t.cpu().numpy(), oracle.c_fill_uniform(12345, 42, 777))


def test_host_apply(cp, oracle):
    n = (32, 16, 24)
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(int(np.prod(n)), 1)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        x = plan.apply_host(b)
    assert oracle.rel_l2(x, oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)) < TOL


@pytest.mark.parametrize("n", [(256, 256, 256), (512, 512, 512)])
def test_full_size_residual(cp, n):
    """Size-independent property at the bench sizes: ||C x - b|| / ||b|| and round trip."""
    N = int(np.prod(n))
    lam = (0.6, 0.15, 0.02)
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 20251017)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        x = plan.apply(b)
        r = apply_C_torch(x, n, lam) - b
        assert float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b)) < 1e-12
        del r
        f = plan.forward(b)
        plan.backward(f, out=f)
        f /= N
        assert float(torch.linalg.vector_norm(f - b) / torch.linalg.vector_norm(b)) < 1e-13
        assert all(p["fast"] for p in plan.passes())


def test_three_pass_512(cp):
    """The 3-sweep schedule at 512^3 (r04: N1 = 32 x N2 = 16, P2 on 32 columns in XCD order):
    residual of C x = b, in place, and against the 5-pass schedule."""
    n = (512, 512, 512)
    N = 512 ** 3
    lam = (0.3 + 0.2j, 1.1, 0.7 - 0.4j)
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 512)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("three")
        assert [p["mode"] for p in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
        x = plan.apply(b)
        r = apply_C_torch(x, n, lam) - b
        assert float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b)) < 1e-12
        del r
        plan.set_schedule("five")
        x5 = plan.apply(b)
        assert float((x5 - x).abs().max() / x5.abs().max()) < 1e-13
        del x5
        for mid in ("lane64", "blocked", "blocked32", "rowsalt"):  # LDS phase A; blocks of 2 / 8 x; other row sync
            plan.set_schedule("three").set_three_pass_shape(0, mid)
            assert float((plan.apply(b) - x).abs().max() / x.abs().max()) < 1e-13
        plan.set_three_pass_shape(0, "default").set_schedule("three")
        plan.apply(b, out=b)  # in place
        assert torch.equal(b, x)


def test_max_size_1024_cubed(cp):
    """The largest fast-path grid, 1024^3 (2^30 points, 16 GiB per vector): residual of C x = b
    with in-place device arithmetic (peak ~4 vectors of HBM)."""
    n = (1024, 1024, 1024)
    N = 1024 ** 3
    lam = (0.6, 0.15, 0.02)
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 20251017)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        assert all(p["fast"] for p in plan.passes())
        x = plan.apply(b)
    u = x.view(1024, 1024, 1024)
    y = x.clone().view(1024, 1024, 1024)
    y.mul_(1 + sum(lam))
    for l, dim in ((lam[0], 2), (lam[1], 1), (lam[2], 0)):
        y.sub_(torch.roll(u, shifts=1, dims=dim), alpha=l)
    y = y.view(-1)
    y.sub_(b)
    rel = float(torch.linalg.vector_norm(y) / torch.linalg.vector_norm(b))
    del x, u, y, b
    torch.cuda.empty_cache()
    assert rel < 1e-12


LONG = [(8192, 1, 1), (10000, 1, 1), (4097, 1, 1), (4100, 3, 1), (6, 5000, 2), (3, 2, 4608), (65536, 1, 1),
        (5000, 4, 6)]


@pytest.mark.parametrize("n", LONG, ids=lambda n: "x".join(map(str, n)))
def test_long_axes_vs_oracle(cp, oracle, n):
    """Axes above 4096 (four-step split n = n1 n2): 1-D (the standalone divide) and mixed grids
    (the short axis carries the fused pass), in place and out of place."""
    N = int(np.prod(n))
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(N, 4)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL, plan.passes()
        t = _dev(b)
        plan.apply(t, out=t)
        assert _rel(t, ref) < TOL


def test_long_axes_2d_residual(cp):
    """8192 x 8192 (both axes long: 9 sweeps with the standalone divide), ||C x - b|| / ||b||."""
    n = (8192, 8192, 1)
    N = 8192 * 8192
    lam = (0.6, 0.15, 0.0)
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 11)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        modes = [p["mode"] for p in plan.passes()]
        assert "sym_divide" in modes and len(modes) == 9
        x = plan.apply(b)
    r = apply_C_torch(x, n, lam) - b
    assert float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b)) < 1e-12


def test_long_axes_limits(cp):
    with pytest.raises(cp.CirculantError):
        cp.CirculantPlan((4099, 1, 1))  # prime above 4096
    with cp.CirculantPlan((8192, 1, 1)) as plan:
        with pytest.raises(cp.CirculantError):
            plan.forward(torch.zeros(8192, dtype=torch.complex128, device="cuda"))
        with pytest.raises(cp.CirculantError):
            plan.set_diag(torch.ones(8192, dtype=torch.complex128, device="cuda"))


def test_errors(cp):
    with pytest.raises(cp.CirculantError):
        cp.CirculantPlan((0, 4, 4))
    with pytest.raises(cp.CirculantError):
        cp.CirculantPlan((8198, 1, 1))  # 2 x 4099: no split into two factors <= 4096
    with cp.CirculantPlan((8, 8, 8)) as plan:
        b = torch.zeros(512, dtype=torch.complex128, device="cuda")
        with pytest.raises(cp.CirculantError):
            plan.apply(b)  # no symbol yet: PETSC_ERR_ARG_WRONGSTATE


@pytest.mark.parametrize("n,chunk", [((64, 32, 48), 16), ((64, 32, 48), 20), ((32, 32, 32), 1), ((20, 12, 9), 4),
                                     ((128, 128, 128), 32)])
def test_chunked_schedule_vs_oracle(cp, oracle, n, chunk):
    lam = (0.6, 0.15, 0.02 + 0.01j)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 31)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_chunking(chunk)
        nch = -(-n[2] // chunk)
        assert len(plan.passes()) == 4 * nch + 1
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t = _dev(b)
        plan.apply(t, out=t)
        assert _rel(t, ref) < TOL


# ------------------------------------------------------------------ 3-sweep schedule (256^3)
@pytest.mark.parametrize("lam", [(0.6, 0.15, 0.02), (55.6, 0.0, 0.0), (0.3 + 0.2j, 1.1, 0.7 - 0.4j)],
                         ids=["bench", "transport", "complex"])
def test_three_pass_vs_oracle(cp, oracle, lam):
    n = (256, 256, 256)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 97)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("three")
        modes = [p["mode"] for p in plan.passes()]
        assert modes == ["rows_fwd", "mid_fused", "rows_inv"]
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t = _dev(b)
        plan.apply(t, out=t)  # in place (b == x), as KSPSolve(ksp, Un, Un) hands it
        assert torch.equal(t, x)
        plan.set_schedule("five")
        assert len(plan.passes()) == 5
        x5 = plan.apply(_dev(b))
        assert _rel(x5, x) < 1e-13


def test_three_pass_schedule_rules(cp):
    n = (256, 256, 256)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert len(plan.passes()) == 3  # default (AUTO) at 256^3: the 3-sweep schedule
        plan.set_schedule("five")
        assert len(plan.passes()) == 5
        plan.set_schedule("auto").set_chunking(32)
        assert len(plan.passes()) == 4 * 8 + 1  # chunking asked for: the chunked 5-pass schedule
        plan.set_chunking(0).set_schedule("three")
        assert len(plan.passes()) == 3
        d = torch.ones(256 ** 3, dtype=torch.complex128, device="cuda") * 2.0
        b = torch.ones_like(d)
        x = plan.apply_with_diag(d, b)  # explicit Diag: the 5-pass fused-Diag path serves it
        assert torch.allclose(x, b / 2.0)
        for n1, mid in ((16, 0), (32, 9), (32, 8), (64, 5), (-1, 0), (0, -1), (0, 9)):  # only built shapes; nothing from the environment
            with pytest.raises(cp.CirculantError):
                plan.set_three_pass_shape(n1, mid)
    with cp.CirculantPlan((64, 64, 64)) as plan:
        with pytest.raises(cp.CirculantError):
            plan.set_schedule("three")
        plan.set_transport_symbol((0.5, 0.5, 0.5)).set_schedule("five")
        assert len(plan.passes()) == 5


@pytest.mark.parametrize("n1,mid", [(0, "default"), (0, "lane64"), (0, "swap64"), (32, "default"), (16, "lane32"),
                                    (16, "lane64"), (16, "swap64"), (0, "rowsalt")])
@pytest.mark.parametrize("lam", [(0.6, 0.15, 0.02), (0.3 + 0.2j, 1.1, 0.7 - 0.4j)], ids=["bench", "complex"])
def test_three_pass_128_vs_oracle(cp, oracle, lam, n1, mid):
    """The 3-sweep schedule at 128^3 (N1 = 32 x N2 = 4; AUTO there): the default kernels (8
    points per thread, whole-complex exchanges) and the round-2 ones (lane64): against the
    oracle, in place, and against the 5-pass schedule."""
    n = (128, 128, 128)
    b = oracle.c_fill_uniform(128 ** 3, 31)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("three").set_three_pass_shape(n1, mid)
        assert [p["mode"] for p in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t = _dev(b)
        plan.apply(t, out=t)
        assert torch.equal(t, x)
        plan.set_schedule("five")
        assert _rel(plan.apply(_dev(b)), x) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("mid", ["default", "lane64", "lane32"])
def test_three_pass_100_vs_oracle(cp, oracle, mid):
    """The 3-sweep schedule at the reference's default mesh 100^3 (cfp_three_pass_sq.hip: y split
    10 x 10, radix-10 FFTs; mid = the middle kernel's x tile 4 / 2 / 5): against the oracle,
    in place, and against the 5-pass and plane schedules."""
    n = (100, 100, 100)
    lam = (0.3 + 0.2j, 1.1, 0.7 - 0.4j)
    b = oracle.c_fill_uniform(100 ** 3, 43)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("three").set_three_pass_shape(0, mid)
        assert [p["mode"] for p in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t = _dev(b)
        plan.apply(t, out=t)
        assert torch.equal(t, x)
        plan.set_schedule("five")
        assert _rel(plan.apply(_dev(b)), x) < 1e-13
        plan.set_schedule("plane")
        assert _rel(plan.apply(_dev(b)), x) < 1e-13


# ------------------------------------------------------------------ plane schedule (n_x = n_y)
@pytest.mark.parametrize("n", [(100, 100, 100), (64, 64, 64), (128, 128, 128), (100, 100, 7), (64, 64, 2),
                               (128, 128, 10), (32, 32, 32), (32, 32, 5)], ids=lambda n: "x".join(map(str, n)))
def test_plane_vs_oracle(cp, oracle, n):
    """x + y DFTs of whole z-planes | fused z | inverse planes: against the oracle (separable
    symbol and explicit Diag), in place, and against the 5-pass schedule."""
    lam = (0.3 + 0.2j, 1.1, 0.7 - 0.4j)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 41)
    diag = oracle.c_build_diag_transport(n, lam)
    ref = oracle.c_solve_3d(diag, b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("plane")
        assert [p["mode"] for p in plan.passes()] == ["plane_fwd", "fused_sep", "plane_inv"]
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t = _dev(b)
        plan.apply(t, out=t)
        assert torch.equal(t, x)
        assert _rel(plan.apply_with_diag(_dev(diag), _dev(b)), ref) < TOL
        plan.set_schedule("five")
        assert len(plan.passes()) == 5
        assert _rel(plan.apply(_dev(b)), x) < 1e-13


def test_plane_schedule_rules(cp):
    with cp.CirculantPlan((100, 100, 100)) as plan:
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert [p["mode"] for p in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]  # AUTO at 100^3 (r04)
        plan.set_chunking(10)
        assert len(plan.passes()) == 4 * 10 + 1  # chunking asked for: the chunked 5-pass schedule
        plan.set_chunking(0).set_schedule("five")
        assert len(plan.passes()) == 5
    for n in ((64, 32, 16), (256, 256, 256), (100, 100, 1), (50, 50, 50)):
        with cp.CirculantPlan(n) as plan:
            with pytest.raises(cp.CirculantError):
                plan.set_schedule("plane")
    with cp.CirculantPlan((100, 100, 7)) as plan:  # 100^2 planes, another n_z: planes
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert [p["mode"] for p in plan.passes()] == ["plane_fwd", "fused_sep", "plane_inv"]
    with cp.CirculantPlan((64, 64, 64)) as plan:  # AUTO: planes for 64^2 too
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert len(plan.passes()) == 3
    with cp.CirculantPlan((32, 32, 32)) as plan:  # ... and for 32^2 (BASELINE config 1; r06z2)
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert [p["mode"] for p in plan.passes()] == ["plane_fwd", "fused_sep", "plane_inv"]
    with cp.CirculantPlan((128, 128, 128)) as plan:  # ... but not for 128^3: 3 sweeps there (r03m)
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert [p["mode"] for p in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
    with cp.CirculantPlan((128, 128, 64)) as plan:  # 128^2 planes, another n_z: 5 passes
        plan.set_transport_symbol((0.5, 0.5, 0.5))
        assert len(plan.passes()) == 5


@pytest.fixture(scope="module")
def tp_case(oracle):
    n, lam = (256, 256, 256), (0.3 + 0.2j, 1.1, 0.7 - 0.4j)
    b = oracle.c_fill_uniform(256 ** 3, 5)
    return n, lam, b, oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)


@pytest.mark.parametrize("n1,mid", [(64, "lane64"), (64, "lane32"), (32, "lane64"), (32, "lane32"), (0, "default"),
                                    (32, "swap64"), (64, "swap64"), (32, "swap64pf"), (64, "swap64pf"),
                                    (0, "blocked"), (32, "blocked"), (0, "blocked32"), (32, "blocked32"),
                                    (0, "swap32x"), (32, "swap32x"), (0, "rowsalt")])
def test_three_pass_variants(cp, tp_case, n1, mid):
    """Both y splits (64 x 4 with a 4-lane y2 DFT, 32 x 8 with an 8-lane one) and both P2 tile
    widths, selected per plan through cfp_plan_set_three_pass_shape."""
    n, lam, b, ref = tp_case
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_schedule("three").set_three_pass_shape(n1, mid)
        x = plan.apply(_dev(b))
        assert _rel(x, ref) < TOL
        t_ = _dev(b)
        plan.apply(t_, out=t_)
        assert torch.equal(t_, x)


@pytest.mark.parametrize("mid", ["default", "blocked", "blocked32"])
def test_three_pass_8_byte_aligned(cp, tp_case, mid):
    """The 3-sweep apply on buffers that are 8- but not 16-byte aligned (the LDS-DMA prefetch of
    the middle kernel needs 16-byte addresses; such buffers run it without the prefetch)."""
    n, lam, b, ref = tp_case
    N = 256 ** 3
    raw = torch.empty(2 * N + 1, dtype=torch.float64, device="cuda")  # raw[1:] starts 8 bytes past a 16-byte boundary
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam).set_three_pass_shape(0, mid)
        bd = _dev(b)
        x = plan.apply(bd)
        assert _rel(x, ref) < TOL
        # drive the ABI directly with an 8-byte offset into a float64 buffer holding b
        raw[1:].copy_(torch.view_as_real(bd).reshape(-1))
        ptr = raw.data_ptr() + 8
        from circulantpreconditioner_amd._lib import check, lib
        check(lib().cfp_plan_apply(plan._h, ptr, ptr, None))
        torch.cuda.synchronize()
        got = torch.view_as_complex(raw[1:].clone().reshape(-1, 2))
        assert torch.equal(got, x)


def _random_grids(count=48, seed=2025, max_points=1 << 21):
    menu = [1, 2, 3, 4, 5, 7, 8, 10, 11, 12, 13, 16, 20, 24, 25, 27, 30, 31, 32, 36, 40, 49, 50, 60, 64, 81, 96,
            97, 100, 125, 128, 200, 243, 256, 300, 512]
    rng = np.random.default_rng(seed)
    grids = []
    while len(grids) < count:
        n = tuple(int(v) for v in rng.choice(menu, 3))
        if int(np.prod(n)) <= max_points and n not in grids:
            grids.append(n)
    return grids


@pytest.mark.parametrize("n", _random_grids(), ids=lambda n: "x".join(map(str, n)))
def test_random_grids_vs_oracle(cp, oracle, n):
    """Seeded sweep over the kernel dispatch table: power-of-two, radix-10, mixed-radix and prime
    sides in every axis position, each grid with its own complex lambda."""
    N = int(np.prod(n))
    rng = np.random.default_rng(sum(n) * 7919 + n[0])
    lam = tuple(complex(rng.uniform(0.01, 2.0), rng.uniform(-0.5, 0.5)) for _ in range(3))
    b = oracle.c_fill_uniform(N, 1000 + sum(n))
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        assert _rel(plan.apply(_dev(b)), ref) < TOL, plan.passes()


@pytest.mark.parametrize("n", [(64, 32, 48), (256, 256, 256), (20, 12, 9), (32, 1, 16)])
def test_y_fused_schedule_vs_oracle(cp, oracle, n):
    lam = (0.6, 0.15 + 0.05j, 0.02)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 41)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        plan.set_schedule("five_y")  # after the symbol: the tables are rebuilt for y
        ps = plan.passes()
        if n[1] > 1 and n[2] > 1:
            assert [p["axis"] for p in ps] == ["x", "z", "y", "z", "x"]
        assert _rel(plan.apply(_dev(b)), ref) < TOL
    with cp.CirculantPlan(n) as plan:
        plan.set_schedule("five_y").set_transport_symbol(lam)  # before the symbol
        assert _rel(plan.apply(_dev(b)), ref) < TOL


def test_profile_mode_records_the_callers_applies(cp, oracle):
    """cfp_plan_profile_begin/_end: one event per launch inside ordinary applies (bench.py's
    timed-region kernel times); results unchanged, counts and times sane, capacity respected."""
    n = (64, 32, 16)
    N = int(np.prod(n))
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(N, 3)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        tb, x = _dev(b), torch.empty(N, dtype=torch.complex128, device="cuda")
        plan.profile_begin(3)
        for _ in range(5):  # two more than the capacity: they run unrecorded
            plan.apply(tb, out=x)
        ms, napp = plan.profile_end()
        assert napp == 3 and len(ms) == len(plan.passes())
        plan.profile_begin(100, every=4)  # sampling: applies 0, 4, 8 of 10
        for _ in range(10):
            plan.apply(tb, out=x)
        ms4, napp4 = plan.profile_end()
        assert napp4 == 3 and all(m > 0 for m in ms4)
        assert all(0.0 < m < 100.0 for m in ms)
        assert _rel(x, ref) < TOL
        with pytest.raises(Exception):
            plan.profile_end()  # not started


def test_profile_mode_stamps_the_three_sweep_dispatches(cp):
    """At 256^3 the profile mode stamps each 3-sweep kernel's own dispatch
    (hipExtLaunchKernelGGL start / stop events, r03z): three positive times whose sum matches the
    apply's own duration (kernels back to back), where separate event packets added ~5 us each."""
    g = (256, 256, 256)
    N = g[0] * g[1] * g[2]
    b = torch.empty(N, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 7)
    x = torch.empty_like(b)
    with cp.CirculantPlan(g) as plan:
        plan.set_transport_symbol((0.6, 0.15, 0.02))
        assert [q["mode"] for q in plan.passes()] == ["rows_fwd", "mid_fused", "rows_inv"]
        for _ in range(20):
            plan.apply(b, out=x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(40):
            plan.apply(b, out=x)
        e1.record()
        torch.cuda.synchronize()
        apply_ms = e0.elapsed_time(e1) / 40
        plan.profile_begin(20, every=2)
        for _ in range(40):
            plan.apply(b, out=x)
        ms, napp = plan.profile_end()
    assert napp == 20 and len(ms) == 3 and all(m > 0 for m in ms)
    assert 0.85 < sum(ms) / apply_ms < 1.05, (ms, apply_ms)


# ------------------------------------------------------------------ HIP-graph replay
@pytest.mark.parametrize("n", [(32, 32, 32), (100, 100, 100), (64, 32, 16), (256, 256, 256)])
def test_graph_replay_vs_oracle(cp, oracle, n):
    """cfp_plan_set_graph: replayed applies equal the eager apply bit for bit, follow a new
    symbol, a new schedule and an in-place pair, and match the oracle."""
    lam = (0.6, 0.15, 0.02)
    lam2 = (1.3 - 0.2j, 0.4, 2.0)
    N = int(np.prod(n))
    b_h = oracle.c_fill_uniform(N, 77)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b_h, n)
    ref2 = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam2), b_h, n)
    b = _dev(b_h)
    with cp.CirculantPlan(n) as plan:
        plan.set_transport_symbol(lam)
        eager = plan.apply(b)
        plan.set_graph(True)
        x = torch.empty_like(b)
        for _ in range(3):  # miss (eager + capture), then two replays
            x.zero_()
            plan.apply(b, out=x)
            torch.cuda.synchronize()
            assert torch.equal(x, eager)
        assert _rel(x, ref) < TOL
        plan.set_transport_symbol(lam2)  # moves the symbol buffers: the graphs are dropped
        for _ in range(2):
            plan.apply(b, out=x)
        assert _rel(x, ref2) < TOL
        plan.set_schedule("five")
        for _ in range(2):
            plan.apply(b, out=x)
        assert _rel(x, ref2) < TOL
        t = b.clone()
        for _ in range(2):  # in place: each replay solves against the previous result
            t.copy_(b)
            plan.apply(t, out=t)
        assert _rel(t, ref2) < TOL
        plan.set_graph(False)
        assert torch.equal(plan.apply(b), x)
