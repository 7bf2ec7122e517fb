"""The Krylov step fused into the apply (r06): cfp_plan_apply_ex and the
PCSHELL's applyBA inside the stand-in GMRES (config 3, 256^3 transport).

- Plan level: x = apply(A b) with A the transport operator in row-class diagonal form, and the
  Gram-Schmidt dots v_j^H x, against the same three steps done separately (scipy SpMV on the
  host, the plain apply, torch dots).  The 256^3 3-sweep schedule fuses them (P1 forms A b from the
  rows it loads, P3 reads the v_j beside its stores); other grids and stencils that leave the
  x-line run them as separate kernels -- both must give the same numbers.
- Solver level: config 3's GMRES step with the fused applyBA against the same step with
  MatMult + PCApply (fuse = 0): same iteration count, same iterate to rounding.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import circulantpreconditioner_amd as cp
from circulantpreconditioner_amd import transport as T
from circulantpreconditioner_amd.plan import row_class_form

pytestmark = pytest.mark.gpu


def _operator(dims, a, sign, dt):
    h = [1.0 / d for d in dims]
    rp, col, val = T.transport_csr(dims, h, dt, a, sign, 1.0)
    n = int(np.prod(dims))
    return sp.csr_matrix((val, col, rp), shape=(n, n))


def _stencil_dev(A, nx, dev):
    cls, mask, tab, offs, xl = row_class_form(A.indptr, A.indices, A.data, nx)
    return (torch.from_numpy(cls).to(dev), torch.from_numpy(mask).to(dev),
            torch.from_numpy(np.ascontiguousarray(tab).reshape(-1)).to(dev), [int(o) for o in offs], xl)


def _rel(a, b):
    return float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))


@pytest.mark.parametrize("n,sign,a,want_fused", [
    (256, "fixed", (1.0, 0.0, 0.0), 1),        # config 3's operator: fused
    (256, "reference", (1.0, 0.0, 0.0), 1),    # the reference's inflow sign: still x-local
    (256, "fixed", (1.0, 0.5, 0.0), 0),        # couples y-neighbours: separate kernels
    (128, "fixed", (1.0, 0.0, 0.0), 0),        # no fused kernels at 128^3: separate kernels
])
def test_apply_ex_matches_separate_steps(n, sign, a, want_fused):
    dims = (n, n, n)
    dev = torch.device("cuda", 0)
    dt = 0.2 / n
    A = _operator(dims, a, sign, dt)
    st = _stencil_dev(A, n, dev)
    assert st[4] == (a[1] == 0.0 and a[2] == 0.0)
    lam = (a[0] * dt * n, a[1] * dt * n, a[2] * dt * n)
    plan = cp.CirculantPlan(dims, device=0).set_transport_symbol(lam)
    N = n ** 3
    b = torch.empty(N, dtype=torch.complex128, device=dev)
    cp.fill_uniform(b, 11)
    v0 = torch.empty_like(b)
    cp.fill_uniform(v0, 12)
    v1 = torch.empty_like(b)
    cp.fill_uniform(v1, 13)
    x = torch.empty_like(b)
    dots, fused = plan.apply_ex(b, x, stencil=st, dots_with=(v0, v1, None))
    torch.cuda.synchronize()
    assert fused == want_fused
    y = torch.from_numpy(A @ b.cpu().numpy()).to(dev)
    xr = plan.apply(y)
    torch.cuda.synchronize()
    assert _rel(x, xr) < 1e-13
    ref = torch.stack([torch.vdot(v0, xr), torch.vdot(v1, xr), torch.vdot(xr, xr)])
    assert _rel(dots, ref) < 1e-12
    # the dots alone (no stencil), up to 4 vectors in the fused P3
    dots2, fused2 = plan.apply_ex(b, x, dots_with=(None, v1, v0, v1))
    torch.cuda.synchronize()
    assert fused2 == (1 if n == 256 else 0)
    xb = plan.apply(b)
    ref2 = torch.stack([torch.vdot(xb, xb), torch.vdot(v1, xb), torch.vdot(v0, xb), torch.vdot(v1, xb)])
    assert _rel(x, xb) < 1e-15 and _rel(dots2, ref2) < 1e-12
    plan.close()


def test_apply_ex_argument_checks():
    dims = (256, 256, 256)
    dev = torch.device("cuda", 0)
    plan = cp.CirculantPlan(dims, device=0).set_transport_symbol((1.0, 0.0, 0.0))
    b = torch.zeros(256 ** 3, dtype=torch.complex128, device=dev)
    A = _operator(dims, (1.0, 0.0, 0.0), "fixed", 1e-3)
    st = _stencil_dev(A, 256, dev)
    with pytest.raises(cp.CirculantError):
        plan.apply_ex(b, b, stencil=st)  # b aliases x with a stencil
    with pytest.raises(cp.CirculantError):
        plan.apply_ex(b, torch.empty_like(b), dots_with=tuple([None] * 9))
    plan.close()


def test_config3_fused_equals_unfused():
    """Config 3 (256^3 transport, GMRES + FFT PCSHELL, fixed sign): the fused applyBA and dots
    give the iteration count and the step of MatMult + PCApply + VecMDot."""
    rf, Uf = T.run(T.config(256, pc="fft", sign="fixed", device=True, steps=2), return_field=True)
    ru, Uu = T.run(T.config(256, pc="fft", sign="fixed", device=True, steps=2, fuse=0), return_field=True)
    assert rf["all_converged"] == ru["all_converged"] == 1
    assert rf["total_its"] == ru["total_its"] and rf["pc_calls"] == ru["pc_calls"]
    assert rf["fused_dots"] == rf["total_its"] and rf["fused_norms"] == rf["steps"]
    assert ru["fused_dots"] == 0
    assert np.linalg.norm(Uf - Uu) <= 1e-11 * np.linalg.norm(Uu)


def test_config1_dots_fall_back():
    """Config 1 (32^3): no fused kernels there, the dots come from the separate kernels; the
    iterate is unchanged by the request path."""
    rf, Uf = T.run(T.config(32, pc="fft", sign="fixed", device=True, steps=2), return_field=True)
    ru, Uu = T.run(T.config(32, pc="fft", sign="fixed", device=True, steps=2, fuse=0), return_field=True)
    assert rf["total_its"] == ru["total_its"]
    assert np.linalg.norm(Uf - Uu) <= 1e-11 * np.linalg.norm(Uu)


def test_device_copy():
    """cfp_device_copy (the stand-in VecCopy's kernel): aligned sizes on the 16-byte-lane kernel,
    odd sizes and offsets through hipMemcpyAsync, zero bytes a no-op; bit-exact."""
    from circulantpreconditioner_amd._lib import check, lib
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randint(0, 256, (1 << 22,), dtype=torch.uint8, device="cuda", generator=g)
    for off, nb in ((0, 1 << 22), (0, 16 * 12345), (16, 16 * 777), (3, 1001), (0, 7), (0, 0)):
        c = torch.zeros_like(a)
        check(lib().cfp_device_copy(c.data_ptr() + off, a.data_ptr() + off, nb, None))
        torch.cuda.synchronize()
        assert torch.equal(c[off:off + nb], a[off:off + nb])
        assert int(c[:off].sum()) == 0 and int(c[off + nb:].sum()) == 0


@pytest.mark.parametrize("n", [1, 1000, 256 * 1024 + 3, 0])
def test_axpy_norm_partials_follow_the_vector_state(n):
    """VecAXPY on a device Vec leaves the |y|^2 partials of its result; VecNorm(NORM_2) sums them
    while the vector is unchanged (the time loops' VecAXPY(dU, -1, U); VecNorm(dU)), and any later
    write -- VecScale, VecSet, another AXPY, a VecHIPGetArray write, a host-side set -- is seen.
    Norms agree with numpy to 1e-12; NORM_1 / NORM_INFINITY never take the partials."""
    from circulantpreconditioner_amd import petsc as P
    rng = np.random.default_rng(7)
    a = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    b = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    y, x = P.Vec.seq_hip(n).set_array(a), P.Vec.seq_hip(n).set_array(b)

    def close(v, want):
        assert abs(v - want) <= 1e-12 * max(want, 1e-300)

    y.axpy(-0.5 + 0.25j, x)
    ref = a + (-0.5 + 0.25j) * b
    close(y.norm(), np.linalg.norm(ref))
    close(y.norm(), np.linalg.norm(ref))  # twice: still unchanged
    close(y.norm(P.NORM_1), np.abs(ref.real).sum() + np.abs(ref.imag).sum())
    close(y.norm(P.NORM_INFINITY), np.abs(ref).max(initial=0.0))
    y.scale(3.0)
    ref = 3.0 * ref
    close(y.norm(), np.linalg.norm(ref))
    y.axpy(1.0, x)
    ref = ref + b
    close(y.norm(), np.linalg.norm(ref))
    if n:
        from circulantpreconditioner_amd._lib import check, lib
        t = torch.full((n,), 2.0 + 0j, dtype=torch.complex128, device="cuda")
        with y.hip_array() as p:  # a raw device write between the AXPY and the norm
            torch.cuda.synchronize()
            check(lib().cfp_device_copy(p, t.data_ptr(), 16 * n, None))
            torch.cuda.synchronize()
        close(y.norm(), 2.0 * np.sqrt(n))
    y.axpy(1.0, x)
    y.set_array(a)  # host-side write after the AXPY
    close(y.norm(), np.linalg.norm(a))
    y.axpy(2.0, x)
    y.set(1.0)
    close(y.norm(), np.sqrt(n))
