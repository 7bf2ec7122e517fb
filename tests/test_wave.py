"""Row f2 (BASELINE config 4): wave-system operator, block-circulant
preconditioner (HIP) and the implicit GMRES loop.

Oracle: oracle/wave.py (reference assembly restated as a face loop, explicit 4x4 block symbol
and numpy block-circulant solve, pinned to the assembly by the periodic round trip below)."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from circulantpreconditioner_amd import petsc as P
from circulantpreconditioner_amd import wave as W

from oracle import transport as OT
from oracle import wave as OW


def _csr(dims, h, dt, bc, shift=0.0, c0=700.0, dim=3):
    rp, col, val = W.wave_csr(dims, h, dt, c0, bc, shift, dim=dim)
    m = (dim + 1) * int(np.prod(dims))
    return sp.csr_matrix((val, col, rp), shape=(m, m))


CASES = [((4, 3, 5), (0.25, 1 / 3, 0.2), 1e-3), ((6, 2, 1), (1 / 6, 0.5, 1.0), 2e-4), ((2, 2, 2), (0.5, 0.5, 0.5), 5e-4),
         ((1, 1, 3), (1.0, 1.0, 1 / 3), 1e-4)]


@pytest.mark.parametrize("bc", ["wall", "periodic", "neumann"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[0])))
def test_wave_csr_matches_face_loop(case, bc):
    dims, h, dt = case
    A = _csr(dims, h, dt, bc, shift=1.0)
    R = OW.wave_matrix(dims, h, dt, bc=bc, shift=1.0)
    scale = max(1.0, abs(R).max())
    np.testing.assert_allclose(A.toarray(), R.toarray(), rtol=0, atol=1e-13 * scale)
    assert A.has_sorted_indices
    m = A.shape[0]
    assert all(r in A.indices[A.indptr[r]:A.indptr[r + 1]] for r in range(m))


# 1-D and 2-D meshes: nbComp = dim + 1 unknowns per cell and faces along dim axes only
# (src/WaveSystem.cxx:111-113); the reference mains' default mesh is the 2-D 50 x 50 square
CASES_LOWDIM = [((5, 4, 1), (0.2, 0.25, 1.0), 2e-4, 2), ((6, 1, 1), (1 / 6, 1.0, 1.0), 3e-4, 2),
                ((1, 1, 1), (1.0, 1.0, 1.0), 1e-4, 2), ((7, 1, 1), (1 / 7, 1.0, 1.0), 5e-4, 1),
                ((2, 1, 1), (0.5, 1.0, 1.0), 1e-4, 1)]


@pytest.mark.parametrize("bc", ["wall", "periodic", "neumann"])
@pytest.mark.parametrize("case", CASES_LOWDIM, ids=lambda c: f"{c[3]}d-" + "x".join(map(str, c[0])))
def test_wave_csr_lowdim_matches_face_loop(case, bc):
    dims, h, dt, dim = case
    A = _csr(dims, h, dt, bc, shift=1.0, dim=dim)
    R = OW.wave_matrix(dims, h, dt, bc=bc, shift=1.0, dim=dim)
    assert A.shape == ((dim + 1) * int(np.prod(dims)),) * 2
    scale = max(1.0, abs(R).max())
    np.testing.assert_allclose(A.toarray(), R.toarray(), rtol=0, atol=1e-13 * scale)
    m = A.shape[0]
    assert all(r in A.indices[A.indptr[r]:A.indptr[r + 1]] for r in range(m))


@pytest.mark.parametrize("dim,dims,h", [(2, (5, 4), (0.2, 0.25)), (1, (9,), (1 / 9,))], ids=["2d", "1d"])
def test_block_solve_inverts_periodic_assembly_lowdim(dim, dims, h):
    dt = 4e-4
    kappa = [dt / v for v in h] + [0.0] * (3 - dim)
    A = OW.wave_matrix(dims, h, dt, bc="periodic", shift=1.0, dim=dim)
    rng = np.random.default_rng(5)
    b = rng.standard_normal(A.shape[0]) + 1j * rng.standard_normal(A.shape[0])
    x = OW.block_solve(dims, kappa, b, dim=dim)
    assert np.linalg.norm(A @ x - b) <= 1e-12 * np.linalg.norm(b)


def test_wave_csr_lowdim_errors():
    with pytest.raises(Exception):
        W.wave_csr((4, 4, 2), (0.25, 0.25, 0.5), 1e-4, dim=2)  # nz > 1 in 2-D
    with pytest.raises(Exception):
        W.wave_csr((4, 2, 1), (0.25, 0.5, 1.0), 1e-4, dim=1)  # ny > 1 in 1-D
    with pytest.raises(Exception):
        W.wave_csr((4, 1, 1), (0.25, 1.0, 1.0), 1e-4, dim=4)


def test_wave_initial_condition_2d():
    dims = (10, 8, 1)
    v = P.Vec.seq(3 * int(np.prod(dims)))
    lo, hi = (ctypes.c_double * 3)(-0.5, -0.5, -0.5), (ctypes.c_double * 3)(0.5, 0.5, 0.5)
    P.PetscCall(P.lib().initial_conditions_shock_wave(*dims, lo, hi, v.h))
    np.testing.assert_array_equal(v.array(), OW.initial_conditions_shock_wave(dims, dim=2))
    bad = P.Vec.seq(5 * int(np.prod(dims)))
    with pytest.raises(P.PetscError):
        P.PetscCall(P.lib().initial_conditions_shock_wave(*dims, lo, hi, bad.h))


def test_wave_config_reference_main_default():
    """The reference main's default: 2-D 50 x 50 square, cfl = 1e3 / 2 (impl_seq.cxx:182-212)."""
    cfg = W.config(50, dim=2)
    assert (cfg.nx, cfg.ny, cfg.nz, cfg.dim) == (50, 50, 1, 2)
    assert cfg.cfl == 500.0 and cfg.c0 == 700.0 and cfg.tmax == 0.05


def test_wave_driver_2d_pcnone_host_matches_oracle():
    dims = (12, 10, 1)
    res, U = W.run(W.config(dims, dim=2, pc="none", device=False, steps=3), return_field=True)
    dt, kappa, h = OW.dt_and_kappa(dims, dim=2)
    assert res["dt"] == pytest.approx(dt, rel=1e-15)
    assert res["kappa"] == pytest.approx(kappa, rel=1e-15)
    A = OW.wave_matrix(dims, h, dt, bc="wall", shift=1.0, dim=2)
    Uo = OW.initial_conditions_shock_wave(dims, dim=2)
    its = 0
    for _ in range(3):
        Uo, k, reason, _, _ = OT.gmres(A, Uo, rtol=1e-5, abstol=1e-5, maxits=1000)
        its += k
    assert abs(res["total_its"] - its) <= 3
    # three rtol = 1e-5 solves in a row: the two GMRES agree to the solver tolerance
    np.testing.assert_allclose(U, Uo, rtol=0, atol=1e-5 * np.abs(Uo).max())


def test_block_solve_inverts_periodic_assembly():
    """Pin: the block-circulant inverse of the oracle undoes the reference's periodic assembly."""
    dims, h = (4, 3, 5), (0.25, 1 / 3, 0.2)
    dt = 3e-4
    kappa = [dt / v for v in h]
    A = OW.wave_matrix(dims, h, dt, bc="periodic", shift=1.0)
    rng = np.random.default_rng(0)
    b = rng.standard_normal(A.shape[0]) + 1j * rng.standard_normal(A.shape[0])
    x = OW.block_solve(dims, kappa, b)
    assert np.linalg.norm(A @ x - b) <= 1e-12 * np.linalg.norm(b)


def test_arrowhead_closed_form_equals_block_symbol():
    """The kernel's closed form (cfp_fft_device.h wave_solve) against the explicit symbol."""
    dims, kappa, c0 = (5, 4, 3), (0.07, 0.03, 0.11), 700.0
    S = OW.block_symbol(dims, kappa, c0)
    nx, ny, nz = dims
    kz, ky, kx = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    th = (2 * np.pi * kx / nx, 2 * np.pi * ky / ny, 2 * np.pi * kz / nz)
    p = [kappa[d] * c0 * (1 - np.cos(th[d])) for d in range(3)]
    q = [kappa[d] * np.sin(th[d]) for d in range(3)]
    E = np.zeros_like(S)
    E[..., 0, 0] = 1 + p[0] + p[1] + p[2]
    for d in range(3):
        E[..., 0, 1 + d] = 1j * c0 * c0 * q[d]
        E[..., 1 + d, 0] = 1j * q[d]
        E[..., 1 + d, 1 + d] = 1 + p[d]
    np.testing.assert_allclose(S, E, rtol=0, atol=1e-9)


def test_wave_initial_condition():
    dims = (6, 5, 4)
    v = P.Vec.seq(4 * int(np.prod(dims)))
    lo, hi = (ctypes.c_double * 3)(-0.5, -0.5, -0.5), (ctypes.c_double * 3)(0.5, 0.5, 0.5)
    P.PetscCall(P.lib().initial_conditions_shock_wave(*dims, lo, hi, v.h))
    np.testing.assert_array_equal(v.array(), OW.initial_conditions_shock_wave(dims))


def test_wave_csr_errors():
    with pytest.raises(Exception):
        W.wave_csr((0, 2, 2), (1, 1, 1), 1.0)
    with pytest.raises(Exception):
        W.wave_csr((2, 2, 2), (1, 1, 1), 1.0, bc=9)
    with pytest.raises(Exception):
        W.wave_csr((2, 2, 2), (1, 1, 1), 1.0, c0=0.0)


def test_wave_driver_pcnone_host_matches_oracle():
    dims = (6, 5, 4)
    res, U = W.run(W.config(dims, pc="none", device=False), return_field=True)
    dt, kappa, h = OW.dt_and_kappa(dims)
    assert res["dt"] == pytest.approx(dt, rel=1e-15)
    A = _csr(dims, h, dt, "wall", shift=1.0)  # the face-loop match is test_wave_csr_matches_face_loop
    Uo = OW.initial_conditions_shock_wave(dims)
    # the reference loop: while time <= tmax (0.05), time += dt
    steps, t = 0, 0.0
    while t <= 0.05:
        t += dt
        steps += 1
    assert res["steps"] == steps
    its, conv = 0, True
    for _ in range(steps):
        Uo, k, reason, _, _ = OT.gmres(A, Uo, rtol=1e-5, abstol=1e-5, maxits=1000)
        its += k
        conv = conv and reason in (2, 3)
    # a stopping test that lands within rounding of the threshold may move by one iteration
    assert abs(res["total_its"] - its) <= steps and res["all_converged"] == int(conv)
    np.testing.assert_allclose(U, Uo, rtol=0, atol=1e-6 * np.abs(Uo).max())


def test_wave_driver_fft_needs_device():
    with pytest.raises(P.PetscError) as e:
        W.run(W.config(4, pc="fft", device=False))
    assert e.value.code == 56


# --------------------------------------------------------------------------- GPU
def _rand(m, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(m) + 1j * rng.standard_normal(m)


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(16, 16, 16), (32, 16, 8), (8, 8, 64), (64, 32, 16), (6, 5, 7), (12, 10, 3),
                                  (16, 1, 1), (8, 4, 1), (1, 1, 1), (20, 10, 50), (10, 10, 10), (100, 3, 1)],
                         ids=lambda d: "x".join(map(str, d)))
def test_wave_plan_matches_oracle(dims):
    import torch
    kappa = (0.079, 0.05, 0.11)
    m = 4 * int(np.prod(dims))
    b = _rand(m, 1)
    plan = W.WavePlan(dims).set_symbol(kappa)
    x = plan.apply(torch.from_numpy(b).cuda()).cpu().numpy()
    xo = OW.block_solve(dims, kappa, b)
    assert np.linalg.norm(x - xo) <= 1e-12 * np.linalg.norm(xo)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,dims", [(2, (16, 16)), (2, (50, 50)), (2, (12, 10)), (2, (64, 32)), (2, (128, 128)),
                                      (2, (7, 1)), (2, (1, 1)), (2, (256, 8)), (1, (16,)), (1, (50,)), (1, (7,)),
                                      (1, (1024,)), (1, (1,))],
                         ids=lambda v: str(v) if isinstance(v, int) else "x".join(map(str, v)))
def test_wave_plan_lowdim_matches_oracle(dim, dims):
    """1-D / 2-D wave systems (2 or 3 interleaved unknowns per cell) against the oracle."""
    import torch
    kappa = (0.079, 0.05, 0.0)
    m = (dim + 1) * int(np.prod(dims))
    b = _rand(m, 11)
    plan = W.WavePlan(dims, dim=dim).set_symbol(kappa)
    x = plan.apply(torch.from_numpy(b).cuda()).cpu().numpy()
    xo = OW.block_solve(dims, kappa, b, dim=dim)
    assert np.linalg.norm(x - xo) <= 1e-12 * np.linalg.norm(xo)
    t = torch.from_numpy(b).cuda()
    plan.apply(t, out=t)  # in place
    assert np.linalg.norm(t.cpu().numpy() - xo) <= 1e-12 * np.linalg.norm(xo)


@pytest.mark.gpu
def test_wave_plan_lowdim_errors():
    with pytest.raises(Exception):
        W.WavePlan((8, 8, 2), dim=2)
    with pytest.raises(Exception):
        W.WavePlan((8, 2), dim=1)
    with pytest.raises(Exception):
        W.WavePlan((8, 8), dim=0)


@pytest.mark.gpu
def test_wave_plan_aliasing_and_transforms():
    import torch
    dims = (16, 8, 32)
    m = 4 * int(np.prod(dims))
    b = _rand(m, 2)
    plan = W.WavePlan(dims).set_symbol((0.08, 0.08, 0.08))
    t = torch.from_numpy(b).cuda()
    ref = plan.apply(t)
    t2 = t.clone()
    plan.apply(t2, out=t2)
    assert torch.equal(ref, t2)
    F = plan.forward(t).cpu().numpy().reshape(dims[2], dims[1], dims[0], 4)
    Fo = np.fft.fftn(b.reshape(dims[2], dims[1], dims[0], 4), axes=(0, 1, 2))
    assert np.linalg.norm(F - Fo) <= 1e-12 * np.linalg.norm(Fo)
    Bk = plan.backward(torch.from_numpy(Fo.reshape(-1)).cuda()).cpu().numpy()
    assert np.linalg.norm(Bk / np.prod(dims) - b) <= 1e-12 * np.linalg.norm(b)


@pytest.mark.gpu
def test_wave_plan_128_inverts_periodic_operator():
    """Config 4 size, size-independent check: the periodic operator (reference assembly,
    host SpMV) applied to the HIP solve returns b."""
    import torch
    dims = (128, 128, 128)
    dt, kappa, h = OW.dt_and_kappa(dims)
    m = 4 * 128 ** 3
    b = _rand(m, 3)
    x = W.WavePlan(dims).set_symbol(kappa).apply(torch.from_numpy(b).cuda()).cpu().numpy()
    A = _csr(dims, h, dt, "periodic", shift=1.0)
    assert np.linalg.norm(A @ x - b) <= 1e-11 * np.linalg.norm(b)


@pytest.mark.gpu
@pytest.mark.parametrize("kappa", [(0.079, 0.079, 0.079), (0.31, 0.05, 0.11)], ids=["config4", "anisotropic"])
def test_wave_plan_128_three_sweep_matches_oracle(kappa):
    """The 3-sweep wave apply (cfp_wave_three.hip, AUTO at 128^3): against the oracle's block
    solve, against the 5-sweep schedule, in place; schedule rules."""
    import torch
    dims = (128, 128, 128)
    m = 4 * 128 ** 3
    b = _rand(m, 5)
    xo = OW.block_solve(dims, kappa, b)
    plan = W.WavePlan(dims).set_symbol(kappa)
    assert plan.num_passes() == 3
    bd = torch.from_numpy(b).cuda()
    x3 = plan.apply(bd)
    assert np.linalg.norm(x3.cpu().numpy() - xo) <= 1e-12 * np.linalg.norm(xo)
    t = bd.clone()
    plan.apply(t, out=t)
    assert torch.equal(t, x3)
    plan.set_schedule("five")
    assert plan.num_passes() == 5
    x5 = plan.apply(bd)
    assert float(torch.linalg.vector_norm(x5 - x3) / torch.linalg.vector_norm(x5)) < 1e-13
    plan.set_schedule("three")
    assert plan.num_passes() == 3
    small = W.WavePlan((64, 64, 64))
    assert small.set_symbol(kappa).num_passes() == 5
    with pytest.raises(Exception):
        small.set_schedule("three")
    with pytest.raises(Exception):
        W.WavePlan((128, 128), dim=2).set_schedule("three")


@pytest.mark.gpu
def test_wave_plan_errors():
    import torch
    plan = W.WavePlan((8, 8, 8))
    x = torch.zeros(4 * 512, dtype=torch.complex128, device="cuda")
    with pytest.raises(Exception):
        plan.apply(x)  # no symbol
    with pytest.raises(Exception):
        plan.set_symbol((0.1, 0.1, 0.1), c0=-1.0)
    plan.set_symbol((0.1, 0.1, 0.1))
    with pytest.raises(ValueError):
        plan.apply(torch.zeros(4 * 511, dtype=torch.complex128, device="cuda"))


@pytest.mark.gpu
def test_wave_driver_pcnone_device_equals_host():
    dims = (8, 8, 8)
    rh, Uh = W.run(W.config(dims, pc="none", device=False), return_field=True)
    rd, Ud = W.run(W.config(dims, pc="none", device=True), return_field=True)
    # the device SpMV sums a row's nonzeros in lane-strided partial sums (cfp::blas_csr_spmv),
    # the host loop in order: ten unpreconditioned rtol = 1e-5 solves in a row (c0^2 = 4.9e5
    # couples pressure and momentum) may then stop an iteration apart, and the two rounding
    # paths agree to the solver tolerance, not to rounding
    assert abs(rd["total_its"] - rh["total_its"]) <= 2, (rd["total_its"], rh["total_its"])
    np.testing.assert_allclose(Ud, Uh, rtol=0, atol=1e-5 * np.abs(Uh).max())


@pytest.mark.gpu
def test_wave_driver_fft_pc_matches_oracle():
    dims = (16, 16, 16)
    res, U = W.run(W.config(dims, pc="fft", steps=2), return_field=True)
    dt, kappa, h = OW.dt_and_kappa(dims)
    assert res["kappa"] == pytest.approx(kappa, rel=1e-14)
    A = OW.wave_matrix(dims, h, dt, bc="wall", shift=1.0)
    U0 = OW.initial_conditions_shock_wave(dims)
    M = lambda v: OW.block_solve(dims, kappa, v)  # noqa: E731
    its = []
    Uo = U0
    for _ in range(2):
        Uo, k, reason, _, _ = OT.gmres(A, Uo, M=M, rtol=1e-5, abstol=1e-5, maxits=1000)
        its.append(k)
    assert res["all_converged"] == 1
    assert abs(res["total_its"] - sum(its)) <= max(1, sum(its) // 100)
    Us = U0
    for _ in range(2):
        Us = spla.spsolve(A.tocsc(), Us)
    assert np.linalg.norm(U - Us) <= 10 * np.linalg.norm(Uo - Us) + 1e-10 * np.linalg.norm(Us)


@pytest.mark.gpu
def test_wave_fft_pc_cuts_iterations():
    r_none = W.run(W.config(32, pc="none"))
    r_fft = W.run(W.config(32, pc="fft"))
    assert r_fft["all_converged"] == 1
    assert r_none["all_converged"] == 0 or r_fft["total_its"] * 3 <= r_none["total_its"]


@pytest.mark.gpu
def test_wave_driver_2d_fft_pc_matches_oracle():
    dims = (32, 24, 1)
    res, U = W.run(W.config(dims, dim=2, pc="fft", steps=2), return_field=True)
    dt, kappa, h = OW.dt_and_kappa(dims, dim=2)
    assert res["kappa"] == pytest.approx(kappa, rel=1e-14)
    A = OW.wave_matrix(dims, h, dt, bc="wall", shift=1.0, dim=2)
    U0 = OW.initial_conditions_shock_wave(dims, dim=2)
    M = lambda v: OW.block_solve(dims, kappa, v, dim=2)  # noqa: E731
    its, Uo = [], U0
    for _ in range(2):
        Uo, k, reason, _, _ = OT.gmres(A, Uo, M=M, rtol=1e-5, abstol=1e-5, maxits=1000)
        its.append(k)
    assert res["all_converged"] == 1
    assert abs(res["total_its"] - sum(its)) <= max(1, sum(its) // 100)
    Us = U0
    for _ in range(2):
        Us = spla.spsolve(A.tocsc(), Us)
    assert np.linalg.norm(U - Us) <= 10 * np.linalg.norm(Uo - Us) + 1e-10 * np.linalg.norm(Us)


@pytest.mark.gpu
def test_wave_reference_default_2d_50x50():
    """The reference main's own case (2-D 50 x 50 square, wall boundaries, cfl 500, tmax 0.05):
    the whole time loop with PCNONE and with the block-circulant PCSHELL."""
    r_none = W.run(W.config(50, dim=2, pc="none"))
    r_fft = W.run(W.config(50, dim=2, pc="fft"))
    assert r_fft["steps"] == r_none["steps"] > 0
    assert r_fft["all_converged"] == 1
    assert r_none["all_converged"] == 0 or r_fft["total_its"] * 3 <= r_none["total_its"]


@pytest.mark.gpu
@pytest.mark.parametrize("dims,dim,bc", [((20, 16, 12), 3, "wall"), ((12, 10, 8), 3, "periodic"),
                                         ((9, 7, 5), 3, "neumann"), ((2, 2, 2), 3, "periodic"),
                                         ((50, 50), 2, "wall"), ((24, 18), 2, "periodic"), ((40,), 1, "wall")])
def test_wave_operator_block_row_class_spmv(dims, dim, bc):
    """The stand-in AIJ stores the interleaved wave operator in block row-class form (B = d + 1
    blocks on <= 16 block diagonals, one class byte per cell) and its device MatMult equals
    scipy's CSR product; MatShift rebuilds it."""
    d3 = tuple(dims) + (1,) * (3 - len(dims))
    h = [1.0 / v for v in d3]
    A = _csr(d3, h, 3e-4, bc, shift=1.0, dim=dim)
    m = A.shape[0]
    M = P.Mat.aij(A.indptr.astype(np.int64), A.indices.astype(np.int64), A.data, A.shape)
    rng = np.random.default_rng(3)
    x = rng.standard_normal(m) + 1j * rng.standard_normal(m)
    xv, yv = P.Vec.seq_hip(m).set_array(x), P.Vec.seq_hip(m)
    M.mult(xv, yv)
    # 1-D (2 unknowns, 3 cells) and a 2 x 2 x 2 periodic grid have few enough distinct diagonals
    # (<= 8) that the scalar row-class form fits and is preferred
    want = "dia" if dim == 1 or max(d3) <= 2 else "bdia"
    assert M.aij_format() == want
    ref = A @ x
    assert np.linalg.norm(yv.array() - ref) <= 1e-14 * np.linalg.norm(ref)
    M.shift(0.25 + 0.5j)
    assert M.aij_format() == "none"
    M.mult(xv, yv)
    assert M.aij_format() == want
    ref = ref + (0.25 + 0.5j) * x
    assert np.linalg.norm(yv.array() - ref) <= 1e-14 * np.linalg.norm(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("grid,want_fused", [((128, 128, 128), 1), ((32, 24, 16), 0)])
def test_wave_apply_dots_match_separate_steps(grid, want_fused):
    """cfp_wave_plan_apply_dots: x = S^{-1} b and the Gram-Schmidt dots v_j^H x.  On the 128^3
    3-sweep schedule they ride in P3w's stores; elsewhere one multi-dot sweep follows.  Either way
    the same numbers as the plain apply and torch's dots."""
    import torch
    from circulantpreconditioner_amd.plan import fill_uniform
    wp = W.WavePlan(grid).set_symbol((0.079, 0.05, 0.11))
    n = 4 * int(np.prod(grid))
    b = torch.empty(n, dtype=torch.complex128, device="cuda")
    fill_uniform(b, 11)
    vs = [torch.empty_like(b) for _ in range(3)]
    for i, v in enumerate(vs):
        fill_uniform(v, 100 + i)
    xr = wp.apply(b)
    for dots_with in ([None], [vs[0]], [vs[0], vs[1]], [vs[0], vs[1], vs[2], None]):
        x, dots, fused = wp.apply_dots(b, dots_with=dots_with)
        assert fused == want_fused
        assert float(torch.linalg.vector_norm(x - xr) / torch.linalg.vector_norm(xr)) < 1e-15
        ref = torch.stack([torch.vdot(v if v is not None else xr, xr) for v in dots_with])
        assert float(torch.linalg.vector_norm(dots - ref) / torch.linalg.vector_norm(ref)) < 1e-12
    # more than 4 vectors: the separate sweep, same numbers
    x, dots, fused = wp.apply_dots(b, dots_with=[vs[0], vs[1], vs[2], None, vs[0]])
    assert fused == 0
    ref = torch.stack([torch.vdot(v if v is not None else xr, xr) for v in [vs[0], vs[1], vs[2], xr, vs[0]]])
    assert float(torch.linalg.vector_norm(dots - ref) / torch.linalg.vector_norm(ref)) < 1e-12
    wp.close()


@pytest.mark.gpu
def test_wave_gmres_fused_dots_equal_unfused():
    """Config 4's implicit step with the Gram-Schmidt dots and the residual norm computed inside
    the block PCSHELL's 3-sweep apply, against the same loop with separate sweeps: same
    iterations, same iterate to rounding."""
    rf, Uf = W.run(W.config(128, pc="fft", steps=2, fuse=1), return_field=True)
    ru, Uu = W.run(W.config(128, pc="fft", steps=2, fuse=0), return_field=True)
    assert rf["all_converged"] == ru["all_converged"] == 1
    assert rf["total_its"] == ru["total_its"]
    assert rf["fused_dots"] == rf["total_its"] and rf["fused_norms"] == rf["steps"]
    assert ru["fused_dots"] == 0 and ru["fused_norms"] == 0
    assert np.linalg.norm(Uf - Uu) <= 1e-11 * np.linalg.norm(Uu)
