"""Row f1: transport operator, KSPGMRES and the GMRES time loop with the
circulant FFT PCSHELL.  CPU tests use host Vecs (the stand-in runs every Vec/Mat op on the
host for them); GPU tests run the same solves on HIP Vecs with the HIP SpMV/BLAS and the
HIP preconditioner.

Oracles: oracle/transport.py (operator restated as the reference's cell/face loop, PETSc
GMRES restated, the PCSHELL apply via numpy FFT) and scipy's sparse direct solve."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from circulantpreconditioner_amd import petsc as P
from circulantpreconditioner_amd import transport as T

from oracle import transport as OT


def _lib_csr(dims, h, dt, a, sign, shift=0.0):
    rp, col, val = T.transport_csr(dims, h, dt, a, sign, shift)
    n = int(np.prod(dims))
    return sp.csr_matrix((val, col, rp), shape=(n, n))


CSR_CASES = [
    ((5, 4, 3), (0.2, 0.25, 1 / 3), 0.7, (1.0, 0.0, 0.0)),
    ((6, 5, 7), (0.1, 0.3, 0.05), 0.013, (0.3, -1.2, 0.7)),
    ((8, 1, 1), (0.125, 1.0, 1.0), 6.9, (1.0, 0.0, 0.0)),
    ((4, 6, 1), (0.25, 1 / 6, 1.0), 0.4, (-0.5, 0.8, 0.0)),
    ((1, 1, 1), (1.0, 1.0, 1.0), 1.0, (1.0, 1.0, 1.0)),
]


@pytest.mark.parametrize("sign", ["reference", "fixed"])
@pytest.mark.parametrize("case", CSR_CASES, ids=lambda c: "x".join(map(str, c[0])))
def test_csr_matches_face_loop(case, sign):
    dims, h, dt, a = case
    A = _lib_csr(dims, h, dt, a, sign, shift=1.0)
    R = OT.divergence_matrix(dims, h, dt, a, sign, shift=1.0)
    R.sort_indices()
    # same sparsity (plus the always-stored diagonal), values to rounding of dt|F|/|C|
    assert A.has_sorted_indices
    np.testing.assert_allclose(A.toarray(), R.toarray(), rtol=0, atol=1e-13 * max(1.0, abs(R).max()))
    # off-diagonal sparsity identical; the diagonal is stored in every row
    offA = {(r, c) for r in range(A.shape[0]) for c in A.indices[A.indptr[r]:A.indptr[r + 1]] if c != r}
    offR = {(r, c) for r in range(R.shape[0]) for c in R.indices[R.indptr[r]:R.indptr[r + 1]] if c != r}
    assert offA == offR
    assert all(r in A.indices[A.indptr[r]:A.indptr[r + 1]] for r in range(A.shape[0]))


def test_fixed_sign_interior_rows_equal_golden_circulant(oracle):
    """Pin for the operator: away from the border the fixed-sign upwind operator IS the
    circulant 1 + sum_d lambda_d (I - S_d) whose symbol the golden fixtures pin."""
    dims, h, dt, a = (6, 5, 4), (1 / 6, 0.2, 0.25), 0.05, (0.7, 1.1, -0.4)
    lam = [a[d] * dt / h[d] for d in range(3)]
    A = _lib_csr(dims, h, dt, a, "fixed", shift=1.0).toarray()
    # the circulant for a_d < 0 is upwind from the other side: transpose that axis' factor
    C = oracle.np_dense_C(dims, [abs(v) for v in lam])
    nx, ny, nz = dims
    if a[2] < 0:
        from scipy.linalg import circulant
        Cz = np.kron(circulant(oracle.np_transport_col(nz)), np.eye(nx * ny))
        C = C - abs(lam[2]) * Cz + abs(lam[2]) * Cz.T
    interior = [i + nx * (j + ny * k) for k in range(1, nz - 1) for j in range(1, ny - 1) for i in range(1, nx - 1)]
    np.testing.assert_allclose(A[interior], C[interior], rtol=0, atol=1e-13)


def test_csr_errors():
    with pytest.raises(Exception):
        T.transport_csr((0, 4, 4), (1, 1, 1), 1.0, (1, 0, 0))
    with pytest.raises(Exception):
        T.transport_csr((4, 4, 4), (1, -1, 1), 1.0, (1, 0, 0))
    with pytest.raises(Exception):
        T.transport_csr((4, 4, 4), (1, 1, 1), 1.0, (1, 0, 0), sign=7)


def test_min_ratio_and_defaults():
    assert T.min_ratio_vol_surf(3, (0.1, 0.1, 0.1)) == pytest.approx(0.1 / 6, rel=1e-15)
    assert T.min_ratio_vol_surf(3, (0.1, 0.2, 0.4)) == pytest.approx(OT.min_ratio_vol_surf((0.1, 0.2, 0.4)))
    cfg = T.config(32)
    assert (cfg.nx, cfg.ny, cfg.nz) == (32, 32, 32)
    assert cfg.cfl == pytest.approx(1e3 / 3) and cfg.precision == 1e-5 and cfg.max_its == 1000
    assert list(cfg.a) == [1.0, 0.0, 0.0] and cfg.restart == 30 and cfg.tmax == 0.05


def test_initial_condition_matches_oracle():
    dims = (10, 12, 8)
    v = P.Vec.seq(int(np.prod(dims)))
    xmin, xmax = (ctypes.c_double * 3)(-0.5, -0.5, -0.5), (ctypes.c_double * 3)(0.5, 0.5, 0.5)
    P.PetscCall(P.lib().initial_conditions_shock_cartesian(*dims, xmin, xmax, v.h))
    np.testing.assert_array_equal(v.array(), OT.initial_conditions_shock(dims))


def _host_aij(A: sp.csr_matrix) -> P.Mat:
    return P.Mat.aij(A.indptr.astype(np.int64), A.indices.astype(np.int64), A.data, A.shape)


def _random_system(n, seed, shift=4.0):
    rng = np.random.default_rng(seed)
    A = sp.random(n, n, density=0.05, random_state=seed, dtype=np.float64)
    A = (A + 1j * sp.random(n, n, density=0.05, random_state=seed + 1)).tocsr()
    A = (A + shift * sp.identity(n, format="csr")).tocsr()
    A.sort_indices()
    b = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    return A, b


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("restart", [30, 5])
def test_ksp_gmres_host_matches_oracle(side, restart):
    n = 200
    A, b = _random_system(n, 3, shift=7.0)
    ksp = P.KSP().set_tolerances(1e-10, 1e-50, P.PETSC_DEFAULT, 500).set_restart(restart)
    ksp.set_pc_side(P.PC_LEFT if side == "left" else P.PC_RIGHT)
    ksp.get_pc().set_none()
    M = _host_aij(A)
    ksp.set_operators(M)
    bv = P.Vec.seq(n).set_array(b)
    xv = P.Vec.seq(n)
    reason = ksp.solve(bv, xv)
    xo, its_o, reason_o, rn_o, _ = OT.gmres(A, b, rtol=1e-10, maxits=500, restart=restart, side=side)
    assert reason == reason_o == 2
    assert ksp.its == its_o
    assert ksp.rnorm == pytest.approx(rn_o, rel=1e-6)
    np.testing.assert_allclose(xv.array(), xo, rtol=0, atol=1e-10 * np.abs(xo).max())
    xs = spla.spsolve(A.tocsc(), b)
    assert np.linalg.norm(xv.array() - xs) <= 1e-8 * np.linalg.norm(xs)
    ksp.destroy()


def test_ksp_b_equals_x_and_maxits():
    n = 120
    A, b = _random_system(n, 9, shift=7.0)
    M = _host_aij(A)
    ksp = P.KSP().set_tolerances(1e-12, 1e-50, P.PETSC_DEFAULT, 7)
    ksp.get_pc().set_none()
    ksp.set_operators(M)
    v = P.Vec.seq(n).set_array(b)
    reason = ksp.solve(v, v)  # KSPSolve(ksp, Un, Un) as the reference driver does
    assert reason == -3 and ksp.its == 7  # KSP_DIVERGED_ITS
    xo, its_o, reason_o, _, _ = OT.gmres(A, b, rtol=1e-12, maxits=7)
    assert its_o == 7 and reason_o == -3
    np.testing.assert_allclose(v.array(), xo, rtol=0, atol=1e-10 * np.abs(xo).max())
    # in place across restarts: b lives in x until the first update, then in the KSP's copy
    for side in ("left", "right"):
        ksp.set_tolerances(1e-10, 1e-50, P.PETSC_DEFAULT, 500).set_restart(3)
        ksp.set_pc_side(P.PC_LEFT if side == "left" else P.PC_RIGHT)
        v = P.Vec.seq(n).set_array(b)
        assert ksp.solve(v, v) == 2
        xo, its_o, reason_o, _, _ = OT.gmres(A, b, rtol=1e-10, maxits=500, restart=3, side=side)
        assert ksp.its == its_o and reason_o == 2
        np.testing.assert_allclose(v.array(), xo, rtol=0, atol=1e-9 * np.abs(xo).max())
    # b = 0: converged before any update, x = 0 whatever it held
    v = P.Vec.seq(n).set_array(np.zeros(n, dtype=complex))
    ksp.set_tolerances(1e-10, 1e-50, P.PETSC_DEFAULT, 500)
    xz = P.Vec.seq(n).set_array(np.ones(n, dtype=complex))
    ksp.solve(v, xz)
    assert ksp.its == 0 and np.array_equal(xz.array(), np.zeros(n))


def test_ksp_errors():
    ksp = P.KSP()
    with pytest.raises(P.PetscError):
        ksp.set_type("cg")
    with pytest.raises(P.PetscError):
        ksp.set_restart(0)
    v = P.Vec.seq(4)
    with pytest.raises(P.PetscError) as e:
        ksp.solve(v, P.Vec.seq(4))
    assert e.value.code == 73  # no operators: PETSC_ERR_ARG_WRONGSTATE


def _driver_reference(dims, sign, pc_lam=None, steps=1, rtol=1e-5, h=None):
    """The time loop restated: U <- GMRES((I + dt A), U) steps times (oracle GMRES)."""
    n = int(np.prod(dims))
    hh = h or [1.0 / d for d in dims]
    dt = (1e3 / 3) * OT.min_ratio_vol_surf(hh) / 1.0
    A = OT.divergence_matrix(dims, hh, dt, (1.0, 0.0, 0.0), sign, shift=1.0)
    U = OT.initial_conditions_shock(dims)
    M = OT.fft_preconditioner(dims, pc_lam) if pc_lam is not None else None
    its = []
    for _ in range(steps):
        U, k, reason, _, _ = OT.gmres(A, U, M=M, rtol=rtol, abstol=rtol, maxits=1000)
        its.append(k)
    return U, its, dt, A


@pytest.mark.parametrize("sign", ["reference", "fixed"])
def test_driver_pcnone_host_matches_oracle(sign):
    dims = (12, 10, 6)
    cfg = T.config(dims, pc="none", sign=sign, device=False, steps=2)
    res, U = T.run(cfg, return_field=True)
    Uo, its, dt, A = _driver_reference(dims, sign, steps=2)
    assert res["steps"] == 2 and res["dt"] == pytest.approx(dt, rel=1e-15)
    assert res["all_converged"] == 1
    assert res["max_step_its"] == max(its) and res["min_step_its"] == min(its)
    np.testing.assert_allclose(U, Uo, rtol=0, atol=1e-8 * np.abs(Uo).max())


def test_driver_reference_loop_takes_one_step():
    """With the reference main's cfl = 1e3/3 and tmax = 0.05, dt = 55.6 h > tmax: one solve."""
    cfg = T.config(8, pc="none", device=False)
    res = T.run(cfg)
    assert res["steps"] == 1 and res["dt"] > 0.05


def test_driver_fft_pc_needs_device():
    with pytest.raises(P.PetscError) as e:
        T.run(T.config(8, pc="fft", device=False))
    assert e.value.code == 56


# --------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("sign", ["reference", "fixed"])
def test_driver_pcnone_device_equals_host(sign):
    dims = (16, 12, 10)
    rh, Uh = T.run(T.config(dims, pc="none", sign=sign, device=False, steps=2), return_field=True)
    rd, Ud = T.run(T.config(dims, pc="none", sign=sign, device=True, steps=2), return_field=True)
    assert rd["total_its"] == rh["total_its"]
    np.testing.assert_allclose(Ud, Uh, rtol=0, atol=1e-9 * np.abs(Uh).max())


@pytest.mark.gpu
@pytest.mark.parametrize("sign", ["reference", "fixed"])
@pytest.mark.parametrize("lam", ["matched", "reference"])
def test_driver_fft_pc_matches_oracle(sign, lam):
    """Config 1 (32^3): GMRES + FFT PCSHELL against the oracle GMRES with the numpy FFT
    preconditioner.  Short solves (fixed sign, matched lambda: 2 iterations) must agree in
    iteration count and to 1e-8; the long ones (hundreds of iterations over restarts, where
    rounding may move the stopping iteration) to one iteration in a hundred and 1e-6."""
    dims = (32, 32, 32)
    steps = 2 if (sign, lam) == ("fixed", "matched") else 1
    res, U = T.run(T.config(dims, pc="fft", sign=sign, lam=lam, device=True, steps=steps), return_field=True)
    h = 1.0 / 32
    dt = res["dt"]
    lam_v = [dt / h, 0.0, 0.0] if lam == "matched" else [dt * h, 0.0, 0.0]
    assert res["lambda"] == pytest.approx(lam_v, rel=1e-14)
    Uo, its, _, A = _driver_reference(dims, sign, pc_lam=lam_v, steps=steps)
    assert res["all_converged"] == 1
    assert res["pc_calls"] >= res["total_its"]
    if max(its) <= 30:
        assert res["total_its"] == sum(its)
        np.testing.assert_allclose(U, Uo, rtol=0, atol=1e-8 * np.abs(Uo).max())
    else:
        # long solves: two rtol=1e-5 iterates of an ill-conditioned preconditioned system may
        # differ by more than rounding; both must be as close to the exact step as each other
        assert abs(res["total_its"] - sum(its)) <= max(1, sum(its) // 100)
        Us = spla.spsolve(A.tocsc(), OT.initial_conditions_shock(dims))
        err, err_o = np.linalg.norm(U - Us), np.linalg.norm(Uo - Us)
        assert err <= 10 * err_o + 1e-10 * np.linalg.norm(Us)


@pytest.mark.gpu
@pytest.mark.parametrize("sign", ["reference", "fixed"])
@pytest.mark.parametrize("case", CSR_CASES + [((64, 48, 40), (1 / 64, 1 / 48, 1 / 40), 0.02, (0.3, -0.5, 0.7))],
                         ids=lambda c: "x".join(map(str, c[0])))
def test_aij_row_class_spmv(case, sign):
    """the stand-in AIJ stores a Cartesian stencil in row-class diagonal form
    (one class byte per row, a table of the distinct rows) and its device MatMult equals scipy's
    CSR product; MatShift rebuilds it.  A general sparse matrix keeps the CSR kernels."""
    dims, h, dt, a = case
    A = _lib_csr(dims, h, dt, a, sign, shift=1.0)
    n = A.shape[0]
    M = _host_aij(A)
    rng = np.random.default_rng(7)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    xv, yv = P.Vec.seq_hip(n).set_array(x), P.Vec.seq_hip(n)
    M.mult(xv, yv)
    assert M.aij_format() == "dia"
    ref = A @ x
    assert np.linalg.norm(yv.array() - ref) <= 1e-14 * np.linalg.norm(ref)
    M.shift(0.5 - 0.25j)
    assert M.aij_format() == "none"
    M.mult(xv, yv)
    assert M.aij_format() == "dia"
    ref = ref + (0.5 - 0.25j) * x
    assert np.linalg.norm(yv.array() - ref) <= 1e-14 * np.linalg.norm(ref)
    R = _random_system(200, 3)[0]
    MR = _host_aij(R)
    xr = rng.standard_normal(200) + 0j
    xrv, yrv = P.Vec.seq_hip(200).set_array(xr), P.Vec.seq_hip(200)
    MR.mult(xrv, yrv)
    assert MR.aij_format() == "csr"
    assert np.linalg.norm(yrv.array() - R @ xr) <= 1e-13 * np.linalg.norm(R @ xr)


@pytest.mark.gpu
def test_fft_pc_cuts_iterations():
    """The point of row f1: at the reference's cfl = 1e3/3 the fixed-sign upwind step does not
    converge in 1000 unpreconditioned GMRES iterations at 32^3, and converges in a handful
    with the circulant preconditioner."""
    r_none = T.run(T.config(32, pc="none", sign="fixed", device=True))
    r_fft = T.run(T.config(32, pc="fft", sign="fixed", device=True))
    assert r_fft["all_converged"] == 1 and r_fft["total_its"] <= 5
    assert r_none["all_converged"] == 0 or r_none["total_its"] >= 20 * r_fft["total_its"]


@pytest.mark.gpu
def test_ksp_device_pcshell_random_rhs():
    """KSP through the Python mirror: the transport operator + PCSHELL on HIP Vecs, a random
    right-hand side, solution checked against scipy's direct solve."""
    dims = (16, 16, 16)
    n = 16 ** 3
    h = [1 / 16] * 3
    dt = 0.3
    A = _lib_csr(dims, h, dt, (1.0, 0.5, 0.25), "fixed", shift=1.0)
    M = _host_aij(A)
    ksp = P.KSP().set_tolerances(1e-10, 1e-50, P.PETSC_DEFAULT, 200)
    lam = [dt / h[0] * 1.0, dt / h[1] * 0.5, dt / h[2] * 0.25]
    ctx = P.make_context(dims, lam)
    ksp.get_pc().set_shell(ctx)
    ksp.set_operators(M)
    rng = np.random.default_rng(5)
    b = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    bv = P.Vec.seq_hip(n).set_array(b)
    xv = P.Vec.seq_hip(n)
    assert ksp.solve(bv, xv) == 2
    xs = spla.spsolve(A.tocsc(), b)
    assert np.linalg.norm(xv.array() - xs) <= 1e-8 * np.linalg.norm(xs)
    xo, its_o, _, _, _ = OT.gmres(A, b, M=OT.fft_preconditioner(dims, lam), rtol=1e-10, maxits=200)
    assert ksp.its == its_o
    ksp.destroy()


@pytest.mark.gpu
def test_config3_256_converges_and_solves():
    """Config 3 (256^3 PCApply inside GMRES, the reference's caller
    tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:120-136, rtol = abstol = 1e-5) at full
    size against the oracle GMRES with the numpy FFT preconditioner on the same operator (the
    library's CSR, pinned to the face loop by test_csr_matches_face_loop): the same iteration
    count, and the iterate to 1e-8, as config 1 at 32^3.  The true residual is checked too."""
    dims = (256, 256, 256)
    res, U = T.run(T.config(256, pc="fft", sign="fixed", device=True), return_field=True)
    assert res["all_converged"] == 1 and res["steps"] == 1
    h = [1 / 256] * 3
    A = _lib_csr(dims, h, res["dt"], (1.0, 0.0, 0.0), "fixed", shift=1.0)
    U0 = OT.initial_conditions_shock(dims)
    lam = [res["dt"] / h[0], 0.0, 0.0]
    Uo, its, reason, _, _ = OT.gmres(A, U0, M=OT.fft_preconditioner(dims, lam), rtol=1e-5, abstol=1e-5, maxits=1000)
    assert reason in (2, 3)
    assert res["total_its"] == its
    assert np.linalg.norm(U - Uo) <= 1e-8 * np.linalg.norm(Uo)
    r = A @ U - U0
    assert np.linalg.norm(r) <= 1e-3 * np.linalg.norm(U0)
