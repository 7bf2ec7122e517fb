"""The real-scalar PETSc boundary on the GPU: libcirculant_fft_real.so,
PetscScalar = double -- the reference's !PETSC_USE_COMPLEX branches of solve_3D
(src/FftLinearSolver_3D.c:6-78, 166-190) and the PCSHELL (src/PCSHELLFft_3D.cxx:10-99) on real
host and HIP Vecs, against the oracle's solve of the same real b (the correct real arithmetic,
not the reference's loop bound of 2 (size/4 + 1) entries and 2/size scale).
FFT_MAT's spectral side is FFTW's r2c half spectrum, checked against numpy's rfftn."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-10

# (nx, ny, nz): the real plan's grids (r2c rows: nx/2 a power of two >= 16; 3 sweeps at 128^3 and
# 256^3) and grids it lacks (the complex plan on the promoted b: odd nx, radix-10, tiny)
GRIDS = [(32, 16, 24), (32, 5, 7), (128, 128, 128), (10, 10, 10), (9, 4, 6), (20, 6, 4), (1, 8, 8)]


@pytest.fixture(scope="module")
def R():
    from circulantpreconditioner_amd import petsc_real as R
    R.lib()
    return R


def _half(full, nx):
    """[nz][ny][nx] complex -> the r2c half spectrum as interleaved reals"""
    return np.ascontiguousarray(full[..., : nx // 2 + 1]).view(np.float64).reshape(-1)


def _oracle_solve(oracle, dims, lam, b):
    x = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b.astype(np.complex128), dims)
    assert np.abs(x.imag).max() <= 1e-12 * np.abs(x.real).max()  # real b, real lambda: x is real
    return x.real


# the 256^3 solve on device Vecs only (host staging adds nothing the device one does not check)
@pytest.mark.parametrize("dims,hip", [(d, h) for d in GRIDS for h in (True, False)] + [((256, 256, 256), True)])
def test_real_direct_solver_in_place(R, oracle, dims, hip):
    """PetscFft3DTransportSolver(ctx, Un, Un), two time steps (FFT_MAT survives the first)."""
    nx, ny, nz = dims
    N = nx * ny * nz
    b = oracle.c_fill_uniform(N, 41).real.copy()
    a, dt, h = (1.0, 0.5, 0.25), 0.02, (1.0 / nx, 1.0 / ny, 1.0 / nz)
    F = R.mat_create_fft([nz, ny, nx])
    ctx = R.StructuredTransportContext(nx, ny, nz, a[0], a[1], a[2], dt, h[0], h[1], h[2], F)
    u = R.Vec.seq(N, hip=hip).set_array(b)
    lam = tuple(a[d] * dt / h[d] for d in range(3))
    ref = b
    for _ in range(2):
        R.PetscCall(R.lib().PetscFft3DTransportSolver(ctx, u.h, u.h))
        ref = _oracle_solve(oracle, dims, lam, ref)
        got = u.array()
        assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < TOL
    if dims in ((32, 16, 24), (128, 128, 128), (256, 256, 256)):  # the real plan served it
        rp = ctypes.c_void_p()
        R.PetscCall(R.lib().MatFFTHIPGetRealPlan(F, ctypes.byref(rp)))
        assert rp.value
    u.destroy()
    R.PetscCall(R.lib().MatDestroy(ctypes.byref(F)))


@pytest.mark.parametrize("dims", GRIDS)
@pytest.mark.parametrize("hip", [True, False])
def test_real_pcshell(R, oracle, dims, hip):
    """The PCSHELL registered as ToDo.md:1 intends, on real Vecs: PCApply with the symbol setup
    materialised (register fast path), then with a Diag changed by the caller (explicit path)."""
    nx, ny, nz = dims
    N = nx * ny * nz
    lam = (0.6, 0.15, 0.02)
    ctx = R.FFTPrecTransportContext(3, nx, ny, nz, lam[0], lam[1], lam[2], None, None, None, None, None)
    pc = R.pc_shell(ctx)
    b = oracle.c_fill_uniform(N, 43).real.copy()
    vb, vx = R.Vec.seq(N, hip=hip).set_array(b), R.Vec.seq(N, hip=hip)
    R.PetscCall(R.lib().PCApply(pc, vb.h, vx.h))
    d0 = oracle.c_build_diag_transport(dims, lam)
    ref = _oracle_solve(oracle, dims, lam, b)
    assert np.linalg.norm(vx.array() - ref) / np.linalg.norm(ref) < TOL
    diag = R.Vec(ctypes.c_void_p(ctx.Diag))
    np.testing.assert_allclose(diag.array(), _half(d0.reshape(nz, ny, nx), nx), rtol=0, atol=1e-14)
    R.PetscCall(R.lib().VecScale(diag.h, 2.0))  # the caller changes Diag: solve_3D divides by it
    R.PetscCall(R.lib().PCApply(pc, vb.h, vx.h))
    ref2 = oracle.c_solve_3d(2 * d0, b.astype(np.complex128), dims).real
    assert np.linalg.norm(vx.array() - ref2) / np.linalg.norm(ref2) < TOL
    own, expl = ctypes.c_int64(), ctypes.c_int64()
    R.PetscCall(R.lib().MatFFTHIPGetSolveCounts(ctypes.c_void_p(ctx.FFT_MAT), ctypes.byref(own), ctypes.byref(expl)))
    assert (own.value, expl.value) == (1, 1)
    vb.destroy()
    vx.destroy()
    pcp = ctypes.c_void_p(pc.value)
    R.PetscCall(R.lib().PCDestroy(ctypes.byref(pcp)))


@pytest.mark.parametrize("dims", [(32, 16, 24), (9, 4, 6), (10, 10, 10), (16, 1, 1)])
def test_real_matmult_is_fftw_r2c(R, dims):
    """MatMult = r2c (FFTW_FORWARD, unnormalised) into the half spectrum; MatMultTranspose = c2r
    (unnormalised): numpy's rfftn and irfftn * N."""
    nx, ny, nz = dims
    N = nx * ny * nz
    F = R.mat_create_fft([nz, ny, nx])
    x, y, z = R.mat_create_vecs_fftw(F)
    assert x.size == N and y.size == 2 * (nx // 2 + 1) * ny * nz and z.size == N
    c = np.random.default_rng(4).standard_normal(N)
    x.set_array(c)
    R.PetscCall(R.lib().MatMult(F, x.h, y.h))
    want = np.fft.rfftn(c.reshape(nz, ny, nx))
    got = y.array().view(np.complex128).reshape(want.shape)
    assert np.linalg.norm(got - want) / np.linalg.norm(want) < 1e-13
    R.PetscCall(R.lib().MatMultTranspose(F, y.h, z.h))
    assert np.linalg.norm(z.array() - N * c) / np.linalg.norm(N * c) < 1e-13
    for v in (x, y, z):
        v.destroy()
    R.PetscCall(R.lib().MatDestroy(ctypes.byref(F)))


@pytest.mark.parametrize("dims", [(32, 16, 24), (9, 4, 6), (10, 10, 10)])
def test_real_build_diag_and_solve_3D(R, oracle, dims):
    """The reference's own Diag construction on a real-scalar PETSc (src/PCSHELLFft_3D.cxx:39-69):
    1-D MATFFTWs of the transport columns, then build_diag_mat_vec_3D; solve_3D with that Diag."""
    L = R.lib()
    nx, ny, nz = dims
    N = nx * ny * nz
    lam = (0.6, 0.15, 0.02)
    hats = []
    keep = []
    for n in (nx, ny, nz):
        F1 = R.mat_create_fft([n])
        c, ch, _ = R.mat_create_vecs_fftw(F1)
        R.PetscCall(L.build_transport_col(c.h, n))
        R.PetscCall(L.MatMult(F1, c.h, ch.h))
        hats.append(ch)
        keep.append((F1, c, _))
    F = R.mat_create_fft([nz, ny, nx])
    _, diag, _ = R.mat_create_vecs_fftw(F)
    R.PetscCall(L.build_diag_mat_vec_3D(diag.h, hats[0].h, hats[1].h, hats[2].h, nx, ny, nz, *lam))
    d0 = oracle.c_build_diag_transport(dims, lam)
    np.testing.assert_allclose(diag.array(), _half(d0.reshape(nz, ny, nx), nx), rtol=0, atol=1e-14)
    b = oracle.c_fill_uniform(N, 45).real.copy()
    vb, vx, bh = R.Vec.seq(N, hip=True).set_array(b), R.Vec.seq(N, hip=True), R.Vec.seq(diag.size, hip=True)
    R.PetscCall(L.solve_3D(F, vx.h, diag.h, vb.h, bh.h, N))
    ref = _oracle_solve(oracle, dims, lam, b)
    assert np.linalg.norm(vx.array() - ref) / np.linalg.norm(ref) < TOL
    for F1, c, z in keep:
        R.PetscCall(L.MatDestroy(ctypes.byref(F1)))


def test_real_gmres_with_pcshell(R, oracle):
    """The stand-in KSPGMRES on real Vecs with the real PCSHELL (BASELINE config 1's operator,
    fixed sign, matched lambda), against the oracle's PETSc-restated GMRES."""
    from oracle import transport as OT
    L = R.lib()
    n = 32
    dims, h = (n, n, n), (1.0 / n,) * 3
    a, dt = (1.0, 0.0, 0.0), 1e3 / 3 * OT.min_ratio_vol_surf(h)
    A = OT.divergence_matrix(dims, h, dt, a, sign="fixed", shift=1.0).real.tocsr()
    A.sort_indices()
    lam = (a[0] * dt / h[0], 0.0, 0.0)
    b = OT.initial_conditions_shock(dims)
    M = R.mat_aij(A)
    ksp = ctypes.c_void_p()
    R.PetscCall(L.KSPCreate(R.PETSC_COMM_SELF, ctypes.byref(ksp)))
    R.PetscCall(L.KSPSetType(ksp, b"gmres"))
    R.PetscCall(L.KSPSetOperators(ksp, M, M))
    R.PetscCall(L.KSPSetTolerances(ksp, 1e-10, 1e-50, 1e5, 1000))
    pc = ctypes.c_void_p()
    R.PetscCall(L.KSPGetPC(ksp, ctypes.byref(pc)))
    ctx = R.FFTPrecTransportContext(3, n, n, n, lam[0], lam[1], lam[2], None, None, None, None, None)
    R.PetscCall(L.PCSetType(pc, b"shell"))
    R.PetscCall(L.PCShellSetContext(pc, ctypes.addressof(ctx)))
    R.PetscCall(L.PCShellSetSetUp(pc, R.fn("setupFFTPrec3D")))
    R.PetscCall(L.PCShellSetApply(pc, R.fn("applyFFT3DPrecTransport")))
    R.PetscCall(L.PCShellSetDestroy(pc, R.fn("destroyFFTPrec3D")))
    u = R.Vec.seq(n ** 3, hip=True).set_array(b)
    R.PetscCall(L.KSPSolve(ksp, u.h, u.h))  # KSPSolve(ksp, Un, Un), as the reference driver
    its, reason = ctypes.c_int64(), ctypes.c_int()
    R.PetscCall(L.KSPGetIterationNumber(ksp, ctypes.byref(its)))
    R.PetscCall(L.KSPGetConvergedReason(ksp, ctypes.byref(reason)))
    xo, its_o, reason_o, _, _ = OT.gmres(A.astype(np.complex128), b, M=OT.fft_preconditioner(dims, lam), rtol=1e-10,
                                          maxits=1000)
    assert reason.value > 0 and reason.value == reason_o and its.value == its_o
    assert np.linalg.norm(u.array() - xo.real) <= 1e-9 * np.linalg.norm(xo.real)
    R.PetscCall(L.KSPDestroy(ctypes.byref(ksp)))
    R.PetscCall(L.MatDestroy(ctypes.byref(M)))
