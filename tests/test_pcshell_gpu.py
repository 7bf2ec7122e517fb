"""GPU parity through the reference's PETSc-facing interface (PCSHELL callbacks, direct
solver chain), driven exactly as a PETSc caller would register them (ToDo.md:1)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module")
def P():
    from circulantpreconditioner_amd import petsc
    assert torch.cuda.is_available()
    return petsc


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.complex128)).cuda()


def _lam(case):
    return tuple(complex(re, im) for re, im in case["lam"])


@pytest.mark.parametrize("name", ["kat3d_4x3x2", "py3d_10x25x40", "kat1d_4", "py2d_12x10", "rand16_A", "odd6x5x7"])
def test_pcshell_apply_golden(P, golden, name):
    c = golden[name]
    n = tuple(c["n"])
    ctx = P.make_context(n, _lam(c))
    pc = P.PC.shell(ctx)
    pc.setup()  # setupFFTPrec3D: FFT matrix, Diag, work vectors
    assert ctx.FFT_MAT and ctx.Diag and ctx.b_hat and ctx.b_cartesien and P.context_plan(ctx)
    tb, tx = _dev(c["b"]), torch.zeros(int(np.prod(n)), dtype=torch.complex128, device="cuda")
    b, x = P.Vec.from_tensor(tb), P.Vec.from_tensor(tx)
    pc.apply(b, x)  # PCApply -> applyFFT3DPrecTransport
    torch.cuda.synchronize()
    got = tx.cpu().numpy()
    assert np.linalg.norm(got - c["x"]) / np.linalg.norm(c["x"]) < TOL
    # Diag materialised by setup equals the reference's Kronecker Diag
    d = P.Vec.borrow(ctx.Diag).array()
    assert np.linalg.norm(d - c["diag"]) / np.linalg.norm(c["diag"]) < 1e-14
    np.testing.assert_array_equal(tb.cpu().numpy(), c["b"])  # b untouched
    pc.destroy()  # destroyFFTPrec3D
    assert not ctx.FFT_MAT and not ctx.Diag


def test_pcshell_host_vectors(P, oracle):
    """VECSEQ (host) vectors take the PCIe staging path and give the same answer."""
    n = (32, 16, 8)
    lam = (0.6, 0.15, 0.02)
    b = oracle.c_fill_uniform(int(np.prod(n)), 5)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    ctx = P.make_context(n, lam)
    pc = P.PC.shell(ctx).setup()
    vb, vx = P.Vec.seq(b.size).set_array(b), P.Vec.seq(b.size)
    pc.apply(vb, vx)
    assert oracle.rel_l2(vx.array(), ref) < TOL
    pc.destroy()


def test_pcshell_from_factory(P, oracle):
    # getFFTPrec3DContext on a 32^3 unit cube, a = (1,0,0), cfl-like dt (reference formula)
    ctx = P.getFFTPrec3DContext(3, 10.0, 32 ** 3, 1.0, 0.0, 0.0, -0.5, -0.5, -0.5, 0.5, 0.5, 0.5)
    lam = (complex(ctx.lambda_x), complex(ctx.lambda_y), complex(ctx.lambda_z))
    n = (32, 32, 32)
    pc = P.PC.shell(ctx).setup()
    b = oracle.c_fill_uniform(32 ** 3, 1)
    tb, tx = _dev(b), torch.empty(32 ** 3, dtype=torch.complex128, device="cuda")
    pc.apply(P.Vec.from_tensor(tb), P.Vec.from_tensor(tx))
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b, n)
    assert oracle.rel_l2(tx.cpu().numpy(), ref) < TOL
    pc.destroy()


def test_solve_3D_honours_the_diag_it_is_given(P, oracle):
    """solve_3D divides by the Diag it is handed (src/FftLinearSolver_3D.c:174): after
    VecScale(ctx->Diag, 2), after a device write through VecHIPGetArray/Restore and after a
    symbol change on FFT_MAT, the apply must follow the new Diag; an untouched Diag keeps the
    register-symbol fast path."""
    from circulantpreconditioner_amd._lib import check, lib
    n, lam = (32, 16, 8), (0.6, 0.15 - 0.1j, 0.02)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 8)
    d0 = oracle.c_build_diag_transport(n, lam)
    ctx = P.make_context(n, lam)
    pc = P.PC.shell(ctx).setup()
    F = P.Mat(ctypes_handle(ctx.FFT_MAT), owned=False)
    diag = P.Vec.borrow(ctx.Diag)
    tb, tx = _dev(b), torch.empty(N, dtype=torch.complex128, device="cuda")
    vb, vx = P.Vec.from_tensor(tb), P.Vec.from_tensor(tx)

    def apply_and_check(dref, counts):
        pc.apply(vb, vx)
        torch.cuda.synchronize()
        assert oracle.rel_l2(tx.cpu().numpy(), oracle.c_solve_3d(dref, b, n)) < TOL
        assert F.solve_counts() == counts

    apply_and_check(d0, (1, 0))           # untouched: the plan's own symbol, no Diag read
    apply_and_check(d0, (2, 0))
    s0 = diag.state()
    diag.scale(2.0)                       # VecScale(ctx->Diag, 2)
    assert diag.state() > s0
    apply_and_check(2 * d0, (2, 1))
    with diag.hip_array() as p:           # a device write through VecHIPGetArray/Restore
        check(lib().cfp_scale(p, 0.5, 0.25, N, None))
        torch.cuda.synchronize()
    apply_and_check(2 * d0 * (0.5 + 0.25j), (2, 2))
    # a symbol change on FFT_MAT (another lambda through the direct-solver chain) with the
    # untouched-since-setup Diag restored: setup's Diag no longer matches the plan's symbol
    pc.destroy()
    ctx2 = P.make_context(n, lam)
    pc2 = P.PC.shell(ctx2).setup()
    F2 = P.Mat(ctypes_handle(ctx2.FFT_MAT), owned=False)
    lam2 = (1.5, 0.0, 0.3)
    P.FftTransportSolver(n[0], n[1], n[2], *lam2, vx, vb, F2)  # symbol now lam2
    pc2.apply(vb, vx)
    torch.cuda.synchronize()
    assert oracle.rel_l2(tx.cpu().numpy(), oracle.c_solve_3d(d0, b, n)) < TOL  # ctx2.Diag still holds lam
    assert F2.solve_counts() == (0, 1)
    pc2.destroy()


def ctypes_handle(h):
    import ctypes
    return h if isinstance(h, ctypes.c_void_p) else ctypes.c_void_p(h)


def test_pcapply_requires_distinct_vectors(P):
    ctx = P.make_context((8, 8, 8), (1, 1, 1))
    pc = P.PC.shell(ctx).setup()
    t = torch.zeros(512, dtype=torch.complex128, device="cuda")
    v = P.Vec.from_tensor(t)
    with pytest.raises(P.PetscError) as e:
        pc.apply(v, v)
    assert e.value.code == 61
    pc.destroy()


def test_solve_3D_explicit_diag_chain(P, golden):
    """The reference's own setup chain: 1-D MatCreateFFT of each transport column, MatMult,
    build_diag_mat_vec_3D, then solve_3D(FFT_MAT, X, Diag, b, b_hat, size)."""
    c = golden["py3d_10x25x40"]
    nx, ny, nz = c["n"]
    lam = _lam(c)
    hats = []
    for n in (nx, ny, nz):
        A = P.Mat.create_fft([n])
        col, hat = A.create_vecs(2)
        P.build_transport_col(col, n)
        A.mult(col, hat)
        hats.append(hat)
        hats[-1]._A = A
    F = P.Mat.create_fft([nz, ny, nx])
    Diag, b_hat = F.create_vecs(2)
    P.build_diag_mat_vec_3D(Diag, *hats, nx, ny, nz, *lam)
    d = Diag.array()
    assert np.linalg.norm(d - c["diag"]) / np.linalg.norm(c["diag"]) < 1e-14
    tb = _dev(c["b"])
    tx = torch.empty_like(tb)
    P.solve_3D(F, P.Vec.from_tensor(tx), Diag, P.Vec.from_tensor(tb), b_hat, nx * ny * nz)
    assert np.linalg.norm(tx.cpu().numpy() - c["x"]) / np.linalg.norm(c["x"]) < TOL


def test_matmult_is_unnormalised_fftw(P, oracle):
    n = (12, 10, 8)
    F = P.Mat.create_fft([n[2], n[1], n[0]])
    b = oracle.c_fill_uniform(int(np.prod(n)), 2)
    x, y = F.create_vecs(2)
    x.set_array(b)
    F.mult(x, y)
    assert oracle.rel_l2(y.array(), oracle.c_fft3d(b, n, -1)) < 1e-13
    F.mult_transpose(x, y)
    assert oracle.rel_l2(y.array(), oracle.c_fft3d(b, n, +1)) < 1e-13


@pytest.mark.parametrize("inplace", [False, True])
def test_direct_solver_chain(P, oracle, inplace):
    """PetscFft3DTransportSolver(ctx, Un, Un) as tests/TransportEquationFFT_..._mpi.cxx:111."""
    nx, ny, nz = 20, 10, 10
    a, dt, dlt = (1.0, 0.0, 0.0), 1e3 / 3 / 20, (1 / 20, 1 / 10, 1 / 10)
    F = P.Mat.create_fft([nz, ny, nx])
    ctx = P.StructuredContext(nx, ny, nz, *a, dt, *dlt, F)
    b = oracle.c_fill_uniform(nx * ny * nz, 3)
    lam = tuple(a[i] * dt / dlt[i] for i in range(3))
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport((nx, ny, nz), lam), b, (nx, ny, nz))
    tb = _dev(b)
    vb = P.Vec.from_tensor(tb)
    if inplace:
        P.PetscFft3DTransportSolver(ctx, vb, vb)
        got = tb.cpu().numpy()
    else:
        tx = torch.empty_like(tb)
        P.PetscFft3DTransportSolver(ctx, vb, P.Vec.from_tensor(tx))
        got = tx.cpu().numpy()
    assert oracle.rel_l2(got, ref) < TOL
    # the caller's FFT_MAT survives (the reference destroys it, App. A item 6): reuse it
    P.PetscFft3DTransportSolver(ctx, vb, vb)


def test_fft2d_fft1d_solvers(P, oracle, golden):
    c = golden["py2d_12x10"]
    F = P.Mat.create_fft([10, 12])
    tb = _dev(c["b"])
    tx = torch.empty_like(tb)
    l = _lam(c)
    # lambda = a dt / delta with dt = 1, delta = 1
    P.Fft2DTransportSolver(12, 10, l[0], l[1], 1.0, 1.0, 1.0, P.Vec.from_tensor(tx), P.Vec.from_tensor(tb), F)
    assert np.linalg.norm(tx.cpu().numpy() - c["x"]) / np.linalg.norm(c["x"]) < TOL
    c1 = golden["kat1d_4"]
    F1 = P.Mat.create_fft([4])
    tb = _dev(c1["b"])
    tx = torch.empty_like(tb)
    P.Fft1DTransportSolver(4, 0.5, 1.0, 1.0, P.Vec.from_tensor(tx), P.Vec.from_tensor(tb), F1)
    np.testing.assert_allclose(tx.cpu().numpy().real, [6.7, 2.9, 6.3, 20.1], atol=1e-12)


def test_intersection_matrix_remap(P, oracle):
    """A permutation intersectionMatrix (mesh numbering -> Cartesian) is applied before the solve."""
    n = (8, 8, 8)
    N = 512
    lam = (0.6, 0.15, 0.02)
    perm = np.random.default_rng(0).permutation(N)
    rowptr = np.arange(N + 1)
    A = P.Mat.aij(rowptr, perm, np.ones(N), (N, N))  # (A b)[i] = b[perm[i]]
    ctx = P.make_context(n, lam)
    ctx.intersectionMatrix = A.h.value
    pc = P.PC.shell(ctx).setup()
    b = oracle.c_fill_uniform(N, 4)
    tb, tx = _dev(b), torch.empty(N, dtype=torch.complex128, device="cuda")
    pc.apply(P.Vec.from_tensor(tb), P.Vec.from_tensor(tx))
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(n, lam), b[perm], n)
    assert oracle.rel_l2(tx.cpu().numpy(), ref) < TOL
    pc.destroy()


@pytest.mark.parametrize("mean", [1, 2, 3, 7, 13, 40])
def test_aij_device_spmv_row_lengths(P, mean):
    """MatMult of the stand-in AIJ on device Vecs (cfp::blas_csr_spmv: one thread per row up to
    ~1 nonzero per row, 2 / 4 / 8 / 16 lanes per row above) against scipy, with empty rows, rows
    far longer than the lanes and unsorted columns."""
    import scipy.sparse as sp
    rng = np.random.default_rng(mean)
    m, n = 4099, 3001
    lens = rng.integers(0, 2 * mean + 1, m)
    lens[::17] = 0
    lens[5] = 5 * mean + 37
    rowptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(rowptr[-1])
    col = rng.integers(0, n, nnz).astype(np.int64)
    val = rng.standard_normal(nnz) + 1j * rng.standard_normal(nnz)
    A = P.Mat.aij(rowptr, col, val, (m, n))
    xs = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    ty = torch.empty(m, dtype=torch.complex128, device="cuda")
    A.mult(P.Vec.from_tensor(_dev(xs)), P.Vec.from_tensor(ty))
    ref = sp.csr_matrix((val, col, rowptr), shape=(m, n)) @ xs
    assert np.linalg.norm(ty.cpu().numpy() - ref) <= 1e-13 * np.linalg.norm(ref)
    A.destroy()


def test_device_vec_kernels(P):
    rng = np.random.default_rng(1)
    a = rng.standard_normal(3000) + 1j * rng.standard_normal(3000)
    bb = rng.standard_normal(3000) + 1j * rng.standard_normal(3000)
    x, y = P.Vec.from_tensor(_dev(a)), P.Vec.from_tensor(_dev(bb))
    assert abs(x.dot(y) - np.vdot(bb, a)) < 1e-10
    assert abs(x.norm(P.NORM_2) - np.linalg.norm(a)) < 1e-10
    assert abs(x.norm(P.NORM_1) - np.sum(np.abs(a.real) + np.abs(a.imag))) < 1e-9
    assert abs(x.norm(P.NORM_INFINITY) - np.abs(a).max()) < 1e-12
    x.axpy(0.5j, y)
    np.testing.assert_allclose(x.array(), a + 0.5j * bb, rtol=1e-14)


@pytest.mark.parametrize("explicit", [False, True], ids=["own_symbol", "explicit_diag"])
def test_solve_3D_in_place_host_vec(P, oracle, explicit):
    """solve_3D(FFT_MAT, X, Diag, X, ...) on a host (VECSEQ) Vec, in place: staged through the
    plan's persistent device buffer with checked copies (no per-call allocation), for the
    plan's own symbol and for an explicit (scaled) Diag."""
    n, lam = (32, 16, 8), (0.6, 0.15, 0.02)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 21)
    d0 = oracle.c_build_diag_transport(n, lam)
    ctx = P.make_context(n, lam)
    pc = P.PC.shell(ctx).setup()
    F = P.Mat(ctypes_handle(ctx.FFT_MAT), owned=False)
    diag = P.Vec.borrow(ctx.Diag)
    if explicit:
        diag.scale(0.5 + 0.5j)
    vx = P.Vec.seq(N).set_array(b)
    for k in range(3):  # repeated in-place solves reuse the staging buffer
        vx.set_array(b)
        P.solve_3D(F, vx, diag, vx, None, N)
        dref = d0 * (0.5 + 0.5j) if explicit else d0
        assert oracle.rel_l2(vx.array(), oracle.c_solve_3d(dref, b, n)) < TOL
    assert F.solve_counts() == ((0, 3) if explicit else (3, 0))
    pc.destroy()


def test_symbol_set_on_the_plan_directly_leaves_the_fast_path(P, oracle):
    """A symbol set on the plan behind FFT_MAT (MatFFTHIPGetPlan + cfp_plan_set_*) bumps the
    plan's own symbol version: solve_3D then divides by the Diag it is given, not by the new
    register symbol."""
    from circulantpreconditioner_amd._lib import check, lib
    import ctypes
    n, lam = (16, 16, 8), (0.6, 0.15, 0.02)
    N = int(np.prod(n))
    b = oracle.c_fill_uniform(N, 3)
    d0 = oracle.c_build_diag_transport(n, lam)
    ctx = P.make_context(n, lam)
    pc = P.PC.shell(ctx).setup()
    F = P.Mat(ctypes_handle(ctx.FFT_MAT), owned=False)
    v0, v1 = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().cfp_plan_symbol_version(ctypes.c_void_p(P.context_plan(ctx)), ctypes.byref(v0)))
    lam2 = (ctypes.c_double * 6)(2.0, 0.0, 0.5, 0.0, 0.1, 0.0)
    check(lib().cfp_plan_set_symbol_transport(ctypes.c_void_p(P.context_plan(ctx)), lam2))
    check(lib().cfp_plan_symbol_version(ctypes.c_void_p(P.context_plan(ctx)), ctypes.byref(v1)))
    assert v1.value > v0.value
    tb, tx = _dev(b), torch.empty(N, dtype=torch.complex128, device="cuda")
    pc.apply(P.Vec.from_tensor(tb), P.Vec.from_tensor(tx))
    torch.cuda.synchronize()
    assert oracle.rel_l2(tx.cpu().numpy(), oracle.c_solve_3d(d0, b, n)) < TOL
    assert F.solve_counts() == (0, 1)
    pc.destroy()
