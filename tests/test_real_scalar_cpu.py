"""The real-scalar build of the PETSc boundary (libcirculant_fft_real.so, PetscScalar = double)
on CPU: it loads beside the complex library, exports every entry point of the PETSc-typed
headers, and its host Vecs and GMRES (PCNONE) match numpy / scipy.  GPU parity of the FFT
paths: tests/test_real_scalar_gpu.py."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def test_real_library_loads_and_exports():
    from circulantpreconditioner_amd import petsc_real as R
    from circulantpreconditioner_amd._lib import _parse_decls, lib
    lib()  # the complex library in the same process (RTLD_GLOBAL): the real one must not bind to it
    L = R.lib()
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    names = _parse_decls(os.path.join(inc, "pcshell_fft3d.h")) + _parse_decls(os.path.join(inc, "petsc_mini.h"))
    names += _parse_decls(os.path.join(inc, "circulant_fft.h")) + _parse_decls(os.path.join(inc, "circulant_fft_real.h"))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert hasattr(L, "MatFFTHIPGetRealPlan")


def test_real_host_vec_ops():
    from circulantpreconditioner_amd import petsc_real as R
    rng = np.random.default_rng(3)
    a, b = rng.standard_normal(101), rng.standard_normal(101)
    va, vb = R.Vec.seq(101).set_array(a), R.Vec.seq(101).set_array(b)
    d, nrm = np.zeros(1), np.zeros(1)
    import ctypes
    dd, nn = ctypes.c_double(), ctypes.c_double()
    R.PetscCall(R.lib().VecDot(va.h, vb.h, ctypes.byref(dd)))
    R.PetscCall(R.lib().VecNorm(va.h, R.NORM_2, ctypes.byref(nn)))
    assert dd.value == pytest.approx(a @ b, rel=1e-14) and nn.value == pytest.approx(np.linalg.norm(a), rel=1e-14)
    R.PetscCall(R.lib().VecAXPY(vb.h, 2.5, va.h))
    np.testing.assert_allclose(vb.array(), b + 2.5 * a, rtol=1e-15)
    R.PetscCall(R.lib().VecScale(vb.h, -0.5))
    np.testing.assert_allclose(vb.array(), -0.5 * (b + 2.5 * a), rtol=1e-15)
    va.destroy()
    vb.destroy()


def test_real_host_gmres_pcnone():
    import ctypes
    from circulantpreconditioner_amd import petsc_real as R
    n = 150
    A = (sp.random(n, n, density=0.05, random_state=5) + 6.0 * sp.identity(n)).tocsr()
    A.sort_indices()
    b = np.random.default_rng(6).standard_normal(n)
    L = R.lib()
    M = R.mat_aij(A)
    ksp = ctypes.c_void_p()
    R.PetscCall(L.KSPCreate(R.PETSC_COMM_SELF, ctypes.byref(ksp)))
    R.PetscCall(L.KSPSetType(ksp, b"gmres"))
    R.PetscCall(L.KSPSetOperators(ksp, M, M))
    R.PetscCall(L.KSPSetTolerances(ksp, 1e-12, 1e-50, 1e5, 500))
    pc = ctypes.c_void_p()
    R.PetscCall(L.KSPGetPC(ksp, ctypes.byref(pc)))
    R.PetscCall(L.PCSetType(pc, b"none"))
    vb, vx = R.Vec.seq(n).set_array(b), R.Vec.seq(n)
    R.PetscCall(L.KSPSolve(ksp, vb.h, vx.h))
    reason = ctypes.c_int()
    R.PetscCall(L.KSPGetConvergedReason(ksp, ctypes.byref(reason)))
    assert reason.value > 0
    xs = spla.spsolve(A.tocsc(), b)
    assert np.linalg.norm(vx.array() - xs) <= 1e-10 * np.linalg.norm(xs)
    R.PetscCall(L.KSPDestroy(ctypes.byref(ksp)))
    R.PetscCall(L.MatDestroy(ctypes.byref(M)))


@pytest.mark.parametrize("dims", [(8, 6, 4), (9, 5, 7), (1, 4, 4), (2, 3, 3), (16, 1, 8)])
def test_half_spectrum_row_padding_is_c2r(dims):
    """The identity the real-scalar slab path rests on (pcshell_fft3d_real.cpp, cfp_half_spectrum_pad):
    for ANY half spectrum H ([nz][ny][nx/2 + 1]), Re IDFT(pad(H)) -- pad: weight 1 on kx = 0 and,
    nx even, nx/2, weight 2 on the other kx <= nx/2, 0 above -- equals Re IDFT of H's Hermitian
    extension (FFTW's c2r), and it needs no value from another z-plane."""
    nx, ny, nz = dims
    M = nx // 2 + 1
    rng = np.random.default_rng(3)
    H = rng.standard_normal((nz, ny, M)) + 1j * rng.standard_normal((nz, ny, M))
    ext = np.empty((nz, ny, nx), complex)
    ext[..., :M] = H
    for kx in range(M, nx):
        ext[:, :, kx] = np.conj(H[(-np.arange(nz)) % nz][:, (-np.arange(ny)) % ny, nx - kx])
    pad = np.zeros((nz, ny, nx), complex)
    w = np.full(M, 2.0)
    w[0] = 1.0
    if nx % 2 == 0:
        w[M - 1] = 1.0
    pad[..., :M] = H * w
    a = np.fft.ifftn(ext).real
    b = np.fft.ifftn(pad).real
    assert np.abs(a - b).max() <= 1e-13 * max(1.0, np.abs(a).max())
    # and for a Hermitian-consistent H (the r2c of real data) both are FFTW's c2r = N * irfftn
    x = rng.standard_normal((nz, ny, nx))
    Hr = np.fft.rfftn(x)
    padr = np.zeros((nz, ny, nx), complex)
    padr[..., :M] = Hr * w
    assert np.abs(np.fft.ifftn(padr).real - x).max() < 1e-13
