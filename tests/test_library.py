"""CPU tests of the C ABI library: it loads, exports every symbol include/*.h declares, and
its host-only logic (slab layout, PETSc stand-in on host vectors, context factory) behaves
as the reference's interface.  No GPU compute is issued here."""
import os
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def L():
    import circulantpreconditioner_amd as cp
    return cp.lib()


def test_loads_and_version(L):
    assert b"gfx950" in L.cfp_version()


def test_exports_every_declared_symbol(L):
    from circulantpreconditioner_amd import _lib
    names = _lib.exported_symbols()
    assert len(names) > 100
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    for must in ("applyFFT3DPrecTransport", "setupFFTPrec3D", "destroyFFTPrec3D", "solve_3D",
                 "PetscFft3DTransportSolver", "build_diag_mat_vec_3D", "cfp_plan_apply", "cfp_dist_plan_apply"):
        assert must in names


def test_library_is_gfx950_code_object():
    import subprocess
    from circulantpreconditioner_amd import LIB_PATH
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB_PATH], capture_output=True, text=True)
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_transport_symbol_1d(oracle):
    import circulantpreconditioner_amd as cp
    for n in (1, 2, 3, 4, 10, 256):
        ref = np.fft.fft(oracle.np_transport_col(n))
        np.testing.assert_allclose(cp.transport_symbol_1d(n), ref, atol=2e-15)


@pytest.mark.parametrize("dims,P", [((256, 256, 256), 8), ((512, 512, 512), 8), ((64, 32, 16), 4),
                                    ((10, 6, 4), 2), ((8, 8, 8), 1)])
def test_slab_layout(dims, P):
    from circulantpreconditioner_amd.distributed import slab_layout
    nx, ny, nz = dims
    tot = 0
    for r in range(P):
        L = slab_layout(dims, P, r)
        assert L["nz_local"] == nz // P and L["ny_local"] == ny // P
        assert L["z0"] == r * nz // P and L["y0"] == r * ny // P
        assert L["local_size"] == nx * ny * nz // P
        assert L["chunk"] * P == L["local_size"]
        assert L["local_offset"] == tot  # PETSC_DECIDE contiguous blocks
        tot += L["local_size"]
    assert tot == nx * ny * nz


@pytest.mark.parametrize("dims,P,rows", [((64, 30, 32), 4, [8, 8, 8, 6]), ((8, 3, 8), 4, [1, 1, 1, 0]),
                                         ((256, 100, 256), 8, [13] * 7 + [9]), ((64, 40, 32), 4, [10] * 4)])
def test_slab_layout_uneven_y(dims, P, rows):
    """P need not divide ny: FFTW-MPI's blocks of ceil(ny / P) z-pencil rows, padded chunks."""
    from circulantpreconditioner_amd.distributed import slab_layout
    nx, ny, nz = dims
    nyp = -(-ny // P)
    for r in range(P):
        L = slab_layout(dims, P, r)
        assert L["ny_local"] == rows[r] and L["y0"] == r * nyp and L["ny_chunk"] == nyp
        assert L["chunk"] == (nz // P) * nyp * nx
        assert L["local_size"] == nx * ny * nz // P and L["local_offset"] == r * L["local_size"]
        assert L["work_size"] == max(L["local_size"], P * L["chunk"])
    assert sum(rows) == ny


def test_slab_layout_errors():
    import circulantpreconditioner_amd as cp
    from circulantpreconditioner_amd.distributed import slab_layout
    with pytest.raises(cp.CirculantError) as e:
        slab_layout((64, 64, 12), 8, 0)  # 8 does not divide nz
    assert e.value.code == 60
    with pytest.raises(cp.CirculantError):
        slab_layout((64, 64, 64), 4, 4)


# ---------------------------------------------------------------- PETSc stand-in, host only
def test_host_vec_ops():
    from circulantpreconditioner_amd import petsc as P
    rng = np.random.default_rng(0)
    a = rng.standard_normal(50) + 1j * rng.standard_normal(50)
    b = rng.standard_normal(50) + 1j * rng.standard_normal(50) + 3
    x, y = P.Vec.seq(50).set_array(a), P.Vec.seq(50).set_array(b)
    assert abs(x.dot(y) - np.vdot(b, a)) < 1e-12  # VecDot = y^H x
    assert abs(x.norm(P.NORM_2) - np.linalg.norm(a)) < 1e-12
    assert abs(x.norm(P.NORM_1) - np.sum(np.abs(a.real) + np.abs(a.imag))) < 1e-12
    assert abs(x.norm(P.NORM_INFINITY) - np.abs(a).max()) < 1e-12
    x.axpy(2 - 1j, y)
    np.testing.assert_allclose(x.array(), a + (2 - 1j) * b, rtol=1e-14)
    w = P.Vec.seq(50)
    P.PetscCall(P.lib().VecPointwiseDivide(w.h, x.h, y.h))
    np.testing.assert_allclose(w.array(), (a + (2 - 1j) * b) / b, rtol=1e-14)
    # PETSc's VecPointwiseDivide: a zero divisor gives 0 (bvec2.c), not inf / NaN
    bz = b.copy()
    bz[[3, 17]] = 0
    y.set_array(bz)
    P.PetscCall(P.lib().VecPointwiseDivide(w.h, x.h, y.h))
    ref = (a + (2 - 1j) * b) / np.where(bz != 0, bz, 1)
    ref[[3, 17]] = 0
    np.testing.assert_allclose(w.array(), ref, rtol=1e-14)


def test_pc_none_and_identical_vectors():
    from circulantpreconditioner_amd import petsc as P
    v = P.Vec.seq(8).set_array(np.arange(8) + 1j)
    u = P.Vec.seq(8)
    pc = P.PC.none()
    pc.apply(v, u)
    np.testing.assert_array_equal(u.array(), np.arange(8) + 1j)
    with pytest.raises(P.PetscError) as e:
        pc.apply(v, v)  # PCApply requires x != y
    assert e.value.code == 61  # PETSC_ERR_ARG_IDN


def test_pcshell_context_roundtrip():
    from circulantpreconditioner_amd import petsc as P
    ctx = P.make_context((8, 4, 2), (0.5, 0.25, 0.1))
    pc = P.PC.shell(ctx)
    got = ctypes.c_void_p()
    P.PetscCall(P.lib().PCShellGetContext(pc.h, ctypes.byref(got)))
    assert got.value == ctypes.addressof(ctx)


def test_getFFTPrec3DContext_formula():
    from circulantpreconditioner_amd import petsc as P
    # src/PCSHELLFft_3D.cxx:122-148: n = floor(cbrt(nbCells)), lambda = a dt (max-min)/n
    ctx = P.getFFTPrec3DContext(3, 0.01, 32 ** 3, 1.0, 2.0, 0.0, -0.5, -0.5, -0.5, 0.5, 0.5, 0.5)
    assert (ctx.spaceDim, ctx.n_x, ctx.n_y, ctx.n_z) == (3, 32, 32, 32)
    assert abs(complex(ctx.lambda_x) - 0.01 / 32) < 1e-18
    assert abs(complex(ctx.lambda_y) - 0.02 / 32) < 1e-18
    ctx2 = P.getFFTPrec3DContext(2, 1.0, 100, 1, 1, 1, 0, 0, 0, 1, 1, 1)
    assert (ctx2.n_x, ctx2.n_y, ctx2.n_z) == (10, 10, 1)
    ctx1 = P.getFFTPrec3DContext(1, 1.0, 7, 1, 1, 1, 0, 0, 0, 1, 1, 1)
    assert (ctx1.n_x, ctx1.n_y, ctx1.n_z) == (7, 1, 1)
    with pytest.raises(P.PetscError) as e:
        P.getFFTPrec3DContext(4, 1.0, 8, 1, 1, 1, 0, 0, 0, 1, 1, 1)
    assert e.value.code == 63  # PETSC_ERR_ARG_OUTOFRANGE, "Dimension should be 1, 2 or 3"


def test_mat_create_fft_rejects_other_types():
    from circulantpreconditioner_amd import petsc as P
    h = ctypes.c_void_p()
    d = (ctypes.c_int64 * 3)(4, 4, 4)
    rc = P.lib().MatCreateFFT(0, 3, d, b"aij", ctypes.byref(h))
    assert rc == 56  # PETSC_ERR_SUP


REF_CALLER = r"""
#include <cstdio>
#include <complex>
#include "pcshell_fft3d.h"
static double re(double v) { return v; }
static double re(std::complex<double> v) { return v.real(); }
struct Mesh { long cells; double bbox[6]; };  // stands for SOLVERLAB's Mesh, passed by value
int main() {
  Mesh m{4096, {0, 1, 0, 2, 0, 4}};
  // the reference's call, unchanged (src/PCSHELLFft_3D.hxx:27-41)
  PetscErrorCode ierr = getFFTPrec3DContext(3, 0.5, m.cells, 1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0, 2.0, 4.0, m);
  const FFTPrecTransportContext *c = FFTPrecTransportContextLast();
  FFTPrecTransportContext mine;
  PetscErrorCode ierr2 = getFFTPrec3DContext(2, 1.0, 100, 1.0, 1.0, 1.0, 0, 0, 0, 1, 1, 1, &mine);
  // ADVICE r04: NULL / 0 / nullptr as the last argument reach the C function's NULL check, not
  // the Mesh template (which would succeed and write the library slot)
  PetscErrorCode e0 = getFFTPrec3DContext(3, 0.5, 64, 1.0, 1.0, 1.0, 0, 0, 0, 1, 1, 1, NULL);
  PetscErrorCode e1 = getFFTPrec3DContext(3, 0.5, 64, 1.0, 1.0, 1.0, 0, 0, 0, 1, 1, 1, 0);
  PetscErrorCode e2 = getFFTPrec3DContext(3, 0.5, 64, 1.0, 1.0, 1.0, 0, 0, 0, 1, 1, 1, nullptr);
  std::printf("%d %d %ld %ld %ld %.17g %.17g %.17g %ld %ld %d %d %d %ld\n", (int)ierr, (int)ierr2, (long)c->n_x,
              (long)c->n_y, (long)c->n_z, re(c->lambda_x), re(c->lambda_y), re(c->lambda_z),
              (long)mine.n_x, (long)mine.n_z, (int)e0, (int)e1, (int)e2, (long)FFTPrecTransportContextLast()->n_x);
  return 0;
}
"""


@pytest.mark.parametrize("real", [False, True])
def test_reference_caller_compiles_unchanged(tmp_path, real):
    """the reference's 13-argument getFFTPrec3DContext(..., Mesh srcMesh)
    compiles and links against include/pcshell_fft3d.h; the context lands in the library slot."""
    import shutil
    import subprocess
    from circulantpreconditioner_amd import LIB_PATH
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    lib = LIB_PATH if not real else LIB_PATH.replace("libcirculant_fft.so", "libcirculant_fft_real.so")
    src = tmp_path / "caller.cpp"
    src.write_text(REF_CALLER)
    exe = tmp_path / "caller"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    cmd = ["g++", "-std=c++17", "-I", inc, str(src), "-o", str(exe), lib, "-Wl,-rpath," + os.path.dirname(lib)]
    if real:
        cmd.insert(1, "-DCFP_REAL_SCALAR")
    subprocess.run(cmd, check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert out[:5] == ["0", "0", "16", "16", "16"]
    # lambda_d = a_d dt (max - min) / n (src/PCSHELLFft_3D.cxx:146-148)
    np.testing.assert_allclose([float(v) for v in out[5:8]], [1 * .5 * 1 / 16, 2 * .5 * 2 / 16, 3 * .5 * 4 / 16])
    assert out[8:10] == ["10", "1"]
    assert out[10:13] == ["85", "85", "85"]  # PETSC_ERR_ARG_NULL
    assert out[13] == "16"  # the slot still holds the Mesh call's context
