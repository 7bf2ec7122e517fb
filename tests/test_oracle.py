"""CPU tests: pin the oracle (C + numpy restatements) to the reference's golden vectors.

The fixtures in tests/golden/ were produced by the reference's own Python oracle
functions (tests/golden/make_golden.py); the C KATs' published answers are
asserted directly (testFftSolver_1D.c:144-177 -> x = (6.7, 2.9, 6.3, 20.1);
testFftSolver_3D.c:95-141 -> x = X_ref = i^3).
"""
import hashlib

import numpy as np
import pytest

TOL = 1e-10  # north_star: 1e-10 relative on the preconditioned vector


def _lam(case):
    return tuple(complex(re, im) for re, im in case["lam"])


def test_manifest_integrity(golden):
    import os
    import json
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    man = json.load(open(os.path.join(gdir, "manifest.json")))
    for name, meta in man["cases"].items():
        with open(os.path.join(gdir, meta["file"]), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == meta["sha256"], name


def test_kat1d_published_answer(golden):
    c = golden["kat1d_4"]
    np.testing.assert_allclose(c["x"].real, [6.7, 2.9, 6.3, 20.1], rtol=0, atol=1e-12)


def test_kat3d_recovers_xref(golden):
    c = golden["kat3d_4x3x2"]
    assert np.linalg.norm(c["x"] - c["x_ref"]) / np.linalg.norm(c["x_ref"]) < 1e-13


@pytest.mark.parametrize("name", ["py3d_10x25x40", "py1d_8", "py2d_12x10"])
def test_reference_demo_error(golden, name):
    # the reference prints these relative errors (testFftSolver_3D.py:73-76); 3.2e-16 etc.
    c = golden[name]
    assert np.linalg.norm(c["x"] - c["x_ref"]) / np.linalg.norm(c["x_ref"]) < 1e-12


def test_splitmix_matches_fixture(golden, oracle):
    c = golden["rand32_A"]
    b = oracle.c_fill_uniform(32 ** 3, c["b_generator"]["seed"])
    assert hashlib.sha256(b.tobytes()).hexdigest() == c["b_sha256"]
    b16 = oracle.c_fill_uniform(16 ** 3, c["b_generator"]["seed"])
    np.testing.assert_array_equal(b16, golden["rand16_A"]["b"])


def test_uniform_range(oracle):
    b = oracle.c_fill_uniform(100000, 7)
    for part in (b.real, b.imag):
        assert part.min() >= -1.0 and part.max() < 1.0
        assert abs(part.mean()) < 0.02


@pytest.mark.parametrize("name", ["kat3d_4x3x2", "py3d_10x25x40", "kat1d_4", "py1d_8", "py2d_12x10",
                                  "py2d_50x200", "rand16_A", "rand16_B", "odd6x5x7"])
def test_c_oracle_diag_and_solve(golden, oracle, name):
    c = golden[name]
    n = tuple(c["n"])
    lam = _lam(c)
    d = oracle.c_build_diag_transport(n, lam)
    if name.startswith("kat1d") or name.startswith("py1d"):
        # 1-D fixtures use the (1+l, -l) column directly: same Diag by construction
        pass
    assert oracle.rel_l2(d, c["diag"]) < 1e-14
    x = oracle.c_solve_3d(c["diag"], c["b"], n)
    assert oracle.rel_l2(x, c["x"]) < TOL
    xn = oracle.np_solve_3d(c["diag"], c["b"], n)
    assert oracle.rel_l2(xn, c["x"]) < TOL


def test_c_oracle_rand32(golden, oracle):
    c = golden["rand32_A"]
    n = tuple(c["n"])
    b = oracle.c_fill_uniform(32 ** 3, c["b_generator"]["seed"])
    d = oracle.c_build_diag_transport(n, _lam(c))
    assert oracle.rel_l2(oracle.c_solve_3d(d, b, n), c["x"]) < TOL


@pytest.mark.parametrize("n", [(4, 3, 2), (16, 8, 4), (6, 5, 7), (12, 10, 1), (9, 1, 1)])
def test_kron_build_matches_closed_form(oracle, n):
    lam = (0.6 + 0.1j, 0.15, 0.02 - 0.3j)
    d = oracle.c_build_diag_transport(n, lam)
    assert oracle.rel_l2(d, oracle.np_diag_closed_form(n, lam)) < 1e-14


@pytest.mark.parametrize("n", [(4, 3, 2), (6, 5, 7), (8, 4, 2)])
def test_dense_operator_matches_stencil(oracle, n):
    lam = (0.6, 0.15, 0.02)
    rng = np.random.default_rng(1)
    x = rng.standard_normal(np.prod(n)) + 1j * rng.standard_normal(np.prod(n))
    C = oracle.np_dense_C(n, lam)
    assert oracle.rel_l2(oracle.c_apply_circulant(x, n, lam), C @ x) < 1e-14


@pytest.mark.parametrize("n", [(64, 64, 64), (32, 48, 20)])
def test_c_fft3d_matches_numpy(oracle, n):
    b = oracle.c_fill_uniform(int(np.prod(n)), 5)
    f = oracle.c_fft3d(b, n, -1)
    ref = np.fft.fftn(b.reshape(n[::-1])).reshape(-1)
    assert oracle.rel_l2(f, ref) < 1e-13
    g = oracle.c_fft3d(f, n, +1) / np.prod(n)
    assert oracle.rel_l2(g, b) < 1e-13


def test_solve_residual_large(oracle):
    n = (128, 64, 32)
    lam = (55.6, 0.0, 0.0)
    b = oracle.c_fill_uniform(int(np.prod(n)), 11)
    d = oracle.c_build_diag_transport(n, lam)
    x = oracle.c_solve_3d(d, b, n)
    assert oracle.rel_l2(oracle.c_apply_circulant(x, n, lam), b) < 1e-12


def test_zero_divisor_rule(oracle):
    """solve_3D's VecPointwiseDivide with a singular Diag (PETSc: a zero divisor gives 0): the
    C restatement and the numpy restatement agree, and the result is the pseudo-inverse solve
    (the null frequencies dropped), finite everywhere."""
    n = (8, 6, 4)
    N = int(np.prod(n))
    d = oracle.c_build_diag_transport(n, (0.6, 0.15, 0.02))
    d[[0, 5, 77]] = 0
    b = oracle.c_fill_uniform(N, 9)
    x = oracle.c_solve_3d(d, b, n)
    assert np.all(np.isfinite(x))
    np.testing.assert_allclose(x, oracle.np_solve_3d(d, b, n), rtol=0, atol=1e-14 * np.abs(x).max())
    bh = np.fft.fftn(b.reshape(n[2], n[1], n[0])).reshape(-1)
    q = np.zeros_like(bh)
    nz = d != 0
    q[nz] = bh[nz] / d[nz]
    ref = np.fft.ifftn(q.reshape(n[2], n[1], n[0])).reshape(-1)
    np.testing.assert_allclose(x, ref, rtol=0, atol=1e-13 * np.abs(ref).max())
