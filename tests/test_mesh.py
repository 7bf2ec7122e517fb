"""Row f3: unstructured meshes, the mesh -> Cartesian intersection matrix of the
PCSHELL (src/PCSHELLFft_3D.hxx:17, ToDo.md:12) and the transport operator over mesh faces
(src/TransportEquation.cxx:75-133) -- host-side set-up, checked on CPU.

Inputs are the reference's own FVCA6 meshes (tests/golden/meshes/: Gmsh copies that sit beside
the reference's .med files, data only).  Oracle: oracle/mesh.py (independent algorithms:
divergence-theorem geometry, polytope volumes by vertex enumeration).  MEDCoupling,
whose getCrudeMatrix the reference wants, is absent: the intersection matrix is pinned by the
independent oracle and by exact properties (row sums = Cartesian cell volumes, column sums =
mesh cell volumes, the aligned hexahedral mesh gives a permutation) -- parity unpinned against
MEDCoupling itself."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from circulantpreconditioner_amd import CirculantError
from circulantpreconditioner_amd import mesh as M
from circulantpreconditioner_amd import transport as T

from oracle import mesh as OM

MDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "meshes")
MESHES = ["mesh_tetra_0.msh", "mesh_hexa_2.msh", "3DKershawTetra1.msh", "mesh_tetra_1.msh"]


def _path(name):
    return os.path.join(MDIR, name)


@pytest.fixture(scope="module")
def meshes():
    out = {}
    for name in MESHES:
        xyz, cells = OM.read_gmsh(_path(name))
        out[name] = (M.Mesh.read(_path(name)), xyz, cells)
    return out


@pytest.mark.parametrize("name", MESHES)
def test_reader_and_geometry(meshes, name):
    m, xyz, cells = meshes[name]
    info = m.info()
    assert info["nnodes"] == len(xyz) and info["ncells"] == len(cells)
    assert np.allclose(info["bbox"], [0, 1, 0, 1, 0, 1])  # the unit cube of meshes/README.md
    vol, ctr = m.geometry()
    ovol, octr = OM.geometry(xyz, cells)
    np.testing.assert_allclose(vol, ovol, rtol=1e-12, atol=0)
    np.testing.assert_allclose(ctr, octr, rtol=0, atol=1e-13)
    assert abs(vol.sum() - 1.0) < 1e-12  # the cells tile the cube


@pytest.mark.parametrize("name", MESHES)
def test_faces(meshes, name):
    m, xyz, cells = meshes[name]
    c0, c1, meas, nrm = m.faces()
    F = OM.faces(xyz, cells)
    assert len(c0) == len(F)
    # same faces, same cells, measures and normals (matched through the cell pair + the normal)
    def key(c0_, c1_, n_):
        return (c0_, c1_) + tuple(np.round(n_, 8))
    ours = sorted((key(a, b, n) + (m_, tuple(n)) for a, b, m_, n in zip(c0.tolist(), c1.tolist(), meas, nrm)))
    theirs = sorted((key(v[0], v[1], v[3]) + (float(v[2]), tuple(v[3])) for v in F.values()))
    ours = [(o[0], o[1], o[-2], o[-1]) for o in ours]
    theirs = [(t[0], t[1], t[-2], t[-1]) for t in theirs]
    assert [o[:2] for o in ours] == [t[:2] for t in theirs]
    np.testing.assert_allclose([o[2] for o in ours], [t[2] for t in theirs], rtol=1e-12)
    np.testing.assert_allclose([o[3] for o in ours], [t[3] for t in theirs], atol=1e-12)
    border = c1 < 0
    if name == "3DKershawTetra1.msh":
        # this file is not conforming: 832 internal triangles (7.24 of area) match no neighbour
        # face, so they are border faces here exactly as in the oracle's independent face loop
        assert meas[border].sum() > 6.0
    else:
        assert abs(meas[border].sum() - 6.0) < 1e-11  # the cube's surface
    np.testing.assert_allclose(np.linalg.norm(nrm, axis=1), 1.0, atol=1e-14)
    # every cell is closed: sum over its faces of |F| n_out = 0
    acc = np.zeros((m.ncells, 3))
    np.add.at(acc, c0, meas[:, None] * nrm)
    np.add.at(acc, c1[~border], -(meas[~border, None] * nrm[~border]))
    assert np.abs(acc).max() < 1e-13
    assert abs(m.min_ratio_vol_surf() - OM.min_ratio_vol_surf(xyz, cells)) < 1e-15


CRUDE_CASES = [("mesh_tetra_0.msh", (4, 4, 4)), ("mesh_tetra_0.msh", (3, 5, 2)), ("mesh_hexa_2.msh", (3, 3, 3)),
               ("3DKershawTetra1.msh", (2, 3, 2))]


@pytest.mark.parametrize("name,dims", CRUDE_CASES, ids=lambda v: str(v))
def test_crude_matrix_vs_polytope_oracle(meshes, name, dims):
    m, xyz, cells = meshes[name]
    rp, cl, vl = m.crude_matrix(dims)
    N = int(np.prod(dims))
    V = sp.csr_matrix((vl, cl, rp), shape=(N, m.ncells))
    only = None
    if len(cells) > 2000:  # the oracle is slow: every 8th cell of the large mesh
        only = list(range(0, len(cells), 8))
        V = V[:, only]
    W = OM.crude_matrix(xyz, cells, dims, only=only)
    if only is not None:
        W = W[:, only]
    assert abs(V - W).max() <= 1e-12 * (1.0 / N)
    # entries that one side dropped as touching-only are below the threshold on the other
    assert abs(V.nnz - W.nnz) <= max(2, W.nnz // 1000)


@pytest.mark.parametrize("name,dims", [("mesh_tetra_1.msh", (8, 8, 8)), ("3DKershawTetra1.msh", (6, 5, 7)),
                                       ("mesh_hexa_2.msh", (5, 3, 7)), ("mesh_tetra_0.msh", (1, 1, 1))])
def test_crude_matrix_sums(meshes, name, dims):
    m, _, _ = meshes[name]
    rp, cl, vl = m.crude_matrix(dims)
    N = int(np.prod(dims))
    V = sp.csr_matrix((vl, cl, rp), shape=(N, m.ncells))
    vol, _ = m.geometry()
    np.testing.assert_allclose(np.asarray(V.sum(axis=1)).ravel(), 1.0 / N, rtol=1e-11)
    np.testing.assert_allclose(np.asarray(V.sum(axis=0)).ravel(), vol, rtol=1e-11)
    assert np.all(np.diff(rp) >= 0) and rp[-1] == len(cl)
    for r in range(N):
        assert np.all(np.diff(cl[rp[r]:rp[r + 1]]) > 0)


def test_aligned_hexa_is_a_permutation(meshes):
    m, _, _ = meshes["mesh_hexa_2.msh"]  # 4^3 uniform hexahedra
    rp, cl, vl = m.crude_matrix((4, 4, 4))
    assert np.all(np.diff(rp) == 1) and sorted(cl.tolist()) == list(range(64))
    np.testing.assert_allclose(vl, 1 / 64, rtol=1e-13)
    _, ctr = m.geometry()
    # Cartesian cell i holds the mesh cell whose barycentre is its centre
    idx = np.arange(64)
    centre = np.stack([(idx % 4 + 0.5) / 4, (idx // 4 % 4 + 0.5) / 4, (idx // 16 + 0.5) / 4], axis=1)
    np.testing.assert_allclose(ctr[cl], centre, atol=1e-14)


@pytest.mark.parametrize("sign", ["reference", "fixed"])
@pytest.mark.parametrize("name", ["mesh_tetra_0.msh", "mesh_hexa_2.msh", "3DKershawTetra1.msh"])
def test_transport_csr_vs_face_loop(meshes, name, sign):
    m, xyz, cells = meshes[name]
    dt, a = 0.37, (1.0, -0.4, 0.25)
    rp, cl, vl = m.transport_csr(dt, a, sign, shift=1.0)
    n = m.ncells
    A = sp.csr_matrix((vl, cl, rp), shape=(n, n))
    B = OM.transport_csr(xyz, cells, dt, a, sign, shift=1.0)
    assert abs(A - B).max() <= 1e-13 * abs(B).max()
    assert all(rp[j] < rp[j + 1] and j in cl[rp[j]:rp[j + 1]] for j in range(n))  # diagonal stored


def test_aligned_hexa_transport_equals_cartesian(meshes):
    """On the uniform hexahedral mesh the face loop must give the Cartesian operator (after the
    cell permutation), which is itself pinned to the circulant golden fixtures."""
    m, _, _ = meshes["mesh_hexa_2.msh"]
    rp, cl, vl = m.crude_matrix((4, 4, 4))
    perm = cl  # Cartesian row r holds mesh cell perm[r]
    dt, a = 0.37, (1.0, -0.4, 0.25)
    for sign in ("reference", "fixed"):
        mr, mc, mv = m.transport_csr(dt, a, sign, shift=1.0)
        A = sp.csr_matrix((mv, mc, mr), shape=(64, 64))[perm][:, perm]
        cr, cc, cv = T.transport_csr((4, 4, 4), (0.25, 0.25, 0.25), dt, a, sign, shift=1.0)
        C = sp.csr_matrix((cv, cc, cr), shape=(64, 64))
        assert abs(A - C).max() < 1e-13


def test_mesh_from_arrays_and_errors(tmp_path):
    # one unit cube as 1 hexahedron and as 5 tetrahedra: same volume, same bbox
    xyz = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], float)
    hexm = M.Mesh.from_arrays(xyz, [list(range(8))])
    v, c = hexm.geometry()
    assert abs(v[0] - 1) < 1e-15 and np.allclose(c[0], 0.5)
    tets = [(0, 1, 3, 4), (1, 2, 3, 6), (1, 4, 5, 6), (3, 4, 6, 7), (1, 3, 4, 6)]
    tm = M.Mesh.from_arrays(xyz, tets)
    v, _ = tm.geometry()
    assert abs(v.sum() - 1) < 1e-15
    rp, cl, vl = tm.crude_matrix((2, 2, 2))
    assert abs(vl.sum() - 1) < 1e-14
    with pytest.raises(CirculantError):
        M.Mesh.from_arrays(xyz, [(0, 1, 2)])  # 3-node cell
    with pytest.raises(CirculantError):
        M.Mesh.from_arrays(xyz, [(0, 1, 2, 99)])  # bad node
    with pytest.raises(CirculantError):
        M.Mesh.from_arrays(xyz, [(0, 1, 2, 3)])  # flat tet (z = 0 for all four)
    with pytest.raises(CirculantError):
        M.Mesh.read(str(tmp_path / "missing.msh"))
    bad = tmp_path / "bad.msh"
    bad.write_text("$MeshFormat\n4.1 0 8\n$EndMeshFormat\n")
    with pytest.raises(CirculantError):
        M.Mesh.read(str(bad))


def test_remap_matrices_host(meshes):
    m, xyz, cells = meshes["mesh_tetra_0.msh"]
    toCart, toMesh = m.remap((3, 3, 3))
    from circulantpreconditioner_amd import petsc as P
    n = m.ncells
    b = np.random.default_rng(3).standard_normal(n) + 1j * np.random.default_rng(4).standard_normal(n)
    vb = P.Vec.seq(n).set_array(b)
    vc = P.Vec.seq(27)
    toCart.mult(vb, vc)
    vm = P.Vec.seq(n)
    toMesh.mult(vc, vm)
    R, B = OM.remap_matrices(OM.crude_matrix(xyz, cells, (3, 3, 3)))
    np.testing.assert_allclose(vc.array(), R @ b, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(vm.array(), B @ (R @ b), rtol=1e-12, atol=1e-12)
    # constants are preserved both ways (intensive remap)
    vb.set(2.5)
    toCart.mult(vb, vc)
    np.testing.assert_allclose(vc.array(), 2.5, rtol=1e-13)
