"""The reference's PETSc boundary on a communicator of several ranks, on the GPU.

The reference builds its FFT matrix on PETSC_COMM_WORLD (src/PCSHELLFft_3D.cxx:34-37) and its
direct-solve driver distributes Un with VecCreateMPI(PETSC_COMM_WORLD, PETSC_DECIDE, N)
(tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:66,100,111), so solve_3D and the
PCSHELL apply run on every rank's block of rows.  Here 2 (and 4) fresh processes share cuda:0;
PETSC_COMM_WORLD is a communicator whose collectives are torch.distributed's (gloo), so
MatCreateFFTHIP backs the FFT matrix with the z-slab plan and its exchanges go through the
communicator.  Each rank runs the reference's calls on its slab:
  setupFFTPrec3D, PCApply -> applyFFT3DPrecTransport, PetscFft3DTransportSolver(ctx, Un, Un)
  (device and host Vecs), solve_3D with a changed Diag, MatMult / MatMultTranspose;
the gathered results are compared with the oracle (1e-10).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, dims, lam, pieces, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from circulantpreconditioner_amd import petsc as P
        from circulantpreconditioner_amd._lib import check, lib
        from oracle import oracle as O
        torch.cuda.set_device(0)
        comm = P.Comm.torch().set_world()
        nx, ny, nz = dims
        N = nx * ny * nz
        b = O.c_fill_uniform(N, 31)
        out = {}
        # --- PCSHELL registered as ToDo.md:1 intends, on PETSC_COMM_WORLD
        ctx = P.make_context(dims, lam)
        pc = P.PC.shell(ctx).setup()
        F = P.Mat(ctx.FFT_MAT, owned=False)
        import ctypes
        dp = ctypes.c_void_p()
        P.PetscCall(lib().MatFFTHIPGetDistPlan(ctx.FFT_MAT, ctypes.byref(dp)))
        assert dp.value, "several ranks: the FFT matrix is backed by the slab plan"
        if pieces:
            check(lib().cfp_dist_plan_set_pieces(dp, pieces))
        diag = P.Vec.borrow(ctx.Diag)
        lo, hi = diag.ownership_range()
        out["range"] = (lo, hi)
        tb = torch.from_numpy(b[lo:hi].copy()).cuda()
        tx = torch.zeros_like(tb)
        vb, vx = P.Vec.from_tensor_mpi(tb, N), P.Vec.from_tensor_mpi(tx, N)
        pc.apply(vb, vx)
        torch.cuda.synchronize()
        out["pc"] = tx.cpu().numpy()
        out["diag"] = diag.array()
        # --- PetscFft3DTransportSolver(ctx, Un, Un): in place, device and host Vecs
        h = (1.0 / nx, 1.0 / ny, 1.0 / nz)
        a, dt = (1.0, 0.5, 0.25), 0.02
        sc = P.StructuredContext(nx, ny, nz, a[0], a[1], a[2], dt, h[0], h[1], h[2], F)
        tu = torch.from_numpy(b[lo:hi].copy()).cuda()
        vu = P.Vec.from_tensor_mpi(tu, N)
        P.PetscFft3DTransportSolver(sc, vu, vu)
        torch.cuda.synchronize()
        out["direct"] = tu.cpu().numpy()
        hu = P.Vec.mpi(N).set_array(b[lo:hi])
        P.PetscFft3DTransportSolver(sc, hu, hu)
        out["direct_host"] = hu.array()
        # --- solve_3D divides by the Diag it is given: a changed Diag after a different symbol
        diag.scale(2.0)
        pc.apply(vb, vx)
        torch.cuda.synchronize()
        out["pc_2diag"] = tx.cpu().numpy()
        out["counts"] = F.solve_counts()
        # --- MatMult / MatMultTranspose: the unnormalised DFT of the distributed grid
        ty = torch.empty_like(tb)
        vy = P.Vec.from_tensor_mpi(ty, N)
        F.mult(vb, vy)
        out["fwd"] = ty.cpu().numpy()
        F.mult_transpose(vb, vy)
        out["bwd"] = ty.cpu().numpy()
        try:  # the slab plan behind FFT_MAT still uses the communicator: destroy is refused
            comm.destroy()
            out["destroy_refused"] = False
        except P.PetscError:
            out["destroy_refused"] = True
        pc.destroy()
        P.set_comm_world(P.PETSC_COMM_SELF)
        comm.destroy()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dims,world,pieces", [((32, 16, 24), 2, 0), ((64, 64, 64), 2, 4), ((32, 32, 16), 4, 2),
                                               ((32, 30, 16), 4, 0), ((64, 40, 32), 4, 0)])  # P | n_y or not
def test_pcshell_and_direct_solver_on_several_ranks(dims, world, pieces, oracle):
    import torch.multiprocessing as mp
    lam = (0.6, 0.15 - 0.1j, 0.02)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, dims, lam, pieces, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    nx, ny, nz = dims
    N = nx * ny * nz

    def gather(key):
        x = np.empty(N, dtype=np.complex128)
        for r in range(world):
            lo, hi = parts[r]["range"]
            x[lo:hi] = parts[r][key]
        return x

    # PETSC_DECIDE rows = whole z-planes of rank r
    for r in range(world):
        assert parts[r]["range"] == (r * N // world, (r + 1) * N // world)
    b = oracle.c_fill_uniform(N, 31)
    d0 = oracle.c_build_diag_transport(dims, lam)
    assert oracle.rel_l2(gather("diag"), d0) < 1e-14
    assert oracle.rel_l2(gather("pc"), oracle.c_solve_3d(d0, b, dims)) < TOL
    lam_d = (1.0 * 0.02 * nx, 0.5 * 0.02 * ny, 0.25 * 0.02 * nz)  # a dt / delta
    ref_d = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam_d), b, dims)
    assert oracle.rel_l2(gather("direct"), ref_d) < TOL
    assert oracle.rel_l2(gather("direct_host"), ref_d) < TOL
    assert oracle.rel_l2(gather("pc_2diag"), oracle.c_solve_3d(2 * d0, b, dims)) < TOL
    for r in range(world):
        assert parts[r]["counts"] == (1, 1)  # own symbol once, then the changed Diag
        assert parts[r]["destroy_refused"]  # PetscMiniCommDestroy while FFT_MAT's slab plan uses it
    bz = b.reshape(nz, ny, nx)
    f = np.fft.fftn(bz).reshape(-1)
    g = (np.fft.ifftn(bz) * N).reshape(-1)
    assert np.linalg.norm(gather("fwd") - f) / np.linalg.norm(f) < 1e-12
    assert np.linalg.norm(gather("bwd") - g) / np.linalg.norm(g) < 1e-12
