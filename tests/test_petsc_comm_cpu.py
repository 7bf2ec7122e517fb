"""The stand-in PETSc's communicators on CPU: world_size-2 and -3 gloo processes.

A communicator of several ranks (PetscMiniCommCreate with torch.distributed collectives) as
PETSC_COMM_WORLD; VecCreateMPI(PETSC_COMM_WORLD, PETSC_DECIDE, N) gives each rank its
PETSC_DECIDE block of rows (tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:66),
and VecDot / VecNorm / VecMDot reduce over the ranks.  Host vectors only: no GPU work.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, P, port, N, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from circulantpreconditioner_amd import petsc as Pm
        comm = Pm.Comm.torch().set_world()
        assert (comm.size, comm.rank) == (P, rank)
        rng = np.random.default_rng(7)
        a = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        b = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        va, vb = Pm.Vec.mpi(N), Pm.Vec.mpi(N)
        lo, hi = va.ownership_range()
        assert va.size == N and va.local_size == hi - lo
        va.set_array(a[lo:hi])
        vb.set_array(b[lo:hi])
        out = {"range": (lo, hi), "dot": va.dot(vb), "n2": va.norm(Pm.NORM_2), "n1": va.norm(Pm.NORM_1),
               "ninf": va.norm(Pm.NORM_INFINITY)}
        # VecSetValue with global indices keeps this rank's rows
        vc = Pm.Vec.mpi(N).set(0.0)
        for i in range(N):
            Pm.PetscCall(Pm.lib().VecSetValue(vc.h, i, Pm._S(complex(i, -i)), Pm.INSERT_VALUES))
        out["setvalues"] = np.array_equal(vc.array(), np.arange(lo, hi) * (1 - 1j))
        # the reference MPI driver's pattern (TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:
        # 69-92): rank 0 alone sets every global row, VecAssemblyBegin/End ships them to their owners
        ve = Pm.Vec.mpi(N).set(0.0)
        if rank == 0:
            for i in range(N):
                Pm.PetscCall(Pm.lib().VecSetValue(ve.h, i, Pm._S(complex(2 * i, 1)), Pm.INSERT_VALUES))
        Pm.PetscCall(Pm.lib().VecAssemblyBegin(ve.h))
        Pm.PetscCall(Pm.lib().VecAssemblyEnd(ve.h))
        out["rank0_fill"] = np.array_equal(ve.array(), 2 * np.arange(lo, hi) + 1j)
        # ADD_VALUES from every rank to every row (own rows at once, the others at assembly)
        vf = Pm.Vec.mpi(N).set(0.5)
        for i in range(N):
            Pm.PetscCall(Pm.lib().VecSetValue(vf.h, i, Pm._S(complex(rank + 1, 0)), Pm.ADD_VALUES))
        Pm.PetscCall(Pm.lib().VecAssemblyBegin(vf.h))
        Pm.PetscCall(Pm.lib().VecAssemblyEnd(vf.h))
        out["add_all"] = np.array_equal(vf.array(), np.full(hi - lo, 0.5 + P * (P + 1) / 2))
        out["max"] = comm.allreduce([rank, -rank], op=1).tolist()
        # the local sizes given, N determined (PETSC_DETERMINE) and the row start from them
        vd = Pm.Vec.mpi(-1, nlocal=rank + 1)
        out["determine"] = (vd.size, vd.ownership_range())
        Pm.set_comm_world(Pm.PETSC_COMM_SELF)
        comm.destroy()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,N", [(2, 1000), (3, 1001)])
def test_comm_vec_reductions(P, N):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, P, port, N, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(P))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7)
    a = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    b = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    # PETSC_DECIDE: N // P rows, the first N % P ranks one more
    start = 0
    for r in range(P):
        n = N // P + (1 if r < N % P else 0)
        assert res[r]["range"] == (start, start + n)
        start += n
        assert res[r]["dot"] == pytest.approx(np.vdot(b, a), rel=1e-13)  # PETSc: y^H x
        assert res[r]["n2"] == pytest.approx(np.linalg.norm(a), rel=1e-13)
        assert res[r]["n1"] == pytest.approx(np.abs(a.real).sum() + np.abs(a.imag).sum(), rel=1e-13)
        assert res[r]["ninf"] == pytest.approx(np.abs(a).max(), rel=1e-13)
        assert res[r]["setvalues"]
        assert res[r]["rank0_fill"] and res[r]["add_all"]
        assert res[r]["max"] == [P - 1, 0]
        tot = P * (P + 1) // 2
        assert res[r]["determine"] == (tot, (r * (r + 1) // 2, r * (r + 1) // 2 + r + 1))
