"""N > 1 path on CPU: world_size-2 (and 4) gloo runs of the z-slab decomposition.

Each rank takes its slab from the library's host-side layout (cfp_slab_layout: PETSc's
PETSC_DECIDE rows = FFTW-MPI z-slabs), performs the same schedule as cfp_dist.hip --
x/y forward passes writing per-peer chunks [nz_l][ny_l][nx], all-to-all, z forward /
divide by the rank-local closed-form symbol / z inverse, all-to-all back, y/x inverse,
1/N -- with numpy FFTs standing in for the HIP axis passes, and the exchange through
torch.distributed (gloo).  The gathered result must equal the single-process oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _alltoall(chunks_out, P):
    """list of P equal numpy chunks -> list of P received chunks (gloo: isend/irecv pairs)."""
    r = dist.get_rank()
    recv = [None] * P
    reqs = []
    bufs = []
    for q in range(P):
        if q == r:
            recv[q] = chunks_out[q].copy()
            continue
        t_out = torch.from_numpy(np.ascontiguousarray(chunks_out[q]))
        t_in = torch.empty_like(t_out)
        bufs.append((q, t_in))
        reqs.append(dist.isend(t_out, q))
        reqs.append(dist.irecv(t_in, q))
    for rq in reqs:
        rq.wait()
    for q, t in bufs:
        recv[q] = t.numpy()
    return recv


def _worker(rank, P, port, dims, lam, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from circulantpreconditioner_amd.distributed import slab_layout
        from oracle import oracle as O
        nx, ny, nz = dims
        L = slab_layout(dims, P, rank)
        nzl, nyl = L["nz_local"], L["ny_local"]
        b = O.c_fill_uniform(L["local_size"], 77, L["local_offset"]).reshape(nzl, ny, nx)
        # x, y forward on the local z-planes
        a = np.fft.fft(np.fft.fft(b, axis=2), axis=1)
        # y-forward output written straight into per-peer chunks: chunk q = y in [q nyl, (q+1) nyl)
        send = [a[:, q * nyl:(q + 1) * nyl, :] for q in range(P)]
        recv = _alltoall(send, P)
        zs = np.concatenate(recv, axis=0)  # [nz][nyl][nx], z = p nzl + iz
        assert zs.shape == (nz, nyl, nx)
        # z forward, divide by the closed-form symbol at global frequencies, z inverse
        f = np.fft.fft(zs, axis=0)
        kz, kyl, kx = np.meshgrid(np.arange(nz), np.arange(nyl), np.arange(nx), indexing="ij")
        ky = L["y0"] + kyl
        d = np.ones_like(f)
        for l, k, n in ((lam[0], kx, nx), (lam[1], ky, ny), (lam[2], kz, nz)):
            if n > 1:
                d = d + l * (1 - np.exp(-2j * np.pi * k / n))
        g = np.fft.ifft(f / d, axis=0) * nz  # unnormalised backward
        send = [g[p * nzl:(p + 1) * nzl] for p in range(P)]
        recv = _alltoall(send, P)  # from q: [nzl][nyl (q's y)][nx]
        h = np.concatenate(recv, axis=1)  # [nzl][ny][nx]
        x = np.fft.ifft(np.fft.ifft(h, axis=1), axis=2) * (ny * nx) / (nx * ny * nz)
        q.put((rank, L["local_offset"], x.reshape(-1)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,dims", [(2, (16, 8, 12)), (2, (10, 6, 4)), (4, (8, 16, 8))])
def test_slab_decomposition_gloo(P, dims, oracle):
    lam = (0.6, 0.15 + 0.05j, 0.02)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, P, port, dims, lam, q)) for r in range(P)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=120) for _ in range(P)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nx, ny, nz = dims
    N = nx * ny * nz
    x = np.empty(N, dtype=np.complex128)
    for _, off, part in parts:
        x[off:off + part.size] = part
    b = oracle.c_fill_uniform(N, 77)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    assert oracle.rel_l2(x, ref) < 1e-12
