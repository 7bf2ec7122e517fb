"""N > 1 path on CPU: world_size-2 (and 4) gloo runs of the library's own slab schedule.

Each rank asks the library for the steps its cfp_dist_plan_apply runs
(cfp_slab_step_info: the same host code that builds the GPU plan's launches -- axis, mode,
column and point addressing of every pass, including the y passes that write and read
the per-peer exchange chunks, and the two all-to-alls) and replays them on the CPU: an axis
pass becomes a gather through the step's own addressing, a numpy DFT, a divide by the
closed-form symbol at the step's global frequencies and a scatter; an all-to-all goes
through torch.distributed (gloo).  The gathered result must equal the single-process
oracle, so a wrong stride, chunk offset, step order or exchange direction in the library's
schedule fails here without a GPU.
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


def _index(st, side, g, k):
    """Element index of (column g, point k) on one side of a step (circulant_fft_dist.h)."""
    return ((g % st["inner_n"]) * st[side + "_inner"] + (g // st["inner_n"]) * st[side + "_outer"]
            + (k // st[side + "_seg_len"]) * st[side + "_seg_stride"] + (k % st[side + "_seg_len"]) * st[side + "_pt"])


def _replay_pass(st, bufs, L, dims, lam):
    g = np.arange(st["ncols"])[:, None]
    k = np.arange(st["n"])[None, :]
    src = bufs[st["src"]][_index(st, "in", g, k)]  # [ncols][n]
    n = st["n"]
    if st["mode"] == 0:  # forward, e^{-}
        out = np.fft.fft(src, axis=1)
    elif st["mode"] == 1:  # unnormalised backward, e^{+}
        out = np.fft.ifft(src, axis=1) * n
    elif st["mode"] == 2:  # DFT, divide by the separable symbol, IDFT (the z pass of the slab)
        assert st["axis"] == 2
        nx, ny, nz = dims
        kx = g % nx
        ky = L["y0"] + g // nx  # z-pass columns g = ix + nx * iyl of the y-slab
        d = np.ones((st["ncols"], n), dtype=np.complex128)
        for lv, kk, nn in ((lam[0], kx, nx), (lam[1], ky, ny), (lam[2], k, nz)):
            if nn > 1:
                d = d + lv * (1 - np.exp(-2j * np.pi * kk / nn))
        out = np.fft.ifft(np.fft.fft(src, axis=1) / d, axis=1) * n
    else:
        raise AssertionError(f"unexpected mode {st['mode']}")
    bufs[st["dst"]][_index(st, "out", g, k)] = out * st["scale"]


def _worker(rank, P, port, dims, lam, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from circulantpreconditioner_amd.distributed import slab_layout, slab_steps
        from oracle import oracle as O
        L = slab_layout(dims, P, rank)
        steps = slab_steps(dims, P, rank)
        assert [s["kind"] for s in steps].count(1) == 2, "two all-to-alls per apply"
        n = L["local_size"]
        b = O.c_fill_uniform(n, 77, L["local_offset"])
        bufs = {0: b.copy(), 1: np.full(n, np.nan + 0j), 2: np.full(n, np.nan + 0j)}
        for st in steps:
            if st["kind"] == 0:
                _replay_pass(st, bufs, L, dims, lam)
                continue
            c = L["chunk"]
            src = torch.view_as_real(torch.from_numpy(np.ascontiguousarray(bufs[st["src"]]))).contiguous()
            dst = torch.empty_like(src)
            dist.all_to_all_single(dst, src)  # chunk q -> rank q, stored as chunk `rank`
            assert dst.shape[0] == P * c
            bufs[st["dst"]][:] = torch.view_as_complex(dst).numpy()
        q.put((rank, L["local_offset"], bufs[1].copy(), np.array_equal(bufs[0], b)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,dims", [(2, (16, 8, 12)), (2, (10, 6, 4)), (4, (8, 16, 8)), (2, (1, 4, 6))])
def test_slab_schedule_gloo(P, dims, oracle):
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
    for _, off, part, b_untouched in parts:
        assert b_untouched, "the apply must not write b"
        x[off:off + part.size] = part
    b = oracle.c_fill_uniform(N, 77)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    assert oracle.rel_l2(x, ref) < 1e-12


def test_slab_steps_shape():
    """The step list itself: x/y forward, all-to-all, fused z, all-to-all, y/x inverse, 1/N last."""
    from circulantpreconditioner_amd.distributed import slab_steps
    st = slab_steps((16, 8, 12), 2, 1)
    assert [(s["kind"], s["axis"], s["mode"]) for s in st] == [
        (0, 0, 0), (0, 1, 0), (1, -1, -1), (0, 2, 2), (1, -1, -1), (0, 1, 1), (0, 0, 1)]
    assert [s["scale"] for s in st if s["kind"] == 0][-1] == pytest.approx(1.0 / (16 * 8 * 12))
    with pytest.raises(Exception):
        slab_steps((16, 8, 12), 5, 0)  # 5 does not divide nz
