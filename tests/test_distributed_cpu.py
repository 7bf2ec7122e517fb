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
    base = st["src_off"] if side == "in" else st["dst_off"]
    return (base + (g % st["inner_n"]) * st[side + "_inner"] + (g // st["inner_n"]) * st[side + "_outer"]
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


def _replay_repack(st, bufs, L, dims):
    """natural planes [planes][ny][nx] <-> per-peer chunks (circulant_fft_dist.h, kind 3)"""
    nx, ny, _ = dims
    nyp, c = L["ny_chunk"], L["chunk"]
    i = np.arange(st["ncols"] * ny * nx)
    x, row = i % nx, i // nx
    y, z = row % ny, row // ny
    ci = (y // nyp) * c + (z * nyp + y % nyp) * nx + x
    src, dst = bufs[st["src"]], bufs[st["dst"]]
    if st["axis"]:  # to chunks
        dst[st["dst_off"] + ci] = src[st["src_off"] + i]
    else:
        dst[st["dst_off"] + i] = src[st["src_off"] + ci]


def _exchange_piece(st, bufs, P):
    """peer q gets src[q chunk + off, + cnt) and stores it at dst[rank chunk + off]"""
    c, off, cnt = st["chunk"], st["ex_off"], st["ex_cnt"]
    src = bufs[st["src"]]
    send = np.concatenate([src[q * c + off:q * c + off + cnt] for q in range(P)])
    st_send = torch.view_as_real(torch.from_numpy(send)).contiguous()
    recv = torch.empty_like(st_send)
    dist.all_to_all_single(recv, st_send)
    r = torch.view_as_complex(recv).numpy()
    for q in range(P):
        bufs[st["dst"]][q * c + off:q * c + off + cnt] = r[q * cnt:(q + 1) * cnt]


def _replay(steps, bufs, L, dims, lam, P):
    for st in steps:
        if st["kind"] == 0:
            _replay_pass(st, bufs, L, dims, lam)
        elif st["kind"] == 1:
            _exchange_piece(st, bufs, P)
        elif st["kind"] == 3:
            _replay_repack(st, bufs, L, dims)
        else:
            raise AssertionError("3-sweep stages are checked for layout only")


def _worker(rank, P, port, dims, lam, pieces, lists, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from circulantpreconditioner_amd.distributed import slab_layout, slab_steps
        from oracle import oracle as O
        L = slab_layout(dims, P, rank)
        n = L["local_size"]
        b = O.c_fill_uniform(n, 77, L["local_offset"])
        out = {}
        for lst in lists:
            steps = slab_steps(dims, P, rank, schedule="five", pieces=pieces, list_=lst)
            nex = [s["kind"] for s in steps].count(1)
            assert nex == (2 * pieces if lst == "apply" else 2), (lst, nex)
            w = L["work_size"]
            bufs = {0: b.copy(), 1: np.full(n, np.nan + 0j), 2: np.full(w, np.nan + 0j), 3: np.full(w, np.nan + 0j)}
            _replay(steps, bufs, L, dims, lam, P)
            out[lst] = (bufs[1].copy(), np.array_equal(bufs[0], b))
        q.put((rank, L["local_offset"], out))
    finally:
        dist.destroy_process_group()


def _run(P, dims, lam, pieces, lists):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, P, port, dims, lam, pieces, lists, q)) for r in range(P)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=120) for _ in range(P)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nx, ny, nz = dims
    N = nx * ny * nz
    res = {}
    for lst in lists:
        x = np.empty(N, dtype=np.complex128)
        for _, off, out in parts:
            part, b_untouched = out[lst]
            assert b_untouched, "the apply must not write b"
            x[off:off + part.size] = part
        res[lst] = x
    return res


@pytest.mark.parametrize("P,dims,pieces", [(2, (16, 8, 12), 1), (2, (10, 6, 4), 1), (4, (8, 16, 8), 1),
                                           (2, (1, 4, 6), 1), (2, (16, 8, 12), 2), (2, (16, 8, 12), 3),
                                           (2, (16, 8, 12), 6), (4, (8, 16, 8), 2), (2, (10, 6, 8), 4),
                                           (2, (1, 4, 6), 3),
                                           # P does not divide ny (FFTW-MPI's ceil(ny / P) row blocks)
                                           (2, (8, 7, 6), 1), (4, (16, 10, 8), 1), (4, (16, 10, 8), 2),
                                           (4, (6, 3, 8), 1), (3, (5, 7, 9), 3), (4, (64, 30, 32), 1)])
def test_slab_schedule_gloo(P, dims, pieces, oracle):
    """The library's apply step list (five passes, `pieces` exchange pieces), replayed across
    P gloo processes, against the oracle's full-grid solve."""
    lam = (0.6, 0.15 + 0.05j, 0.02)
    x = _run(P, dims, lam, pieces, ["apply"])["apply"]
    N = int(np.prod(dims))
    b = oracle.c_fill_uniform(N, 77)
    ref = oracle.c_solve_3d(oracle.c_build_diag_transport(dims, lam), b, dims)
    assert oracle.rel_l2(x, ref) < 1e-12


@pytest.mark.parametrize("P,dims", [(2, (16, 8, 12)), (4, (8, 16, 8))])
def test_slab_transforms_gloo(P, dims):
    """The distributed MatMult / MatMultTranspose step lists (x, y -> chunks, exchange, z,
    exchange back, repack): the unnormalised 3-D DFT of the slab-distributed grid in natural
    order, as numpy's fftn / ifftn * N."""
    from oracle import oracle as O
    res = _run(P, dims, (0, 0, 0), 1, ["forward", "backward"])
    nx, ny, nz = dims
    N = nx * ny * nz
    b = O.c_fill_uniform(N, 77).reshape(nz, ny, nx)
    f = np.fft.fftn(b).reshape(-1)
    g = (np.fft.ifftn(b) * N).reshape(-1)
    assert np.linalg.norm(res["forward"] - f) / np.linalg.norm(f) < 1e-12
    assert np.linalg.norm(res["backward"] - g) / np.linalg.norm(g) < 1e-12


def test_slab_steps_shape():
    """The step list itself: x/y forward, all-to-all, fused z, all-to-all, y/x inverse, 1/N last."""
    from circulantpreconditioner_amd.distributed import slab_steps
    st = slab_steps((16, 8, 12), 2, 1)
    assert [(s["kind"], s["axis"], s["mode"]) for s in st] == [
        (0, 0, 0), (0, 1, 0), (1, -1, -1), (0, 2, 2), (1, -1, -1), (0, 1, 1), (0, 0, 1)]
    assert [s["scale"] for s in st if s["kind"] == 0][-1] == pytest.approx(1.0 / (16 * 8 * 12))
    with pytest.raises(Exception):
        slab_steps((16, 8, 12), 5, 0)  # 5 does not divide nz
    with pytest.raises(Exception):
        slab_steps((16, 8, 12), 2, 0, pieces=4)  # 4 does not divide the 6 local planes


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_slab_steps_pieces_layout(P):
    """Pieces: the forward pieces cover every chunk exactly once and each waits for the y pass
    of its own block; the backward inverse passes of block k wait for piece k; 1/N rides on the
    last launch of every block; the old round-2 entry points still describe the one-piece list."""
    from circulantpreconditioner_amd.distributed import slab_layout, slab_steps
    dims = (32, 16, 64)
    for r in range(P):
        L = slab_layout(dims, P, r)
        for K in [k for k in (1, 2, 4, 8) if L["nz_local"] % k == 0]:
            st = slab_steps(dims, P, r, pieces=K)
            ex = [i for i, s in enumerate(st) if s["kind"] == 1]
            assert len(ex) == 2 * K
            fwd, bwd = ex[:K], ex[K:]
            for half in (fwd, bwd):
                cover = sorted((st[i]["ex_off"], st[i]["ex_cnt"]) for i in half)
                assert cover[0][0] == 0 and sum(c for _, c in cover) == L["chunk"]
                assert all(a + c == b for (a, c), (b, _) in zip(cover, cover[1:]))
            for k, i in enumerate(fwd):
                w = st[st[i]["wait"]]
                assert w["kind"] == 0 and w["axis"] == 1 and w["mode"] == 0
                assert w["dst_off"] == st[i]["ex_off"]  # the y pass that wrote this piece
            z = [i for i, s in enumerate(st) if s["kind"] == 0 and s["axis"] == 2]
            assert len(z) == 1 and st[z[0]]["wait"] == fwd[-1]
            for i in bwd:
                assert st[i]["wait"] == z[0]
                y = st[i + 1]
                assert y["kind"] == 0 and y["axis"] == 1 and y["mode"] == 1 and y["wait"] == i
                assert y["src_off"] == st[i]["ex_off"]
            last = [s for s in st if s["kind"] == 0 and s["axis"] == 0 and s["mode"] == 1]
            assert len(last) == K and all(s["scale"] == pytest.approx(1.0 / (32 * 16 * 64)) for s in last)
            # K > 1 lands the exchanges in W2 (no pass writes what a piece reads or receives)
            m = 1 if K == 1 else 3
            assert all(st[i]["dst"] == m for i in fwd) and all(st[i]["src"] == m for i in bwd)


@pytest.mark.parametrize("n,P", [(256, 1), (256, 2), (256, 4), (256, 8), (256, 16), (512, 2), (512, 8), (512, 16)])
@pytest.mark.parametrize("pieces", [1, 2, 4])
def test_slab_three_sweep_layout(n, P, pieces):
    """the 3-sweep slab schedule (AUTO at 256^3 and 512^3 for every P | 32 up to 16
    since r05) is described too: P1 blocks write block k of every chunk (offsets k B nyl nx), P2
    runs on the rank's k1 rows [r nyl / N2, ...) (N2 = 8 at 256^3, 16 at 512^3), the chunk and row
    bookkeeping the kernels receive, and the exchange pieces tile the chunk."""
    from circulantpreconditioner_amd.distributed import slab_layout, slab_steps
    dims = (n, n, n)
    n2 = 16 if n == 512 else 8
    for r in range(P):
        L = slab_layout(dims, P, r)
        st = slab_steps(dims, P, r, schedule="auto", pieces=pieces)
        kinds = [s["kind"] for s in st]
        assert kinds.count(2) == 2 * pieces + 1 and kinds.count(1) == 2 * pieces and kinds.count(0) == 0
        B = L["nz_local"] // pieces
        p1 = [s for s in st if s["kind"] == 2 and s["axis"] == 0]
        p3 = [s for s in st if s["kind"] == 2 and s["axis"] == 2]
        (p2,) = [s for s in st if s["kind"] == 2 and s["axis"] == 1]
        for k, (a, c) in enumerate(zip(p1, p3)):
            assert a["ncols"] == B and c["ncols"] == B
            assert a["src_off"] == k * B * n * n and a["dst_off"] == k * B * L["ny_local"] * n
            assert c["src_off"] == k * B * L["ny_local"] * n and c["dst_off"] == k * B * n * n
            assert c["scale"] == pytest.approx(1.0 / n ** 3)
        assert p2["k1_off"] == r * (L["ny_local"] // n2) and 1 << p2["lnyl"] == L["ny_local"]
        assert all(s["chunk"] == L["chunk"] == L["nz_local"] * L["ny_local"] * n for s in st)
        ex = [s for s in st if s["kind"] == 1]
        assert sum(s["ex_cnt"] for s in ex[:pieces]) == L["chunk"]
    # the round-2 entry point describes the five-pass list only (its docstring says so)
    assert all(s["kind"] in (0, 1) for s in slab_steps(dims, 2, 0))
