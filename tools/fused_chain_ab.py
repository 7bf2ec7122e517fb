"""A/B of the fused Krylov apply at 256^3 (r06): the 3-sweep chain with P1 forming A b (the x-local
transport stencil) and P3 the dots with one or two basis vectors, against the plain chain, in
steady state (back-to-back applies after a settle).  Run under rocprofv3 --kernel-trace; the
per-kernel medians per variant come from tools/fused_chain_ab.py --summary <trace dir>.

    python tools/fused_chain_ab.py [--iters 60]
"""
import argparse
import csv
import glob
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = ["plain", "pre", "pre_x", "pre_post1", "pre_post2", "post1", "plain2"]


def run(iters):
    import numpy as np
    import scipy.sparse as sp
    import torch
    import circulantpreconditioner_amd as cp
    from circulantpreconditioner_amd import transport as T
    from circulantpreconditioner_amd.plan import row_class_form
    n = 256
    dev = torch.device("cuda", 0)
    h = [1.0 / n] * 3
    dt = (1e3 / 3) * T.min_ratio_vol_surf(3, h)
    rp, col, val = T.transport_csr((n, n, n), h, dt, (1.0, 0.0, 0.0), "fixed", 1.0)
    A = sp.csr_matrix((val, col, rp), shape=(n ** 3, n ** 3))
    cls, mask, tab, offs, xl = row_class_form(A.indptr, A.indices, A.data, n)
    st = (torch.from_numpy(cls).to(dev), torch.from_numpy(mask).to(dev),
          torch.from_numpy(np.ascontiguousarray(tab).reshape(-1)).to(dev), [int(o) for o in offs], xl)
    assert np.array_equal(cls.reshape(-1, n), np.broadcast_to(cls[:n], (cls.size // n, n)))
    st_x = st + (torch.from_numpy(cls[:n].copy()).to(dev),)  # classes by x alone
    plan = cp.CirculantPlan((n, n, n), device=0).set_transport_symbol((dt * n, 0.0, 0.0))
    b = torch.empty(n ** 3, dtype=torch.complex128, device=dev)
    cp.fill_uniform(b, 1)
    v0, v1, x = torch.empty_like(b), torch.empty_like(b), torch.empty_like(b)
    cp.fill_uniform(v0, 2)
    cp.fill_uniform(v1, 3)
    calls = {"plain": lambda: plan.apply(b, out=x),
             "pre": lambda: plan.apply_ex(b, x, stencil=st),
             "pre_x": lambda: plan.apply_ex(b, x, stencil=st_x),
             "pre_post1": lambda: plan.apply_ex(b, x, stencil=st_x, dots_with=(v0,)),
             "pre_post2": lambda: plan.apply_ex(b, x, stencil=st_x, dots_with=(v0, v1)),
             "post1": lambda: plan.apply_ex(b, x, dots_with=(v0,)),
             "plain2": lambda: plan.apply(b, out=x)}
    for name in VARIANTS:
        f = calls[name]
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:  # settle
            f()
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        time.sleep(0.05)  # a gap in the trace marks the variant's timed block
        for _ in range(iters):
            f()
        torch.cuda.synchronize()
        time.sleep(0.05)
        print(name, "done", flush=True)


def summary(tdir):
    f = glob.glob(os.path.join(tdir, "*", "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # blocks separated by >= 40 ms gaps: settle, then the timed block, per variant
    blocks, cur, prev = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if prev is not None and s - prev > 40e6:
            blocks.append(cur)
            cur = []
        cur.append(r)
        prev = int(r["End_Timestamp"])
    blocks.append(cur)
    timed = [b for b in blocks if len(b) > 100]
    for name, blk in zip(VARIANTS, timed[1::2] if len(timed) >= 2 * len(VARIANTS) else timed):
        by = {}
        for r in blk:
            k = r["Kernel_Name"].replace("void cfp::", "")[:28]
            by.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        parts = " | ".join(f"{k} {statistics.median(v):.1f} us (n={len(v)})" for k, v in sorted(by.items()))
        print(f"{name:10s} {parts}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--summary", default=None)
    a = ap.parse_args()
    if a.summary:
        summary(a.summary)
    else:
        run(a.iters)
