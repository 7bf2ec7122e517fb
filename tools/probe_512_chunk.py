#!/usr/bin/env python3
"""VERDICT r03 item 2, option (ii): 512^3 (BASELINE config 5's grid) with the x and y passes run
over blocks of C z-planes (cfp_plan_set_chunking), so that each block's y pass reads what its x
pass just wrote while it is still in the 256 MB Infinity Cache (a 16-plane block is 64 MiB).
PCApply/s per chunk size against the unchunked 5-pass schedules, same output.  GPU only."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
lam = (0.6, 0.15, 0.02)
N = n ** 3
b = torch.empty(N, dtype=torch.complex128, device="cuda")
cp.fill_uniform(b, 20251017)
x = torch.empty_like(b)
ref = None
cases = [("five", 0), ("five_y", 0), ("five", 4), ("five", 8), ("five", 16), ("five", 32), ("five", 64)]
for rnd in range(2):
    for sched, C in cases:
        with cp.CirculantPlan((n, n, n)) as p:
            p.set_transport_symbol(lam).set_schedule(sched).set_chunking(C)
            for _ in range(3):
                p.apply(b, out=x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 10
            e0.record()
            for _ in range(it):
                p.apply(b, out=x)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / it
            if ref is None:
                ref = x.clone()
            err = float(torch.linalg.vector_norm(x - ref) / torch.linalg.vector_norm(ref))
            print(json.dumps({"round": rnd, "schedule": sched, "chunk_planes": C, "ms": round(ms, 4),
                              "PCApply_per_s": round(1e3 / ms, 2), "rel_diff_vs_first": err,
                              "launches": len(p.passes())}), flush=True)
