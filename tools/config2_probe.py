#!/usr/bin/env python3
"""Why does bench.py's config2_128 leg (after the 256^3 headline) read ~17.1k applies/s when a
--grid 128 process reads 18.4-19k?  Runs a 256^3 warm phase, then times the 128^3 apply with
several settle lengths and with a host-side clock beside the events (host-bound check)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402
from bench import event_ms  # noqa: E402

LAM = (0.6, 0.15, 0.02)


def leg(g, settle, iters=2000):
    with cp.CirculantPlan(g, device=0) as p:
        p.set_transport_symbol(LAM)
        b = torch.empty(g[0] * g[1] * g[2], dtype=torch.complex128, device="cuda:0")
        cp.fill_uniform(b, 20251017)
        x = torch.empty_like(b)
        ms = event_ms(lambda: p.apply(b, out=x), iters, settle)
        t0 = time.perf_counter()
        for _ in range(iters):
            p.apply(b, out=x)
        host = (time.perf_counter() - t0) / iters * 1e3  # enqueue time per call (ms)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / iters * 1e3
    return ms, host, wall


print("128^3 cold process:", ["%.4f" % v for v in leg([128] * 3, 150)], flush=True)
print("256^3 warm phase:", ["%.4f" % v for v in leg([256] * 3, 2000, 200)], flush=True)
for settle in (150, 500, 1500):
    print(f"128^3 after 256^3, settle {settle} ms:", ["%.4f" % v for v in leg([128] * 3, settle)], flush=True)
