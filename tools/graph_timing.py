#!/usr/bin/env python3
"""Host-synchronous PCApply latency with and without HIP-graph replay (cfp_plan_set_graph).

Each timed call is apply + stream synchronize, as inside GMRES or the reference's direct
time loop (tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx:111), where the host
waits for every apply; the bench's queued throughput loop hides launch cost, this does not.

    python3 tools/graph_timing.py [--grids 32 64 100 128 256] [--iters 400]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", type=int, nargs="+", default=[32, 64, 100, 128, 256])
    ap.add_argument("--iters", type=int, default=400)
    args = ap.parse_args()
    import torch

    import circulantpreconditioner_amd as cp

    for n in args.grids:
        N = n ** 3
        b = torch.empty(N, dtype=torch.complex128, device="cuda:0")
        cp.fill_uniform(b, 20251017)
        x = torch.empty_like(b)
        res = {"grid": n}
        ref = None
        for mode in ("eager", "graph", "eager2", "graph2"):
            with cp.CirculantPlan((n, n, n), device=0) as plan:
                plan.set_transport_symbol((0.6, 0.15, 0.02)).set_graph(mode.startswith("graph"))
                iters = max(50, args.iters if n < 256 else args.iters // 4)
                for _ in range(20):
                    plan.apply(b, out=x)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    plan.apply(b, out=x)
                    torch.cuda.synchronize()
                res[mode + "_us"] = round((time.perf_counter() - t0) / iters * 1e6, 2)
                if ref is None:
                    ref = x.clone()
                else:
                    assert torch.equal(ref, x), f"{mode} result differs at {n}^3"
                res["passes"] = len(plan.passes())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
