#!/usr/bin/env python3
"""A/B of apply schedules / 3-sweep shapes on one grid (GPU only; measurement tool, not a test).

  python tools/ab_sched.py 100 plane three:0,default three:0,lane64 three:0,lane32 five
  python tools/ab_sched.py 256 real:three real:three_alt     # RealPlan schedules on the real part of b

Every variant applies the same b (SplitMix64 U[-1,1) complex, the bench's transport symbol) in
place on the current stream, timed with HIP events over `--iters` back-to-back applies; the
variants are interleaved over `--rounds` rounds.  Prints one JSON line per variant: PCApply/s of
each round and the max relative difference of its x to the first variant's (of the same kind).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("grid", type=int)
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lam", type=float, nargs=3, default=[0.6, 0.15, 0.02])
    ap.add_argument("--lib", default=None, help="another build of libcirculant_fft.so (A/B of two builds)")
    args = ap.parse_args()
    if args.lib:
        import circulantpreconditioner_amd._lib as L
        L.LIB_PATH = os.path.abspath(args.lib)
    n = (args.grid,) * 3
    N = args.grid ** 3
    g = torch.Generator(device="cpu").manual_seed(20251017)
    b = (torch.rand(N, generator=g, dtype=torch.float64) * 2 - 1 +
         1j * (torch.rand(N, generator=g, dtype=torch.float64) * 2 - 1)).to("cuda")
    br = b.real.contiguous()
    plans = []
    for v in args.variants:
        if v.startswith("real:"):
            p = cp.RealPlan(n)
            p.set_transport_symbol(tuple(args.lam))
            p.set_schedule(v[5:])
            plans.append(p)
            continue
        p = cp.CirculantPlan(n)
        p.set_transport_symbol(tuple(args.lam))
        sched, _, shape = v.partition(":")
        p.set_schedule(sched)
        if shape:
            n1, mid = shape.split(",")
            p.set_three_pass_shape(int(n1), mid)
        plans.append(p)
    ref = {}
    res = {}
    for v, p in zip(args.variants, plans):
        real = v.startswith("real:")
        res[v] = {"rates": [], "rel_diff": None}
        if real:
            res[v]["stage_ms"] = [round(t, 4) for t in p.time_passes(br, torch.empty_like(br), iters=20)]
        else:
            res[v]["passes"] = [q["mode"] for q in p.passes()]
        x = p.apply(br if real else b)
        r = ref.setdefault(real, x)
        res[v]["rel_diff"] = float((x - r).abs().max() / r.abs().max())
    for _ in range(args.rounds):
        for v, p in zip(args.variants, plans):
            bb = br if v.startswith("real:") else b
            x = torch.empty_like(bb)
            for _ in range(50):
                p.apply(bb, out=x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                p.apply(bb, out=x)
            e1.record()
            e1.synchronize()
            res[v]["rates"].append(round(args.iters / (e0.elapsed_time(e1) * 1e-3), 1))
    for v in args.variants:
        print(json.dumps({"grid": args.grid, "variant": v, "lib": args.lib or "in-tree", **res[v]}), flush=True)
    for p in plans:
        p.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
