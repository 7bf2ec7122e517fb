#!/usr/bin/env python3
"""Why is the 256^3 PCApply slower inside GMRES / the direct loop than in bench.py?
  The per-launch times of the 3-sweep apply (HIP events on the launch
stream, cfp_plan_profile_begin) in different surroundings:

  back-to-back    apply(b -> x) repeated (bench.py's loop)
  host-sync       apply + hipStreamSynchronize each time (the PCSHELL's contract)
  copy-before     a 256 MiB device copy of another vector, then the apply (the direct loop's
                  VecCopy(Un, dUn) before PetscFft3DTransportSolver)
  write-before    a kernel writing another 256 MiB vector, then the apply (GMRES: MatMult /
                  VecMAXPY output just before PCApply)
  in-place        apply(x -> x) (the direct solver's Un, Un)

    python tools/p2_context_probe.py [--reps 40]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--grid", type=int, default=256)
    a = ap.parse_args()
    import torch
    import circulantpreconditioner_amd as cp
    n = a.grid
    N = n ** 3
    dev = torch.device("cuda", 0)
    b = torch.empty(N, dtype=torch.complex128, device=dev)
    cp.fill_uniform(b, 1)
    x = torch.empty_like(b)
    other = torch.empty_like(b)
    other2 = torch.empty_like(b)
    plan = cp.CirculantPlan((n, n, n), device=0).set_transport_symbol((0.6, 0.15, 0.02))
    for _ in range(50):  # clocks up
        plan.apply(b, out=x)
    torch.cuda.synchronize()
    names = [f"{p['axis']}:{p['mode']}" for p in plan.passes()]

    def run(label, body):
        plan.profile_begin(a.reps, 1)
        for _ in range(a.reps):
            body()
        torch.cuda.synchronize()
        ms, k = plan.profile_end()
        line = {"case": label, "applies": k, "us": {nm: round(m * 1e3, 1) for nm, m in zip(names, ms)},
                "sum_us": round(sum(ms) * 1e3, 1)}
        print(json.dumps(line), flush=True)

    run("back-to-back", lambda: plan.apply(b, out=x))

    def hs():
        plan.apply(b, out=x)
        torch.cuda.synchronize()
    run("host-sync", hs)

    def cb():
        other.copy_(b)
        plan.apply(b, out=x)
    run("copy-before", cb)

    def wb():
        torch.add(b, x, out=other)  # reads 2, writes 1 vector, like VecWAXPY / MatMult output
        plan.apply(other, out=x)
    run("write-before", wb)

    def wbs():
        torch.add(b, x, out=other)
        torch.cuda.synchronize()
        plan.apply(other, out=x)
        torch.cuda.synchronize()
    run("write-before+sync", wbs)

    def ip():
        other2.copy_(b)
        plan.apply(other2, out=other2)
    run("copy+in-place", ip)


if __name__ == "__main__":
    main()
