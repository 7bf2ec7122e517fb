"""GMRES transport benchmark: BASELINE.json configs 1 and 3.

The implicit upwind transport step of tests/TransportEquation_SphericalExplosion_impl_mpi.cxx
(cfl 1e3/3, a = (1,0,0), GMRES with rtol = abstol = 1e-5, 1000 iterations max) on an n^3
Cartesian grid, solved by the stand-in KSPGMRES on one MI355X with PCNONE (the reference
driver's choice) and with the circulant FFT PCSHELL (the wiring ToDo.md:1 asks for).

One JSON line per (grid, sign, pc, lambda) case: GMRES iterations, wall time per solve and
per iteration, PCApply calls and the host wall time spent inside them.

    python bench_transport.py                      # configs 1 (32^3) and 3 (256^3)
    python bench_transport.py --grid 128 --sign fixed --pc fft --steps 5
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs="*", default=[32, 256])
    ap.add_argument("--sign", nargs="*", default=["fixed", "reference"], choices=["fixed", "reference"])
    ap.add_argument("--pc", nargs="*", default=["none", "fft"], choices=["none", "fft"])
    ap.add_argument("--lam", nargs="*", default=["matched"], choices=["matched", "reference"])
    ap.add_argument("--steps", type=int, default=None,
                    help="time steps (default: the reference loop, tmax = 0.05, i.e. one step)")
    ap.add_argument("--max-its", type=int, default=1000)
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file")
    args = ap.parse_args(argv)

    import torch
    if not torch.cuda.is_available():
        print("bench_transport.py needs a HIP device", file=sys.stderr)
        return 2
    from circulantpreconditioner_amd import transport as T

    lines = []
    for n in args.grid:
        for sign in args.sign:
            for pc in args.pc:
                for lam in (args.lam if pc == "fft" else ["-"]):
                    kw = dict(pc=pc, sign=sign, device=True, max_its=args.max_its)
                    if pc == "fft":
                        kw["lam"] = lam
                    if args.steps:
                        kw["steps"] = args.steps
                    t0 = time.perf_counter()
                    r = T.run(T.config(n, **kw))
                    wall = time.perf_counter() - t0
                    its = max(1, r["total_its"])
                    line = {
                        "metric": "GMRES transport step", "config": f"{n}^3 transport, GMRES(30), 1 MI355X",
                        "grid": n, "sign": sign, "pc": pc, "lambda_mode": lam, "steps": r["steps"],
                        "dt": r["dt"], "lambda": r["lambda"], "gmres_its": r["total_its"],
                        "its_per_step": [r["min_step_its"], r["max_step_its"]],
                        "converged": bool(r["all_converged"]), "last_reason": r["last_reason"],
                        "last_residual": r["last_residual"],
                        "solve_s": r["solve_seconds"], "ms_per_solve": 1e3 * r["solve_seconds"] / max(1, r["steps"]),
                        "ms_per_iteration": 1e3 * r["solve_seconds"] / its,
                        "pc_calls": r["pc_calls"], "pc_s": r["pc_seconds"],
                        "pc_share": r["pc_seconds"] / r["solve_seconds"] if r["solve_seconds"] > 0 else None,
                        "setup_s": r["setup_seconds"], "wall_s": wall,
                    }
                    print(json.dumps(line), flush=True)
                    lines.append(line)
    if args.out:
        with open(args.out, "a") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
