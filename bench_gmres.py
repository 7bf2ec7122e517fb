"""GMRES benchmarks: BASELINE.json configs 1 and 3 (transport) and
config 4 (wave system with the block-circulant preconditioner, row f2).

The implicit upwind transport step of tests/TransportEquation_SphericalExplosion_impl_mpi.cxx
(cfl 1e3/3, a = (1,0,0), GMRES with rtol = abstol = 1e-5, 1000 iterations max) on an n^3
Cartesian grid, solved by the stand-in KSPGMRES on one MI355X with PCNONE (the reference
driver's choice) and with the circulant FFT PCSHELL (the wiring ToDo.md:1 asks for).

The wave system (tests/WaveSystem_SphericalExplosion_impl_seq.cxx: c0 = 700, cfl 1e3/3,
wall boundaries, GMRES rtol = abstol = 1e-5) runs with PCNONE and with the block-circulant
PCSHELL; its block apply is also timed alone (PCApply/s and HBM GB/s).

One JSON line per case: GMRES iterations, wall time per solve and per iteration, PCApply
calls and the host wall time spent inside them.

    python bench_gmres.py                          # configs 1, 3 and 4
    python bench_gmres.py --system transport --grid 128 --sign fixed --pc fft --steps 5
    python bench_gmres.py --system wave --wave-grid 64 --wave-steps 3
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", nargs="*", default=["transport", "wave"], choices=["transport", "wave", "wave2d", "mesh", "direct"])
    ap.add_argument("--direct-grid", type=int, nargs="*", default=[10, 100, 256],
                    help="--system direct: the direct-solver loop (TransportEquationFFT_impl) on n^3")
    ap.add_argument("--mesh", nargs="*", default=["mesh_tetra_1.msh", "3DKershawTetra1.msh", "mesh_hexa_3.msh"],
                    help="tests/golden/meshes/ files for --system mesh (row f3: the PCSHELL with the remap)")
    ap.add_argument("--wave-grid", type=int, nargs="*", default=[128])
    ap.add_argument("--wave2d-grid", type=int, nargs="*", default=[50, 1024],
                    help="2-D wave system (3 unknowns per cell): 50 is the reference main's default mesh")
    ap.add_argument("--wave2d-loop-max", type=int, default=256,
                    help="run the whole time loop (to tmax = 0.05) only up to this many cells a side")
    ap.add_argument("--wave-steps", type=int, default=1,
                    help="wave time steps (the reference loop to tmax = 0.05 is ~81 steps at 128^3)")
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
        print("bench_gmres.py needs a HIP device", file=sys.stderr)
        return 2
    from circulantpreconditioner_amd import transport as T

    lines = []
    if "wave" in args.system:
        lines += wave_lines(args)
    if "wave2d" in args.system:
        lines += wave2d_lines(args)
    if "mesh" in args.system:
        lines += mesh_lines(args)
    if "direct" in args.system:
        lines += direct_lines(args)
    for n in (args.grid if "transport" in args.system else []):
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
                        "pc_ms_per_call": 1e3 * r["pc_seconds"] / max(1, r["pc_calls"]),
                        "pc_share": r["pc_seconds"] / r["solve_seconds"] if r["solve_seconds"] > 0 else None,
                        "pc_timing": "device time of each PCApply on the Vec stream: the 3-sweep apply's own first-kernel start to last-kernel end (dispatch stamps), else HIP events around it",
                        "setup_s": r["setup_seconds"], "wall_s": wall,
                    }
                    print(json.dumps(line), flush=True)
                    lines.append(line)
    if args.out:
        with open(args.out, "a") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")
    return 0


def direct_lines(args) -> list:
    """The reference's direct-solver loop (tests/TransportEquationFFT_SphericalExplosion_impl_mpi.cxx,
    ctests "10 10 10" and "100 100 100"): the reference run (tmax = 0.05: one step at cfl 1e3/3)
    and 20 timed steps (one PetscFft3DTransportSolver(ctx, Un, Un) each, host-synchronous)."""
    from circulantpreconditioner_amd import transport as T
    out = []
    for n in args.direct_grid:
        for label, kw in (("reference run", {}), ("20 steps", {"steps": 20, "precision": 1e-30})):
            t0 = time.perf_counter()
            r = T.run_direct(T.config(n, device=True, **kw))
            wall = time.perf_counter() - t0
            line = {"metric": "direct FFT transport solve", "config": f"{n}^3 TransportEquationFFT, 1 MI355X",
                    "grid": n, "run": label, "steps": r["steps"], "dt": r["dt"], "lambda": r["lambda"],
                    "ms_per_step": 1e3 * r["solve_seconds"] / max(1, r["steps"]),
                    "solves_per_s": r["steps"] / r["solve_seconds"] if r["solve_seconds"] > 0 else None,
                    "setup_s": r["setup_seconds"], "wall_s": wall}
            print(json.dumps(line), flush=True)
            out.append(line)
    return out


def mesh_lines(args) -> list:
    """The transport step on the reference's unstructured meshes (Mesh(filename) in
    tests/TransportEquation_SphericalExplosion_impl_mpi.cxx:248-250) with PCNONE and with the
    FFT PCSHELL behind the mesh -> Cartesian remap (row f3)."""
    import os
    from circulantpreconditioner_amd import mesh as M
    from circulantpreconditioner_amd import transport as T
    out = []
    mdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "meshes")
    for name in args.mesh:
        m = M.Mesh.read(os.path.join(mdir, name))
        for sign in args.sign:
            for pc in args.pc:
                kw = dict(pc=pc, sign=sign, device=True, max_its=args.max_its, lam="matched")
                if args.steps:
                    kw["steps"] = args.steps
                t0 = time.perf_counter()
                r = M.run_transport(m, T.config(8, **kw))
                wall = time.perf_counter() - t0
                its = max(1, r["total_its"])
                line = {"metric": "GMRES transport step on a mesh", "mesh": name, "cells": m.ncells,
                        "fft_grid": int(m.ncells ** (1 / 3) + 1e-9), "sign": sign, "pc": pc,
                        "steps": r["steps"], "dt": r["dt"], "lambda": r["lambda"], "gmres_its": r["total_its"],
                        "converged": bool(r["all_converged"]), "last_reason": r["last_reason"],
                        "ms_per_solve": 1e3 * r["solve_seconds"] / max(1, r["steps"]),
                        "ms_per_iteration": 1e3 * r["solve_seconds"] / its, "pc_calls": r["pc_calls"],
                        "pc_s": r["pc_seconds"], "setup_s": r["setup_seconds"], "wall_s": wall}
                print(json.dumps(line), flush=True)
                out.append(line)
    return out


def wave_lines(args) -> list:
    import torch
    from circulantpreconditioner_amd import wave as W
    out = []
    for n in args.wave_grid:
        # the block apply alone (config 4's PCApply): 5 sweeps of 4 components
        dims = (n, n, n)
        h = 1.0 / n
        dt = (1e3 / 3) * (h / 6) / W.C0
        plan = W.WavePlan(dims).set_symbol([dt / h] * 3)
        m = 4 * n ** 3
        b = torch.randn(m, dtype=torch.complex128, device="cuda")
        x = torch.empty_like(b)
        for _ in range(5):
            plan.apply(b, x)
        torch.cuda.synchronize()
        iters = max(10, int(2e9 / (m * 16)))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            plan.apply(b, x)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        passes = plan.time_passes(b, x, iters=5)
        # the 5-sweep schedule on the same vectors, for the A/B (AUTO takes 3 sweeps at 128^3)
        ms5 = None
        if len(passes) == 3:
            plan.set_schedule("five")
            for _ in range(3):
                plan.apply(b, x)
            e0.record()
            for _ in range(iters):
                plan.apply(b, x)
            e1.record()
            torch.cuda.synchronize()
            ms5 = e0.elapsed_time(e1) / iters
            plan.set_schedule("auto")
        line = {"metric": "wave block PCApply", "config": f"WaveSystem {n}^3, 4x4 block-circulant, 1 MI355X",
                "grid": n, "pcapply_per_s": 1e3 / ms, "ms_per_apply": ms, "sweeps": len(passes),
                "hbm_gbps_moved": len(passes) * 2 * m * 16 / (ms * 1e-3) / 1e9,
                "hbm_gbps_b_alg_1024N": 1024 * n ** 3 / (ms * 1e-3) / 1e9,
                "passes_ms": passes, "five_sweep_ms_per_apply": ms5}
        print(json.dumps(line), flush=True)
        out.append(line)
        del plan, b, x
        for pc in args.pc:
            t0 = time.perf_counter()
            r = W.run(W.config(n, pc=pc, steps=args.wave_steps, max_its=args.max_its))
            wall = time.perf_counter() - t0
            its = max(1, r["total_its"])
            line = {"metric": "GMRES wave step", "config": f"WaveSystem {n}^3 implicit, GMRES(30), 1 MI355X",
                    "grid": n, "pc": pc, "steps": r["steps"], "dt": r["dt"], "kappa": r["kappa"],
                    "gmres_its": r["total_its"], "its_per_step": [r["min_step_its"], r["max_step_its"]],
                    "converged": bool(r["all_converged"]), "last_reason": r["last_reason"],
                    "last_residual": r["last_residual"], "solve_s": r["solve_seconds"],
                    "ms_per_solve": 1e3 * r["solve_seconds"] / max(1, r["steps"]),
                    "ms_per_iteration": 1e3 * r["solve_seconds"] / its, "pc_calls": r["pc_calls"],
                    "pc_s": r["pc_seconds"], "setup_s": r["setup_seconds"], "wall_s": wall}
            print(json.dumps(line), flush=True)
            out.append(line)
    return out


def _time_apply(plan, b, x):
    import torch
    for _ in range(5):
        plan.apply(b, x)
    torch.cuda.synchronize()
    iters = max(20, int(2e9 / (b.numel() * 16)))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        plan.apply(b, x)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def wave2d_lines(args) -> list:
    """The reference mains' own wave case: a 2-D square, 3 interleaved unknowns per cell
    (tests/WaveSystem_SphericalExplosion_impl_seq.cxx:182-212, nx = ny = 50, cfl = 1e3/2)."""
    import torch
    from circulantpreconditioner_amd import wave as W
    out = []
    for n in args.wave2d_grid:
        dims = (n, n, 1)
        h = 1.0 / n
        dt = (1e3 / 2) * (h / 4) / W.C0
        plan = W.WavePlan(dims, dim=2).set_symbol([dt / h, dt / h, 0.0])
        m = 3 * n * n
        b = torch.randn(m, dtype=torch.complex128, device="cuda")
        x = torch.empty_like(b)
        ms = _time_apply(plan, b, x)
        passes = plan.time_passes(b, x, iters=5)
        line = {"metric": "wave 2-D block PCApply", "config": f"WaveSystem {n}x{n} (2-D), 3x3 block-circulant, 1 MI355X",
                "grid": n, "pcapply_per_s": 1e3 / ms, "ms_per_apply": ms,
                "hbm_gbps_moved": len(passes) * 2 * m * 16 / (ms * 1e-3) / 1e9, "passes_ms": passes}
        print(json.dumps(line), flush=True)
        out.append(line)
        del plan, b, x
        if n > args.wave2d_loop_max:
            continue
        for pc in args.pc:
            t0 = time.perf_counter()
            r = W.run(W.config(n, dim=2, pc=pc, max_its=args.max_its))
            wall = time.perf_counter() - t0
            its = max(1, r["total_its"])
            line = {"metric": "GMRES wave 2-D time loop", "config": f"WaveSystem {n}x{n} implicit to tmax=0.05, "
                    "GMRES(30), 1 MI355X", "grid": n, "pc": pc, "steps": r["steps"], "dt": r["dt"],
                    "kappa": r["kappa"], "gmres_its": r["total_its"], "its_per_step": [r["min_step_its"],
                    r["max_step_its"]], "converged": bool(r["all_converged"]), "last_reason": r["last_reason"],
                    "solve_s": r["solve_seconds"], "ms_per_solve": 1e3 * r["solve_seconds"] / max(1, r["steps"]),
                    "ms_per_iteration": 1e3 * r["solve_seconds"] / its, "pc_calls": r["pc_calls"],
                    "pc_s": r["pc_seconds"], "wall_s": wall}
            print(json.dumps(line), flush=True)
            out.append(line)
    return out


if __name__ == "__main__":
    sys.exit(main())
