#!/usr/bin/env python3
"""Device time per implicit step of a GMRES run, by kernel, from a rocprofv3 kernel trace.

The solve region starts after the setup (vector fills, the Diag build) with the first step's
leading copies; the number of implicit steps comes from --steps (the run's own count).  Prints
per-kernel calls, median and total microseconds, and the device busy time per step, split into
KSPSolve's own kernels and the reference time loop's vector operations around it
(TransportEquation_impl_mpi.cxx:131-166: VecCopy(Un, dUn) -- a copy of more than 20 us --,
VecAXPY(dUn, -1, Un) and VecNorm(dUn) -- a k_axpy followed by a k_reduce).  Since r06 the
copy is k_copy16, and since r06z5 the AXPY writes the norm partials itself (one k_maxpy<T, false,
true> with no k_reduce after it, the same kernel as the unfused Gram-Schmidt MAXPY), so on later
traces the split below counts that AXPY as KSPSolve's; the device time per step is unaffected.

    python tools/gmres_step_kernels.py gpurun_out/r04a_gmres256_trace [--steps 6]
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    paths = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    first = next(i for i, r in enumerate(rows) if "_spmv" in r[2])
    # back over the kernels queued before the first SpMV, to the end of the setup's fills
    while first > 0 and "fillBufferAligned" not in rows[first - 1][2] and "k_build_diag" not in rows[first - 1][2]:
        first -= 1
    # the solve region starts with the first step's VecCopy(Un, dUn) (a copy of more than 20 us);
    # the setup's MatMult(A, Un, dUn) before it (transport_cartesian.cpp, the device copy of A
    # made before the timed steps) stays outside
    first = next((i for i in range(first, len(rows))
                  if "copyBuffer" in rows[i][2] and (rows[i][1] - rows[i][0]) / 1e3 > 20.0), first)
    sol = rows[first:]
    by = collections.defaultdict(list)
    for s, e, n in sol:
        key = n.split("(")[0][:60]
        by[key].append((e - s) / 1e3)
    tot = sum(sum(v) for v in by.values())
    print(f"solve region: {len(sol)} kernels, device busy {tot:.1f} us, {tot / a.steps:.1f} us per step "
          f"({a.steps} steps), span {(sol[-1][1] - sol[0][0]) / 1e3 / a.steps:.1f} us per step")
    loop = set()
    for i, (s, e, n) in enumerate(sol):
        if ("copyBuffer" in n or "k_copy16" in n) and (e - s) / 1e3 > 20.0:
            loop.add(i)
        if "k_axpy" in n and i + 1 < len(sol) and "k_reduce" in sol[i + 1][2]:
            loop.update((i, i + 1))
    lt = sum((sol[i][1] - sol[i][0]) / 1e3 for i in loop)
    print(f"  KSPSolve's kernels {(tot - lt) / a.steps:.1f} us per step; the time loop's VecCopy / VecAXPY / "
          f"VecNorm around it {lt / a.steps:.1f} us per step ({len(loop)} launches)")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:60s} calls {len(v):4d}  median {statistics.median(v):7.1f} us  total {sum(v):8.1f} us  "
              f"per step {sum(v) / a.steps:7.1f} us")


if __name__ == "__main__":
    main()
