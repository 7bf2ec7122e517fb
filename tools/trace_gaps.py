#!/usr/bin/env python3
"""Per-PCApply breakdown from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

An apply is the run of launches from the first pass of the schedule (`--first`, substring of
the kernel name) to its last pass (`--last`).  For every apply it reports the kernel time of
each of its launches, the idle gaps between them, the wall span first-start -> last-end, and
the gap since the previous kernel on the device ended (host time the caller spent between
launches: stream syncs, Vec bookkeeping).  Used for VERDICT r02 item 4 (PCApply inside GMRES
vs the bare apply at 256^3).

    python tools/trace_gaps.py gpurun_out/r03d_gmres256 --first "k_tp_rows<false" --last "k_tp_rows<true"
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import statistics


def load(d):
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name: str) -> str:
    n = name.split("(")[0]
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--first", required=True)
    ap.add_argument("--last", required=True)
    ap.add_argument("--skip", type=int, default=2, help="applies to skip (warm-up)")
    a = ap.parse_args()
    rows = load(a.dir)
    applies = []
    i = 0
    while i < len(rows):
        if a.first in rows[i][2]:
            j = i
            while j < len(rows) and a.last not in rows[j][2]:
                j += 1
            if j == len(rows):
                break
            prev_end = rows[i - 1][1] if i > 0 else None
            prev_name = short(rows[i - 1][2]) if i > 0 else "-"
            ks = rows[i:j + 1]
            applies.append({
                "span_us": (ks[-1][1] - ks[0][0]) / 1e3,
                "kernel_us": [(k[1] - k[0]) / 1e3 for k in ks],
                "inner_gaps_us": [(ks[m + 1][0] - ks[m][1]) / 1e3 for m in range(len(ks) - 1)],
                "gap_before_us": (ks[0][0] - prev_end) / 1e3 if prev_end else None,
                "prev": prev_name,
                "next_gap_us": (rows[j + 1][0] - ks[-1][1]) / 1e3 if j + 1 < len(rows) else None,
            })
            i = j + 1
        else:
            i += 1
    applies = applies[a.skip:]
    if not applies:
        raise SystemExit("no complete applies found")
    nk = len(applies[0]["kernel_us"])
    med = statistics.median
    print(f"applies: {len(applies)} (after skipping {a.skip})")
    print(f"span first-start -> last-end: median {med(x['span_us'] for x in applies):.1f} us")
    for m in range(nk):
        print(f"  launch {m}: median {med(x['kernel_us'][m] for x in applies):.1f} us")
    for m in range(nk - 1):
        print(f"  gap {m}->{m + 1}: median {med(x['inner_gaps_us'][m] for x in applies):.2f} us")
    gb = [x["gap_before_us"] for x in applies if x["gap_before_us"] is not None]
    ga = [x["next_gap_us"] for x in applies if x["next_gap_us"] is not None]
    if gb:
        print(f"gap since the previous kernel ended: median {med(gb):.1f} us (min {min(gb):.1f}, max {max(gb):.1f})")
    if ga:
        print(f"gap until the next kernel starts:   median {med(ga):.1f} us")
    prevs = {}
    for x in applies:
        prevs[x["prev"]] = prevs.get(x["prev"], 0) + 1
    print("kernel before each apply:", ", ".join(f"{k} x{v}" for k, v in sorted(prevs.items(), key=lambda t: -t[1])))


if __name__ == "__main__":
    main()
