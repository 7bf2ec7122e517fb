#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (sqlite .db or *_kernel_stats.csv)
into a small markdown table for profiles/.

    python tools/prof_summary.py gpurun_out/prof1 --grid 256 256 256 > profiles/r01_256_kernel_stats.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sqlite3


def from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4])) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            # rocprofv3 stats: Name, Calls, TotalDurationNs, AverageNs, Percentage, ...
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["Percentage"])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--grid", type=int, nargs=3, default=None)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    N = a.grid[0] * a.grid[1] * a.grid[2] if a.grid else None
    print(f"# rocprofv3 kernel stats {a.title}".rstrip())
    print()
    print(f"source: `{(csvs or dbs)[0]}` (rocprofv3 --kernel-trace --stats)")
    if N:
        print(f"grid: {a.grid}, N = {N}; GB/s column = 32 N bytes (read + write one c128 grid) / average")
    print()
    print("| kernel | calls | total us | avg us | % | GB/s (32N/avg) |")
    print("|---|---|---|---|---|---|")
    for name, calls, tot, avg, pct in rows:
        short = name.replace("HIP_vector_type<double, 2u>", "cd").replace("cfp::", "")
        short = short.split("(")[0]
        gbs = f"{32 * N / (avg * 1e-6) / 1e9:.0f}" if (N and ("k_axis" in name or "k_tp_" in name)) else ""
        print(f"| `{short}` | {calls} | {tot:.1f} | {avg:.2f} | {pct:.1f} | {gbs} |")


if __name__ == "__main__":
    main()
