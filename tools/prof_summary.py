#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (sqlite .db or *_kernel_stats.csv)
into a small markdown table for profiles/.

    python tools/prof_summary.py gpurun_out/prof1 --grid 256 256 256 > profiles/r01_256_kernel_stats.md
    python tools/prof_summary.py gpurun_out/r05g_prof_bench --bench > profiles/r05g_bench_kernel_stats.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sqlite3

# --bench: the complex 3-sweep kernels of bench.py's legs, each with its own grid edge
# (template arguments as cfp_three_pass.hip instantiates them; real-data and wave kernels
# move a different byte count per grid and are left blank).
BENCH_GRIDS = [
    (r"k_tp_mid_sw<64, 8, 256, 0, true, 256,", 256),
    (r"k_tp_rows<(true|false), 20[0-9][0-9], 32, 256,", 256),
    (r"k_tp_mid<0, 32, 16, 512,", 512),
    (r"k_tp_rows<(true|false), 20[0-9][0-9], 32, 512,", 512),
    (r"k_tp_mid<0, 32, 8, 128,", 128),
    (r"k_tp_rows<(true|false), 2048, 16, 128,", 128),
]


def bench_grid(name):
    for pat, n in BENCH_GRIDS:
        if re.search(pat, name):
            return n ** 3
    return None


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
    ap.add_argument("--bench", action="store_true", help="per-kernel grid for bench.py's complex legs")
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    N = a.grid[0] * a.grid[1] * a.grid[2] if a.grid else None
    print(f"# rocprofv3 kernel stats {a.title}".rstrip())
    print()
    print(f"source: `{(csvs or dbs)[0]}` (rocprofv3 --kernel-trace --stats)")
    if a.bench:
        print("GB/s column = 32 N bytes (read + write one c128 grid) / average, N = the kernel's own grid "
              "(256^3, 512^3 or 128^3 complex 3-sweep legs; blank for the other legs)")
    elif N:
        print(f"grid: {a.grid}, N = {N}; GB/s column = 32 N bytes (read + write one c128 grid) / average")
    print()
    print("| kernel | calls | total us | avg us | % | GB/s (32N/avg) |")
    print("|---|---|---|---|---|---|")
    for name, calls, tot, avg, pct in rows:
        short = name.replace("HIP_vector_type<double, 2u>", "cd").replace("cfp::", "")
        short = short.split("(")[0]
        n = bench_grid(name) if a.bench else (N if ("k_axis" in name or "k_tp_" in name) else None)
        gbs = f"{32 * n / (avg * 1e-6) / 1e9:.0f}" if n else ""
        print(f"| `{short}` | {calls} | {tot:.1f} | {avg:.2f} | {pct:.1f} | {gbs} |")


if __name__ == "__main__":
    main()
