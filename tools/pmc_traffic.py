#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (separate passes, csv) into per-launch
HBM bytes for each axis-pass kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:

    hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024

(FETCH_SIZE, in KiB, reads exactly half of a 16-B/lane coalesced streaming read on gfx950;
WRITE_SIZE is exact for 16-B/lane stores).  Kernels are mapped to the bench's pass names
through the template arguments <N, PTS, R0, ROW, T, MODE> and the 5-launch schedule, or
the 3-sweep schedule's k_tp_rows / k_tp_mid.

    python tools/pmc_traffic.py --grid 256 --fetch gpurun_out/pmc256_fetch --write gpurun_out/pmc256_write \
        --out profiles/pmc_traffic.json
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def load(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, path


def pass_name(kname: str):
    # the 3-sweep schedule's kernels (cfp_three_pass.hip): rows fwd / mid fused / rows inv
    t = re.search(r"k_tp_rows<(true|false)", kname)
    if t:
        return "pass2_xy_rows_inv" if t.group(1) == "true" else "pass0_xy_rows_fwd"
    if re.search(r"k_tp_mid(_sw)?<", kname):
        return "pass1_yz_mid_fused"
    m = re.search(r"k_axis_fast<(\d+), (\d+), (\d+), (true|false), (\d+), (\d+)(?:, \d+)?>", kname)
    if not m:
        return None
    row, mode = m.group(4) == "true", int(m.group(6))
    if mode == 0:
        return "pass0_x_fwd" if row else "pass1_y_fwd"
    if mode == 1:
        return "pass4_x_inv" if row else "pass3_y_inv"
    return "pass2_z_fused_sep" if mode == 2 else "pass2_z_fused_diag"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs="+", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    g = a.grid * 3 if len(a.grid) == 1 else a.grid
    N = g[0] * g[1] * g[2]
    fetch, fp = load(a.fetch, "FETCH_SIZE")
    write, wp = load(a.write, "WRITE_SIZE")
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    key = f"{g[0]}x{g[1]}x{g[2]}"
    ent = {}
    for k in fetch:
        name = pass_name(k)
        if not name or k not in write:
            continue
        hbm = 2 * fetch[k] * 1024 + write[k] * 1024
        ent[name] = {"kernel": k.split("(")[0], "FETCH_SIZE_KiB": fetch[k], "WRITE_SIZE_KiB": write[k],
                     "hbm_bytes_per_launch": int(hbm), "alg_bytes_32N": 32 * N,
                     "ratio_to_32N": round(hbm / (32 * N), 4)}
    ent["_source"] = {"fetch_csv": fp, "write_csv": wp,
                      "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM)"}
    data.setdefault(key, {}).update(ent)  # keep other schedules' kernels of the same grid
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    for n, e in sorted(ent.items()):
        if not n.startswith("_"):
            print(f"{key} {n:22s} hbm/launch={e['hbm_bytes_per_launch'] / 1e6:9.1f} MB  ratio to 32N={e['ratio_to_32N']}")


if __name__ == "__main__":
    main()
