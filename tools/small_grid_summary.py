#!/usr/bin/env python3
"""Markdown summary of tools/prof_small_grids.sh: per apply kernel of the
128^3 / 100^3 benches, the rocprofv3 mean duration, the HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE,
MI355X_MICROARCH.md's gfx950 correction) and the SQ occupancy / wait counters.

    python tools/small_grid_summary.py gpurun_out r03i > profiles/r03i_small_grids.md
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def stats(d):
    p = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    if p:
        for r in csv.DictReader(open(p[0])):
            out[r["Name"].split("(")[0]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    return out


def counters(d):
    p = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    if p:
        for r in csv.DictReader(open(p[0])):
            acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    base, tag = sys.argv[1], sys.argv[2]
    print(f"# Launch-bound configs: kernel profile ({tag}, one MI355X)\n")
    print("rocprofv3 --kernel-trace --stats of `bench.py --grid G --steps 200` (trace overhead included in")
    print("the bench value of that run); counters from separate `--pmc` passes of 20 steps.  Bytes per launch =")
    print("2 FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the gfx950 correction of MI355X_MICROARCH.md).  Occupancy")
    print("= SQ_WAVE_CYCLES / SQ_BUSY_CYCLES (mean waves resident while the SQ is busy, summed over CUs);")
    print("wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES.\n")
    for g in (128, 100):
        bj = os.path.join(base, f"{tag}_bench{g}.json")
        if not os.path.exists(bj):
            continue
        b = json.load(open(bj))
        st = stats(os.path.join(base, f"{tag}_trace{g}"))
        sq = counters(os.path.join(base, f"{tag}_sq{g}"))
        fe = counters(os.path.join(base, f"{tag}_fetch{g}"))
        wr = counters(os.path.join(base, f"{tag}_write{g}"))
        N = g ** 3
        print(f"## {g}^3: {b['value']:.0f} PCApply/s under the tracer, {b['ms_per_step'] * 1e3:.1f} us per apply\n")
        print("passes (live events): " + ", ".join(f"{p['axis']}:{p['mode']} {p['ms'] * 1e3:.1f} us" for p in b["passes"]) + "\n")
        print("| kernel | calls | mean us | bytes/launch (x 32N) | GB/s | waves | occupancy | wait share |")
        print("|---|---|---|---|---|---|---|---|")
        for name, (calls, us) in sorted(st.items(), key=lambda t: -t[1][1] * t[1][0]):
            if "cfp::" not in name or calls < 100:
                continue
            f = fe.get((name, "FETCH_SIZE"))
            w = wr.get((name, "WRITE_SIZE"))
            byt = (2 * f + w) * 1024 if f is not None and w is not None else None
            wv = sq.get((name, "SQ_WAVES"))
            busy = sq.get((name, "SQ_BUSY_CYCLES"))
            wcyc = sq.get((name, "SQ_WAVE_CYCLES"))
            wait = sq.get((name, "SQ_WAIT_ANY"))
            occ = wcyc / busy if wcyc and busy else None
            short = name.replace("void ", "").replace("cfp::", "")
            print(f"| `{short}` | {calls} | {us:.2f} | "
                  f"{'%.3f' % (byt / (32 * N)) if byt else '-'} | {'%.0f' % (byt / (us * 1e-6) / 1e9) if byt else '-'} | "
                  f"{int(wv) if wv else '-'} | {'%.1f' % occ if occ else '-'} | {'%.2f' % (wait / wcyc) if wait and wcyc else '-'} |")
        print()
    wj = os.path.join(base, f"{tag}_wave128.jsonl")
    st = stats(os.path.join(base, f"{tag}_wave128"))
    if st:
        print("## wave system 128^3 (config 4), bench_gmres.py --system wave\n")
        if os.path.exists(wj):
            for line in open(wj):
                if line.startswith("{"):
                    d = json.loads(line)
                    keep = {k: d[k] for k in d if k in ("pc", "gmres_its", "ms_per_solve", "apply_ms", "applies_per_s",
                                                         "GBps", "frac_hbm", "pass_ms", "pcapply_per_s",
                                                         "ms_per_apply", "sweeps", "passes_ms",
                                                         "five_sweep_ms_per_apply")}
                    print("- " + json.dumps(keep))
        print("\n| kernel | calls | mean us |\n|---|---|---|")
        for name, (calls, us) in sorted(st.items(), key=lambda t: -t[1][1] * t[1][0])[:12]:
            print(f"| `{name.replace('void ', '')[:90]}` | {calls} | {us:.2f} |")


if __name__ == "__main__":
    main()
