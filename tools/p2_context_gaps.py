#!/usr/bin/env python3
"""Why is P2 slower inside GMRES (136-139 us) than back to back (120 us)?  Runs the 256^3 apply in
contexts that separate the candidate causes, each as its own labelled block of applies, for a
rocprofv3 kernel trace (GPU only; measurement tool):

  A  back to back (bench.py's loop)
  B  a host synchronisation after every apply (GMRES's reductions wait for the host)
  C  B plus 50 us of host idle after every sync (the GPU drops to idle clocks)
  D  a 256 MiB device copy (dirty lines in the caches) before every apply, back to back
  E  a 256 MiB copy into the apply's input before every apply (the SpMV's output feeds P1)

    rocprofv3 --kernel-trace --output-format csv -d OUT -- python3 tools/p2_context_gaps.py
    python3 tools/p2_context_gaps.py --summary OUT
"""
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BLOCK = 40


def run():
    import torch
    import circulantpreconditioner_amd as cp
    n = 256
    b = torch.empty(n ** 3, dtype=torch.complex128, device="cuda")
    cp.fill_uniform(b, 20251017)
    x, y, z = torch.empty_like(b), torch.empty_like(b), torch.empty_like(b)
    p = cp.CirculantPlan((n, n, n)).set_transport_symbol((0.6, 0.15, 0.02))
    for _ in range(50):
        p.apply(b, out=x)
    torch.cuda.synchronize()

    def spin(us):
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e6 < us:
            pass

    for ctx in "ABCDE":
        # a marker kernel between blocks: a tiny fill the summary splits on
        z[:1].fill_(0)
        torch.cuda.synchronize()
        for _ in range(BLOCK):
            if ctx == "D":
                y.copy_(z)
            if ctx == "E":
                y.copy_(b)
                p.apply(y, out=x)
            else:
                p.apply(b, out=x)
            if ctx in "BC":
                torch.cuda.synchronize()
            if ctx == "C":
                spin(50)
        torch.cuda.synchronize()
    print("ok", flush=True)


def summary(d):
    import csv
    import statistics
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # blocks start after each single-element fill (the marker); the warm-up precedes the first
    marks = [i for i, r in enumerate(rows) if "fill" in r[2].lower() or "FillBuffer" in r[2]]
    marks = marks[-5:]
    for k, ctx in enumerate("ABCDE"):
        lo = marks[k]
        hi = marks[k + 1] if k + 1 < len(marks) else len(rows)
        seg = rows[lo:hi]
        out = []
        for key in ("k_tp_rows<false", "k_tp_mid_sw", "k_tp_rows<true"):
            t = [(e - s) / 1e3 for s, e, nm in seg if key in nm]
            out.append(f"{key:18s} {statistics.median(t):7.1f} us (n={len(t)})" if t else f"{key}: -")
        print(ctx, " | ".join(out))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
