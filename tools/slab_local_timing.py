#!/usr/bin/env python3
"""Local pass time per rank of the z-slab plan (GPU only): rank 0 of P ranks, the library's three
kernel segments on one stream, exchanges skipped (they are timed by bench.py --gpus N on a real
node).  Compares the 3-sweep and the 5-pass slab schedules.

    python tools/slab_local_timing.py [--grid 256] [--ranks 1 2 4 8] [--iters 50]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402
from circulantpreconditioner_amd._lib import check, lib  # noqa: E402
from circulantpreconditioner_amd.distributed import slab_layout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    n = a.grid
    lam = (ctypes.c_double * 6)(0.6, 0.0, 0.15, 0.0, 0.02, 0.0)
    for P in a.ranks:
        L = slab_layout((n, n, n), P, 0)
        loc = L["local_size"]
        b = torch.empty(loc, dtype=torch.complex128, device="cuda")
        cp.fill_uniform(b, 3)
        x = torch.empty_like(b)
        h = ctypes.c_void_p()
        check(lib().cfp_dist_plan_create_external(ctypes.byref(h), n, n, n, P, 0, 0))
        check(lib().cfp_dist_plan_set_symbol_transport(h, lam))
        res = {}
        for name, sched in (("three", 2), ("five", 1)):
            if lib().cfp_dist_plan_set_schedule(h, sched) != 0:
                res[name] = None
                continue
            s = torch.cuda.current_stream()
            seg = lambda k: check(lib().cfp_dist_plan_run_segment(h, k, b.data_ptr(), x.data_ptr(),
                                                                  ctypes.c_void_p(s.cuda_stream)))
            for _ in range(5):
                for k in range(3):
                    seg(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                for k in range(3):
                    seg(k)
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) / a.iters * 1e3
        check(lib().cfp_dist_plan_destroy(h))
        moved3, moved5 = 96 * loc, 160 * loc
        t3 = (f"3-sweep {res['three']:.1f} us ({moved3 / res['three'] / 1e6:.2f} TB/s moved)"
              if res["three"] else "3-sweep n/a (not built for this shape)")
        print(f"{n}^3 P={P}: local {loc} points; {t3}, 5-pass {res['five']:.1f} us "
              f"({moved5 / res['five'] / 1e6:.2f} TB/s moved)", flush=True)


if __name__ == "__main__":
    main()
