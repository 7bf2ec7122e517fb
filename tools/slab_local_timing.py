#!/usr/bin/env python3
"""Local pass time per rank of the z-slab plan (GPU only): rank 0 of P ranks runs the kernel
steps of its step list on one stream, exchanges skipped (they are timed by bench.py --gpus N on
a real node).  For each schedule and pipeline depth K (pieces) it reports the local kernel time
split into the forward part (before the first exchange piece), the middle (z) and the backward
part, and a model of the whole apply over xGMI: one link of ~150 GB/s per peer (7 links on an
8-GPU node), each all-to-all moving 16 N/P (P-1)/P bytes out of every GPU.

  unpipelined (K = 1):  fwd + X + mid + X + bwd
  pipelined  (K > 1):   max(fwd, X) + min(fwd, X)/K + mid + max(bwd, X) + min(bwd, X)/K
                        (X: one all-to-all; the first / last piece cannot overlap)

    python tools/slab_local_timing.py [--grid 512] [--ranks 2 4 8] [--pieces 1 4 8] [--iters 20] [--lib SO]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402
from circulantpreconditioner_amd._lib import check, lib  # noqa: E402
from circulantpreconditioner_amd.distributed import STEP_KEYS, slab_layout  # noqa: E402

LINK_GBS = 150.0


def steps_of(h):
    n = ctypes.c_int()
    check(lib().cfp_dist_plan_num_steps(h, ctypes.byref(n)))
    out = []
    for i in range(n.value):
        d = (ctypes.c_int64 * len(STEP_KEYS))()
        check(lib().cfp_dist_plan_step(h, i, d))
        out.append(dict(zip(STEP_KEYS, list(d))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=512)
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--pieces", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="another build of libcirculant_fft.so (A/B of two builds)")
    a = ap.parse_args()
    if a.lib:
        import circulantpreconditioner_amd._lib as Lib
        Lib.LIB_PATH = os.path.abspath(a.lib)
    n = a.grid
    lam = (ctypes.c_double * 6)(0.6, 0.0, 0.15, 0.0, 0.02, 0.0)
    for P in a.ranks:
        L = slab_layout((n, n, n), P, 0)
        loc = L["local_size"]
        b = torch.empty(loc, dtype=torch.complex128, device="cuda")
        cp.fill_uniform(b, 3)
        x = torch.empty_like(b)
        w, w2 = torch.empty_like(b), torch.empty_like(b)
        h = ctypes.c_void_p()
        check(lib().cfp_dist_plan_create_external(ctypes.byref(h), n, n, n, P, 0, 0))
        check(lib().cfp_dist_plan_set_work_buffers(h, w.data_ptr(), w2.data_ptr()))
        check(lib().cfp_dist_plan_set_symbol_transport(h, lam))
        links = max(1, min(P - 1, 7))
        x_us = 16 * loc * (P - 1) / P / (links * LINK_GBS * 1e9) * 1e6  # one all-to-all
        for name, sched in (("three", 2), ("five", 1)):
            if lib().cfp_dist_plan_set_schedule(h, sched) != 0:
                continue
            for K in a.pieces:
                if lib().cfp_dist_plan_set_pieces(h, K) != 0:
                    continue
                st = steps_of(h)
                s = torch.cuda.current_stream()
                seg_t = []
                for seg in (0, 1, 2):
                    idx = [i for i, d in enumerate(st) if d["kind"] != 1 and d["seg"] == seg]

                    def run():
                        for i in idx:
                            check(lib().cfp_dist_plan_run_step(h, i, b.data_ptr(), x.data_ptr(),
                                                               ctypes.c_void_p(s.cuda_stream)))
                    for _ in range(3):
                        run()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    seg_t.append(e0.elapsed_time(e1) / a.iters * 1e3)
                fwd, mid, bwd = seg_t
                if K == 1:
                    model = fwd + x_us + mid + x_us + bwd
                else:
                    model = max(fwd, x_us) + min(fwd, x_us) / K + mid + max(bwd, x_us) + min(bwd, x_us) / K
                print(f"{n}^3 P={P} {name} K={K}: local kernels fwd {fwd:.1f} + mid {mid:.1f} + bwd {bwd:.1f} = "
                      f"{fwd + mid + bwd:.1f} us; all-to-all model {x_us:.1f} us ({links} x {LINK_GBS:.0f} GB/s); "
                      f"apply model {model:.1f} us = {1e6 / model:.0f} PCApply/s", flush=True)
        check(lib().cfp_dist_plan_destroy(h))
        del b, x, w, w2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
