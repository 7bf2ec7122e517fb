#!/usr/bin/env python3
"""r04: copy floors of the 3-sweep chain's access patterns, natural against the blocked
intermediate layout (tools/kexp/seg.hip seg_chain).  Interleaved rounds, min over rounds.  GPU only."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "seg.so"))
L.seg_chain.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
N = 256 ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
res = {0: [], 1: []}
for rnd in range(4):
    for bl in (0, 1):
        us = (ctypes.c_double * 4)()
        assert L.seg_chain(bl, b.data_ptr(), x.data_ptr(), 40, us) == 0
        res[bl].append(list(us))
for bl, name in ((0, "natural (128-B P2 runs)"), (1, "blocked (1 KiB P2 runs)")):
    best = [min(r[k] for r in res[bl]) for k in range(4)]
    tb = [2 * N * 16 / (t * 1e-6) / 1e12 for t in best[:3]]
    print(f"{name:26s} P1 {best[0]:6.1f} us ({tb[0]:.2f} TB/s)  P2 {best[1]:6.1f} us ({tb[1]:.2f})  "
          f"P3 {best[2]:6.1f} us ({tb[2]:.2f})  sum {sum(best[:3]):6.1f}  chain {best[3]:6.1f} us")
