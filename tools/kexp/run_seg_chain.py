#!/usr/bin/env python3
"""r04: copy floors of the 3-sweep chain's access patterns for several intermediate layouts
and P2 tile widths (tools/kexp/seg.hip seg_chain).  Interleaved rounds, min over rounds.  GPU only."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "seg.so"))
L.seg_chain.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                        ctypes.POINTER(ctypes.c_double)]
N = 256 ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
cases = [(0, 64, "natural, P2 64 cols (8 x 128 B runs / z): today"), (1, 64, "blocked8, P2 64 cols (1 KiB run / z)"),
         (0, 32, "natural, P2 32 cols (8 x 64 B runs / z)"), (1, 32, "blocked8, P2 32 cols (8 x 64 B in 1 KiB / z)"),
         (2, 32, "blocked4, P2 32 cols (512 B run / z)"), (2, 64, "blocked4, P2 64 cols (2 x 512 B / z)")]
res = {c[:2]: [] for c in cases}
for rnd in range(4):
    for mode, T, _ in cases:
        us = (ctypes.c_double * 4)()
        assert L.seg_chain(mode, T, b.data_ptr(), x.data_ptr(), 40, us) == 0
        res[(mode, T)].append(list(us))
for mode, T, name in cases:
    best = [min(r[k] for r in res[(mode, T)]) for k in range(4)]
    tb = [2 * N * 16 / (t * 1e-6) / 1e12 for t in best[:3]]
    print(f"{name:48s} P1 {best[0]:6.1f} us ({tb[0]:.2f} TB/s)  P2 {best[1]:6.1f} us ({tb[1]:.2f})  "
          f"P3 {best[2]:6.1f} us ({tb[2]:.2f})  sum {sum(best[:3]):6.1f}  chain {best[3]:6.1f} us")
