#!/usr/bin/env python3
"""Decompose the 256^3 middle kernel's time with the tp_probe.hip variants (GPU only).
Each probe drops part of P2's work; the times bound what each part costs and what overlaps."""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "tp_probe.so"))
L.tp_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = 256
N = n ** 3
data = torch.randn(N, dtype=torch.complex128, device="cuda")
tw = torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda")
colsym = torch.full((n * n,), 0.5 + 0.1j, dtype=torch.complex128, device="cuda")
axsym = torch.full((n,), 0.25, dtype=torch.complex128, device="cuda")
NAMES = {32: "full, s_setprio 1 on the second half of the waves", 0: "full (product: swap64 + prefetch)", 100: "full (lane DFT, product default)", 1: "no y2 DFT", 2: "no z math+divide",
         3: "no y2, no z math (mem + exchanges)", 4: "no exchanges", 6: "no z math, no exchanges",
         7: "mem only (no math, no exchanges)", 8: "no loads", 16: "no stores", 24: "no loads, no stores (compute+xchg)",
         26: "no mem, no z math (y2 + xchg)", 28: "no mem, no xchg (y2 + z math)", 29: "no mem, no xchg, no y2 (z math)",
         30: "no mem, no xchg, no z math (y2 only)", 31: "nothing (loop + twiddle)"}
cases = [0, 32, 100, 1, 2, 3, 4, 6, 7, 8, 16, 24, 26, 28, 29, 30, 31, 1000, 1007]
res = {c: [] for c in cases}
for rnd in range(3):
    for c in cases:
        ms = ctypes.c_float()
        rc = L.tp_probe(c, data.data_ptr(), tw.data_ptr(), colsym.data_ptr(), axsym.data_ptr(), 30, ctypes.byref(ms))
        assert rc == 0, (c, rc)
        res[c].append(ms.value * 1e3)
torch.cuda.synchronize()
for c in cases:
    base = NAMES[c % 1000] + (" [1 WG per unit]" if c >= 1000 else "")
    t = sorted(res[c])
    print(f"{c:5d} {base:44s} min {t[0]:7.1f} us  med {t[1]:7.1f} us  ({2 * N * 16 / (t[0] * 1e-6) / 1e12:5.2f} TB/s eq)")
