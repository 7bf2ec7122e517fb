#!/usr/bin/env python3
"""Cache-policy A/B of the 256^3 3-sweep apply chain (tp_chain.hip) with the lane-pair P1/P3 (r03z), interleaved rounds."""
import ctypes
import os

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tp_chain.so"))
L.tp_chain.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = 256
b = torch.randn(n ** 3, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
tw = torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda")
cs = torch.full((n * n,), 0.5 + 0.1j, dtype=torch.complex128, device="cuda")
ax = torch.full((n,), 0.25, dtype=torch.complex128, device="cuda")
P1 = ["nt-ld", "plain", "nt-ld+st", "nt-st"]
P2 = ["plain", "nt-st"]
P3 = ["nt-st", "nt-ld+st", "plain"]
import sys
BASE = int(sys.argv[1]) if len(sys.argv) > 1 else 64  # 64: lane-pair rows; + 4096: P2 NT loads
cases = [BASE + q1 + 4 * q2 + 16 * q3 for q3 in range(3) for q2 in range(2) for q1 in range(4)]
res = {c: [] for c in cases}
for rnd in range(3):
    for c in cases:
        ms = ctypes.c_float()
        assert L.tp_chain(c, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(), 40,
                          ctypes.byref(ms)) == 0
        res[c].append(ms.value * 1e3)
for c in sorted(cases, key=lambda c: min(res[c])):
    q1, q2, q3 = c & 3, (c >> 2) & 3, (c >> 4) & 3
    print(f"P1 {P1[q1]:9s} P2 {P2[q2]:6s} P3 {P3[q3]:9s}  {min(res[c]):6.1f} us  ({', '.join('%.1f' % t for t in res[c])})")
