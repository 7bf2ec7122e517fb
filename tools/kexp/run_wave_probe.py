#!/usr/bin/env python3
"""Decompose the wave 3-sweep middle kernel's time (P2w, 128^3) with the wave_probe.hip
variants (GPU only).  Each probe drops part of P2w's work; the times bound what each part costs."""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "wave_probe.so"))
L.wave_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_double, ctypes.c_int,
                                                                   ctypes.POINTER(ctypes.c_float)]
n = 128
data = torch.randn(4 * n ** 3, dtype=torch.complex128, device="cuda")
tw = torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda")
th = 2 * np.pi * np.arange(n) / n
tab = torch.from_numpy(np.stack([0.079 * (1 - np.cos(th)), 0.079 * np.sin(th)], 1).copy()).to("cuda")
NAMES = {0: "full", 100: "full, whole-complex LDS (1 WG/CU)", 1: "no y2 DFT", 2: "no solve", 3: "no y2, no solve",
         4: "no loads", 8: "no stores", 12: "no loads, no stores", 13: "no mem, no y2", 14: "no mem, no solve",
         15: "no mem, no y2, no solve (z FFTs + exchanges)"}
for k in [0, 1, 2, 3, 4, 8, 12, 13, 14, 15]:
    NAMES[200 + k] = "ct: " + NAMES[k]
    NAMES[300 + k] = "ct2: " + NAMES[k]
    NAMES[400 + k] = "ct2 pf: " + NAMES[k]
    NAMES[500 + k] = "ct3: " + NAMES[k]
    NAMES[600 + k] = "ct3 pf: " + NAMES[k]
cases = [0, 100, 1, 2, 3, 4, 8, 12, 13, 14, 15] + [200 + k for k in [0, 1, 2, 3, 4, 8, 12, 13, 14, 15]] + [300 + k for k in [0, 1, 2, 3, 4, 8, 12, 13, 14, 15]] + [400 + k for k in [0, 1, 3, 8, 15]] + [500 + k for k in [0, 1, 3, 15]] + [600 + k for k in [0, 1, 3]]
res = {c: [] for c in cases}
for rnd in range(3):
    for c in cases:
        ms = ctypes.c_float()
        rc = L.wave_probe(c, data.data_ptr(), tw.data_ptr(), tab.data_ptr(), tab.data_ptr(), tab.data_ptr(), 1.0, 50,
                          ctypes.byref(ms))
        assert rc == 0, (c, rc)
        res[c].append(ms.value * 1e3)
for c in cases:
    print(f"{NAMES[c]:48s} {min(res[c]):7.1f} us  (rounds: {', '.join('%.1f' % t for t in res[c])})")
