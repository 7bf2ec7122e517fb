#!/usr/bin/env python3
"""Whole 5-launch applies at 512^3 (interleaved rounds, one process): y-fused order
(x, z, y*, z, x; the product's AUTO order at 512^3) and z-fused order, over fused / column shapes
68..82 of kexp.so."""
import ctypes
import os
import statistics

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kexp.so"))
L.kexp_chain_axes.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)] + \
    [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.kexp_name.restype = ctypes.c_char_p
n = 512
N = n ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
k = np.arange(n, dtype=np.longdouble)
tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
YF, ZF = (0, 2, 1, 2, 0), (0, 1, 2, 1, 0)
sets = {"yf_product": ((81, 75, 73, 78, 82), YF)}
for v in (68, 69, 70, 71, 72, 74):
    sets[f"yf_fused{v}"] = ((81, 75, v, 78, 82), YF)
for v in (73, 68, 70, 71):
    sets[f"zf_fused{v}"] = ((81, 75, v, 78, 82), ZF)
sets["yf_col76_79"] = ((81, 76, 73, 79, 82), YF)
sets["yf_col77"] = ((81, 77, 73, 78, 82), YF)
sets["yf_col80"] = ((81, 80, 73, 78, 82), YF)
res = {s: [] for s in sets}
for rnd in range(5):
    for name, (vs, axs) in sets.items():
        ms = ctypes.c_double()
        rc = L.kexp_chain_axes(5, (ctypes.c_int * 5)(*vs), (ctypes.c_int * 5)(*axs), b.data_ptr(), x.data_ptr(),
                               tw.data_ptr(), cs.data_ptr(), ax.data_ptr(), 4, ctypes.byref(ms))
        assert rc == 0, (name, rc)
        res[name].append(ms.value)
for name, t in res.items():
    med = statistics.median(t)
    vs = sets[name][0]
    print(f"{name:14s} apply {med:7.3f} ms  min {min(t):7.3f}  -> {1e3 / med:6.1f}/s   "
          + " | ".join(L.kexp_name(v).decode() for v in vs), flush=True)
