#!/usr/bin/env python3
"""Whole 5-launch applies in two axis orders at 256^3 (interleaved rounds, one process):
z-fused (x, y, z*, y, x; the product's AUTO order) vs x-fused (z, y, x*, y, z) with row-mode
fused-pass shapes 60..67 of kexp.so."""
import ctypes
import os
import statistics

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kexp.so"))
L.kexp_chain_axes.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)] + \
    [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.kexp_name.restype = ctypes.c_char_p
n = 256
N = n ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
k = np.arange(n, dtype=np.longdouble)
tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
sets = {"zfused_product": ((1, 4, 42, 5, 2), (0, 1, 2, 1, 0))}
for v in range(60, 68):
    sets[f"xfused_v{v}"] = ((4, 4, v, 5, 5), (2, 1, 0, 1, 2))
sets["xfused_v61_ldz"] = ((4, 3, 61, 5, 5), (2, 1, 0, 1, 2))
res = {s: [] for s in sets}
for rnd in range(7):
    for name, (vs, axs) in sets.items():
        ms = ctypes.c_double()
        va = (ctypes.c_int * 5)(*vs)
        aa = (ctypes.c_int * 5)(*axs)
        rc = L.kexp_chain_axes(5, va, aa, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                               20, ctypes.byref(ms))
        assert rc == 0, (name, rc)
        res[name].append(ms.value)
for name, t in res.items():
    med = statistics.median(t)
    fused = sets[name][0][2]
    print(f"{name:18s} apply {med * 1e3:7.1f} us  min {min(t) * 1e3:7.1f}  -> {1e3 / med:7.1f}/s   fused "
          f"{L.kexp_name(fused).decode()}", flush=True)
