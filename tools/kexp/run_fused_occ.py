#!/usr/bin/env python3
"""Whole 5-launch applies at 256^3 with the fused z pass at higher occupancy (variants 83..87:
8-wave requests with PTS 8 / PTS 4) against the product's fused shape (42), interleaved rounds."""
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
b = torch.randn(n ** 3, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
k = np.arange(n, dtype=np.longdouble)
tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
ZF = (0, 1, 2, 1, 0)
sets = {f"fused{v}": ((1, 4, v, 5, 2), ZF) for v in (42, 83, 84, 85, 86, 87)}
res = {s: [] for s in sets}
for rnd in range(7):
    for name, (vs, axs) in sets.items():
        ms = ctypes.c_double()
        rc = L.kexp_chain_axes(5, (ctypes.c_int * 5)(*vs), (ctypes.c_int * 5)(*axs), b.data_ptr(), x.data_ptr(),
                               tw.data_ptr(), cs.data_ptr(), ax.data_ptr(), 20, ctypes.byref(ms))
        assert rc == 0, (name, rc)
        res[name].append(ms.value)
for name, t in res.items():
    med = statistics.median(t)
    print(f"{name:9s} apply {med * 1e3:7.1f} us  min {min(t) * 1e3:7.1f}  -> {1e3 / med:7.1f}/s   "
          f"{L.kexp_name(sets[name][0][2]).decode()}", flush=True)
