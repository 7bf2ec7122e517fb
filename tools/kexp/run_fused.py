#!/usr/bin/env python3
"""Whole-apply timing of fused-pass shapes at 256^3: x/y/y-inv/x-inv fixed at the product's
choices, the fused z pass swapped (kexp.so variants), interleaved rounds.  GPU only."""
import ctypes
import os
import statistics

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kexp.so"))
L.kexp_chain.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.kexp_name.restype = ctypes.c_char_p
L.kexp_time.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
n = 256
N = n ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
k = np.arange(n, dtype=np.longdouble)
tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
X, Y, Y2, X2 = 1, 3, 5, 2
fused = [7] + list(range(27, 37))
res = {f: [] for f in fused}
outs = {}
for rnd in range(5):
    for f in fused:
        ms = ctypes.c_double()
        rc = L.kexp_chain(X, Y, f, Y2, X2, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                          20, ctypes.byref(ms))
        assert rc == 0, (f, rc)
        res[f].append(ms.value)
        if rnd == 0:
            outs[f] = x.clone()
ref = outs[7]
for f in fused:
    t = statistics.median(res[f])
    err = float(torch.linalg.vector_norm(outs[f] - ref) / torch.linalg.vector_norm(ref))
    print(f"{L.kexp_name(f).decode():38s} apply {t * 1e3:7.1f} us  min {min(res[f]) * 1e3:7.1f}  rel-diff {err:.1e}")
