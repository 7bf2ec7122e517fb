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
import sys
X, Y, Y2, X2 = 1, 3, 5, 2
if "--rev" in sys.argv:
    chains = {"product": (1, 3, 7, 5, 2), "rev y,y-inv": (1, 38, 7, 40, 2), "rev x,z,x-inv": (37, 3, 39, 5, 41),
              "rev all": (37, 38, 39, 40, 41), "rev y-fwd only": (1, 38, 7, 5, 2), "rev x-inv only": (1, 3, 7, 5, 41)}
elif "--occ" in sys.argv:
    chains = {L.kexp_name(f).decode(): (X, Y, f, Y2, X2) for f in [7] + list(range(42, 50))}
else:
    chains = {L.kexp_name(f).decode(): (X, Y, f, Y2, X2) for f in [7] + list(range(27, 37))}
res = {c: [] for c in chains}
outs = {}
for rnd in range(5):
    for c, idx in chains.items():
        ms = ctypes.c_double()
        rc = L.kexp_chain(*idx, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                          20, ctypes.byref(ms))
        assert rc == 0, (c, rc)
        res[c].append(ms.value)
        if rnd == 0:
            outs[c] = x.clone()
ref = outs[next(iter(chains))]
for c in chains:
    t = statistics.median(res[c])
    err = float(torch.linalg.vector_norm(outs[c] - ref) / torch.linalg.vector_norm(ref))
    print(f"{c:38s} apply {t * 1e3:7.1f} us  min {min(res[c]) * 1e3:7.1f}  rel-diff {err:.1e}")
