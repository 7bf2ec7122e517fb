#!/usr/bin/env python3
"""Exhaustive store/load-policy sweep over the five launches of one apply (x-fwd, y-fwd,
z-fused, y-inv, x-inv), each in {plain, NT loads, NT stores}; whole-apply timing."""
import ctypes
import itertools
import os
import statistics
import sys

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kexp.so"))
L.kexp_chain.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
BASE = {256: (0, 3, 6), 512: (9, 12, 15), 128: (18, 21, 24)}
iters = {128: 100, 256: 10, 512: 2}
POL = ("pl", "ld", "st")
for n in [int(a) for a in sys.argv[1:]] or (256, 512, 128):
    N = n ** 3
    b = torch.randn(N, dtype=torch.complex128, device="cuda")
    x = torch.empty_like(b)
    k = np.arange(n, dtype=np.longdouble)
    tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
    cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
    ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
    rx, ry, rz = BASE[n]
    combos = list(itertools.product(range(3), repeat=5))
    res = {c: [] for c in combos}
    for rnd in range(3):
        for c in combos:
            ids = (rx + c[0], ry + c[1], rz + c[2], ry + c[3], rx + c[4])
            ms = ctypes.c_double()
            rc = L.kexp_chain(*ids, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                              iters[n], ctypes.byref(ms))
            assert rc == 0, rc
            res[c].append(ms.value)
    ranked = sorted(combos, key=lambda c: statistics.median(res[c]))
    base = statistics.median(res[(0, 0, 0, 0, 0)])
    print(f"n={n}: all-plain apply {base * 1e3:.1f} us")
    for c in ranked[:12] + ranked[-3:]:
        med = statistics.median(res[c])
        print(f"  x-fwd={POL[c[0]]} y-fwd={POL[c[1]]} z={POL[c[2]]} y-inv={POL[c[3]]} x-inv={POL[c[4]]}: "
              f"{med * 1e3:8.1f} us  {1e3 / med:8.1f}/s  ({(base / med - 1) * 100:+.1f}%)")
