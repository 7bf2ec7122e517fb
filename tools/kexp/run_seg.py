#!/usr/bin/env python3
"""Copy bandwidth of candidate pass access patterns on a 256^3 c128 grid (tools/kexp/seg.hip).
Each case runs as a ping-pong chain (a->b, b->a) so every launch reads what the previous one
wrote, as in an apply.  GPU only."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "seg.so"))
L.seg_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 2 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
n = 256
N = n ** 3
a = torch.randn(N, dtype=torch.complex128, device="cuda")
b = torch.empty_like(a)
cases = [
    ("rows nr=8 consecutive", 0, 0, 8, 1), ("rows nr=16 consecutive", 0, 0, 16, 1),
    ("rows nr=16 y-stride16", 0, 0, 16, 16), ("rows nr=32 y-stride8", 0, 0, 32, 8),
    ("rows nr=64 y-stride4", 0, 0, 64, 4),
    ("cols tx=16 nr=1 (z pass now)", 1, 16, 1, 0), ("cols tx=32 nr=1", 1, 32, 1, 0),
    ("cols tx=16 nr=2", 1, 16, 2, 0), ("cols tx=16 nr=4", 1, 16, 4, 0),
    ("cols tx=8 nr=4", 1, 8, 4, 0), ("cols tx=8 nr=4 xcd", 1, 8, 4, 1),
    ("cols tx=8 nr=8", 1, 8, 8, 0), ("cols tx=8 nr=8 xcd", 1, 8, 8, 1),
    ("cols tx=4 nr=8", 1, 4, 8, 0), ("cols tx=4 nr=8 xcd", 1, 4, 8, 1),
    ("cols tx=4 nr=16", 1, 4, 16, 0), ("cols tx=4 nr=16 xcd", 1, 4, 16, 1),
    ("cols tx=2 nr=16", 1, 2, 16, 0), ("cols tx=2 nr=16 xcd", 1, 2, 16, 1),
]
res = {c[0]: [] for c in cases}
for rnd in range(3):
    for name, kind, tx, nr, x in cases:
        ms = ctypes.c_double()
        rc = L.seg_run(kind, tx, nr, x, a.data_ptr(), b.data_ptr(), 20, ctypes.byref(ms))
        assert rc == 0, (name, rc)
        res[name].append(ms.value)
        L.seg_run(kind, tx, nr, x, b.data_ptr(), a.data_ptr(), 1, ctypes.byref(ms))
torch.cuda.synchronize()
for name, *_ in cases:
    t = min(res[name])
    print(f"{name:34s} {t * 1e3:8.1f} us  {2 * N * 16 / (t * 1e-3) / 1e12:6.2f} TB/s")
