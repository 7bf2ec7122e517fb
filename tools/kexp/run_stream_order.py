#!/usr/bin/env python3
"""Streaming-kernel unit orders (stream_order.hip; GPU only, measurement tool).

    python tools/kexp/run_stream_order.py
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "stream_order.so"))
L.stream_order.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2 + [ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                                                        ctypes.POINTER(ctypes.c_float)]
N = 256 ** 3
x = torch.randn(N, dtype=torch.complex128, device="cuda")
y = torch.randn(N, dtype=torch.complex128, device="cuda")
part = torch.zeros(1 << 16, dtype=torch.float64, device="cuda")
ORD = {0: "grid-stride", 1: "grid-stride, XCD-contiguous", 2: "contiguous per WG"}
KIND = {0: ("axpy", 3), 1: ("dot", 2), 2: ("copy", 2)}
res = {}
for rnd in range(3):
    for blocks in (1024, 2048, 4096):
        for k in KIND:
            for o in ORD:
                ms = ctypes.c_float()
                rc = L.stream_order(o, k, blocks, y.data_ptr(), x.data_ptr(), N, part.data_ptr(), 50, ctypes.byref(ms))
                assert rc == 0, rc
                res.setdefault((blocks, k, o), []).append(ms.value * 1e3)
for (blocks, k, o), t in sorted(res.items()):
    t = sorted(t)
    name, nv = KIND[k]
    print(f"{name:5s} {blocks:5d} WG  {ORD[o]:28s} min {t[0]:7.1f} us  med {t[1]:7.1f} us  "
          f"({nv * 16 * N / (t[0] * 1e-6) / 1e12:5.2f} TB/s)", flush=True)
