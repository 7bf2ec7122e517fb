#!/usr/bin/env python3
"""Timing probes of the 512^3 (and 256^3) row sweeps P1 / P3 (rows_512.hip; GPU only, measurement tool).

    python tools/kexp/run_rows_512.py     # every sweep x probe, 3 interleaved rounds, min / median
"""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "rows_512.so"))
L.rows_512.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
SWEEPS = {0: ("P1", 512), 1: ("P3", 512), 2: ("P1", 256), 3: ("P3", 256)}
PROBES = {0: "product", 1: "no loads", 2: "no stores", 3: "arithmetic + exchanges alone", 4: "memory alone",
          5: "memory + transpose", 6: "product, z-major units", 7: "memory alone, z-major units",
          8: "product, XCD unit order", 9: "memory alone, XCD unit order",
          10: "memory alone, XCD, 1 WG per CU"}
if os.environ.get("ROWS_PROBES"):
    PROBES = {int(p): PROBES[int(p)] for p in os.environ["ROWS_PROBES"].split(",")}
bufs = {}
for n in (512, 256):
    N = n ** 3
    bufs[n] = (torch.randn(N, dtype=torch.complex128, device="cuda"), torch.empty(N, dtype=torch.complex128, device="cuda"),
               torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda"))


def run(w, iters):
    n = SWEEPS[w % 10][1]
    b, x, tw = bufs[n]
    ms = ctypes.c_float()
    rc = L.rows_512(w, b.data_ptr(), x.data_ptr(), tw.data_ptr(), iters, ctypes.byref(ms))
    assert rc == 0, (w, rc)
    return ms.value * 1e3


res = {}
for rnd in range(3):
    for s in SWEEPS:
        for p in PROBES:
            res.setdefault(10 * p + s, []).append(run(10 * p + s, 10 if SWEEPS[s][1] == 512 else 40))
for s, (name, n) in SWEEPS.items():
    for p, pname in PROBES.items():
        t = sorted(res[10 * p + s])
        print(f"{name} {n}^3 {pname:30s} min {t[0]:8.1f} us  med {t[1]:8.1f} us  "
              f"({32 * n ** 3 / (t[0] * 1e-6) / 1e12:5.2f} TB/s on 32 N)", flush=True)
