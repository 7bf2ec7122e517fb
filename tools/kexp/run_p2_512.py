#!/usr/bin/env python3
"""512^3 P2 variants of p2_512.hip (GPU only, measurement tool).

    python tools/kexp/run_p2_512.py            # time every variant, 3 interleaved rounds
    python tools/kexp/run_p2_512.py W ITERS    # run variant W ITERS times (for rocprofv3 --pmc)
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "p2_512.so"))
L.p2_512.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = 512
N = n ** 3
data = torch.randn(N, dtype=torch.complex128, device="cuda")
tw = torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda")
colsym = torch.full((n * n,), 0.5 + 0.1j, dtype=torch.complex128, device="cuda")
axsym = torch.full((n,), 0.25, dtype=torch.complex128, device="cuda")
NAMES = {0: "product (XCD order, 256 WG)", 1: "NT stores", 2: "128 WG", 3: "64 WG", 4: "blockIdx order",
         5: "probe: no WG barriers", 6: "probe: no loads", 7: "probe: no stores", 8: "probe: math + xchg alone",
         9: "probe: memory alone", 10: "blocks of 8 x: memory alone", 11: "blocks of 8 x",
         12: "blocks of 2 x: memory alone", 13: "blocks of 2 x"}
if os.environ.get("P2_WHICH"):
    NAMES = {int(w): NAMES[int(w)] for w in os.environ["P2_WHICH"].split(",")}


def run(w, iters):
    ms = ctypes.c_float()
    rc = L.p2_512(w, data.data_ptr(), tw.data_ptr(), colsym.data_ptr(), axsym.data_ptr(), iters, ctypes.byref(ms))
    assert rc == 0, (w, rc)
    return ms.value * 1e3


if len(sys.argv) > 1:
    run(int(sys.argv[1]), int(sys.argv[2]))
    torch.cuda.synchronize()
    print("ok", flush=True)
else:
    res = {w: [] for w in NAMES}
    for rnd in range(3):
        for w in NAMES:
            res[w].append(run(w, 10))
    for w, name in NAMES.items():
        t = sorted(res[w])
        print(f"{w} {name:30s} min {t[0]:8.1f} us  med {t[1]:8.1f} us  ({32 * N / (t[0] * 1e-6) / 1e12:5.2f} TB/s on 32 N)",
              flush=True)
