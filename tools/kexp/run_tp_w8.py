#!/usr/bin/env python3
"""A/B of the 256^3 3-sweep chain (tp_chain.hip): the product P2 (k_tp_mid_sw, 16 waves) against
lane-pair phase A (which + 64), product cache policies, interleaved rounds, plus an output
comparison of the two chains on the same input."""
import ctypes
import sys
import os

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tp_chain.so"))
L.tp_chain.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = 256
b = torch.randn(n ** 3, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
tw = torch.from_numpy(np.exp(-2j * np.pi * np.arange(n) / n)).to("cuda")
cs = torch.full((n * n,), 0.5 + 0.1j, dtype=torch.complex128, device="cuda")
ax = torch.full((n,), 0.25, dtype=torch.complex128, device="cuda")
cases = {"product (LP rows, sw P2)": 64, "w8 P2, VPF 0": 64 + 256, "w8 P2, VPF 8": 64 + 512, "w8 P2, VPF 16 (spills)": 64 + 768}
if len(sys.argv) > 1:  # name=which pairs against the product
    cases = {"product (LP rows, sw P2)": 64}
    cases.update({kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[1:]})
outs = {}
for name, c in cases.items():
    ms = ctypes.c_float()
    assert L.tp_chain(c, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(), 1,
                      ctypes.byref(ms)) == 0
    torch.cuda.synchronize()
    outs[name] = x.clone()
ref = outs["product (LP rows, sw P2)"]
for name, o in outs.items():
    print(f"{name:30s} max |x - x_product| / max |x_product| = {float((o - ref).abs().max() / ref.abs().max()):.3e}", flush=True)
res = {c: [] for c in cases.values()}
for rnd in range(5):
    for c in cases.values():
        ms = ctypes.c_float()
        assert L.tp_chain(c, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(), 100,
                          ctypes.byref(ms)) == 0
        res[c].append(ms.value * 1e3)
for name, c in cases.items():
    print(f"{name:30s} min {min(res[c]):6.1f} us  ({', '.join('%.1f' % t for t in res[c])})", flush=True)
