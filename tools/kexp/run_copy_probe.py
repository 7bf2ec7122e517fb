#!/usr/bin/env python3
"""Copy-rate probe (copy_probe.hip) on the 256^3 complex vector (268 MB) and a 2 GB one."""
import ctypes
import os

import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "copy_probe.so"))
L.copy_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                         ctypes.POINTER(ctypes.c_float)]
cus = torch.cuda.get_device_properties(0).multi_processor_count
for n in (256 ** 3, 512 ** 3 // 4):
    a = torch.randn(n, dtype=torch.complex128, device="cuda")
    b = torch.empty_like(a)
    best = []
    for bsel in (0, 1, 2):
        for pol in (0, 1, 2, 3):
            for U in (1, 2, 4, 8):
                w = U + 16 * pol + 64 * bsel
                ms = ctypes.c_float()
                rc = L.copy_probe(w, a.data_ptr(), b.data_ptr(), n, cus, 50, ctypes.byref(ms))
                assert rc == 0, (w, rc)
                tbs = 2 * n * 16 / (ms.value * 1e-3) / 1e12
                best.append((tbs, U, pol, (4, 8, 16)[bsel], ms.value * 1e3))
    best.sort(reverse=True)
    print(f"n = {n} ({n * 16 / 1e6:.0f} MB): best 6 of 48 (TB/s, U, policy 1=nt ld 2=nt st, WG/CU, us)")
    for r in best[:6]:
        print("   %.2f  U=%d pol=%d wg/cu=%d  %.1f us" % r)
    print("   worst: %.2f  U=%d pol=%d wg/cu=%d  %.1f us" % best[-1], flush=True)
    del a, b
    torch.cuda.empty_cache()
