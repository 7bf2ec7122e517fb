#!/usr/bin/env python3
"""Time whole 5-launch applies (x, y, z-fused, y, x; each pass reads the previous output)
for sets of kernel variants of kexp.so, interleaved rounds in one process."""
import ctypes
import os
import statistics

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kexp.so"))
L.kexp_chain.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.kexp_name.restype = ctypes.c_char_p
SETS = {
    256: {"old": (0, 3, 6), "new_ntst": (1, 4, 7), "new_plain": (2, 5, 8), "new_ntldst": (9, 10, 11),
          "new_ntld": (12, 13, 14), "ntst_xy_only": (1, 4, 8), "ntst_yz": (2, 4, 7), "ntst_z_only": (2, 5, 7),
          "ntld_x_ntst_yz": (12, 4, 7)},
    512: {"old": (15, 24, 25), "new_plain": (15, 17, 19), "new_ntst": (16, 18, 20), "new_ntld": (21, 22, 23),
          "ntst_x_only": (16, 17, 19), "ntst_yz": (15, 18, 20)},
}
iters = {256: 20, 512: 4}
for n, sets in SETS.items():
    N = n ** 3
    b = torch.randn(N, dtype=torch.complex128, device="cuda")
    x = torch.empty_like(b)
    k = np.arange(n, dtype=np.longdouble)
    tw = torch.from_numpy((np.cos(2 * np.pi * k / n) - 1j * np.sin(2 * np.pi * k / n)).astype(np.complex128)).cuda()
    cs = torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1
    ax = torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1
    res = {k: [] for k in sets}
    for rnd in range(5):
        for name, (i, j, l) in sets.items():
            ms = ctypes.c_double()
            rc = L.kexp_chain(i, j, l, b.data_ptr(), x.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                              iters[n], ctypes.byref(ms))
            assert rc == 0, rc
            res[name].append(ms.value)
    for name, t in res.items():
        med = statistics.median(t)
        print(f"n={n} {name:18s} apply {med * 1e3:8.1f} us  min {min(t) * 1e3:8.1f}  -> {1e3 / med:8.1f} applies/s   "
              f"[{', '.join(L.kexp_name(v).decode() for v in sets[name])}]")
