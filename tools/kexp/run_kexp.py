#!/usr/bin/env python3
"""Time every kernel variant of kexp.so in one process (interleaved rounds), check each
against the first variant of its (N, row, mode) group, print a table.  GPU only."""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "kexp.so"))
L.kexp_name.restype = ctypes.c_char_p
L.kexp_time.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
nv = L.kexp_count()
info = []
for i in range(nv):
    vals = [ctypes.c_int() for _ in range(6)]
    L.kexp_info(i, *[ctypes.byref(v) for v in vals])
    info.append(dict(zip(("n", "row", "T", "threads", "mode", "flags"), [v.value for v in vals]), name=L.kexp_name(i).decode()))
sizes = sorted({v["n"] for v in info})
only = [int(a) for a in sys.argv[1:]] or sizes
bufs = {}
for n in only:
    N = n ** 3
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(N, dtype=torch.complex128, device="cuda", generator=g)
    k = np.arange(n, dtype=np.longdouble)
    ang = 2 * np.pi * k / n
    tw = torch.from_numpy((np.cos(ang).astype(np.float64) - 1j * np.sin(ang).astype(np.float64))).cuda()
    colsym = (torch.randn(n * n, dtype=torch.complex128, device="cuda") * 0.1)
    axsym = (torch.randn(n, dtype=torch.complex128, device="cuda") * 0.1)
    bufs[n] = (a, torch.empty_like(a), tw, colsym, axsym)
iters = {128: 50, 256: 20, 512: 4, 1024: 2}
runs = []
for i in range(nv):
    if info[i]["n"] not in only:
        continue
    for axis in ((1, 2) if not info[i]["row"] else (0,)):
        runs.append((i, axis))
res = {r: [] for r in runs}
ref_out = {}
for rnd in range(3):
    for (i, axis) in res:
        v = info[i]
        a, o, tw, cs, ax = bufs[v["n"]]
        ms = ctypes.c_double()
        rc = L.kexp_time(i, a.data_ptr(), o.data_ptr(), tw.data_ptr(), cs.data_ptr(), ax.data_ptr(),
                         iters[v["n"]], ctypes.byref(ms), axis)
        if rc:
            print("variant", v["name"], "failed rc", rc)
            continue
        res[(i, axis)].append(ms.value)
        if rnd == 0:
            key = (v["n"], v["row"], v["mode"], axis)
            if key not in ref_out:
                ref_out[key] = o.clone()
                v["err%d" % axis] = 0.0
            else:
                v["err%d" % axis] = float(torch.linalg.vector_norm(o - ref_out[key]) / torch.linalg.vector_norm(ref_out[key]))
print(f"{'variant':44s} ax {'thr':>5s} {'med us':>9s} {'min us':>9s} {'GB/s':>7s} {'relerr':>9s}")
for (i, axis), t in res.items():
    v = info[i]
    if not t:
        continue
    med, mn = statistics.median(t), min(t)
    gbs = 32 * v["n"] ** 3 / (med * 1e-3) / 1e9
    print(f"{v['name']:44s} {'xyz'[axis]}  {v['threads']:5d} {med * 1e3:9.1f} {mn * 1e3:9.1f} {gbs:7.0f} {v.get('err%d' % axis, float('nan')):9.1e}")
