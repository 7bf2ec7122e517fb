#!/usr/bin/env python3
"""Item 6 probe (grid_probe.hip): the cost of one grid barrier in a cooperative launch, and three
streaming sweeps over a 128^3 / 100^3 / 256^3 complex vector as three launches against one
persistent launch with two grid barriers (the most a persistent 3-phase apply can save)."""
import ctypes
import os

import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "grid_probe.so"))
L.grid_probe.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4 + [ctypes.c_long, ctypes.c_int,
                                                                       ctypes.POINTER(ctypes.c_float)]
L.grid_probe_max_wgs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
cus = torch.cuda.get_device_properties(0).multi_processor_count
print(f"CUs: {cus}")


def call(which, tb, wgs, rounds, a, t, u, o, n, iters):
    ms = ctypes.c_float()
    rc = L.grid_probe(which, tb, wgs, rounds, a, t, u, o, n, iters, ctypes.byref(ms))
    assert rc == 0, (which, tb, wgs, rc)
    return ms.value * 1e3


for tb in (256, 1024):
    pc = ctypes.c_int()
    assert L.grid_probe_max_wgs(0, tb, ctypes.byref(pc)) == 0
    for per_cu in sorted({1, min(2, pc.value), pc.value}):
        wgs = cus * per_cu
        for w, name in ((0, "flat"), (3, "two-level")):
            us1 = call(w, tb, wgs, 1, 0, 0, 0, 0, 0, 200)
            us100 = call(w, tb, wgs, 101, 0, 0, 0, 0, 0, 20)
            print(f"barriers ({name}): TB={tb} wgs={wgs} ({per_cu}/CU): one launch with 1 barrier {us1:.2f} us, "
                  f"per extra barrier {(us100 - us1) / 100:.2f} us", flush=True)
    for w, name in ((10, "relaxed atomics, no fence"), (11, "acquire fence only"), (12, "release fence only"),
                    (13, "both fences")):
        us1 = call(w, tb, cus, 1, 0, 0, 0, 0, 0, 200)
        us100 = call(w, tb, cus, 101, 0, 0, 0, 0, 0, 20)
        print(f"barrier cost, {name}: TB={tb} wgs={cus}: per barrier {(us100 - us1) / 100:.2f} us", flush=True)
    us0 = call(1, tb, cus, 0, 0, 0, 0, 0, 0, 200)  # three empty sweeps (n = 0): launch floor
    print(f"three empty launches back to back: TB={tb} wgs={cus}: {us0:.2f} us", flush=True)

for side in (100, 128, 256):
    n = side ** 3
    a = torch.randn(n, dtype=torch.complex128, device="cuda")
    t, u, o = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    for tb in (256, 1024):
        pc = ctypes.c_int()
        assert L.grid_probe_max_wgs(1, tb, ctypes.byref(pc)) == 0
        for per_cu in sorted({1, min(2, pc.value), pc.value}):
            wgs = cus * per_cu
            rows = []
            for rep in range(3):  # interleaved rounds
                sep = call(1, tb, wgs, 0, a.data_ptr(), t.data_ptr(), u.data_ptr(), o.data_ptr(), n, 200)
                per = call(2, tb, wgs, 0, a.data_ptr(), t.data_ptr(), u.data_ptr(), o.data_ptr(), n, 200)
                o.zero_()
                per2 = call(4, tb, wgs, 0, a.data_ptr(), t.data_ptr(), u.data_ptr(), o.data_ptr(), n, 200)
                ok2 = torch.equal(o, a)
                o.zero_()
                per3 = call(14, tb, wgs, 0, a.data_ptr(), t.data_ptr(), u.data_ptr(), o.data_ptr(), n, 200)
                rows.append((sep, per, per2, per3))
            ok = ok2 and torch.equal(o, a)
            sep, per, per2, per3 = (min(r[i] for r in rows) for i in range(4))
            print(f"{side}^3 ({n * 16 / 2**20:.0f} MiB): TB={tb} wgs={wgs} ({per_cu}/CU): 3 launches {sep:.2f} us, "
                  f"1 persistent launch + 2 barriers: flat {per:.2f} us ({(per - sep):+.2f}), two-level "
                  f"{per2:.2f} us ({(per2 - sep):+.2f}), fences once {per3:.2f} us ({(per3 - sep):+.2f}), "
                  f"output ok={ok}", flush=True)
    del a, t, u, o
    torch.cuda.empty_cache()
