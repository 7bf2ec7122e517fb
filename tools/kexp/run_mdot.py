#!/usr/bin/env python3
"""The stand-in's VecMDot (k_mdot + k_mdot_finish) on fresh 256^3 device Vecs, with 1 and 2
vectors, beside torch.vdot -- for rocprofv3 --kernel-trace --stats (GPU only, measurement tool).

    rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/kexp/run_mdot.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from circulantpreconditioner_amd._lib import lib  # noqa: E402
from circulantpreconditioner_amd._lib_ext import PetscScalar  # noqa: E402
from circulantpreconditioner_amd.petsc import Vec  # noqa: E402

N = 256 ** 3
t = [torch.randn(N, dtype=torch.complex128, device="cuda") for _ in range(3)]
V = [Vec.from_tensor(x) for x in t]
ys = (ctypes.c_void_p * 2)(V[1].h.value, V[2].h.value)
vals = (PetscScalar * 2)()
for nv in (1, 2):
    for _ in range(40):
        assert lib().VecMDot(V[0].h, nv, ys, vals) == 0
torch.cuda.synchronize()
for _ in range(40):
    torch.vdot(t[1], t[0])
torch.cuda.synchronize()
print("ok", vals[0].re if hasattr(vals[0], "re") else "", flush=True)
