#!/usr/bin/env python3
"""Achievable copy bandwidth on this GPU for the 256^3 complex vector (268 MB): torch's copy
kernel, out of place and in place of a clone, HIP events over 200 copies (GPU only).  The
apply's passes are judged against it (profiles/r02c_seg_copy_patterns.txt)."""
import torch

N = 256 ** 3
b = torch.randn(N, dtype=torch.complex128, device="cuda")
x = torch.empty_like(b)
for name, fn in (("copy_ b -> x", lambda: x.copy_(b)), ("copy_ x -> b", lambda: b.copy_(x))):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1e3
    print(f"{name}: {us:.1f} us per 2 x {N * 16 / 1e6:.0f} MB = {2 * N * 16 / (us * 1e-6) / 1e12:.2f} TB/s", flush=True)
