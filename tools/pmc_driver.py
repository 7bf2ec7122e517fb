#!/usr/bin/env python3
"""A short apply loop to run under `rocprofv3 --pmc` (GPU only; measurement tool, not a test).

  python tools/pmc_driver.py real 256 [iters]   # RealPlan apply (r2c 3-sweep at 128^3 / 256^3)
  python tools/pmc_driver.py wave 128 [iters]   # WavePlan block apply (3 sweeps at 128^3)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import circulantpreconditioner_amd as cp  # noqa: E402


def main() -> int:
    kind, n = sys.argv[1], int(sys.argv[2])
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    N = n ** 3
    if kind == "real":
        p = cp.RealPlan((n, n, n)).set_transport_symbol((0.6, 0.15, 0.02))
        b = torch.randn(N, dtype=torch.float64, device="cuda")
        x = torch.empty_like(b)
        run = lambda: p.apply(b, x)  # noqa: E731
    elif kind == "wave":
        from circulantpreconditioner_amd.wave import WavePlan
        p = WavePlan((n, n, n)).set_symbol((0.3, 0.3, 0.3))
        b = torch.randn(4 * N, dtype=torch.complex128, device="cuda")
        x = torch.empty_like(b)
        run = lambda: p.apply(b, out=x)  # noqa: E731
    else:
        raise SystemExit(f"unknown kind {kind}")
    for _ in range(iters):
        run()
    torch.cuda.synchronize()
    print(kind, n, "ok", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
