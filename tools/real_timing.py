"""Timing of the real-data plan (f4) at 128/256/512^3 (PCApply/s and per-stage ms).  GPU only."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, circulantpreconditioner_amd as cp
for n in (256, 512, 128):
    N = n ** 3
    p = cp.RealPlan((n, n, n)).set_transport_symbol((0.6, 0.15, 0.02))
    b = torch.randn(N, dtype=torch.float64, device="cuda"); x = torch.empty_like(b)
    for _ in range(5): p.apply(b, x)
    torch.cuda.synchronize()
    it = 200 if n <= 256 else 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): p.apply(b, x)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(n, "real PCApply/s", round(1e3 / ms, 1), "ms", round(ms, 4), "stages", [round(v, 4) for v in p.time_passes(b, x, 10)], "moved GB/s ~", round(80 * N / (ms * 1e-3) / 1e9))
    p.close(); del b, x
