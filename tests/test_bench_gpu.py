"""bench.py's N > 1 launch on the GPU box: `bench.py --gpus 2` without a
launcher starts its two ranks itself and both drive the card (CFP_BENCH_SHARE_DEVICE=1, gloo
process group).  RCCL cannot put two ranks on one GPU, so the line carries the labelled
torch-fallback exchange; the apply's output check still runs on the device."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_gpus_2_self_launched_rehearsal():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "CFP_BENCH_SELF_LAUNCHED")}
    env.update({"CFP_BENCH_SHARE_DEVICE": "1", "CFP_BENCH_BACKEND": "gloo"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--grid", "64",
                        "--scaling-grid", "0", "--no-configs", "--no-real", "--no-cpu-baseline", "--steps", "5",
                        "--warmup", "2", "--settle-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0, p.stderr[-4000:]
    assert len(lines) == 1
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["status"] == "ok" and ln["launcher"] == "self (torch.distributed.run)"
    assert ln["check"]["ok"] and ln["check"]["residual"] < 1e-10
    assert ln["exchange"] in ("rccl", "torch-fallback") and "rccl" in ln["rccl"]["lib"]
