#!/usr/bin/env python3
"""One parameterised GPU-box runner (replaces the round-1 one-off tools/gpu_*.sh scripts).

    gpurun -- python3 tools/gpu_run.py STEP [STEP ...]

Each STEP runs as a child process under its own time limit, writes its output under
gpurun_out/, and the runner stops at the first failing step (no retries, no further GPU
work after a fault, an abort or a time limit).  This process itself never touches the GPU.

Steps (fields separated by '@'; ARGS is a shell-split argument string):
  smoke                         __graft_entry__.smoke()
  tests[@ARGS]                  pytest -m gpu ARGS (default: the whole GPU suite)
  bench@TAG[@ARGS]              python3 bench.py ARGS > gpurun_out/TAG.json
  stats@TAG[@ARGS]              rocprofv3 --kernel-trace --stats around bench.py ARGS
  pmc@TAG@COUNTERS[@ARGS]       one rocprofv3 --pmc pass (COUNTERS comma-separated) around bench.py ARGS
  py@TAG@ARGS                   python3 ARGS > gpurun_out/TAG.txt  (any repo script)
  smi@TAG                       rocm-smi clocks/power snapshot (read only)
"""
from __future__ import annotations

import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = sys.executable or "python3"


def run(tag: str, argv: list[str], limit: int, out_name: str | None = None, cwd: str | None = None) -> int:
    os.makedirs(OUT, exist_ok=True)
    out_path = os.path.join(OUT, out_name or f"{tag}.log")
    err_path = out_path + ".err" if out_name else None
    t0 = time.time()
    print(f"[{time.strftime('%H:%M:%S')}] {tag}: {' '.join(argv)}", flush=True)
    with open(out_path, "w") as fo:
        fe = open(err_path, "w") if err_path else subprocess.STDOUT
        try:
            p = subprocess.run(["timeout", "-k", "10", str(limit)] + argv, stdout=fo, stderr=fe,
                               cwd=cwd or ROOT, env=dict(os.environ, PYTHONUNBUFFERED="1"))
        finally:
            if err_path:
                fe.close()
    rc = p.returncode
    print(f"    rc={rc} in {time.time() - t0:.1f} s -> {os.path.relpath(out_path, ROOT)}", flush=True)
    tail = open(out_path).read().strip().splitlines()[-3:]
    for line in tail:
        print("    | " + line[:300], flush=True)
    return rc


def prof_env():
    os.environ["TMPDIR"] = "/tmp"


def step(spec: str) -> int:
    f = spec.split("@")
    kind = f[0]
    if kind == "smoke":
        return run("smoke", [PY, "-c", "import __graft_entry__ as g; g.smoke()"], 300)
    if kind == "tests":
        extra = shlex.split(f[1]) if len(f) > 1 else []
        return run("tests" if len(f) < 3 else f[2],
                   [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-q", "--timeout", "300",
                    "--timeout-method", "thread"] + extra, 1100)
    if kind == "bench":
        tag, extra = f[1], shlex.split(f[2]) if len(f) > 2 else []
        return run(tag, [PY, os.path.join(ROOT, "bench.py")] + extra, 600, out_name=f"{tag}.json")
    if kind == "stats":
        tag, extra = f[1], shlex.split(f[2]) if len(f) > 2 else []
        prof_env()
        return run(tag, ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d",
                         os.path.join(OUT, tag), "-o", "run", "--", PY, os.path.join(ROOT, "bench.py")] + extra,
                   400, cwd="/tmp")
    if kind == "pmc":
        tag, counters, extra = f[1], f[2].split(","), shlex.split(f[3]) if len(f) > 3 else []
        prof_env()
        return run(tag, ["rocprofv3", "--pmc"] + counters + ["--kernel-trace", "--output-format", "csv", "-d",
                                                            os.path.join(OUT, tag), "-o", "run", "--", PY,
                                                            os.path.join(ROOT, "bench.py")] + extra,
                   180, cwd="/tmp")
    if kind == "py":
        return run(f[1], [PY] + shlex.split(f[2]), 900, out_name=f"{f[1]}.txt")
    if kind == "smi":
        return run(f[1], ["rocm-smi", "--showclocks", "--showpower", "--showtemp"], 60, out_name=f"{f[1]}.txt")
    print(f"unknown step {spec!r}", flush=True)
    return 2


def main() -> int:
    for spec in sys.argv[1:]:
        rc = step(spec)
        if rc != 0:
            print(f"stopping after {spec!r} (rc={rc})", flush=True)
            return rc
    print("all steps ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
