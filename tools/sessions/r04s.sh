#!/bin/bash
# r04s GPU session: real plan variants (Nyquist launch at 4 points per thread, P3r whole-complex):
# parity, then its stage time in two bench runs.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_real_gpu.py > $OUT/r04s_tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --scaling-grid 0 --no-cpu-baseline --no-configs > $OUT/r04s_bench_$rep.json 2> $OUT/r04s_bench_$rep.err
done
