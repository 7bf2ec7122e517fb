#!/bin/bash
# r04h GPU session: real plan with non-temporal b loads (P1r) and x stores (P3r): parity, then
# its timing in two bench runs.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_real_gpu.py tests/test_real_scalar_gpu.py > $OUT/r04h_tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --scaling-grid 0 --no-cpu-baseline --no-configs > $OUT/r04h_bench_$rep.json 2> $OUT/r04h_bench_$rep.err
done
timeout -k 10 200 python tools/real_timing.py > $OUT/r04h_real_timing.txt 2>&1
