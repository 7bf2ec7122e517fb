#!/bin/bash
# r04x GPU session: wave P3w store policy A/B (bench other_configs, two runs).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_wave.py -k "three" > $OUT/r04x_tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --scaling-grid 0 --no-cpu-baseline --no-real > $OUT/r04x_bench_$rep.json 2> $OUT/r04x_bench_$rep.err
done
