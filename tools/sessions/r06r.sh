#!/bin/bash
# r06r: the wave dots inside P3w: their tests, then same-box A/B of config 4's step, ab_v6/ (dots
# as separate sweeps) against the working tree, 3 alternating rounds
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wave.py tests/test_wave_mpi_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06r_tests.log 2>&1
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then T=$ROOT/ab_v6; else T=$ROOT; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 --legs 4 >> $OUT/r06r_${side}.jsonl 2>> $OUT/r06r_${side}.err
  done
done
