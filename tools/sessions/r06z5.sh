#!/bin/bash
# r06z5: VecAXPY leaves the |y|^2 partials for the following VecNorm: its tests and the GMRES
# drivers' tests, then same-box A/B of the three GMRES legs (ab_v12/ = the previous commit)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_transport.py tests/test_wave.py tests/test_mpi_gmres_gpu.py tests/test_pcshell_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06z5_tests.log 2>&1
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then T=$ROOT/ab_v12; else T=$ROOT; fi
    timeout -k 10 300 python3 $T/tools/gmres_legs.py --steps 20 >> $OUT/r06z5_${side}.jsonl 2>> $OUT/r06z5_${side}.err
  done
done
