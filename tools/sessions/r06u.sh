#!/bin/bash
# r06u: unrolled MAXPY kernels: the solver tests, then
# same-box A/B of the GMRES legs, ab_v9/ (previous MAXPY kernels) against the working tree
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_transport.py tests/test_fused_gpu.py tests/test_wave.py tests/test_mpi_gmres_gpu.py tests/test_wave_mpi_gpu.py -q -m gpu --timeout 250 --timeout-method thread > $OUT/r06u_tests.log 2>&1 || true
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then T=$ROOT/ab_v9; else T=$ROOT; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 >> $OUT/r06u_${side}.jsonl 2>> $OUT/r06u_${side}.err
  done
done
