#!/bin/bash
# r06z6: block SpMV software-pipelined over its grid-stride rows (CFP_BDIA_PF, 2 workgroups per
# CU): its tests, then same-box A/B of config 4's step (ab_v13: the same source with
# -DCFP_BDIA_PF=0) and the tree's kernels under rocprofv3
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wave.py tests/test_wave_mpi_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06z6_tests.log 2>&1
for r in 1 2 3; do
  for side in ab_v13 tree; do
    if [ $side = tree ]; then T=$ROOT; else T=$ROOT/$side; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 --legs 4 >> $OUT/r06z6_${side}.jsonl 2>> $OUT/r06z6_${side}.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06z6_prof -- python3 $ROOT/tools/gmres_legs.py --steps 10 --legs 4 > $OUT/r06z6_prof.log 2>&1
