#!/bin/bash
# r06t: software-pipelined block SpMV: its tests, then same-box A/B of config 4's step and the
# kernel under rocprofv3 (ab_v8/ = previous kernel)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wave.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06t_tests.log 2>&1
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then T=$ROOT/ab_v8; else T=$ROOT; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 --legs 4 >> $OUT/r06t_${side}.jsonl 2>> $OUT/r06t_${side}.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06t_prof -- python3 $ROOT/tools/gmres_legs.py --steps 10 --legs 4 > $OUT/r06t_prof.log 2>&1
