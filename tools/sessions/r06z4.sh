#!/bin/bash
# r06z4: block SpMV with XCD-contiguous cells (CFP_BDIA_XCD) and real-coefficient products
# (CFP_BDIA_RE): its tests, then same-box A/B of config 4's step over four builds of the same
# source (ab_v9: neither, ab_v10: XCD only, ab_v11: RE only, the tree: both) and the tree's
# kernels under rocprofv3
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wave.py tests/test_wave_mpi_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06z4_tests.log 2>&1
for r in 1 2 3; do
  for side in ab_v9 ab_v10 ab_v11 tree; do
    if [ $side = tree ]; then T=$ROOT; else T=$ROOT/$side; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 --legs 4 >> $OUT/r06z4_${side}.jsonl 2>> $OUT/r06z4_${side}.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06z4_prof -- python3 $ROOT/tools/gmres_legs.py --steps 10 --legs 4 > $OUT/r06z4_prof.log 2>&1
