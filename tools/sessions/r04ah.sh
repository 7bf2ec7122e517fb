#!/bin/bash
# r04ah GPU session: 100^3 S2 with two units per workgroup and a register prefetch of the
# second (shapes swap64 = 2 x tiles, swap64pf = 1 x tiles): parity, A/B, profile.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass_100" > $OUT/r04ah_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 100 three:0,default three:0,swap64 three:0,swap64pf --iters 3000 --rounds 3 > $OUT/r04ah_ab100.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04ah_prof100 -- python3 $ROOT/tools/ab_sched.py 100 three:0,default three:0,swap64 three:0,swap64pf --iters 500 --rounds 1 > $OUT/r04ah_prof100.log 2>&1
