#!/bin/bash
# r04ak GPU session: 128^3 P2 at 16 points per thread (shapes t16s / t16w): parity, A/B, profile.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass_128 or schedule_rules" > $OUT/r04ak_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 128 three:0,default three:0,t16s three:16,t16w --iters 3000 --rounds 3 > $OUT/r04ak_ab128.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04ak_prof128 -- python3 $ROOT/tools/ab_sched.py 128 three:0,default three:0,t16s three:16,t16w --iters 300 --rounds 1 > $OUT/r04ak_prof128.log 2>&1
