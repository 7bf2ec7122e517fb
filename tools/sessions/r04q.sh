#!/bin/bash
# r04q GPU session: 128^3 y split 16 x 8 shapes: parity, A/B, kernel profile.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_128 or schedule_rules" > $OUT/r04q_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 128 three:32,default three:0,default three:16,lane64 three:16,swap64 --iters 3000 --rounds 3 > $OUT/r04q_ab128.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04q_prof128 -- python3 $ROOT/tools/ab_sched.py 128 three:16,lane64 three:16,swap64 --iters 2000 --rounds 1 > $OUT/r04q_prof128.log 2>&1
