#!/bin/bash
# r04ag GPU session: 512^3 P2 at 32 points per thread (shape p32): parity, A/B, profile.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass_512 or schedule_rules" > $OUT/r04ag_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 512 three:0,default three:0,p32 --iters 30 --rounds 3 > $OUT/r04ag_ab512.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04ag_prof512 -- python3 $ROOT/tools/ab_sched.py 512 three:0,default three:0,p32 --iters 10 --rounds 1 > $OUT/r04ag_prof512.log 2>&1
