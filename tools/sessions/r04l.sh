#!/bin/bash
# r04l GPU session: 100^3 middle kernel with padded transposes: parity, A/B, kernel profile.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_100 or plane" > $OUT/r04l_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 100 plane three:0,default three:0,lane64 three:0,lane32 > $OUT/r04l_ab100.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04l_prof100 -- python3 $ROOT/tools/ab_sched.py 100 three --iters 2000 --rounds 1 > $OUT/r04l_prof100.log 2>&1
