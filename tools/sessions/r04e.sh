#!/bin/bash
# r04e GPU session: parity of the 512^3 blocked shape and the XCD-ordered blocked32 rows, the
# 512^3 shape A/B with its kernel profile, and the 256^3 blocked32 A/B against the default.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass" > $OUT/r04e_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 512 auto three three:0,blocked --iters 20 --rounds 2 > $OUT/r04e_ab512.jsonl 2>&1
timeout -k 10 150 python tools/ab_sched.py 256 three:0,default three:0,blocked32 --iters 500 --rounds 3 > $OUT/r04e_ab256.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04e_prof512 -- python3 $ROOT/tools/ab_sched.py 512 three:0,blocked --iters 10 --rounds 1 > $OUT/r04e_prof512.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04e_prof256 -- python3 $ROOT/tools/ab_sched.py 256 three:0,blocked32 --iters 200 --rounds 1 > $OUT/r04e_prof256.log 2>&1
