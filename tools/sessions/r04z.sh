#!/bin/bash
# r04z GPU session: 128^3 P2 on 4 x times 8 y2 tiles in XCD order (lane32 at n1 = 16): parity, A/B.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_128" > $OUT/r04z_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 128 three:0,default three:16,lane32 three:16,swap64 --iters 3000 --rounds 3 > $OUT/r04z_ab128.jsonl 2>&1
