#!/bin/bash
# r04y GPU session: 512^3 P2 with non-temporal loads: parity, A/B.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_512" > $OUT/r04y_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 512 three five_y --iters 20 --rounds 3 > $OUT/r04y_ab512.jsonl 2>&1
