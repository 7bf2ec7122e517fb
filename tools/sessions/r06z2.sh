#!/bin/bash
# r06z2: the 32-point plane kernel: its parity tests, then 32^3 five passes against the plane schedule
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "plane" --timeout 200 --timeout-method thread > $OUT/r06z2_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 32 five plane --iters 2000 --rounds 3 > $OUT/r06z2_ab32.jsonl 2> $OUT/r06z2_ab32.err
timeout -k 10 200 python tools/ab_sched.py 64 five plane --iters 2000 --rounds 3 > $OUT/r06z2_ab64.jsonl 2> $OUT/r06z2_ab64.err
