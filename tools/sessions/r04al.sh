#!/bin/bash
# r04al GPU session: 256^3 P2 (default shape) with its units in XCD order (shape xcd): parity, A/B.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass_variants or schedule_rules" > $OUT/r04al_tests.log 2>&1
timeout -k 10 250 python tools/ab_sched.py 256 three:0,default three:0,xcd --iters 600 --rounds 4 > $OUT/r04al_ab256.jsonl 2>&1
