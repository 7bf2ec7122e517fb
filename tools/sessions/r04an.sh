#!/bin/bash
# r04an GPU session (experiment): real 256^3 P3r with split exchanges at three workgroups per CU
# (real:three_alt, 72 B/lane of scratch) against the whole-complex two per CU (real:three).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_real_gpu.py -k "real_three_sweep" > $OUT/r04an_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 256 real:three real:three_alt --iters 1000 --rounds 3 > $OUT/r04an_ab.jsonl 2>&1
