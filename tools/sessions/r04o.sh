#!/bin/bash
# r04o GPU session: 128^3 rows with the default cache policy (b and x stay in the Infinity Cache)
# against the 256^3 NT policy (shape swap64): parity, A/B, bench other_configs.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_128" > $OUT/r04o_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 128 three:0,default three:0,swap64 five --iters 3000 --rounds 3 > $OUT/r04o_ab128.jsonl 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --scaling-grid 0 --no-cpu-baseline --no-real > $OUT/r04o_bench.json 2> $OUT/r04o_bench.err
