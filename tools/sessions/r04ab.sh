#!/bin/bash
# r04ab GPU session: P1 / P3 row FFT with wave-local exchanges (complex 128/256/512, default now;
# shape rowsalt = the r04 barriers) and the real rows (default now; real:three_alt = r04): parity, A/B.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_real_gpu.py -k "three_pass or real_three_sweep or real_plan" > $OUT/r04ab_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 256 three:0,default three:0,rowsalt real:three real:three_alt --iters 500 --rounds 3 > $OUT/r04ab_ab256.jsonl 2>&1
timeout -k 10 200 python tools/ab_sched.py 128 three:0,default three:0,rowsalt real:three real:three_alt --iters 2000 --rounds 3 > $OUT/r04ab_ab128.jsonl 2>&1
timeout -k 10 200 python tools/ab_sched.py 512 three:0,default three:0,rowsalt --iters 30 --rounds 2 > $OUT/r04ab_ab512.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04ab_prof256 -- python3 $ROOT/tools/ab_sched.py 256 three:0,default three:0,rowsalt real:three real:three_alt --iters 200 --rounds 1 > $OUT/r04ab_prof256.log 2>&1
