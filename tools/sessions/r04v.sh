#!/bin/bash
# r04v GPU session: 100^3 middle kernel in XCD-aware unit order: parity, A/B, HBM traffic.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass_100 or plane" > $OUT/r04v_tests.log 2>&1
timeout -k 10 150 python tools/ab_sched.py 100 plane three:0,default three:0,lane64 three:0,lane32 > $OUT/r04v_ab100.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04v_pmc100_fetch -- python3 $ROOT/tools/ab_sched.py 100 three --iters 50 --rounds 1 > $OUT/r04v_pmc100_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04v_pmc100_write -- python3 $ROOT/tools/ab_sched.py 100 three --iters 50 --rounds 1 > $OUT/r04v_pmc100_write.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04v_prof100 -- python3 $ROOT/tools/ab_sched.py 100 three --iters 2000 --rounds 1 > $OUT/r04v_prof100.log 2>&1
