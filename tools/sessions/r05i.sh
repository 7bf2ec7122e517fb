#!/bin/bash
# r05i: 512^3 blocked intermediate layouts -- P2 probes, parity, whole-schedule A/B, kernel stats
set -e
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p $OUT
P2_WHICH=0,9,10,11,12,13 timeout -k 10 300 python -u tools/kexp/run_p2_512.py > $OUT/r05i_p2_512_blocked.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "three_pass_512" --timeout 240 --timeout-method thread > $OUT/r05i_parity.log 2>&1
timeout -k 10 300 python -u tools/ab_sched.py 512 three:0,default three:0,blocked three:0,blocked32 --iters 200 --rounds 3 > $OUT/r05i_ab512.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/r05i_prof_ab512 -- python3 $ROOT/tools/ab_sched.py 512 three:0,default three:0,blocked32 --iters 100 --rounds 1 > $ROOT/$OUT/r05i_prof_ab512.log 2>&1
