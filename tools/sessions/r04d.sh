#!/bin/bash
# r04d GPU session: parity of the r04 changes since r04c (wave P2w with two lane maps, 512^3
# lane-pair rows, AUTO 3 sweeps at 100^3), the P2w probes, the 512^3 3-sweep profile, then the
# copy floors of the intermediate layouts and the 256^3 3-sweep shape A/B (bench + rocprof).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_wave.py > $OUT/r04d_tests.log 2>&1
timeout -k 10 300 $T tests/test_gpu_parity.py -k "three_pass or plane_schedule" >> $OUT/r04d_tests.log 2>&1
timeout -k 10 150 python tools/kexp/run_wave_probe.py > $OUT/r04d_wave_probe.txt 2>&1
timeout -k 10 150 python tools/ab_sched.py 512 auto three three:0,lane64 --iters 20 --rounds 2 > $OUT/r04d_ab512.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04d_prof512 -- python3 $GRAFT_REPO_ROOT/tools/ab_sched.py 512 three --iters 10 --rounds 1 > $OUT/r04d_prof512.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/kexp/run_seg_chain.py > $OUT/r04d_seg_chain.txt 2>&1
bash tools/ab_blocked.sh r04d
