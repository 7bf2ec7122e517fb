#!/bin/bash
# r04aa GPU session: 256^3 permlane P2 on 32 columns in XCD order (swap32x): parity, A/B, profile;
# real 256^3 row sweeps with wave-local exchanges (three_alt): parity, A/B.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_real_gpu.py -k "three_pass_variants or three_pass_schedule or three_pass_vs or real_three_sweep" > $OUT/r04aa_tests.log 2>&1
timeout -k 10 200 python tools/ab_sched.py 256 three:0,default three:0,swap32x --iters 500 --rounds 3 > $OUT/r04aa_ab256.jsonl 2>&1
timeout -k 10 200 python tools/ab_sched.py 256 real:three real:three_alt --iters 500 --rounds 3 > $OUT/r04aa_abreal.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04aa_prof256 -- python3 $ROOT/tools/ab_sched.py 256 three:0,swap32x real:three_alt --iters 200 --rounds 1 > $OUT/r04aa_prof256.log 2>&1
