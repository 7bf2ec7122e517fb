#!/bin/bash
# r05f GPU session: the new GPU tests (a missing RCCL peer times out; single-GPU 512^3 AUTO vs the
# oracle), and the self-launched N = 2 / 4 rehearsals of bench.py on one GPU (gloo, ranks share the card).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "missing_peer or single_gpu_512 or rccl_single" > $OUT/r05f_tests.log 2>&1
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r05f_rehearsal_n2.json 2> $OUT/r05f_rehearsal_n2.err
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r05f_rehearsal_n4.json 2> $OUT/r05f_rehearsal_n4.err
