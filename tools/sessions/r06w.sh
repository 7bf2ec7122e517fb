#!/bin/bash
# r06w: the self-launched N = 2 / 4 rehearsals of bench.py on one GPU (gloo, ranks share the card)
# with the final round-6 tree (rccl mode field, copy rate, the new legs on one rank only)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r06w_rehearsal_n2.json 2> $OUT/r06w_rehearsal_n2.err
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r06w_rehearsal_n4.json 2> $OUT/r06w_rehearsal_n4.err
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline --rccl-blocking > $OUT/r06w_rehearsal_n2_blocking.json 2> $OUT/r06w_rehearsal_n2_blocking.err
