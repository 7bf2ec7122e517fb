#!/bin/bash
# r05a GPU session: the non-blocking RCCL communicator at world 1, bench.py's self-launched N = 2
# rehearsal (test), the driver's N = 1 bench command, and the self-launched N = 2 / 4 rehearsals
# on one GPU (gloo group, ranks share the card).
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_bench_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "rccl or bench" > $OUT/r05a_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r05a_bench.json 2> $OUT/r05a_bench.err
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r05a_rehearsal_n2.json 2> $OUT/r05a_rehearsal_n2.err
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r05a_rehearsal_n4.json 2> $OUT/r05a_rehearsal_n4.err
