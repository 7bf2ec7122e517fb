#!/bin/bash
# r04n GPU session: the N = 2 bench path rehearsed on one GPU (two ranks share the device, gloo
# process group, the torch all_to_all fallback exchange), 256^3 headline + 512^3 scaling leg.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline > $OUT/r04n_rehearsal_n2.json 2> $OUT/r04n_rehearsal_n2.err
