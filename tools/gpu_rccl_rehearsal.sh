# Rehearse the N>1 bench path (RCCL slab plan) with 2 ranks sharing the one GPU of the box.
# RCCL may refuse two ranks on one device; the run is bounded by timeout either way.
set -o pipefail
mkdir -p gpurun_out
export CFP_BENCH_SHARE_DEVICE=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --grid 64 --steps 5 --warmup 1 > gpurun_out/rccl2.out 2> gpurun_out/rccl2.err
echo "rc=$?"
cat gpurun_out/rccl2.out
tail -20 gpurun_out/rccl2.err
