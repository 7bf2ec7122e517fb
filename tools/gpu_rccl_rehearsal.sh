# Rehearse the N > 1 bench path on a one-GPU box: RCCL refuses two ranks on one device
# ("Duplicate GPU detected"), so the ranks share cuda:0 over gloo and the slab plan's two
# all-to-alls go through torch.distributed (exchange "torch").  Everything else -- the slab
# kernels, the barrier / max-over-ranks timing, the phase report -- is the N > 1 code path.
set -o pipefail
mkdir -p gpurun_out
export CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo CFP_EXCHANGE=torch
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2961$n bench.py --gpus $n --grid 128 --steps 10 --warmup 2 > gpurun_out/rehearse$n.out 2> gpurun_out/rehearse$n.err
  rc=$?
  echo "n=$n rc=$rc"
  cat gpurun_out/rehearse$n.out
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/rehearse$n.err; exit $rc; fi
done
