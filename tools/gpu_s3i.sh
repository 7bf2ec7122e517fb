set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/s3i_tests.log; [ $rc -ne 0 ] && exit $rc
export CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo CFP_EXCHANGE=torch
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2962$n bench.py --gpus $n --grid 128 --steps 10 --warmup 2 --scaling-grid 256 --scaling-steps 2 \
    > gpurun_out/s3i_rehearse$n.out 2> gpurun_out/s3i_rehearse$n.err
  rc=$?; echo "rehearse n=$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s3i_rehearse$n.err; exit $rc; }
done
exit 0
