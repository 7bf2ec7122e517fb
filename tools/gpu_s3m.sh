set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/s3m_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/s3m_bench.json 2> gpurun_out/s3m_bench.err || exit $?
export CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo CFP_EXCHANGE=torch
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29632 bench.py --gpus 2 --grid 128 --steps 10 --warmup 2 --scaling-grid 256 --scaling-steps 2 \
  > gpurun_out/s3m_rehearse2.out 2> gpurun_out/s3m_rehearse2.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s3m_rehearse2.err; exit $rc; }
exit 0
