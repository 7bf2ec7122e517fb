# wave 1-D/2-D parity + full wave GPU tests, bench with the 512^3 scaling line, 2-D wave bench,
# gloo rehearsal of the N > 1 scaling block
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wave.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3a_wave.log 2>&1
rc=$?; echo "wave tests rc=$rc"; tail -3 gpurun_out/s3a_wave.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/s3a_bench.json 2> gpurun_out/s3a_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s3a_bench.err; exit $rc; }
timeout -k 10 300 python bench_gmres.py --system wave2d > gpurun_out/s3a_wave2d.jsonl 2> gpurun_out/s3a_wave2d.err
rc=$?; echo "wave2d rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s3a_wave2d.err; exit $rc; }
export CFP_BENCH_SHARE_DEVICE=1 CFP_BENCH_BACKEND=gloo CFP_EXCHANGE=torch
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29612 bench.py --gpus 2 --grid 128 --steps 10 --warmup 2 --scaling-grid 256 --scaling-steps 3 \
  > gpurun_out/s3a_rehearse2.out 2> gpurun_out/s3a_rehearse2.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/s3a_rehearse2.err; exit $rc; }
exit 0
