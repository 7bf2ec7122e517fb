#!/bin/bash
# r05q: middle sweeps of the wave (k_wtp_mid_ct2) and real-data (k_tp_mid_sw, NX = 128) 3-sweeps
# in XCD unit order, against a -DCFP_WAVE_MID_XCD=0 -DCFP_REAL_MID_XCD=0 build (ab_v3/lib),
# alternating processes; parity of both paths
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_real_gpu.py tests/test_wave.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05q_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u tools/ab_sched.py 256 real:three --iters 3000 --rounds 2 >> $OUT/r05q_real_ab.jsonl 2>> $OUT/r05q_ab.err
  timeout -k 10 200 python -u tools/ab_sched.py 256 real:three --iters 3000 --rounds 2 --lib ab_v3/lib/libcirculant_fft.so >> $OUT/r05q_real_ab.jsonl 2>> $OUT/r05q_ab.err
  timeout -k 10 200 python -u tools/ab_wave.py --iters 2000 >> $OUT/r05q_wave_ab.jsonl 2>> $OUT/r05q_ab.err
  timeout -k 10 200 python -u tools/ab_wave.py --iters 2000 --lib ab_v3/lib/libcirculant_fft.so >> $OUT/r05q_wave_ab.jsonl 2>> $OUT/r05q_ab.err
done
