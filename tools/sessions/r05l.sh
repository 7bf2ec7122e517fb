#!/bin/bash
# r05l: XCD-ordered row sweeps everywhere (slab executor, real-data P1r / P3r, wave P1w / P3w) --
# distributed parity, 3-sweep parity, per-rank slab local time and whole-apply A/B against the
# -DCFP_ROWS_XCD=0 build (ab_v2/lib), alternating processes
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_real_gpu.py tests/test_wave.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05l_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u tools/slab_local_timing.py --grid 512 --ranks 8 16 --pieces 1 4 >> $OUT/r05l_slab512.txt 2>&1
  timeout -k 10 200 python -u tools/slab_local_timing.py --grid 512 --ranks 8 16 --pieces 1 4 --lib ab_v2/lib/libcirculant_fft.so >> $OUT/r05l_slab512_ab.txt 2>&1
  timeout -k 10 200 python -u tools/slab_local_timing.py --grid 256 --ranks 2 4 --pieces 1 4 >> $OUT/r05l_slab256.txt 2>&1
  timeout -k 10 200 python -u tools/slab_local_timing.py --grid 256 --ranks 2 4 --pieces 1 4 --lib ab_v2/lib/libcirculant_fft.so >> $OUT/r05l_slab256_ab.txt 2>&1
  timeout -k 10 200 python -u tools/ab_sched.py 256 real:three --iters 3000 --rounds 2 >> $OUT/r05l_real_ab.jsonl 2>> $OUT/r05l_ab.err
  timeout -k 10 200 python -u tools/ab_sched.py 256 real:three --iters 3000 --rounds 2 --lib ab_v2/lib/libcirculant_fft.so >> $OUT/r05l_real_ab.jsonl 2>> $OUT/r05l_ab.err
  timeout -k 10 200 python -u tools/ab_wave.py --iters 2000 >> $OUT/r05l_wave_ab.jsonl 2>> $OUT/r05l_ab.err
  timeout -k 10 200 python -u tools/ab_wave.py --iters 2000 --lib ab_v2/lib/libcirculant_fft.so >> $OUT/r05l_wave_ab.jsonl 2>> $OUT/r05l_ab.err
done
