#!/bin/bash
# r05k: P1 / P3 units in XCD order (kRowsXCD) -- whole-apply A/B against a -DCFP_ROWS_XCD=0 build
# (ab_v2/lib), alternating processes; 3-sweep parity; one bench line
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "three_pass" --timeout 240 --timeout-method thread > $OUT/r05k_parity.log 2>&1
for r in 1 2; do
  for g in 256 512 128; do
    it=2000; [ $g = 512 ] && it=200; [ $g = 128 ] && it=10000
    timeout -k 10 200 python -u tools/ab_sched.py $g three --iters $it --rounds 2 >> $OUT/r05k_ab.jsonl 2>> $OUT/r05k_ab.err
    timeout -k 10 200 python -u tools/ab_sched.py $g three --iters $it --rounds 2 --lib ab_v2/lib/libcirculant_fft.so >> $OUT/r05k_ab.jsonl 2>> $OUT/r05k_ab.err
  done
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r05k_bench.json 2> $OUT/r05k_bench.err
