#!/bin/bash
# r05o: 256^3 slab local kernels at P = 8 / 16 (3-sweep against 5-pass; the AUTO rule picks
# 5 passes above P = 4)
set -e
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python -u tools/slab_local_timing.py --grid 256 --ranks 4 8 16 --pieces 1 2 4 >> $OUT/r05o_slab256.txt 2>&1
done
