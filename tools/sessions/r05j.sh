#!/bin/bash
# r05j: where the 512^3 row sweeps' time goes (k_tp_rows probes, 256^3 for comparison)
set -e
OUT=gpurun_out
mkdir -p $OUT
ROWS_PROBES=0,4,6,7,8,9 timeout -k 10 300 python -u tools/kexp/run_rows_512.py > $OUT/r05j_rows_order.txt 2>&1
