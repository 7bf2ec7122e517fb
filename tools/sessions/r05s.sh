#!/bin/bash
# r05s: row sweeps at one workgroup per CU (256^3 against its default two)
set -e
OUT=gpurun_out
mkdir -p $OUT
ROWS_PROBES=0,8,9,10 timeout -k 10 300 python -u tools/kexp/run_rows_512.py > $OUT/r05s_rows_occupancy.txt 2>&1
