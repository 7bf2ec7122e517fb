#!/bin/bash
# r05h: where the 512^3 P2 time goes (probes of k_tp_mid<.., 32, 16, 512, ..>)
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/kexp/run_p2_512.py > $OUT/r05h_p2_512_probes.txt 2>&1
