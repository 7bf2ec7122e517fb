#!/bin/bash
# r05m: unit order of streaming (BLAS-1) kernels: grid-stride / XCD-contiguous / contiguous per WG
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/kexp/run_stream_order.py > $OUT/r05m_stream_order.txt 2>&1
