#!/bin/bash
# r05p: AUTO 3-sweep slab schedule at every supported P -- distributed GPU tests and the
# self-launched N = 2 rehearsal
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_bench_gpu.py tests/test_pcshell_mpi_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/r05p_tests.log 2>&1
