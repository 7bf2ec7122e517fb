#!/bin/bash
# r06j: the whole -m gpu suite on the r06 tree (fused Krylov step, distributed AIJ, pinned results)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/r06j_gpu_tests.log 2>&1
