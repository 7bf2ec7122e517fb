#!/bin/bash
# r04i GPU session: the whole -m gpu suite (as the driver runs it), then the 256^3 GMRES trace.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/r04i_gpu_tests.log 2>&1
bash tools/gmres_trace.sh r04i
