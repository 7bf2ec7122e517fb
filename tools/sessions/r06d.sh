#!/bin/bash
# r06d: fused P1 with the edge neighbours through LDS, fusion only where the plan fuses (tests, trace, bench)
set -e
TAG=${1:-r06d}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_transport.py -x -v -m gpu --timeout 240 --timeout-method thread > $OUT/${TAG}_gpu_tests.log 2>&1
bash tools/gmres_trace.sh ${TAG}
timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline --scaling-grid 0 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
