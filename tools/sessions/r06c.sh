#!/bin/bash
# r06c: the fused Krylov step after the DPP neighbours and the setup-time row-class form (tests,
# GMRES trace, bench with the GMRES legs), then the distributed transport GMRES on 2 / 4 ranks
set -e
TAG=${1:-r06c}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_transport.py -x -v -m gpu --timeout 240 --timeout-method thread > $OUT/${TAG}_gpu_tests.log 2>&1
bash tools/gmres_trace.sh ${TAG}
timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline --scaling-grid 0 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
timeout -k 10 500 python -u -m pytest tests/test_mpi_gmres_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/${TAG}_mpi_gmres.log 2>&1
