#!/bin/bash
# r06z7: the tree after the block SpMV restructure (prefetch off): wave + fused tests, smoke,
# the driver's bench command
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_wave.py tests/test_wave_mpi_gpu.py tests/test_fused_gpu.py tests/test_transport.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06z7_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r06z7_smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r06z7_bench.json 2> $OUT/r06z7_bench.err
