#!/bin/bash
# r04g GPU session: AUTO 3-sweep grids with the z-fused tables (the 512^3 AUTO fix), then the
# driver's bench command and smoke().
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "full_size_residual or three_pass or plane" > $OUT/r04g_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04g_bench.json 2> $OUT/r04g_bench.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r04g_smoke.log 2>&1
