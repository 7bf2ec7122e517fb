#!/bin/bash
# r04r GPU session: the whole -m gpu suite, the driver's bench command and smoke().
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/r04r_gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04r_bench.json 2> $OUT/r04r_bench.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r04r_smoke.log 2>&1
