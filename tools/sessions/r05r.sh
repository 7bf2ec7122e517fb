#!/bin/bash
# r05r GPU session (tree as of the round-5 changes): the whole -m gpu suite, smoke(), the driver's
# bench command, and the rocprofv3 kernel summary of the same bench command.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/r05r_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r05r_smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r05r_bench.json 2> $OUT/r05r_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05r_prof_bench -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r05r_prof_bench.log 2>&1
cd $ROOT && bash tools/gmres_trace.sh r05r
