#!/bin/bash
# r06p (final-tree validation): the whole -m gpu suite, smoke(), the driver's bench command, the
# rocprofv3 kernel summary of that same command, and the HBM traffic of the 256^3 3-sweep kernels
# (separate FETCH_SIZE / WRITE_SIZE passes)
set -e
TAG=${1:-r06p}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $OUT/${TAG}_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_bench -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_prof_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${TAG}_pmc256_fetch -- python3 $ROOT/tools/ab_sched.py 256 three --iters 20 --rounds 1 > $OUT/${TAG}_pmc256_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${TAG}_pmc256_write -- python3 $ROOT/tools/ab_sched.py 256 three --iters 20 --rounds 1 > $OUT/${TAG}_pmc256_write.log 2>&1
