#!/bin/bash
# r04am GPU session (final tree): the whole -m gpu suite, the driver's bench command, smoke(), the rocprofv3
# kernel summary of the same bench command, and the HBM traffic (separate FETCH / WRITE passes)
# of the 256^3 3-sweep kernels.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/r04am_gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04am_bench.json 2> $OUT/r04am_bench.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r04am_smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04am_prof_bench -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04am_prof_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04am_pmc256_fetch -- python3 $ROOT/tools/ab_sched.py 256 three --iters 20 --rounds 1 > $OUT/r04am_pmc256_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04am_pmc256_write -- python3 $ROOT/tools/ab_sched.py 256 three --iters 20 --rounds 1 > $OUT/r04am_pmc256_write.log 2>&1
