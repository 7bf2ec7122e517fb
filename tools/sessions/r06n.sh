#!/bin/bash
# r06n: where the wave GMRES step's device time goes (128^3, block PC), the library copy test,
# and the bench's copy-rate legs
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/r06n_fused_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06n_wave_prof -- python3 $ROOT/bench_gmres.py --system wave --wave-grid 128 --wave-steps 4 --pc fft > $OUT/r06n_wave.log 2>&1
cd $ROOT
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-configs --scaling-grid 0 > $OUT/r06n_bench.json 2> $OUT/r06n_bench.err
