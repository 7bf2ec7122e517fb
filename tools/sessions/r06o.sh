#!/bin/bash
# r06o: block row-class SpMV for the wave operator: its tests, the wave suites, and the wave
# GMRES step's kernels again (compare r06n)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wave.py tests/test_wave_mpi_gpu.py tests/test_transport.py tests/test_mpi_gmres_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/r06o_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06o_wave_prof -- python3 $ROOT/bench_gmres.py --system wave --wave-grid 128 --wave-steps 4 --pc fft > $OUT/r06o_wave.log 2>&1
cd $ROOT
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r06o_bench.json 2> $OUT/r06o_bench.err
