#!/bin/bash
# r04ac GPU session: wave-local row FFT in the wave P1w / P3w and the slab rows; tests + bench.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_wave.py tests/test_dist_gpu.py tests/test_gpu_parity.py -k "wave or slab or dist or three_pass" > $OUT/r04ac_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04ac_bench.json 2> $OUT/r04ac_bench.err
