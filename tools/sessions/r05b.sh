#!/bin/bash
# r05b GPU session: the 512^3 3-sweep slab schedule (parity through the group executor) and its
# local kernel time per rank; the row-class diagonal SpMV and config 3's GMRES trace; the
# real-scalar boundary on 2 and 4 ranks.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
# timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread -k "512 or three_sweep or rules or rccl" > $OUT/r05b_tests.log 2>&1
timeout -k 10 400 python tools/slab_local_timing.py --grid 512 --ranks 1 2 4 8 16 --pieces 1 4 --iters 10 > $OUT/r05b_slab_local_512.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_transport.py tests/test_real_scalar_mpi_gpu.py tests/test_real_scalar_gpu.py tests/test_pcshell_mpi_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/r05b_transport_real_tests.log 2>&1
bash tools/gmres_trace.sh r05b
