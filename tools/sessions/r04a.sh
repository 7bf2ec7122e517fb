#!/bin/bash
# r04a GPU session: parity of the touched paths, copy floors, blocked-layout A/B, GMRES trace.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass" > $OUT/r04a_tests.log 2>&1
timeout -k 10 400 $T tests/test_pcshell_mpi_gpu.py tests/test_transport.py tests/test_mesh_gpu.py >> $OUT/r04a_tests.log 2>&1
timeout -k 10 120 python tools/kexp/run_seg_chain.py > $OUT/r04a_seg_chain.txt 2>&1
bash tools/gmres_trace.sh r04a
bash tools/ab_blocked.sh r04a
