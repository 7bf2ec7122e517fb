#!/bin/bash
# r04c GPU session: parity of every path touched this round (3-sweep shapes, real plan with the
# folded Nyquist column, slab layouts with P not dividing ny, multi-rank PCSHELL, GMRES harness,
# the real-scalar build), then copy floors, the 512^3 chunking probe and the 3-sweep shape A/B.
# Each step has its own limit; the first failure ends it.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass" > $OUT/r04c_tests.log 2>&1
timeout -k 10 300 $T tests/test_real_gpu.py tests/test_real_scalar_gpu.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 500 $T tests/test_dist_gpu.py tests/test_pcshell_mpi_gpu.py tests/test_transport.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 120 python tools/kexp/run_seg_chain.py > $OUT/r04c_seg_chain.txt 2>&1
timeout -k 10 240 python tools/probe_512_chunk.py 512 > $OUT/r04c_probe512.jsonl 2>&1
bash tools/ab_blocked.sh r04c
