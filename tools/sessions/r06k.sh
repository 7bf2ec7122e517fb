#!/bin/bash
# r06k: the wave block PCSHELL on 2 and 4 ranks (z-slab plan per component) and the wave tests
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_wave_mpi_gpu.py -x -v --timeout 280 --timeout-method thread > $OUT/r06k_wave_mpi.log 2>&1
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu -k wave --timeout 200 --timeout-method thread > $OUT/r06k_wave_all.log 2>&1
