#!/bin/bash
# r06l: item 6 probe (grid barrier cost; three sweeps as three launches vs one persistent launch)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 240 python -u tools/kexp/run_grid_probe.py > $OUT/r06l_grid_probe.txt 2>&1
