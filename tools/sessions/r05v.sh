#!/bin/bash
# r05v: the stand-in's VecMDot in isolation (fresh vectors) against torch.vdot, kernel trace
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05v_mdot -- python3 $ROOT/tools/kexp/run_mdot.py > $OUT/r05v_mdot.log 2>&1
