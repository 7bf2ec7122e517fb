#!/bin/bash
# ${TAG}: steady-state A/B of the fused 256^3 chain (P1 with the stencil, P3 with the dots) against
# the plain chain, per kernel (tools/fused_chain_ab.py under rocprofv3 --kernel-trace)
set -e
TAG=${1:-r06e}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_chain_trace -- python tools/fused_chain_ab.py > $OUT/${TAG}_chain.log 2>&1
python tools/fused_chain_ab.py --summary $OUT/${TAG}_chain_trace > $OUT/${TAG}_chain_summary.txt
