#!/bin/bash
# r06z3: AUTO picks planes at 32^2: the full GPU suite, then the GMRES legs (config 1 at 32^3)
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r06z3_gpu_tests.log 2>&1
timeout -k 10 300 python tools/gmres_legs.py > $OUT/r06z3_legs.jsonl 2> $OUT/r06z3_legs.err
