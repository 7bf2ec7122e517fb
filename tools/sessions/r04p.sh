#!/bin/bash
# r04p GPU session: P2 probes of the product kernel (prefetch, NT loads) incl. the s_setprio
# experiment.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 200 python tools/kexp/run_tp_probe.py > $OUT/r04p_tp_probe.txt 2>&1
