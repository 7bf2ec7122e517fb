#!/bin/bash
# 256^3 transport GMRES with the FFT PCSHELL (BASELINE config 3): bench_gmres.py
# JSON line, then the same run under rocprofv3 --kernel-trace (per-kernel device time per step).
set -e
TAG=${1:-r04a}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
G="bench_gmres.py --system transport --grid 256 --sign fixed --pc fft --steps 6"
timeout -k 10 150 python $G > $OUT/${TAG}_gmres256.jsonl 2> $OUT/${TAG}_gmres256.err
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_gmres256_trace -- \
  python $G > $OUT/${TAG}_gmres256_traced.jsonl 2> $OUT/${TAG}_gmres256_traced.err
python tools/gmres_step_kernels.py $OUT/${TAG}_gmres256_trace > $OUT/${TAG}_gmres256_kernels.txt
