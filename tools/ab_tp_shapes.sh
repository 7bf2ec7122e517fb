#!/bin/bash
# the 256^3 3-sweep apply with the default shape (N1 = 32, P2 = 8 x * 8 y2,
# 128-byte runs) against N1 = 64 (P2 = 16 x * 4 y2, 256-byte runs; P1/P3 of 64 rows at one
# workgroup per CU), alternating, each under rocprofv3 --kernel-trace --stats.
set -e
TAG=${1:-r03h}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
B="bench.py --steps 200 --warmup 10 --no-real --scaling-grid 0 --no-cpu-baseline"
for rep in 1 2; do
  for shape in 0,default 64,swap64pf 64,default; do
    s=${shape/,/_}
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_${s}_$rep -- \
      python $B --tp-shape $shape > $OUT/${TAG}_${s}_$rep.json 2> $OUT/${TAG}_${s}_$rep.err
  done
done
echo done > $OUT/${TAG}_done
