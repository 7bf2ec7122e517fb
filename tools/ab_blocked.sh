#!/bin/bash
# the 256^3 3-sweep apply, natural intermediate layout (default) against the
# blocked layout (--tp-shape 0,blocked), alternating bench.py runs, then one rocprofv3
# --kernel-trace --stats run of each.  Every step has its own time limit; the first failure ends it.
set -e
TAG=${1:-r04a}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
B="bench.py --steps 200 --warmup 10 --no-real --scaling-grid 0 --no-cpu-baseline --no-configs"
for rep in 1 2; do
  for shape in default blocked blocked32; do
    timeout -k 10 120 python $B --tp-shape 0,$shape > $OUT/${TAG}_${shape}_$rep.json 2> $OUT/${TAG}_${shape}_$rep.err
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for shape in default blocked blocked32; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$shape -- \
    python $B --tp-shape 0,$shape > $OUT/${TAG}_prof_$shape.json 2> $OUT/${TAG}_prof_$shape.err
done
echo done > $OUT/${TAG}_done
