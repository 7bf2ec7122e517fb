#!/bin/bash
# r05d GPU session: the reductions' workgroup counts inside config 3's GMRES loop (MDOT_BLOCKS /
# RED_BLOCKS: working tree 512 / 1024, ab_v1 2048 / 2048, ab_v2 1024 / 2048), rocprofv3 kernel
# traces, two rounds.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
G="bench_gmres.py --system transport --grid 256 --sign fixed --pc fft --steps 6"
for r in 1 2; do
  for t in . ab_v1 ab_v2; do
    tag=$(basename $t); [ "$t" = . ] && tag=v0
    cd $ROOT/$t
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05d_${tag}_$r -- python3 $G > $OUT/r05d_${tag}_$r.jsonl 2> $OUT/r05d_${tag}_$r.err
    python3 $ROOT/tools/gmres_step_kernels.py $OUT/r05d_${tag}_$r > $OUT/r05d_${tag}_$r.txt
  done
done
