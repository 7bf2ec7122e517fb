#!/bin/bash
# r06q: same-box A/B of the GMRES legs: ab_v5/ (blocking stream waits) against the working tree
# (reduction results waited for by a polled event), 3 alternating rounds
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $OUT
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then T=$ROOT/ab_v5; else T=$ROOT; fi
    timeout -k 10 200 python3 $T/tools/gmres_legs.py --steps 20 >> $OUT/r06q_${side}.jsonl 2>> $OUT/r06q_${side}.err
  done
done
