#!/bin/bash
# Same-box A/B of two library builds: ab_old/ (e.g. `git archive HEAD`, built in place) against
# the working tree, bench.py alternating, ROUNDS rounds.  Usage: tools/ab_two_trees.sh TAG "BENCH ARGS" [ROUNDS]
set -e
TAG=$1
ARGS=$2
ROUNDS=${3:-3}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for side in old new; do
    if [ $side = old ]; then B=$ROOT/ab_old/bench.py; else B=$ROOT/bench.py; fi
    timeout -k 10 120 python3 $B $ARGS > $OUT/${TAG}_${side}_$r.json 2> $OUT/${TAG}_${side}_$r.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], [p.get('ms') for p in d.get('passes', [])], flush=True)" \
      $OUT/${TAG}_${side}_$r.json ${side}$r | tee -a $OUT/${TAG}_summary.txt
  done
done
