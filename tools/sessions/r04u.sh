#!/bin/bash
# r04u GPU session: HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes) of the
# r04 3-sweep schedules at 512^3, 128^3 (16 x 8) and 100^3.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
for g in 512 128 100; do
  it=5; [ $g != 512 ] && it=50
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04u_pmc${g}_fetch -- python3 $ROOT/tools/ab_sched.py $g three --iters $it --rounds 1 > $OUT/r04u_pmc${g}_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04u_pmc${g}_write -- python3 $ROOT/tools/ab_sched.py $g three --iters $it --rounds 1 > $OUT/r04u_pmc${g}_write.log 2>&1
done
