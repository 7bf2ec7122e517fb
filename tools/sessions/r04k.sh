#!/bin/bash
# r04k GPU session: kernel profiles of the small grids (100^3 and 128^3 3 sweeps) and the slab
# local timing at 512^3.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04k_prof100 -- python3 $ROOT/tools/ab_sched.py 100 three --iters 2000 --rounds 1 > $OUT/r04k_prof100.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r04k_prof128 -- python3 $ROOT/tools/ab_sched.py 128 three --iters 2000 --rounds 1 > $OUT/r04k_prof128.log 2>&1
cd $ROOT
timeout -k 10 300 python tools/slab_local_timing.py --grid 512 --ranks 2 4 8 --pieces 1 4 > $OUT/r04k_slab_local_512.txt 2>&1
