#!/bin/bash
# Address-translation counters of the 512^3 apply ("the 512^3 z pass runs at 5.1
# TB/s against 6.6 elsewhere, attributed to translation reach, no counters confirm it").  Two
# --pmc passes (<= 4 TCP and 2 GRBM counters each) over a short 512^3 bench plus a kernel trace
# for the per-kernel durations.  Run on the GPU box from the repo root; output gpurun_out/$TAG_*.
set -e
TAG=${1:-r03n}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
B="bench.py --grid 512 --steps 6 --warmup 2 --no-real --scaling-grid 0 --no-cpu-baseline --settle-ms 0"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace -- python $B \
  > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_trace.err
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
  TCP_UTCL1_STALL_MULTI_MISS_sum --output-format csv -d $OUT/${TAG}_pmc1 -- python $B > /dev/null 2> $OUT/${TAG}_pmc1.err
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum \
  TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/${TAG}_pmc2 -- python $B > /dev/null 2> $OUT/${TAG}_pmc2.err
echo done > $OUT/${TAG}_done
