#!/bin/bash
# Kernel traces and counters of the launch-bound configs: 128^3 (config 2,
# 5 passes), 100^3 (the reference's default mesh, plane schedule) and the wave system at 128^3
# (config 4).  Run on the GPU box from the repo root; every step has its own time limit and the
# script stops at the first failure.  Output: gpurun_out/$TAG_*.
set -e
TAG=${1:-r03g}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
B="bench.py --steps 200 --warmup 10 --no-real --scaling-grid 0 --no-cpu-baseline"
for g in 128 100; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace$g -- python $B --grid $g \
    > $OUT/${TAG}_bench$g.json 2> $OUT/${TAG}_bench$g.err
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/${TAG}_sq$g -- \
    python bench.py --steps 20 --warmup 2 --no-real --scaling-grid 0 --no-cpu-baseline --settle-ms 0 --grid $g \
    > /dev/null 2> $OUT/${TAG}_sq$g.err
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${TAG}_fetch$g -- \
    python bench.py --steps 20 --warmup 2 --no-real --scaling-grid 0 --no-cpu-baseline --settle-ms 0 --grid $g \
    > /dev/null 2> $OUT/${TAG}_fetch$g.err
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${TAG}_write$g -- \
    python bench.py --steps 20 --warmup 2 --no-real --scaling-grid 0 --no-cpu-baseline --settle-ms 0 --grid $g \
    > /dev/null 2> $OUT/${TAG}_write$g.err
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_wave128 -- \
  python bench_gmres.py --system wave --wave-grid 128 > $OUT/${TAG}_wave128.jsonl 2> $OUT/${TAG}_wave128.err
echo done > $OUT/${TAG}_done
