#!/bin/bash
# r05e GPU session: wave P2w twiddle-in-rows A/B (ab_v1 = -DCFP_WAVE_TWR=1), config 3's GMRES
# trace with the new reduction defaults, the whole -m gpu suite, the driver's bench command.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
for r in 1 2 3; do
  (cd $ROOT/ab_v1 && timeout -k 10 120 python3 tools/ab_wave.py --tag twr) >> $OUT/r05e_wave_ab.jsonl 2>> $OUT/r05e_wave_ab.err
  (cd $ROOT && timeout -k 10 120 python3 tools/ab_wave.py --tag base) >> $OUT/r05e_wave_ab.jsonl 2>> $OUT/r05e_wave_ab.err
done
bash tools/gmres_trace.sh r05e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05e_p2ctx -- python3 $ROOT/tools/p2_context_gaps.py > $OUT/r05e_p2ctx.log 2>&1
python3 $ROOT/tools/p2_context_gaps.py --summary $OUT/r05e_p2ctx > $OUT/r05e_p2ctx.txt 2>&1 || true
cd $ROOT
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/r05e_gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r05e_bench.json 2> $OUT/r05e_bench.err
