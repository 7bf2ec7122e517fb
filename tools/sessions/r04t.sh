#!/bin/bash
# r04t GPU session: wave P2w at 8 points per thread with whole-complex exchanges and the
# whole-unit prefetch (k_wtp_mid_ct3): parity, probes, bench other_configs.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_wave.py > $OUT/r04t_tests.log 2>&1
timeout -k 10 250 python tools/kexp/run_wave_probe.py > $OUT/r04t_wave_probe.txt 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --scaling-grid 0 --no-cpu-baseline --no-real > $OUT/r04t_bench.json 2> $OUT/r04t_bench.err
