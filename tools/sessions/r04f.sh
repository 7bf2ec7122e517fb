#!/bin/bash
# r04f GPU session: wave parity + P2w probes after the bank-conflict-free column labels, then the
# driver's bench command and smoke().
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_wave.py > $OUT/r04f_tests.log 2>&1
timeout -k 10 150 python tools/kexp/run_wave_probe.py > $OUT/r04f_wave_probe.txt 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04f_bench.json 2> $OUT/r04f_bench.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r04f_smoke.log 2>&1
