#!/bin/bash
# r06m: the whole -m gpu suite on the r06 tree (wave on several ranks, RCCL mode switch), the bench
# with the copy rate in the roofline, smoke()
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/r06m_gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r06m_bench.json 2> $OUT/r06m_bench.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r06m_smoke.log 2>&1
