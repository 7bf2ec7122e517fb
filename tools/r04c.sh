#!/bin/bash
# r04c GPU session: parity of every path touched this round (3-sweep shapes, the wave P2w with the
# comps on lane bits 4-5, real plan with the folded Nyquist column, slab layouts with P not
# dividing ny, multi-rank PCSHELL, GMRES harness, the real-scalar build), then the P2w probes.
# Each step has its own limit; the first failure ends it.  Measurements: tools/r04d.sh.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass" > $OUT/r04c_tests.log 2>&1
timeout -k 10 200 $T tests/test_wave.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 300 $T tests/test_real_gpu.py tests/test_real_scalar_gpu.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 400 $T tests/test_dist_gpu.py tests/test_pcshell_mpi_gpu.py tests/test_transport.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 120 python tools/kexp/run_wave_probe.py > $OUT/r04c_wave_probe.txt 2>&1
