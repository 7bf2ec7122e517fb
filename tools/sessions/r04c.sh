#!/bin/bash
# r04c GPU session: parity of every path touched this round (3-sweep shapes, the wave P2w with the
# comps on lane bits 4-5, real plan with the folded Nyquist column, slab layouts with P not
# dividing ny, multi-rank PCSHELL, GMRES harness, the real-scalar build, the 100^3 3-sweep), then
# the P2w probes and the 100^3 schedule A/B.
# Each step has its own limit; the first failure ends it.  Measurements: tools/r04d.sh.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 200 $T tests/test_gpu_parity.py -k "three_pass" > $OUT/r04c_tests.log 2>&1
timeout -k 10 200 $T tests/test_wave.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 300 $T tests/test_real_gpu.py tests/test_real_scalar_gpu.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 400 $T tests/test_dist_gpu.py tests/test_pcshell_mpi_gpu.py tests/test_transport.py >> $OUT/r04c_tests.log 2>&1
timeout -k 10 120 python tools/kexp/run_wave_probe.py > $OUT/r04c_wave_probe.txt 2>&1
timeout -k 10 150 python tools/ab_sched.py 100 plane three:0,default three:0,lane64 three:0,lane32 five > $OUT/r04c_ab100.jsonl 2>&1
timeout -k 10 150 python tools/ab_sched.py 512 auto three five --iters 20 --rounds 2 > $OUT/r04c_ab512.jsonl 2>&1
