#!/bin/bash
# r04ai GPU session: wave-local row FFT exchanges in the 5-pass axis kernels (k_axis_fast):
# parity, A/B against the previous build (tools/kexp/lib_base) in alternating processes.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_real_gpu.py tests/test_wave.py > $OUT/r04ai_tests.log 2>&1
for r in 1 2; do
  for lib in tools/kexp/lib_base/libcirculant_fft.so circulantpreconditioner_amd/lib/libcirculant_fft.so; do
    timeout -k 10 120 python tools/ab_sched.py 256 five --iters 300 --rounds 1 --lib $lib >> $OUT/r04ai_ab.jsonl 2>/dev/null
    timeout -k 10 120 python tools/ab_sched.py 64 five plane --iters 3000 --rounds 1 --lib $lib >> $OUT/r04ai_ab.jsonl 2>/dev/null
    timeout -k 10 120 python tools/ab_sched.py 512 five --iters 10 --rounds 1 --lib $lib >> $OUT/r04ai_ab.jsonl 2>/dev/null
  done
done
