#!/bin/bash
# r05c GPU session: (1) store policy of the Krylov-vector kernels inside config 3's GMRES loop
# (trees ab_v1..3 built with -DCFP_BLAS_NT=1..3 against the working tree's 0), rocprofv3 kernel
# traces, two rounds; (2) the 512^3 P2 traffic question: variant timings and separate
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes per variant.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
G="bench_gmres.py --system transport --grid 256 --sign fixed --pc fft --steps 6"
for r in 1 2; do
  for t in . ab_v1 ab_v2 ab_v3; do
    tag=$(basename $t); [ "$t" = . ] && tag=v0
    cd $ROOT/$t
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05c_${tag}_$r -- python3 $G > $OUT/r05c_${tag}_$r.jsonl 2> $OUT/r05c_${tag}_$r.err
    python3 $ROOT/tools/gmres_step_kernels.py $OUT/r05c_${tag}_$r > $OUT/r05c_${tag}_$r.txt
    head -3 $OUT/r05c_${tag}_$r.txt
  done
done
cd $ROOT
timeout -k 10 300 python3 tools/kexp/run_p2_512.py > $OUT/r05c_p2_512_times.txt 2>&1
cd /tmp
for w in 0 1 2 3 4; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r05c_pmc_fetch_$w -- python3 $ROOT/tools/kexp/run_p2_512.py $w 3 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r05c_pmc_write_$w -- python3 $ROOT/tools/kexp/run_p2_512.py $w 3 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/r05c_pmc_hit_$w -- python3 $ROOT/tools/kexp/run_p2_512.py $w 3 > /dev/null 2>&1
done
