#!/bin/bash
# r04w GPU session: HBM traffic of the real 256^3 and wave 128^3 3-sweep kernels.
set -e
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
for k in "real 256" "wave 128"; do
  t=${k// /}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04w_pmc_${t}_fetch -- python3 $ROOT/tools/pmc_driver.py $k 20 > $OUT/r04w_pmc_${t}_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04w_pmc_${t}_write -- python3 $ROOT/tools/pmc_driver.py $k 20 > $OUT/r04w_pmc_${t}_write.log 2>&1
done
