# GPU step: SQ counters (wave-cycle breakdown, VALU, LDS bank conflicts) of the 256^3 apply's
# kernels, one rocprofv3 --pmc pass (no tracing domains beside it).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
TAG=${1:-sq}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG.sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.sq.log 2>&1 || exit $?
echo done
