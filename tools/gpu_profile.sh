# GPU step: rocprofv3 kernel stats and separate FETCH_SIZE / WRITE_SIZE PMC passes of the
# complex apply only (--no-real: the real-data variant's half-spectrum passes reuse the same
# kernel instantiations and would mix into the per-kernel averages).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
TAG=${1:-prof}
G=${2:-256}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof$G -o run -- python3 $R/bench.py --grid $G --steps 20 --warmup 3 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.prof$G.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG.pmc${G}_fetch -o run -- python3 $R/bench.py --grid $G --steps 5 --warmup 1 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.pmc_f.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG.pmc${G}_write -o run -- python3 $R/bench.py --grid $G --steps 5 --warmup 1 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.pmc_w.log 2>&1 || exit $?
echo done
