set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=30 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-budget 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit $?
cat gpurun_out/bench1.json
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o prof -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
