# GPU step: full gpu test suite, bench at 256^3 and 512^3, kernel stats and HBM PMC counters.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 1200 python -m pytest tests -q -m gpu --maxfail=30 -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t2.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-budget 15 > gpurun_out/bench256.json 2> gpurun_out/bench256.err || exit $?
cat gpurun_out/bench256.json
timeout -k 10 300 python bench.py --grid 512 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench512.json 2> gpurun_out/bench512.err || exit $?
cat gpurun_out/bench512.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof256 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof256.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc256_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc256_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc256_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc256_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc512_fetch -o run -- python3 $R/bench.py --grid 512 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc512_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc512_write -o run -- python3 $R/bench.py --grid 512 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc512_write.log 2>&1 || exit $?
echo done
