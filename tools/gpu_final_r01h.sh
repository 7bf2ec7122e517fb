# round-1 (session h) closing measurement: GPU suite, bench lines (256 default with 512 scaling item,
# 128, 512), rocprofv3 kernel stats and separate FETCH_SIZE / WRITE_SIZE PMC passes at 256^3
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r01h_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r01h_bench256.json 2> gpurun_out/r01h_bench256.err || exit $?
timeout -k 10 300 python bench.py --grid 128 --no-cpu-baseline --scaling-grid 0 > gpurun_out/r01h_bench128.json 2> gpurun_out/r01h_bench128.err || exit $?
timeout -k 10 300 python bench.py --grid 512 --steps 30 --warmup 3 --no-cpu-baseline --scaling-grid 0 > gpurun_out/r01h_bench512.json 2> gpurun_out/r01h_bench512.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01h.prof256 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01h.prof256.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01h.pmc256_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01h.pmc_f.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01h.pmc256_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01h.pmc_w.log 2>&1 || exit $?
echo done
