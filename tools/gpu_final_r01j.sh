# r01 closing measurement (3-sweep AUTO at 256^3, spill-free): GPU suite, bench lines (AUTO and five), rocprofv3 stats, PMC passes
# and separate FETCH_SIZE / WRITE_SIZE PMC passes at 256^3
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r01j_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r01j_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/r01j_bench256.json 2> gpurun_out/r01j_bench256.err || exit $?
timeout -k 10 300 python bench.py --schedule five --no-cpu-baseline --no-real --scaling-grid 0 > gpurun_out/r01j_bench256_five.json 2> gpurun_out/r01j_bench256_five.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01j.prof256 -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01j.prof256.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01j.pmc256_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01j.pmc_f.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01j.pmc256_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01j.pmc_w.log 2>&1 || exit $?
echo done
