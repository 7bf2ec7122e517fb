# 3-sweep after the P1/P3 spill fix (phase C twiddles from global): parity, bench, rocprofv3 stats, PMC passes
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_direct_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tp4_tests.log 2>&1 || { tail -30 gpurun_out/tp4_tests.log; exit 1; }
tail -1 gpurun_out/tp4_tests.log
B="python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 200"
for rep in 1 2; do
  timeout -k 10 120 $B > gpurun_out/tp4.auto.$rep.json 2>/dev/null || exit $?
  timeout -k 10 120 $B --schedule five > gpurun_out/tp4.five.$rep.json 2>/dev/null || exit $?
  CFP_TP_N1=64 timeout -k 10 120 $B > gpurun_out/tp4.n64.$rep.json 2>/dev/null || exit $?
done
timeout -k 10 300 python bench.py > gpurun_out/r01i4_bench256.json 2> gpurun_out/r01i4_bench256.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01i4.prof256 -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01i4.prof256.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01i4.pmc256_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01i4.pmc_f.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r01i4.pmc256_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real --scaling-grid 0 > $R/gpurun_out/r01i4.pmc_w.log 2>&1 || exit $?
cd $R && python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tp4.*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"], 1), [round(p["ms"] * 1e3, 1) for p in d["passes"]])
PY
