# 3-sweep at 128^3 (and 256^3 regression): parity, bench 128 three vs five, bench 256 auto
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "three_pass" -x -q --timeout 200 --timeout-method thread > gpurun_out/tp6_tests.log 2>&1 || { tail -30 gpurun_out/tp6_tests.log; exit 1; }
tail -1 gpurun_out/tp6_tests.log
for rep in 1 2; do
  timeout -k 10 120 python bench.py --grid 128 --no-cpu-baseline --no-real --scaling-grid 0 --steps 1000 --schedule three > gpurun_out/tp6.128three.$rep.json 2>/dev/null || exit $?
  timeout -k 10 120 python bench.py --grid 128 --no-cpu-baseline --no-real --scaling-grid 0 --steps 1000 --schedule five > gpurun_out/tp6.128five.$rep.json 2>/dev/null || exit $?
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 200 > gpurun_out/tp6.256auto.$rep.json 2>/dev/null || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tp6.*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"], 1), [round(p["ms"] * 1e3, 1) for p in d["passes"]])
PY
