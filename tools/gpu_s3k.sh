set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "profile or vs_oracle" > gpurun_out/s3k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/s3k_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 > gpurun_out/s3k_live.$i.json 2>/dev/null || exit $?
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --no-live-events > gpurun_out/s3k_sep.$i.json 2>/dev/null || exit $?
done
python - <<PY
import json
for t in ("live", "sep"):
    for i in (1, 2):
        d = json.load(open("gpurun_out/s3k_%s.%d.json" % (t, i)))
        print(t, d["value"], d["roofline"]["frac"], [p["ms"] for p in d["passes"]], d["roofline"]["timing"][:40])
PY
