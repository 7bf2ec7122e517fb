# GPU step: full gpu test suite, then bench lines at 256^3 / 512^3 / 128^3 (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG.tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for g in 256 512 128; do
  timeout -k 10 300 python bench.py --grid $g --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/$TAG.bench$g.json 2> gpurun_out/$TAG.bench$g.err || exit $?
done
python - <<PY
import json
for g in (256, 512, 128):
    d = json.load(open("gpurun_out/$TAG.bench%d.json" % g))
    print(g, d["value"], d["ms_per_step"], d["roofline"]["frac"], [(p["axis"], p["mode"], p["ms"]) for p in d["passes"]],
          d.get("real_variant", {}).get("value"))
PY
