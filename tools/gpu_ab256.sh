# A/B of the 256^3 apply: 3 alternating bench runs (no CPU baseline, no extras)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 300 > gpurun_out/ab.$i.json 2>/dev/null || exit $?
done
python - <<PY
import json
for i in (1, 2, 3):
    d = json.load(open("gpurun_out/ab.%d.json" % i))
    print(d["value"], [p["ms"] for p in d["passes"]])
PY
