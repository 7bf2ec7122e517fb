# A/B on one box: the library of an older commit (ab_old/) vs the current tree, alternating
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 300 > ../gpurun_out/abo.$i.json 2>/dev/null) || exit $?
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 300 > gpurun_out/abn.$i.json 2>/dev/null || exit $?
done
python - <<PY
import json
for t in ("abo", "abn"):
    for i in (1, 2, 3):
        d = json.load(open("gpurun_out/%s.%d.json" % (t, i)))
        print(t, d["value"], [p["ms"] for p in d["passes"]])
PY
