# A/B/C on one box: ab_old/ (previous commit), ab_a/ (variant), current tree; alternating rounds
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for d in ab_old ab_a .; do
    t=$(basename $(cd $d && pwd)); [ "$d" = "." ] && t=cur
    (cd $d && timeout -k 10 120 python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 300 > $OLDPWD/gpurun_out/ab3.$t.$i.json 2>/dev/null) || exit $?
  done
done
python - <<PY
import json
for t in ("ab_old", "ab_a", "cur"):
    for i in (1, 2, 3):
        d = json.load(open("gpurun_out/ab3.%s.%d.json" % (t, i)))
        print(t, d["value"], [p["ms"] for p in d["passes"]])
PY
