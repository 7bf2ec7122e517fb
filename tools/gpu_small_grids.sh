# bench lines on the reference's own (mixed-radix) sizes and small power-of-two grids
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-small}
for g in 100 200 64 128 10; do
  timeout -k 10 120 python bench.py --grid $g --no-cpu-baseline --no-real --scaling-grid 0 --steps 200 --warmup 20 \
    > gpurun_out/$TAG.bench$g.json 2> gpurun_out/$TAG.bench$g.err || exit $?
done
python - <<PY
import json
for g in (100, 200, 64, 128, 10):
    d = json.load(open("gpurun_out/$TAG.bench%d.json" % g))
    print(g, round(d["value"]), d["ms_per_step"], [(p["axis"], p["mode"], p["fast"], p["ms"]) for p in d["passes"]])
PY
