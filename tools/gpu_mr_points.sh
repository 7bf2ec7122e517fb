# mixed-radix block size sweep (CFP_MR_POINTS_OVERRIDE) on the reference's own sizes
set -o pipefail
mkdir -p gpurun_out
for pts in 2048 1024 512 256; do
  for g in 100 200 96 10; do
    CFP_MR_POINTS_OVERRIDE=$pts timeout -k 10 120 python bench.py --grid $g --no-cpu-baseline --no-real --scaling-grid 0 \
      --steps 200 --warmup 20 > gpurun_out/mrp.$pts.$g.json 2> gpurun_out/mrp.$pts.$g.err || exit $?
  done
done
python - <<PY
import json
for pts in (2048, 1024, 512, 256):
    for g in (100, 200, 96, 10):
        d = json.load(open("gpurun_out/mrp.%d.%d.json" % (pts, g)))
        print(pts, g, round(d["value"]), [p["ms"] for p in d["passes"]])
PY
