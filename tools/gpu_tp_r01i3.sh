# P2 tile width after the spill fix: T = 64 (128-B runs, 1 WG/CU) vs T = 32 (64-B runs, 2 WG/CU); graft smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
B="python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 200"
for rep in 1 2; do
  timeout -k 10 120 $B > gpurun_out/tp3.t64.$rep.json 2>/dev/null || exit $?
  CFP_TP_MID_T=32 timeout -k 10 120 $B > gpurun_out/tp3.t32.$rep.json 2>/dev/null || exit $?
  CFP_TP_GRID_ALL=1 timeout -k 10 120 $B > gpurun_out/tp3.all.$rep.json 2>/dev/null || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tp3.*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"], 1), [round(p["ms"] * 1e3, 1) for p in d["passes"]])
PY
