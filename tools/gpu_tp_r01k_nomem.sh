# P2 compute-only time: CFP_TP_MID_FLAGS=1024 (F_NO_MEM: register fills, no stores; output invalid) vs default, 2 reps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "three_pass" -x -q --timeout 200 --timeout-method thread > gpurun_out/nm_tests.log 2>&1 || { tail -20 gpurun_out/nm_tests.log; exit 1; }
tail -1 gpurun_out/nm_tests.log
B="python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 300"
for rep in 1 2; do for fl in 0 1024; do
  CFP_TP_MID_FLAGS=$fl timeout -k 10 120 $B > gpurun_out/nm.f$fl.$rep.json 2>/dev/null || exit $?
done; done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/nm.*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"], 1), [round(p["ms"] * 1e3, 1) for p in d["passes"]])
PY
