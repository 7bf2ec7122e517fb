# 3-sweep schedule experiment (cfp_three_pass.hip): parity of every variant, then bench sweeps over
# CFP_TP_N1 x CFP_TP_MID_T x {stagger 0 / 1000 / 2000 ticks of 100 MHz, one unit per workgroup}
# against the 5-pass default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k three_pass -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/tp_tests.log 2>&1 || { tail -40 gpurun_out/tp_tests.log; exit 1; }
tail -3 gpurun_out/tp_tests.log
B="python bench.py --no-cpu-baseline --no-real --scaling-grid 0 --steps 200 --no-live-events"
for rep in 1 2; do
  timeout -k 10 120 $B > gpurun_out/tp.five.$rep.json 2>/dev/null || exit $?
  for n1 in 64 32; do for t in 64 32; do for v in s0 all; do
    st=${v#s}; all=0; [ "$v" = all ] && { st=0; all=1; }
    CFP_TP_N1=$n1 CFP_TP_MID_T=$t CFP_TP_STAGGER=$st CFP_TP_GRID_ALL=$all timeout -k 10 120 $B --schedule three \
      > gpurun_out/tp.$n1.$t.$v.$rep.json 2>/dev/null || exit $?
  done; done; done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tp.*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"], 1), [round(p["ms"] * 1e3, 1) for p in d["passes"]])
PY
