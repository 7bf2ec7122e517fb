# GPU step: full gpu test suite, GMRES bench (configs 1/3/4), bench lines at 256^3 (with CPU baseline), 512^3, 128^3,
# rocprofv3 kernel stats and separate FETCH_SIZE / WRITE_SIZE PMC passes at 256^3.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
TAG=${1:-run}
timeout -k 10 1200 python -m pytest tests -q -m gpu --maxfail=20 -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/$TAG.tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench_gmres.py --out gpurun_out/$TAG.gmres.jsonl > gpurun_out/$TAG.gmres.log 2>&1 || exit $?
cat gpurun_out/$TAG.gmres.jsonl
timeout -k 10 300 python bench.py > gpurun_out/$TAG.bench256.json 2> gpurun_out/$TAG.bench256.err || exit $?
cat gpurun_out/$TAG.bench256.json
timeout -k 10 300 python bench.py --grid 512 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG.bench512.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --grid 128 --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/$TAG.bench128.json 2>/dev/null || exit $?
python - <<PY
import json
for g in (512, 128):
    d = json.load(open("gpurun_out/$TAG.bench%d.json" % g))
    print(g, d["value"], d["ms_per_step"], [(p["axis"], p["mode"], p["ms"]) for p in d["passes"]])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof256 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.prof256.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG.pmc256_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.pmc_f.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG.pmc256_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-real > $R/gpurun_out/$TAG.pmc_w.log 2>&1 || exit $?
echo done
