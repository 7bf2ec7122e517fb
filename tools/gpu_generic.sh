# GPU step: the parity suite, then the non-power-of-two (mixed-radix) apply at the reference's sizes.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-gen}
timeout -k 10 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG.tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for g in 100 96 120 200 10; do
  timeout -k 10 120 python bench.py --grid $g --steps 50 --warmup 5 --no-cpu-baseline --no-real > gpurun_out/$TAG.b$g.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/$TAG.b$g.json'));print($g, d['value'], d['ms_per_step'], [(p['axis'],p['mode'],p['ms']) for p in d['passes']])"
done
