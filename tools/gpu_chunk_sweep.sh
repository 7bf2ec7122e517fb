# GPU step: gpu tests, then bench 256^3 / 512^3 with chunked schedules of several sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -q -m gpu --maxfail=20 -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/t3.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in 0 8 16 32 64 128; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --chunk $c > gpurun_out/b256_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b256_c$c.json'));print('256 chunk $c', d['value'], d['ms_per_step'], [p['ms'] for p in d['passes']][:12])"
done
for c in 0 4 8 16 32; do
  timeout -k 10 200 python bench.py --grid 512 --steps 20 --warmup 3 --no-cpu-baseline --chunk $c > gpurun_out/b512_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b512_c$c.json'));print('512 chunk $c', d['value'], d['ms_per_step'])"
done
