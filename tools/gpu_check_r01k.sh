# r01 last check of the committed tree after build(): graft smoke, GPU suite, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r01k_smoke.log 2>&1 || { tail -20 gpurun_out/r01k_smoke.log; exit 1; }
tail -1 gpurun_out/r01k_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r01k_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r01k_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/r01k_bench256.json 2> gpurun_out/r01k_bench256.err || exit $?
cat gpurun_out/r01k_bench256.json | cut -c1-200
echo done
