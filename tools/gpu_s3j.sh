set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/s3j_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_old.sh
