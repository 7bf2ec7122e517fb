set -o pipefail
TAG=${1:-s3e}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_small_grids.sh $TAG || exit $?
timeout -k 10 300 python bench_gmres.py --system wave2d direct --direct-grid 10 100 > gpurun_out/${TAG}_gmres.jsonl 2> gpurun_out/${TAG}_gmres.err
rc=$?; echo "gmres rc=$rc"; exit $rc
