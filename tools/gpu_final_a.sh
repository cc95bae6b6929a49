# GPU-box, round-end records part A: the GPU test suite, C3 and C5 benches.  Usage: bash tools/gpu_final_a.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; exit 1; }
cat gpurun_out/${TAG}_c3.json
timeout -k 10 300 python tools/stream_bench.py --split-k 16 --kernels gpurun_out/${TAG}_c5_kernels.json > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { echo C5_FAILED; exit 1; }
cat gpurun_out/${TAG}_c5.json
