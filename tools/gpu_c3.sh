# GPU-box: bf16-mode tests (compact layout, full-size C3 exactness, VQ search), then the C3 bench
# with per-kernel tables.  Usage: bash tools/gpu_c3.sh TAG
set -o pipefail
TAG=${1:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c3.py tests/test_gpu_vq.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -40; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; tail -5 gpurun_out/${TAG}_c3.err; exit 1; }
cat gpurun_out/${TAG}_c3.json
python tools/kernel_table.py gpurun_out/${TAG}_c3_kernels_bf16.json | head -12
