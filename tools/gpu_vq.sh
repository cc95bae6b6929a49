# GPU-box: VQ / bf16 / C3 tests, then the default bench (kernel table) and the C3 bench.
# Usage: bash tools/gpu_vq.sh TAG
set -o pipefail
TAG=${1:-vq}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_bf16.py tests/test_gpu_c3.py tests/test_gpu_api.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -40; [ $rc = 0 ] || exit $rc
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json; python tools/kernel_table.py gpurun_out/${TAG}_bench_kernels.json | head -10
DCX_NO_COMPACT=1 DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels_nc.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench_nc.json 2> gpurun_out/${TAG}_bench_nc.err || { echo BENCH_NC_FAILED; exit 1; }
python tools/kernel_table.py gpurun_out/${TAG}_bench_kernels_nc.json | grep -E "vq_|total"
timeout -k 10 400 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; tail -5 gpurun_out/${TAG}_c3.err; exit 1; }
head -1 gpurun_out/${TAG}_c3.json
