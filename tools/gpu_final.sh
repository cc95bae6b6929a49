# GPU-box: the round's evidence in one session: GPU tests, C3 and C5 benches, rocprofv3 trace + PMC
# passes over bench.py, then the default bench (with its CPU-baseline leg).  Usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; exit 1; }
cat gpurun_out/${TAG}_c3.json
timeout -k 10 300 python tools/stream_bench.py --split-k 16 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { echo C5_FAILED; exit 1; }
cat gpurun_out/${TAG}_c5.json
bash tools/gpu_profile.sh $TAG || exit 1
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; exit 1; }
cat gpurun_out/${TAG}_bench.json
