# GPU-box, round-end records part B: rocprofv3 trace + FETCH/WRITE PMC passes over bench.py, then the
# default bench (with its CPU-baseline leg and sub-records).  Usage: bash tools/gpu_final_b.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_profile.sh $TAG || exit 1
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
