# GPU-box: all GPU tests (verbose, per-test time limit), then the default bench and a C4-shaped
# single-GPU bench.  Usage: bash tools/gpu_r2.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-r2}; shift
SEL=${@:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|SNR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40; [ $rc = 0 ] || exit $rc
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench_c4.json 2> gpurun_out/${TAG}_bench_c4.err || { echo C4_FAILED; tail -5 gpurun_out/${TAG}_bench_c4.err; exit 1; }
cat gpurun_out/${TAG}_bench_c4.json
