# GPU-box script: tests, parity report, bench in both GEMM modes.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1; echo TESTS_EXIT $?; tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python tools/parity_report.py > gpurun_out/${TAG}_parity.md 2> gpurun_out/${TAG}_parity.err; echo PARITY_EXIT $?; cat gpurun_out/${TAG}_parity.md
for G in x6 f32; do
  DCX_BENCH_KERNELS=gpurun_out/${TAG}_kernels_$G.json timeout -k 10 600 python bench.py --steps 5 --warmup 2 --gemm $G --no-cpu-baseline > gpurun_out/${TAG}_bench_$G.json 2> gpurun_out/${TAG}_bench_$G.err; echo BENCH_${G}_EXIT $?; cat gpurun_out/${TAG}_bench_$G.json
done
