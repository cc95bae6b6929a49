# GPU-box quick loop: stage parity tests + x6 bench with kernel table.  Usage: bash tools/gpu_quick.sh TAG [bench args]
set -o pipefail
TAG=${1:-q}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_stages.py tests/test_gpu_vq.py -x -q > gpurun_out/${TAG}_tests.log 2>&1; RC=$?; echo TESTS_EXIT $RC; tail -15 gpurun_out/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
DCX_BENCH_KERNELS=gpurun_out/${TAG}_kernels.json timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; echo BENCH_EXIT $?
cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
python tools/kernel_table.py gpurun_out/${TAG}_kernels.json
