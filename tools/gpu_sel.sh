# GPU-box: a pytest selection, then the default bench (kernel table) and the C3 bench.
# Usage: bash tools/gpu_sel.sh TAG "tests/test_a.py tests/test_b.py"
set -o pipefail
TAG=${1:-sel}; SEL=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -20; [ $rc = 0 ] || exit $rc
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
python tools/kernel_table.py gpurun_out/${TAG}_bench_kernels.json | head -14
timeout -k 10 400 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; tail -5 gpurun_out/${TAG}_c3.err; exit 1; }
head -1 gpurun_out/${TAG}_c3.json | cut -c1-300
python tools/kernel_table.py gpurun_out/${TAG}_c3_kernels_bf16.json | head -6
