# GPU-box: split-K latency-mode tests, then the C5 stream bench with and without split-K (per-kernel
# table of the split hop).  Usage: bash tools/gpu_splitk.sh TAG
set -o pipefail
TAG=${1:-sk}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_splitk.py tests/test_gpu_stream.py tests/test_gpu_stream_halo.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|dB" gpurun_out/${TAG}_tests.log | tail -30; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/stream_bench.py --hops 100 --split-k 16 --kernels gpurun_out/${TAG}_c5k.json > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { echo C5_FAILED; tail -5 gpurun_out/${TAG}_c5.err; exit 1; }
cat gpurun_out/${TAG}_c5.json
python tools/kernel_table.py gpurun_out/${TAG}_c5k.json | head -16
