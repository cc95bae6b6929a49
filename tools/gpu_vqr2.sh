# GPU-box: VQ tests, then C3 A/B (DCX_VQ_OLD build vs libdcx.so) and the C2 bench of libdcx.so.
#   bash tools/gpu_vqr2.sh TAG
set -o pipefail
TAG=${1:-vqr2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_c3.py tests/test_gpu_stream.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -30; [ $rc = 0 ] || exit $rc
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/vqold.so distilcodec_nabeel_amd/libdcx.so "vq_|total" || exit 1
DCX_BENCH_KERNELS=gpurun_out/${TAG}_c2.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/${TAG}_c2.out 2>&1 || { tail -5 gpurun_out/${TAG}_c2.out; exit 1; }
echo "== C2: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')" gpurun_out/${TAG}_c2.out)"
python tools/kernel_table.py gpurun_out/${TAG}_c2.json | grep -E "vq_|row_sq|total"
