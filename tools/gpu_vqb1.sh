# GPU-box: vq_prefilter_b1 round-3 check: VQ / bf16 / C3 tests on libdcx.so, then C3 and C2 A/B
# against the DCX_VQ_OLD build (vq_prefilter_bq / _dm) and the ring-depth variants.
#   bash tools/gpu_vqb1.sh TAG
set -o pipefail
TAG=${1:-b1}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_bf16.py tests/test_gpu_c3.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -40; [ $rc = 0 ] || exit $rc
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/vqold.so distilcodec_nabeel_amd/libdcx.so "vq_|total" || exit 1
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/vqns3.so distilcodec_nabeel_amd/vqns5.so "vq_|total" || exit 1
for L in vqold.so libdcx.so; do
  T=$(basename $L .so)
  DCX_LIB=$R/distilcodec_nabeel_amd/$L DCX_BENCH_KERNELS=gpurun_out/${TAG}_c2_$T.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/${TAG}_c2_$T.out 2>&1 || { tail -5 gpurun_out/${TAG}_c2_$T.out; exit 1; }
  echo "== C2 $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')" gpurun_out/${TAG}_c2_$T.out)"
  python tools/kernel_table.py gpurun_out/${TAG}_c2_$T.json | grep -E "vq_|row_sq|total"
done
