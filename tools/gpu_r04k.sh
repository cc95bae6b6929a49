# GPU-box: C5 hop trace; prefilter A/B: 4-wave kernel (DCX_VQ_W4), ring depth 5, L2-resident operands (timing only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_vq.py -k "w4 or many_rows" > gpurun_out/r04k_vqtest.log 2>&1 || { echo VQTEST_FAILED; tail -30 gpurun_out/r04k_vqtest.log; exit 1; }
tail -2 gpurun_out/r04k_vqtest.log
bash tools/gpu_c5trace.sh r04k_c5t && python tools/hop_timeline.py gpurun_out/r04k_c5t_kernel_trace.csv --top 30 > gpurun_out/r04k_c5_timeline.txt || { echo C5T_FAILED; exit 1; }
head -40 gpurun_out/r04k_c5_timeline.txt
cp distilcodec_nabeel_amd/libdcx.so /tmp/w4.so
for r in 1 2; do
  DCX_VQ_W4=0 bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/vns5.so "prefilter" || { echo AB_FAILED; exit 1; }
  DCX_VQ_W4=1 timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/c3w4 > gpurun_out/c3w4.json 2> gpurun_out/c3w4.err || { echo W4_FAILED; tail -5 gpurun_out/c3w4.err; exit 1; }
  echo "== C3 w4: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/c3w4.json)"; python tools/kernel_table.py gpurun_out/c3w4_bf16.json | grep prefilter
done
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/vql2.so distilcodec_nabeel_amd/vns5.so "prefilter" || { echo AB_FAILED; exit 1; }
