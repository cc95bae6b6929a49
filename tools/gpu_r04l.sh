# GPU-box: vq_prefilter_w4 (AGPR accumulators, asm fragment reads): same-results test and C3 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_vq.py -k "w4 or many_rows" > gpurun_out/r04l_vqtest.log 2>&1 || { echo VQTEST_FAILED; tail -30 gpurun_out/r04l_vqtest.log; exit 1; }
tail -2 gpurun_out/r04l_vqtest.log
for r in 1 2; do
  for W in 0 1; do
    DCX_VQ_W4=$W timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/c3w4_$W > gpurun_out/c3w4_$W.json 2> gpurun_out/c3w4_$W.err || { echo W4_FAILED; tail -5 gpurun_out/c3w4_$W.err; exit 1; }
    echo "== C3 w4=$W: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/c3w4_$W.json)"; python tools/kernel_table.py gpurun_out/c3w4_${W}_bf16.json | grep prefilter
  done
done
