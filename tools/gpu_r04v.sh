# GPU-box: bf16dp epilogue composition: table lookups left out (timing build) vs shipped, C3 (two rounds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/lutdiag.so "bf16d" || { echo AB_FAILED; exit 1; }
  DCX_GELU_LUT=0 DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/c3nolut > gpurun_out/c3nolut.json 2>/dev/null || { echo NOLUT_FAILED; exit 1; }
  echo "== C3 evaluated GELU: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/c3nolut.json)"; python tools/kernel_table.py gpurun_out/c3nolut_bf16.json | grep bf16dp
done
