# GPU-box: C3 bench on the epilogue timing builds (bf16dm cost split: GELU / stores / whole epilogue).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in libdcx.so epinogelu.so epinostore.so epinoepi.so; do
  T=$(basename $L .so)
  DCX_LIB=$R/distilcodec_nabeel_amd/$L timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/ed_$T > gpurun_out/ed_$T.json 2> gpurun_out/ed_$T.err || { tail -3 gpurun_out/ed_$T.err; exit 1; }
  echo "== $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/ed_$T.json)"
  python tools/kernel_table.py gpurun_out/ed_${T}_bf16.json | grep -E "bf16dm|prefilter"
done
