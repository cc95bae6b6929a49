# GPU-box: C3 (bf16) kernel tables of three builds: libdcx.so, the GELU timing probe and the
# no-epilogue timing build (conv_gemm_bf16dm fixed per-tile cost).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in libdcx geluprobe noepi; do
  DCX_LIB=$R/distilcodec_nabeel_amd/$L.so timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/epi_$L > gpurun_out/epi_$L.json 2> gpurun_out/epi_$L.err || exit 1
  echo "== $L"; python tools/kernel_table.py gpurun_out/epi_${L}_bf16.json | head -4
done
