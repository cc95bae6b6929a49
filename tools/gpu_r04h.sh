# GPU-box: C3 duplicate-launch epilogue timing (bf16dm), C5 per-kernel table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for M in 1 2; do
  DCX_DIAG_DUP=$M DCX_LIB=$R/distilcodec_nabeel_amd/dup.so timeout -k 10 400 python tools/c3_bench.py --gemm bf16 --steps 2 --kernels gpurun_out/r04h_c3dup$M > gpurun_out/r04h_c3dup$M.json 2> gpurun_out/r04h_c3dup$M.err || { echo DUP_FAILED; tail -3 gpurun_out/r04h_c3dup$M.err; exit 1; }
  echo "== C3 DCX_DIAG_DUP=$M"; python tools/kernel_table.py gpurun_out/r04h_c3dup${M}_bf16.json | sed -n 1,10p
done
timeout -k 10 300 python tools/stream_bench.py --split-k 16 --kernels gpurun_out/r04h_c5_kernels.json > gpurun_out/r04h_c5.json 2> gpurun_out/r04h_c5.err || { echo C5_FAILED; exit 1; }
head -c 600 gpurun_out/r04h_c5.json; echo; python tools/kernel_table.py gpurun_out/r04h_c5_kernels.json | sed -n 1,40p
