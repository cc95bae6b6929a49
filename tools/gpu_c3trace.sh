# GPU-box: per-launch kernel trace of one C3 (bf16) step, for per-shape analysis of conv_gemm_bf16dm.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/c3t_trace -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1 > $R/gpurun_out/c3t.json 2> $R/gpurun_out/c3t.err || { echo TRACE_FAILED; tail -5 $R/gpurun_out/c3t.err; exit 1; }
cp $(find $R/gpurun_out/c3t_trace -name "*kernel_trace.csv" | head -1) $R/gpurun_out/c3t_kernel_trace.csv
echo TRACE_OK
