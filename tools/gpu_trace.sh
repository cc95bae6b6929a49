# GPU-box: per-launch kernel traces (rocprofv3 --kernel-trace) of one C2 step (bench.py) and one C3 step
# (tools/c3_bench.py), for per-launch analysis (tools/launch_table.py).  Usage: bash tools/gpu_trace.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; TAG=${1:-tr}
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
  --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-f32 --no-oracle-codes --no-profile > $R/gpurun_out/${TAG}_c2.out 2> $R/gpurun_out/${TAG}_c2.err \
  || { echo TRACE_FAILED; tail -5 $R/gpurun_out/${TAG}_c2.err; exit 1; }
cp $(find $R/gpurun_out/${TAG}_c2 -name "*kernel_trace.csv" | head -1) $R/gpurun_out/${TAG}_c2_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_c3 -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1 \
  > $R/gpurun_out/${TAG}_c3.out 2> $R/gpurun_out/${TAG}_c3.err || { echo TRACE_FAILED; tail -5 $R/gpurun_out/${TAG}_c3.err; exit 1; }
cp $(find $R/gpurun_out/${TAG}_c3 -name "*kernel_trace.csv" | head -1) $R/gpurun_out/${TAG}_c3_kernel_trace.csv
rm -rf $R/gpurun_out/${TAG}_c2 $R/gpurun_out/${TAG}_c3
echo TRACE_OK
