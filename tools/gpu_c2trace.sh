# GPU-box: per-dispatch kernel trace of C2 bench steps (no sub-records), for per-launch tables
# (tools/launch_table.py).  Usage: bash tools/gpu_c2trace.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
TAG=${1:-c2t}
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-c3 --no-c4 --no-c5 --no-oracle-codes --no-cpu-baseline --no-f32 --no-profile > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo TRACE_FAILED; tail -5 $R/gpurun_out/$TAG.err; exit 1; }
cp $(find $R/gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1) $R/gpurun_out/${TAG}_kernel_trace.csv
rm -rf $R/gpurun_out/${TAG}_trace
echo TRACE_OK
