# GPU-box: per-launch kernel trace of graph-replayed C5 hops (split-K 16) for the hop timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
TAG=${1:-c5t}
cd /tmp && export TMPDIR=/tmp; cd $R
DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 tools/stream_bench.py --split-k 16 --hops 30 --warmup 5 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo TRACE_FAILED; tail -5 $R/gpurun_out/$TAG.err; exit 1; }
cp $(find $R/gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1) $R/gpurun_out/${TAG}_kernel_trace.csv
rm -rf $R/gpurun_out/${TAG}_trace
echo TRACE_OK
