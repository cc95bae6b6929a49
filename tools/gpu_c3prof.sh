# GPU-box: rocprofv3 kernel trace + FETCH/WRITE PMC passes over the C3 bench (bf16 mode), then the
# PMC counter passes over the generator (conv_res_pair MFMA busy).  Usage: bash tools/gpu_c3prof.sh TAG
set -o pipefail
TAG=${1:-c3p}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 2 --kernels $R/gpurun_out/${TAG}_k > $R/gpurun_out/${TAG}_c3.json 2> $R/gpurun_out/${TAG}_trace.err || { echo TRACE_FAILED; tail -5 $R/gpurun_out/${TAG}_trace.err; exit 1; }
echo TRACE_OK
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 > /dev/null 2> $R/gpurun_out/${TAG}_fetch.err || { echo FETCH_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/${TAG}_write -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 > /dev/null 2> $R/gpurun_out/${TAG}_write.err || { echo WRITE_FAILED; exit 1; }
python3 tools/rocprof_summary.py --stats $(find $R/gpurun_out/${TAG}_trace -name "*kernel_stats.csv" | head -1) --fetch $(find $R/gpurun_out/${TAG}_fetch -name "*counter_collection.csv" | head -1) --write $(find $R/gpurun_out/${TAG}_write -name "*counter_collection.csv" | head -1) --bench-kernels $R/gpurun_out/${TAG}_k_bf16.json > $R/gpurun_out/${TAG}_summary.md
head -14 $R/gpurun_out/${TAG}_summary.md
[ -n "$SKIP_GEN" ] || bash tools/gpu_pmc_gen.sh ${TAG}g | tail -60
