# GPU-box: rocprofv3 kernel trace + FETCH/WRITE PMC passes over bench.py.  Usage: bash tools/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cd $R
DCX_BENCH_KERNELS=$R/gpurun_out/${TAG}_kernels.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > $R/gpurun_out/${TAG}_bench_under_rocprof.json 2> $R/gpurun_out/${TAG}_trace.err || { echo TRACE_FAILED; exit 1; }
echo TRACE_OK
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-f32 --no-profile --no-c3 --no-c4 --no-c5 --no-oracle-codes > /dev/null 2> $R/gpurun_out/${TAG}_fetch.err || { echo FETCH_FAILED; exit 1; }
echo FETCH_OK
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/${TAG}_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-f32 --no-profile --no-c3 --no-c4 --no-c5 --no-oracle-codes > /dev/null 2> $R/gpurun_out/${TAG}_write.err || { echo WRITE_FAILED; exit 1; }
echo WRITE_OK
python3 tools/pmc_to_json.py $R/gpurun_out/${TAG}_fetch $R/gpurun_out/${TAG}_write > $R/gpurun_out/${TAG}_pmc.json
python3 tools/rocprof_summary.py --stats $(ls $R/gpurun_out/${TAG}_trace/*kernel_stats.csv $R/gpurun_out/${TAG}_trace/*/*kernel_stats.csv 2>/dev/null | head -1) --fetch $(find $R/gpurun_out/${TAG}_fetch -name "*counter_collection.csv" | head -1) --write $(find $R/gpurun_out/${TAG}_write -name "*counter_collection.csv" | head -1) --bench-kernels $R/gpurun_out/${TAG}_kernels.json > $R/gpurun_out/${TAG}_summary.md
head -12 $R/gpurun_out/${TAG}_summary.md
