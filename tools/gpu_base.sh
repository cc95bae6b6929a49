# GPU-box: baseline measurements without tests: C2 bench (kernel table), C3 and C5 benches.
#   bash tools/gpu_base.sh TAG
set -o pipefail
TAG=${1:-base}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
DCX_BENCH_KERNELS=gpurun_out/${TAG}_kernels.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
python tools/kernel_table.py gpurun_out/${TAG}_kernels.json | sed -n 1,30p
timeout -k 10 300 python tools/c3_bench.py --kernels gpurun_out/${TAG}_c3_kernels > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3_FAILED; exit 1; }
cat gpurun_out/${TAG}_c3.json
timeout -k 10 300 python tools/stream_bench.py --split-k 16 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { echo C5_FAILED; exit 1; }
cat gpurun_out/${TAG}_c5.json
