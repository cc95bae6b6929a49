# GPU-box: A/B of two builds of libdcx.so in one session (conv microbenchmark, then optionally the
# full bench with per-kernel tables).
#   [AB_BENCH=1] bash tools/gpu_ab.sh LIB_A LIB_B [conv_bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
A=$1; B=$2; shift 2
for round in 1 2; do
  for L in $A $B; do
    echo "== $L (round $round)"
    timeout -k 10 300 env DCX_LIB=$R/$L python tools/conv_bench.py "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
if [ -n "$AB_BENCH" ]; then
  for L in $A $B; do
    T=$(basename $L .so)
    DCX_LIB=$R/$L DCX_BENCH_KERNELS=gpurun_out/ab_$T.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$T.out 2>&1 || exit 1
    echo "== bench $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')" gpurun_out/ab_$T.out)"
    python tools/kernel_table.py gpurun_out/ab_$T.json | sed -n 1,9p
  done
fi
