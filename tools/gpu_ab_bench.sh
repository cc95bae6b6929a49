# GPU-box: the GPU test suite, then an A/B of two builds on the full bench (two rounds each, one
# session, so both see the same box and clock).  Usage: bash tools/gpu_ab_bench.sh LIB_A LIB_B [TESTS=0]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
A=$1; B=$2
if [ "${3:-1}" != 0 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/full_tests.log; [ $rc = 0 ] || exit $rc
fi
for round in 1 2; do
  for L in $A $B; do
    T=$(basename $L .so)
    DCX_LIB=$R/$L DCX_BENCH_KERNELS=gpurun_out/ab_$T.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$T.out 2>&1 || exit 1
    echo "== bench $L (round $round): $(tail -1 gpurun_out/ab_$T.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')")"
    python tools/kernel_table.py gpurun_out/ab_$T.json | sed -n 1,8p
  done
done
