# GPU-box: the GPU tests (a selection first, then the rest), then an A/B of one dcx knob (read from the
# environment at dcx_create) on the C2 bench, two rounds each in one session (same box and clock).
# Usage: bash tools/gpu_ab_knob.sh TAG VAR VALUE_B [first pytest selection] [TESTS=1]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; VAR=$2; VB=$3; SEL=${4:-tests/test_gpu_respair.py}
if [ "${5:-1}" != 0 ]; then
  timeout -k 10 300 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_sel.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_sel.log; [ $rc = 0 ] || exit $rc
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
fi
for round in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export $VAR=$VB; else unset $VAR; fi
    DCX_BENCH_KERNELS=gpurun_out/${TAG}_$v.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      --no-c3 --no-c4 --no-f32 --no-oracle-codes > gpurun_out/${TAG}_$v.out 2>&1 || exit 1
    echo "== $v ($VAR=${!VAR:-default}, round $round): $(tail -1 gpurun_out/${TAG}_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s; c5', d.get('c5',{}).get('p50_ms'))")"
    python tools/kernel_table.py gpurun_out/${TAG}_$v.json | sed -n 1,12p
  done
done
