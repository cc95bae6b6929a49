# GPU-box: a pytest selection, then an A/B/.. of several (library, knob) variants on tools/pair_bench.py
# and on the C2 bench (bench.py without the side records), two rounds each in one session.
# Usage: bash tools/gpu_ab_multi.sh TAG "pytest selection|none" "label=lib[,VAR=VAL[,VAR=VAL...]]" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; SEL=$2; shift 2
if [ "$SEL" != none ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
fi
MODE=${AB_MODE:-both}
for round in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; kv=""; [ "$rest" != "$lib" ] && kv=${rest#*,}
    envs="DCX_LIB=$R/$lib"; [ -n "$kv" ] && envs="$envs ${kv//,/ }"
    if [ $MODE != bench ]; then
      env $envs timeout -k 10 120 python tools/pair_bench.py --reps 3 > gpurun_out/${TAG}_${label}_pairs.json || exit 1
      echo "== pairs $label ($envs, round $round): $(cat gpurun_out/${TAG}_${label}_pairs.json)"
    fi
    if [ $MODE != pairs ]; then
      env $envs DCX_BENCH_KERNELS=gpurun_out/${TAG}_${label}.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --no-c3 --no-c4 --no-f32 --no-oracle-codes > gpurun_out/${TAG}_${label}.out 2>&1 || exit 1
      echo "== bench $label (round $round): $(tail -1 gpurun_out/${TAG}_${label}.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s; c5', d.get('c5',{}).get('p50_ms'))")"
      python tools/kernel_table.py gpurun_out/${TAG}_${label}.json | grep -E "${AB_GREP:-res_pair|x6w8<256, 32|x6pf}"
    fi
  done
done
