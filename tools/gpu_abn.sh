# GPU-box A/B of libdcx.so builds in one session: the C2 bench (no sub-records), ROUNDS rounds of
# every library in turn, per-kernel tables of the last round.  Optional C3 leg (AB_C3=1).
#   bash tools/gpu_abn.sh TAG LIB_A LIB_B [LIB_C ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
ROUNDS=${ROUNDS:-2}
for round in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    T=$(basename $L .so)
    DCX_LIB=$R/$L DCX_BENCH_KERNELS=gpurun_out/${TAG}_$T.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
      --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/${TAG}_$T.out 2>&1 || { echo "FAILED $L"; tail -5 gpurun_out/${TAG}_$T.out; exit 1; }
    echo "== $T round $round: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s', d['roofline']['kernel'], d['roofline']['frac'])" gpurun_out/${TAG}_$T.out)"
    if [ -n "$AB_C3" ]; then
      DCX_LIB=$R/$L timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/${TAG}_c3_$T > gpurun_out/${TAG}_c3_$T.out 2>&1 || { echo "C3 FAILED $L"; exit 1; }
      echo "   C3 $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms', d['roofline']['kernel'], d['roofline']['frac'])" gpurun_out/${TAG}_c3_$T.out)"
    fi
  done
done
for L in "$@"; do
  T=$(basename $L .so)
  echo "== kernels $T"
  python tools/kernel_table.py gpurun_out/${TAG}_$T.json | sed -n 1,14p
  [ -n "$AB_C3" ] && python tools/kernel_table.py gpurun_out/${TAG}_c3_${T}_bf16.json | sed -n 1,8p
done
exit 0
