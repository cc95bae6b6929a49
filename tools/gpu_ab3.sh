# GPU-box: A/B/C of the current tree, a DCX_LIB variant of it and an older staged tree (two rounds, C2
# bench with per-kernel tables).  Usage: bash tools/gpu_ab3.sh VARIANT.so OLD_DIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
V=$1; D=$2
FL="--steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-f32 --no-oracle-codes"
for round in 1 2; do
  for T in cur var old; do
    dir=$R; envs=""
    [ $T = var ] && envs="DCX_LIB=$R/$V"
    [ $T = old ] && dir=$R/$D
    (cd $dir && env $envs DCX_BENCH_KERNELS=$R/gpurun_out/ab3_$T.json timeout -k 10 300 python bench.py $FL > $R/gpurun_out/ab3_$T.out 2>&1) || { echo "bench $T failed"; tail -5 gpurun_out/ab3_$T.out; exit 1; }
    echo "== $T (round $round): $(tail -1 gpurun_out/ab3_$T.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')")"
    python tools/kernel_table.py gpurun_out/ab3_$T.json | sed -n 1,12p
  done
done
