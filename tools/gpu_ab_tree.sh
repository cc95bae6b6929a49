# GPU-box: A/B of the current tree against an older tree staged under DIR (its own package, bench.py
# and tools/kernel_table.py; built on the CPU side), two rounds each on the C2 bench with per-kernel
# tables, in one session.  Usage: bash tools/gpu_ab_tree.sh DIR [STEPS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
D=$1; S=${2:-5}
FL="--steps $S --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-f32 --no-oracle-codes"
for round in 1 2; do
  for T in cur old; do
    if [ $T = cur ]; then dir=$R; else dir=$R/$D; fi
    (cd $dir && DCX_BENCH_KERNELS=$R/gpurun_out/abt_$T.json timeout -k 10 300 python bench.py $FL > $R/gpurun_out/abt_$T.out 2>&1) || { echo "bench $T failed"; tail -5 gpurun_out/abt_$T.out; exit 1; }
    echo "== $T (round $round): $(tail -1 gpurun_out/abt_$T.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', round(d['value']/1e6,3), 'M samples/s')")"
    python tools/kernel_table.py gpurun_out/abt_$T.json | sed -n 1,14p
  done
done
