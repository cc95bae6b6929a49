# GPU-box: C5 hop vs the smallest K (steps) a split-K conv may have (DCX_SPLIT_MIN_STEPS), two rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for r in 1 2; do
  for m in 0 32 64 128 256; do
    DCX_LIB=$R/distilcodec_nabeel_amd/minsteps.so DCX_SPLIT_MIN_STEPS=$m timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 > gpurun_out/r04za_${m}_$r.json 2> gpurun_out/r04za_${m}_$r.err || { echo C5_FAILED; tail -5 gpurun_out/r04za_${m}_$r.err; exit 1; }
    echo "== min_steps $m: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[0]); print(d['graph_ms'])" gpurun_out/r04za_${m}_$r.json)"
  done
done
