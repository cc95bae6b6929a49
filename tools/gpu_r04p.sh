# GPU-box: split-K slice bound 16 / 32 / 64 on the C5 hop (A/B, two rounds); split-K tests at 64.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
for r in 1 2; do
  for S in 16 32 64; do
    timeout -k 10 300 python tools/stream_bench.py --split-k $S --hops 100 --warmup 10 > gpurun_out/r04p_c5_$S.json 2> gpurun_out/r04p_c5_$S.err || { echo C5_FAILED; tail -5 gpurun_out/r04p_c5_$S.err; exit 1; }
    echo "== C5 split $S: $(head -1 gpurun_out/r04p_c5_$S.json | cut -c150-330)"
  done
done
timeout -k 10 300 python tools/stream_bench.py --split-k 64 --hops 20 --warmup 5 --kernels gpurun_out/r04p_c5k_64.json > /dev/null 2>&1 && python tools/kernel_table.py gpurun_out/r04p_c5k_64.json | head -8
