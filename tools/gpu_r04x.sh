# GPU-box: half-tile prefilter records (half.so) and the fused split-K reduce (fused.so = both) vs the
# shipped library: tests, C3 A/B (two rounds), C5 A/B (two rounds), C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
DCX_LIB=$R/distilcodec_nabeel_amd/half.so timeout -k 10 600 $PT tests/test_gpu_vq.py tests/test_gpu_c3.py tests/test_gpu_bf16_autocast.py tests/test_gpu_api.py > gpurun_out/r04x_tests_half.log 2>&1 || { echo TESTS_HALF_FAILED; tail -30 gpurun_out/r04x_tests_half.log; exit 1; }
tail -1 gpurun_out/r04x_tests_half.log
DCX_LIB=$R/distilcodec_nabeel_amd/fused.so timeout -k 10 600 $PT tests/test_gpu_splitk.py tests/test_gpu_stream.py tests/test_gpu_stream_halo.py > gpurun_out/r04x_tests_fused.log 2>&1 || { echo TESTS_FUSED_FAILED; tail -30 gpurun_out/r04x_tests_fused.log; exit 1; }
tail -1 gpurun_out/r04x_tests_fused.log
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/half.so "prefilter|pair_eval|certify" || { echo AB_FAILED; exit 1; }
  for L in libdcx fused; do
    DCX_LIB=$R/distilcodec_nabeel_amd/$L.so timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 > gpurun_out/r04x_c5_${L}_$r.json 2> gpurun_out/r04x_c5_${L}_$r.err || { echo C5_FAILED; tail -5 gpurun_out/r04x_c5_${L}_$r.err; exit 1; }
    echo "== C5 $L: $(tail -1 gpurun_out/r04x_c5_${L}_$r.json | cut -c1-300)"
  done
done
for L in libdcx half; do
  DCX_LIB=$R/distilcodec_nabeel_amd/$L.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-c3 --no-c4 --no-c5 --no-oracle-codes --no-cpu-baseline --no-f32 > gpurun_out/r04x_c2_$L.json 2> gpurun_out/r04x_c2_$L.err || { echo BENCH_FAILED; tail -5 gpurun_out/r04x_c2_$L.err; exit 1; }
  echo "== C2 $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms', d['roofline']['frac'])" gpurun_out/r04x_c2_$L.json)"
done
