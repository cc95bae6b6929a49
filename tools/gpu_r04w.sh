# GPU-box: prefilter per-wave half-tile records (half.so) vs shipped: VQ / C3 / API tests, C3 A/B (two rounds), C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
DCX_LIB=$R/distilcodec_nabeel_amd/half.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vq.py tests/test_gpu_c3.py tests/test_gpu_bf16_autocast.py tests/test_gpu_api.py tests/test_gpu_splitk.py > gpurun_out/r04w_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04w_tests.log; exit 1; }
tail -2 gpurun_out/r04w_tests.log
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/half.so "prefilter|pair_eval|certify" || { echo AB_FAILED; exit 1; }
done
for L in libdcx half; do
  DCX_LIB=$R/distilcodec_nabeel_amd/$L.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-c3 --no-c4 --no-c5 --no-oracle-codes --no-cpu-baseline --no-f32 > gpurun_out/r04w_c2_$L.json 2> gpurun_out/r04w_c2_$L.err || { echo BENCH_FAILED; tail -5 gpurun_out/r04w_c2_$L.err; exit 1; }
  echo "== C2 $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms', d['roofline']['frac'])" gpurun_out/r04w_c2_$L.json)"
done
