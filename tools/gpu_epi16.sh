# GPU-box: bf16 staged epilogue A/B: bit digests of both builds, bf16 tests, C3 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in epif32.so libdcx.so; do
  echo "== bits $L"; DCX_LIB=$R/distilcodec_nabeel_amd/$L timeout -k 10 200 python tools/bf16_bits.py 4 10 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/epi16_tests.log 2>&1
rc=$?; tail -3 gpurun_out/epi16_tests.log; [ $rc = 0 ] || exit $rc
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/epif32.so distilcodec_nabeel_amd/libdcx.so "bf16dm|vq_|total" || exit 1
