# GPU-box: bf16-mode parity tests, then a C3 A/B of the branch-free bf16 GELU (libdcx.so) against erff (gelerf.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c3.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gelu_tests.log; [ $rc = 0 ] || exit $rc
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/gelerf.so "bf16dm|prefilter" || exit 1
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/gelerf.so "bf16dm|prefilter"
