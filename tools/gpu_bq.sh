# GPU-box: VQ search parity on the current library, then a C3 A/B of the 16x16x32 bf16 prefilter
# (libdcx.so) against the 32x32x16 form (bk32.so, -DDCX_VQ_BK32).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_bf16.py tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bq_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bq_tests.log; [ $rc = 0 ] || exit $rc
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/bk32.so "prefilter|rescore" || exit 1
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/bk32.so "prefilter|rescore"
