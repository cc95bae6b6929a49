# GPU-box: VQ exactness tests after the prefilter swizzle fix, C3 bench, then the pair-schedule A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_c3.py tests/test_gpu_bf16_autocast.py tests/test_gpu_stages.py tests/test_gpu_modules.py -q --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04g_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/r04g_c3_kernels > gpurun_out/r04g_c3.json 2> gpurun_out/r04g_c3.err || { echo C3_FAILED; tail -3 gpurun_out/r04g_c3.err; exit 1; }
cat gpurun_out/r04g_c3.json; python tools/kernel_table.py gpurun_out/r04g_c3_kernels_bf16.json | head -6
bash tools/gpu_rpsync.sh r04g
