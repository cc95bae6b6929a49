# GPU-box: accumulation probe, bf16-autocast / module / bf16 / api tests, C5 kernel table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/mfma_accum_probe.py > gpurun_out/r04c_accum.json 2>&1; cat gpurun_out/r04c_accum.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_autocast.py tests/test_gpu_modules.py tests/test_gpu_bf16.py tests/test_gpu_api.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?; grep -E "rel |PASS|FAIL|passed|failed|wav rel|codes equal" gpurun_out/r04c_tests.log | tail -80
exit $rc
