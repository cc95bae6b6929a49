# GPU-box: full GPU test suite; prefilter norm-preload A/B on C3 (two rounds); C2 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04q_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04q_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04q_tests.log | tail -3
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/nopre.so distilcodec_nabeel_amd/libdcx.so "prefilter" || { echo AB_FAILED; exit 1; }
done
