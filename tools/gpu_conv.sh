# GPU-box: conv parity tests + microbenchmark.  Usage: bash tools/gpu_conv.sh [conv_bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py -x -q > gpurun_out/conv_tests.log 2>&1; RC=$?; echo CONV_TESTS $RC; tail -5 gpurun_out/conv_tests.log
[ $RC -eq 0 ] || exit 1
timeout -k 10 600 python tools/conv_bench.py "$@" > gpurun_out/conv_bench.txt 2>&1; echo CONV_BENCH $?; grep -v amdgpu.ids gpurun_out/conv_bench.txt
