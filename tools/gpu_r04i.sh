# GPU-box: persistent bf16 pwconv1 (conv_gemm_bf16dp + GELU table): same-bits tests, C3 A/B, C5 kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_bf16_autocast.py > gpurun_out/r04i_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04i_tests.log; exit 1; }
tail -3 gpurun_out/r04i_tests.log
for V in persist nopersist nolut; do
  case $V in persist) E="";; nopersist) E="DCX_BF16_PERSIST=0";; nolut) E="DCX_GELU_LUT=0";; esac
  env $E timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --steps 3 --kernels gpurun_out/r04i_c3_$V > gpurun_out/r04i_c3_$V.json 2> gpurun_out/r04i_c3_$V.err || { echo C3_FAILED $V; tail -5 gpurun_out/r04i_c3_$V.err; exit 1; }
  echo "== C3 $V"; head -c 300 gpurun_out/r04i_c3_$V.json; echo; python tools/kernel_table.py gpurun_out/r04i_c3_${V}_bf16.json | sed -n 1,6p
done
timeout -k 10 300 python tools/stream_bench.py --split-k 16 --kernels gpurun_out/r04i_c5_kernels.json > gpurun_out/r04i_c5.json 2> gpurun_out/r04i_c5.err || { echo C5_FAILED; tail -5 gpurun_out/r04i_c5.err; exit 1; }
head -c 600 gpurun_out/r04i_c5.json; echo; python tools/kernel_table.py gpurun_out/r04i_c5_kernels.json | sed -n 1,40p
