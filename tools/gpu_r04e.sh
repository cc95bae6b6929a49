# GPU-box: bf16 tests (fp64-fold references), then the duplicate-launch epilogue timing on C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_autocast.py tests/test_gpu_bf16.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
grep -E "rel |PASS|FAIL|passed|failed|wav rel|codes equal|snr" gpurun_out/r04e_tests.log | tail -60
for M in 1 2; do
  DCX_DIAG_DUP=$M DCX_LIB=$R/distilcodec_nabeel_amd/dup.so DCX_BENCH_KERNELS=gpurun_out/r04e_dup$M.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/r04e_dup$M.out 2>&1 || { echo DUP_FAILED; tail -5 gpurun_out/r04e_dup$M.out; exit 1; }
  echo "== DCX_DIAG_DUP=$M"
  python tools/kernel_table.py gpurun_out/r04e_dup$M.json | sed -n 1,24p
done
