# GPU-box: bf16dm register epilogue: bf16 / C3 tests, then C3 A/B against the LDS-staged epilogue
# (DCX_BF16_REG_EPI=0), two rounds each, per-kernel tables.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/regepi_tests.log 2>&1
rc=$?; tail -3 gpurun_out/regepi_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    export DCX_BF16_REG_EPI=$v
    timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/re${v}_$r > gpurun_out/re${v}_$r.json 2> gpurun_out/re${v}_$r.err || { tail -3 gpurun_out/re${v}_$r.err; exit 1; }
    echo "== REG_EPI=$v round $r: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/re${v}_$r.json)"
    python tools/kernel_table.py gpurun_out/re${v}_${r}_bf16.json | grep -E "bf16dm|prefilter"
  done
done
