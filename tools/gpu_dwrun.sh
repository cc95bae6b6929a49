# GPU-box: dwconv_ln_run tests, then C3 and C2 A/B against the tiled kernel (DCX_DWCONV_TILED=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dwrun_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dwrun_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    export DCX_DWCONV_TILED=$v
    timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/dw${v}_$r > gpurun_out/dw${v}_$r.json 2> gpurun_out/dw${v}_$r.err || { tail -3 gpurun_out/dw${v}_$r.err; exit 1; }
    echo "== C3 TILED=$v round $r: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/dw${v}_$r.json)"
    python tools/kernel_table.py gpurun_out/dw${v}_${r}_bf16.json | grep -E "dwconv"
  done
done
for v in 0 1; do
  export DCX_DWCONV_TILED=$v
  DCX_BENCH_KERNELS=gpurun_out/dwb${v}_k.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/dwb${v}.json 2> gpurun_out/dwb${v}.err || { tail -3 gpurun_out/dwb${v}.err; exit 1; }
  python - <<PY
import json
d = json.load(open("gpurun_out/dwb${v}.json")); k = json.load(open("gpurun_out/dwb${v}_k.json"))
print("C2 TILED=${v}", d["ms_per_step"], "ms; dwconv_ln", round(k["kernels"]["dwconv_ln"]["ms"] / k["steps"], 3), "ms")
PY
done
