# GPU-box: dwconv_ln_run tests, then C5 hop A/B against the tiled kernel (DCX_DWCONV_TILED=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dwc5_tests.log 2>&1
rc=$?; tail -1 gpurun_out/dwc5_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    DCX_DWCONV_TILED=$v timeout -k 10 200 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 > gpurun_out/dwc5_${v}_$r.out 2>&1 || exit 1
    echo "TILED=$v round $r: $(grep -v amdgpu gpurun_out/dwc5_${v}_$r.out | head -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['graph_ms'])")"
  done
done
