# GPU-box: the graph-captured stream tests first (short limit), then the GPU test suite, then the C3 and
# C2 kernel tables.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_halo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rs_graph.log 2>&1; rc=$?; tail -3 gpurun_out/rs_graph.log; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rs_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rs_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/c3_bench.py --kernels gpurun_out/rs_c3 > gpurun_out/rs_c3.json 2> gpurun_out/rs_c3.err || exit 1
cat gpurun_out/rs_c3.json | cut -c1-200
python tools/kernel_table.py gpurun_out/rs_c3_bf16.json | grep -E "rescore|certify|reset|sqnorm|total"
DCX_BENCH_KERNELS=gpurun_out/rs_c2.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 > gpurun_out/rs_bench.json 2> gpurun_out/rs_bench.err || exit 1
cat gpurun_out/rs_bench.json | cut -c1-300
python tools/kernel_table.py gpurun_out/rs_c2.json | grep -E "rescore|certify|reset|sqnorm|total"
