# GPU-box: chained ParallelBlock-mean group in the split-K mode: tests, C5, hop trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_splitk.py tests/test_gpu_stream.py tests/test_gpu_stream_halo.py > gpurun_out/r04o_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04o_tests.log; exit 1; }
grep -E "passed|failed|dB" gpurun_out/r04o_tests.log | tail -12
timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 200 --warmup 20 > gpurun_out/r04o_c5.json 2> gpurun_out/r04o_c5.err || { echo C5_FAILED; tail -5 gpurun_out/r04o_c5.err; exit 1; }
head -c 1500 gpurun_out/r04o_c5.json
bash tools/gpu_c5trace.sh r04o_c5t && python tools/hop_timeline.py gpurun_out/r04o_c5t_kernel_trace.csv --top 25 > gpurun_out/r04o_c5_timeline.txt || { echo C5T_FAILED; exit 1; }
head -30 gpurun_out/r04o_c5_timeline.txt
