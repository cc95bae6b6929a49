# GPU-box: grouped split-K (C5): split-K / stream tests, C5 A/B (grouped vs per-conv), hop trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_splitk.py tests/test_gpu_stream.py tests/test_gpu_stream_halo.py > gpurun_out/r04m_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04m_tests.log; exit 1; }
grep -E "passed|failed|dB" gpurun_out/r04m_tests.log | tail -12
for r in 1 2; do
  for G in on off; do
    if [ $G = off ]; then export DCX_SPLIT_GROUP_OFF=1; else unset DCX_SPLIT_GROUP_OFF; fi
    timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 > gpurun_out/r04m_c5_$G.json 2> gpurun_out/r04m_c5_$G.err || { echo C5_FAILED; tail -5 gpurun_out/r04m_c5_$G.err; exit 1; }
    echo "== C5 group $G: $(head -1 gpurun_out/r04m_c5_$G.json | cut -c1-330)"
  done
done
unset DCX_SPLIT_GROUP_OFF
bash tools/gpu_c5trace.sh r04m_c5t && python tools/hop_timeline.py gpurun_out/r04m_c5t_kernel_trace.csv --top 25 > gpurun_out/r04m_c5_timeline.txt || { echo C5T_FAILED; exit 1; }
head -30 gpurun_out/r04m_c5_timeline.txt
