# GPU-box: pair kernels on smaller tiles for small batches: same-bits tests, C5 and C2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_respair.py tests/test_gpu_splitk.py > gpurun_out/r04n_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04n_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04n_tests.log | tail -3
for r in 1 2; do
  for V in auto big; do
    if [ $V = big ]; then export DCX_RP_R=496; else unset DCX_RP_R; fi
    timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 --kernels gpurun_out/r04n_c5k_$V.json > gpurun_out/r04n_c5_$V.json 2> gpurun_out/r04n_c5_$V.err || { echo C5_FAILED; tail -5 gpurun_out/r04n_c5_$V.err; exit 1; }
    echo "== C5 pair tiles $V: $(head -1 gpurun_out/r04n_c5_$V.json | cut -c150-330)"
  done
done
unset DCX_RP_R
python tools/kernel_table.py gpurun_out/r04n_c5k_auto.json | head -12
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/r04n_bench.err; exit 1; }
head -c 700 gpurun_out/r04n_bench.json
