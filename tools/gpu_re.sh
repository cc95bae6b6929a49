set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/re_tests.log 2>&1; rc=$?; tail -3 gpurun_out/re_tests.log; [ $rc = 0 ] || exit $rc
DCX_BENCH_KERNELS=gpurun_out/re_kernels.json timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/re_bench.json 2> gpurun_out/re_bench.err || exit 1
cat gpurun_out/re_bench.json; python tools/kernel_table.py gpurun_out/re_kernels.json | head -8
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/vq84.so prefilter || exit 1
bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/vq84.so prefilter
for L in libdcx geluprobe libdcx geluprobe; do
  DCX_LIB=$(pwd)/distilcodec_nabeel_amd/$L.so DCX_BENCH_KERNELS=gpurun_out/ab_$L.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$L.out 2>&1 || exit 1
  echo "== bench $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], 'ms')" gpurun_out/ab_$L.out)"
  python tools/kernel_table.py gpurun_out/ab_$L.json | grep -E "x6dm<256,256>|total"
done
