# GPU-box: bf16 tests after the decode-table fix, then the no-store epilogue A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/bf16_resblock_diag.py > gpurun_out/r04d_rbdiag.txt 2>&1; grep -v amdgpu.ids gpurun_out/r04d_rbdiag.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_autocast.py tests/test_gpu_bf16.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
grep -E "rel |PASS|FAIL|passed|failed|wav rel|codes equal|conv \(|snr" gpurun_out/r04d_tests.log | tail -80
for L in distilcodec_nabeel_amd/base.so distilcodec_nabeel_amd/nostore.so; do
  T=$(basename $L .so)
  DCX_LIB=$R/$L DCX_BENCH_KERNELS=gpurun_out/r04d_ab_$T.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/r04d_ab_$T.out 2>&1 || exit 1
  echo "== $T: $(tail -1 gpurun_out/r04d_ab_$T.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms')")"
  python tools/kernel_table.py gpurun_out/r04d_ab_$T.json | sed -n 1,12p
done
