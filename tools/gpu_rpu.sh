# GPU-box: fused ResBlock pair tests, per-phase stamps, and an A/B generator timing of the shipped
# pair kernels against the round-2 step schedule everywhere (DCX_RP_OLD=1), two rounds each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_respair.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/rpu_tests.log; [ $rc = 0 ] || exit $rc
DCX_LIB=$PWD/distilcodec_nabeel_amd/rp_stamps.so timeout -k 10 120 python -u tools/rp_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DCX_RP_OLD=1; else unset DCX_RP_OLD; fi
    echo "== $v round $r"
    timeout -k 10 120 python -u tools/gen_bench.py --kernels 2>&1 | grep -E "res_pair|generate" || exit 1
  done
done
