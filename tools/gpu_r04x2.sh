# GPU-box: which change breaks the split-K graphed halo stream (half.so / fused.so / fused.so with the
# two-launch reduce), then the C3 and C5 A/Bs.  Assertion failures are recorded and the run goes on;
# a timeout, abort or fault ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PT="python -u -m pytest -q --timeout 300 --timeout-method thread"
T="tests/test_gpu_stream_halo.py tests/test_gpu_splitk.py"
run() {  # tag, env..., then pytest
  local tag=$1; shift
  env "$@" timeout -k 10 600 $PT $T > gpurun_out/r04x2_$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc: $(tail -1 gpurun_out/r04x2_$tag.log)"
  grep "^FAILED" gpurun_out/r04x2_$tag.log | head -5
  if [ $rc -ge 2 ] || grep -q "Timeout" gpurun_out/r04x2_$tag.log; then echo STOP; exit 1; fi
}
run half DCX_LIB=$R/distilcodec_nabeel_amd/half.so
run fused_off DCX_LIB=$R/distilcodec_nabeel_amd/fused.so DCX_SPLIT_FUSED=0
run fused DCX_LIB=$R/distilcodec_nabeel_amd/fused.so
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/half.so "prefilter|pair_eval|certify" || { echo AB_FAILED; exit 1; }
  for L in libdcx fused; do
    DCX_LIB=$R/distilcodec_nabeel_amd/$L.so timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 100 --warmup 10 > gpurun_out/r04x_c5_${L}_$r.json 2> gpurun_out/r04x_c5_${L}_$r.err || { echo C5_FAILED; tail -5 gpurun_out/r04x_c5_${L}_$r.err; exit 1; }
    echo "== C5 $L: $(tail -1 gpurun_out/r04x_c5_${L}_$r.json | cut -c1-300)"
  done
done
