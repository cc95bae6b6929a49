# GPU-box: C2 kernel tables of libdcx.so and the no-epilogue timing build (noepi.so, -DDCX_DIAG_NOEPI;
# wrong numerics, timing only): what the LDS-staged conv epilogues cost per kernel family.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in libdcx noepi; do
  DCX_LIB=$R/distilcodec_nabeel_amd/$L.so DCX_BENCH_KERNELS=gpurun_out/ne_$L.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32 > gpurun_out/ne_$L.out 2>&1 || exit 1
  echo "== $L"; python tools/kernel_table.py gpurun_out/ne_$L.json | head -12
done
