set -o pipefail
mkdir -p gpurun_out
for v in rp_stamps rp_nowait rp_nodma; do
  echo "== $v"
  DCX_LIB=$PWD/distilcodec_nabeel_amd/$v.so timeout -k 10 120 python -u tools/rp_stamps.py > gpurun_out/$v.log 2>&1 || { echo FAIL; tail gpurun_out/$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/$v.log
  DCX_LIB=$PWD/distilcodec_nabeel_amd/$v.so timeout -k 10 120 python -u tools/gen_bench.py --kernels 2>&1 | grep -E "res_pair|generate"
done
