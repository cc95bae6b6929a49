# GPU-box: A/B of two builds on the C3 bench (bf16 token extraction), one session.
#   bash tools/gpu_ab_c3.sh LIB_A LIB_B [kernel-name filter]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in $1 $2; do
  T=$(basename $L .so)
  DCX_LIB=$R/$L timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --kernels gpurun_out/c3ab_$T > gpurun_out/c3ab_$T.json 2> gpurun_out/c3ab_$T.err || exit 1
  echo "== C3 $L: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], 'ms', round(d['value']/1e6, 1), 'M samples/s')" gpurun_out/c3ab_$T.json)"
  python tools/kernel_table.py gpurun_out/c3ab_${T}_bf16.json | grep -E "${3:-.}" | head -6
done
