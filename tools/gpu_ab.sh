# GPU-box: A/B conv microbenchmark of two builds of libdcx.so in one session.
#   bash tools/gpu_ab.sh LIB_A LIB_B [conv_bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
A=$1; B=$2; shift 2
for round in 1 2; do
  for L in $A $B; do
    echo "== $L (round $round)"
    timeout -k 10 300 env DCX_LIB=$R/$L python tools/conv_bench.py "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
