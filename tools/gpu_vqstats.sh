# GPU-box: tools/vq_stats.py on C2 (x6) and C3 (bf16), default list capacity and a large one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for G in "x6 32" "bf16 256"; do
  set -- $G
  timeout -k 10 200 python tools/vq_stats.py --gemm $1 --batch $2 || exit 1
  DCX_VQ_PAIRS_PER_ROW=1024 timeout -k 10 200 python tools/vq_stats.py --gemm $1 --batch $2 || exit 1
done
