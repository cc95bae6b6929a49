# GPU-box: A/B of a runtime switch on the C5 hop (split-K 16, graph-replayed), two rounds each, after a
# pytest selection.  Usage: bash tools/gpu_ab_c5.sh VAR VALUE_A "pytest selection" TAG
# A = VAR set to VALUE_A, B = the shipped default (VAR unset).
set -o pipefail
VAR=$1; VA=$2; SEL=${3:-tests/test_gpu_splitk.py}; TAG=${4:-abc5}
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export $VAR=$VA; else unset $VAR; fi
    timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 200 --warmup 20 --kernels gpurun_out/${TAG}_${v}_k$r.json > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    echo "$v ($VAR=${!VAR:-default}) $(head -c 400 gpurun_out/${TAG}_${v}_$r.json)"
  done
done
