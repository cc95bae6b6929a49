# GPU-box: A/B of two builds on the C5 hop (split-K 16, graph replay), two rounds each, after a pytest
# selection on the default build.  Usage: bash tools/gpu_ab_c5lib.sh LIB_A "pytest selection" TAG
# A = distilcodec_nabeel_amd/LIB_A.so (DCX_LIB), B = the default libdcx.so.
set -o pipefail
LA=$1; SEL=${2:-tests/test_gpu_splitk.py}; TAG=${3:-abc5l}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export DCX_LIB=$R/distilcodec_nabeel_amd/$LA.so; else unset DCX_LIB; fi
    timeout -k 10 300 python tools/stream_bench.py --split-k 16 --hops 200 --warmup 20 > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    echo "$v (${DCX_LIB:-default}) $(python -c "import json;d=json.loads(open('gpurun_out/${TAG}_${v}_$r.json').readline());print(d['graph_ms'])")"
  done
done
