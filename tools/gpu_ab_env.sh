# GPU-box: A/B of a runtime switch (environment variable) on the C3 bench, two rounds each, after a
# pytest selection.  Usage: bash tools/gpu_ab_env.sh VAR VALUE_B "pytest selection"
set -o pipefail
VAR=$1; VB=$2; SEL=${3:-tests/test_gpu_c3.py}
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abenv_tests.log 2>&1; rc=$?; tail -2 gpurun_out/abenv_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export $VAR=$VB; else unset $VAR; fi
    timeout -k 10 300 python tools/c3_bench.py --gemm bf16 --steps 3 --kernels gpurun_out/abenv_$v > gpurun_out/abenv_$v.json 2>/dev/null || exit 1
    echo "$v ($VAR=${!VAR:-default}) $(python -c "import json;d=json.loads(open('gpurun_out/abenv_$v.json').readline());print(d['ms_per_step'])")"; python tools/kernel_table.py gpurun_out/abenv_${v}_bf16.json | sed -n 1,2p
  done
done
