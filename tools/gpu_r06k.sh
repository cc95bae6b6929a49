set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_respair.py tests/test_gpu_h3.py tests/test_gpu_range.py > gpurun_out/r06k_tests.log 2>&1 || { tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -2 gpurun_out/r06k_tests.log
bash tools/gpu_ab_tree.sh abl_r05 > gpurun_out/r06k_ab.log 2>&1 || exit 1
