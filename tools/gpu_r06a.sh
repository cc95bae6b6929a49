# round 6: the h3 range tests and the suites closest to the changed code (range scaling)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -v --maxfail=6 --timeout 300 --timeout-method thread \
  tests/test_gpu_range.py tests/test_gpu_h3.py tests/test_gpu_respair.py tests/test_gpu_modules.py tests/test_gpu_stages.py \
  tests/test_gpu_api.py > gpurun_out/r06a_range.log 2>&1
