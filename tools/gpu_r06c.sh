# round 6: the whole GPU suite, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06c_gpu.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-oracle-codes > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err
