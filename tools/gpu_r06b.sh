set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/range_diag.py > gpurun_out/r06b_diag.log 2>&1
