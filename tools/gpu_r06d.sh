set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/graph_diag.py > gpurun_out/r06d_graph.log 2>&1
