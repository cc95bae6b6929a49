# GPU-box: a round's evidence run: gpu_final.sh (GPU tests, C3, C5, rocprofv3 trace + FETCH/WRITE PMC,
# the default bench with its CPU-baseline leg), then the C2 SQ counter passes.  Usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-evidence}
bash tools/gpu_final.sh $TAG > gpurun_out/${TAG}_final.log 2>&1 || { tail -20 gpurun_out/${TAG}_final.log; exit 1; }
tail -3 gpurun_out/${TAG}_final.log
bash tools/gpu_pmc_c2.sh $TAG > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
