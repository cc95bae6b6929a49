set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_ab_tree.sh abl_r05 > gpurun_out/r06e_ab.log 2>&1 || exit 1
DCX_LIB=$GRAFT_REPO_ROOT/distilcodec_nabeel_amd/rp_stamps.so timeout -k 10 200 python tools/rp_stamps.py > gpurun_out/r06e_stamps.log 2>&1 || exit 1
timeout -k 10 200 python tools/pair_bench.py > gpurun_out/r06e_pair_def.log 2>&1 || exit 1
DCX_LIB=$GRAFT_REPO_ROOT/distilcodec_nabeel_amd/rp_nowload.so timeout -k 10 200 python tools/pair_bench.py > gpurun_out/r06e_pair_nowl.log 2>&1 || exit 1
timeout -k 10 200 python tools/pair_bench.py > gpurun_out/r06e_pair_def2.log 2>&1
