set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_respair.py tests/test_gpu_h3.py tests/test_gpu_range.py > gpurun_out/r06i_tests.log 2>&1 || { tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -2 gpurun_out/r06i_tests.log
DCX_LIB=$GRAFT_REPO_ROOT/distilcodec_nabeel_amd/rp_stamps.so timeout -k 10 200 python tools/rp_stamps.py > gpurun_out/r06i_stamps.log 2>&1 || exit 1
bash tools/gpu_ab3.sh distilcodec_nabeel_amd/norange.so abl_r05 > gpurun_out/r06i_ab.log 2>&1 || exit 1
