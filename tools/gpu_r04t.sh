# GPU-box: prefilter epilogue, 5-op top-2 update: VQ tests, tile timeline, C3 A/B vs the round-3 epilogue (two rounds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export DCX_LIB=$R/distilcodec_nabeel_amd/libdcx.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_vq.py tests/test_gpu_c3.py > gpurun_out/r04t_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04t_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04t_tests.log | tail -2
DCX_LIB=$R/distilcodec_nabeel_amd/tile.so timeout -k 10 300 python tools/tile_diag_vq.py --rows 239872 > gpurun_out/r04t_tiles.txt 2>&1 || { echo TILE_FAILED; tail -5 gpurun_out/r04t_tiles.txt; exit 1; }
grep search gpurun_out/r04t_tiles.txt
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/old.so distilcodec_nabeel_amd/libdcx.so "prefilter" || { echo AB_FAILED; exit 1; }
done
