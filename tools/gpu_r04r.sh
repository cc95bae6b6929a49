# GPU-box: vq_prefilter_b1 per-tile timeline (DCX_TILE_DIAG build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
DCX_LIB=$R/distilcodec_nabeel_amd/tile.so timeout -k 10 300 python tools/tile_diag_vq.py --rows 32768 > gpurun_out/r04r_tiles.txt 2>&1 || { echo TILE_FAILED; tail -5 gpurun_out/r04r_tiles.txt; exit 1; }
DCX_LIB=$R/distilcodec_nabeel_amd/tile.so timeout -k 10 300 python tools/tile_diag_vq.py --rows 239872 >> gpurun_out/r04r_tiles.txt 2>&1 || { echo TILE_FAILED; tail -5 gpurun_out/r04r_tiles.txt; exit 1; }
grep search gpurun_out/r04r_tiles.txt
