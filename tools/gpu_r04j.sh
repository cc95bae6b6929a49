# GPU-box: VQ prefilter segment stamps; static-priority A/B on C3 (two rounds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
DCX_LIB=$R/distilcodec_nabeel_amd/seg.so timeout -k 10 300 python tools/seg_diag_vq.py --rows 65536 > gpurun_out/r04j_seg.txt 2>&1 || { echo SEG_FAILED; tail -5 gpurun_out/r04j_seg.txt; exit 1; }
grep vq_prefilter gpurun_out/r04j_seg.txt
for r in 1 2; do
  bash tools/gpu_ab_c3.sh distilcodec_nabeel_amd/libdcx.so distilcodec_nabeel_amd/sprio.so "prefilter|bf16d" || { echo AB_FAILED; exit 1; }
done
bash tools/gpu_c5trace.sh r04j_c5t && python tools/hop_timeline.py gpurun_out/r04j_c5t_kernel_trace.csv --top 30
