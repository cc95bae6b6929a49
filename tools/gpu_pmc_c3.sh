# GPU-box: PMC counter passes over the C3 bench (bf16 mode: vq_prefilter_bq, conv_gemm_bf16dm).
# Usage: bash tools/gpu_pmc_c3.sh TAG
set -o pipefail
TAG=${1:-pmc3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "PASS $i failed"; tail -5 $R/gpurun_out/${TAG}_p$i.log; exit 1; }
  echo PASS $i ok
done
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_p1 $R/gpurun_out/${TAG}_p2 $R/gpurun_out/${TAG}_p3 > $R/gpurun_out/${TAG}_summary.txt
grep -A 26 "vq_prefilter_bq\|vq_prefilter_bk\|conv_gemm_bf16dm" $R/gpurun_out/${TAG}_summary.txt | grep -E "^dcx|INSTS|MFMA busy|WAIT|BANK|ACTIVE_INST_ANY /"
