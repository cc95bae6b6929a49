# GPU-box: L2 hit / miss and HBM read counters over the h3 kernels (generator ParallelBlocks of the
# C = 512 / 256 stages and two encoder ConvNeXt blocks, tools/seg_diag_h3.py --no-diag), one
# rocprofv3 --pmc pass per counter set.  Usage: bash tools/gpu_pmc_h3.sh TAG
set -o pipefail
TAG=${1:-pmch3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
i=0
for P in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 tools/seg_diag_h3.py --no-diag --stages 0,1 > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "PASS $i failed"; tail -5 $R/gpurun_out/${TAG}_p$i.log; exit 1; }
  echo PASS $i ok
done
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_p1 $R/gpurun_out/${TAG}_p2 $R/gpurun_out/${TAG}_p3 > $R/gpurun_out/${TAG}_summary.txt
grep -A 20 "x3d" $R/gpurun_out/${TAG}_summary.txt | head -60
