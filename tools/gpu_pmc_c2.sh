# GPU-box: the three SQ counter passes of tools/gpu_pmc.sh over C2 only (the h3 kernels, the
# ResBlock pair kernels, the conv family).  Usage: bash tools/gpu_pmc_c2.sh TAG
set -o pipefail
TAG=${1:-pmc_c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA")
for i in 0 1 2; do
  timeout -s KILL 240 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace -d $R/gpurun_out/${TAG}_c2_p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-f32 --no-profile --no-c3 --no-c4 --no-c5 --no-oracle-codes > $R/gpurun_out/${TAG}_c2_p$i.log 2>&1 || { echo "PASS $i failed"; tail -5 $R/gpurun_out/${TAG}_c2_p$i.log; exit 1; }
  echo "PASS $i ok"
done
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_c2_p0 $R/gpurun_out/${TAG}_c2_p1 $R/gpurun_out/${TAG}_c2_p2 > $R/gpurun_out/${TAG}_c2_summary.txt
python3 tools/pmc_table.py $R/gpurun_out/${TAG}_c2_summary.txt > $R/gpurun_out/${TAG}_c2_table.md
cat $R/gpurun_out/${TAG}_c2_table.md
