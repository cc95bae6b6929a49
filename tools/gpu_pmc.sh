# GPU-box: SQ counter passes over C3 (bf16: vq_prefilter_b1, conv_gemm_bf16dm / bf16dp) and C2 (the h3 kernels, the ResBlock
# pair kernels and the conv family), plus FETCH/WRITE over C3.  Usage: bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc5}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA")
run() {  # name counters cmd...
  local n=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/${TAG}_$n -o run --output-format csv -- "$@" > $R/gpurun_out/${TAG}_$n.log 2>&1 || { echo "PASS $n failed"; tail -5 $R/gpurun_out/${TAG}_$n.log; exit 1; }
  echo "PASS $n ok"
}
for i in 0 1 2; do run c3_p$i "${PASSES[$i]}" python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1; done
run c3_fetch FETCH_SIZE python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1
run c3_write WRITE_SIZE python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1
for i in 0 1 2; do run c2_p$i "${PASSES[$i]}" python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-f32 --no-profile --no-c3 --no-c4 --no-c5 --no-oracle-codes; done
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_c3_p0 $R/gpurun_out/${TAG}_c3_p1 $R/gpurun_out/${TAG}_c3_p2 $R/gpurun_out/${TAG}_c3_fetch $R/gpurun_out/${TAG}_c3_write > $R/gpurun_out/${TAG}_c3_summary.txt
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_c2_p0 $R/gpurun_out/${TAG}_c2_p1 $R/gpurun_out/${TAG}_c2_p2 > $R/gpurun_out/${TAG}_c2_summary.txt
python3 tools/pmc_table.py $R/gpurun_out/${TAG}_c3_summary.txt > $R/gpurun_out/${TAG}_c3_table.md
python3 tools/pmc_table.py $R/gpurun_out/${TAG}_c2_summary.txt > $R/gpurun_out/${TAG}_c2_table.md
cat $R/gpurun_out/${TAG}_c3_table.md $R/gpurun_out/${TAG}_c2_table.md
grep -A 30 "vq_prefilter_b1\|conv_gemm_bf16d" $R/gpurun_out/${TAG}_c3_summary.txt | grep -E "^dcx|FETCH|WRITE" | head -20
