# GPU-box: SQ counter passes over the small-C pair kernels alone (tools/pair_bench.py), for the shipped
# kernels and for one knob variant.  Usage: bash tools/gpu_pmc_pairs.sh TAG [VAR VALUE]
set -o pipefail
TAG=${1:-pp}; VAR=$2; VAL=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
        "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum")
timeout -k 10 120 python3 tools/pair_bench.py --reps 3 > $R/gpurun_out/${TAG}_time_A.json || exit 1
echo "A: $(cat $R/gpurun_out/${TAG}_time_A.json)"
if [ -n "$VAR" ]; then
  env $VAR=$VAL timeout -k 10 120 python3 tools/pair_bench.py --reps 3 > $R/gpurun_out/${TAG}_time_B.json || exit 1
  echo "B ($VAR=$VAL): $(cat $R/gpurun_out/${TAG}_time_B.json)"
fi
for v in A B; do
  [ $v = B ] && [ -z "$VAR" ] && break
  for i in 0 1 2 3; do
    if [ $v = B ]; then export $VAR=$VAL; fi
    timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace -d $R/gpurun_out/${TAG}_${v}_p$i -o run --output-format csv -- python3 tools/pair_bench.py --reps 1 > $R/gpurun_out/${TAG}_${v}_p$i.log 2>&1 || { echo "PASS $v $i failed"; tail -5 $R/gpurun_out/${TAG}_${v}_p$i.log; exit 1; }
  done
  unset $VAR 2>/dev/null
  python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_${v}_p0 $R/gpurun_out/${TAG}_${v}_p1 $R/gpurun_out/${TAG}_${v}_p2 $R/gpurun_out/${TAG}_${v}_p3 > $R/gpurun_out/${TAG}_${v}_summary.txt
  rm -rf $R/gpurun_out/${TAG}_${v}_p?
done
grep -E "^dcx|MFMA busy|/ WAVE|INSTS_|TCC_|TCP_|LDS_IDX|GRBM" $R/gpurun_out/${TAG}_A_summary.txt | head -80
