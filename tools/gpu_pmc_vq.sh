# GPU-box: PMC passes over the C3 bench for the VQ search kernels (vq_prefilter_b1, vq_certify,
# vq_pair_eval): HBM bytes, wave waits / instruction mix, L1 / TLB behaviour.  One pass per run.
# Usage: bash tools/gpu_pmc_vq.sh TAG
set -o pipefail
TAG=${1:-pmcvq}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "PASS $i failed"; tail -5 $R/gpurun_out/${TAG}_p$i.log; exit 1; }
  echo PASS $i ok
done
python3 tools/pmc_summary.py $R/gpurun_out/${TAG}_p1 $R/gpurun_out/${TAG}_p2 $R/gpurun_out/${TAG}_p3 $R/gpurun_out/${TAG}_p4 > $R/gpurun_out/${TAG}_summary.txt
grep -A 24 "vq_prefilter_b1\|vq_certify\|vq_pair_eval" $R/gpurun_out/${TAG}_summary.txt
