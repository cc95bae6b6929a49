# GPU-box: A/B of the ResBlock-pair schedules on C2 (one session): the default (step schedule at
# C = 64, barrier-free at C = 32), the barrier-free kernel at C = 64 (DCX_RP_G64=1) and tap-sync
# intervals (DCX_RP_SYNC=n), with per-kernel tables.  Then the pair tests under the chosen switches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-rps}
one() {  # label env...
  local lab=$1; shift
  env "$@" DCX_BENCH_KERNELS=gpurun_out/${TAG}_$lab.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32 --no-c3 --no-c4 --no-c5 --no-oracle-codes > gpurun_out/${TAG}_$lab.out 2>&1 || { echo "FAILED $lab"; tail -3 gpurun_out/${TAG}_$lab.out; exit 1; }
  echo "== $lab: $(tail -1 gpurun_out/${TAG}_$lab.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms')")"
  python tools/kernel_table.py gpurun_out/${TAG}_$lab.json | grep -E "res_pair|x6dm<256,256> "
}
for round in 1 2; do
  one base$round DCX_RP_SYNC=0
  one g64s0_$round DCX_RP_G64=1 DCX_RP_SYNC=0
  one g64s1_$round DCX_RP_G64=1 DCX_RP_SYNC=1
  one g64s2_$round DCX_RP_G64=1 DCX_RP_SYNC=2
  one g64s3_$round DCX_RP_G64=1 DCX_RP_SYNC=3
done
DCX_RP_G64=1 DCX_RP_SYNC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_respair.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; tail -2 gpurun_out/${TAG}_tests.log
