# GPU-box: HBM traffic of the C3 kernels: rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs)
# over tools/c3_bench.py in bf16 mode, then the per-launch table (2*FETCH + WRITE, gfx950 correction).
# Usage: bash tools/gpu_hbm_c3.sh TAG
set -o pipefail
TAG=${1:-hbm3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp; cd $R
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/${TAG}_$C -o run --output-format csv -- python3 tools/c3_bench.py --gemm bf16 --steps 1 > $R/gpurun_out/${TAG}_$C.log 2>&1 || { echo "$C pass failed"; tail -5 $R/gpurun_out/${TAG}_$C.log; exit 1; }
  echo "$C pass ok"
done
python3 tools/pmc_to_json.py $R/gpurun_out/${TAG}_FETCH_SIZE $R/gpurun_out/${TAG}_WRITE_SIZE > $R/gpurun_out/${TAG}_pmc.json
python3 -c "
import json; d=json.load(open('$R/gpurun_out/${TAG}_pmc.json'))['kernels']
for k, v in sorted(d.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'] * kv[1]['launches'])[:8]: print(k, v)"
