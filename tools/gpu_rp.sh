# GPU-box: fused ResBlock pair tests, generator / end-to-end parity, then an A/B bench (fused vs
# per-conv launches, DCX_NO_RESPAIR=1) with per-kernel times.  Usage: bash tools/gpu_rp.sh TAG
set -o pipefail
TAG=${1:-rp}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_respair.py tests/test_gpu_stages.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|SNR|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -40; [ $rc = 0 ] || exit $rc
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
DCX_NO_RESPAIR=1 DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels_off.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench_off.json 2> gpurun_out/${TAG}_bench_off.err || { echo BENCH_OFF_FAILED; exit 1; }
DCX_BENCH_KERNELS=gpurun_out/${TAG}_bench_kernels2.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo BENCH2_FAILED; exit 1; }
python - <<PY
import json
for n in ("${TAG}_bench", "${TAG}_bench_off", "${TAG}_bench2"):
    d = json.load(open(f"gpurun_out/{n}.json"))
    print(n, d["value"], d["ms_per_step"])
for n in ("${TAG}_bench_kernels", "${TAG}_bench_kernels_off"):
    d = json.load(open(f"gpurun_out/{n}.json"))
    k, st = d["kernels"], d["steps"]
    print(n, "(ms per step)")
    for name, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"])[:14]:
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
        print(f"  {name:42s} {v['ms'] / st:8.2f} ms  {v['launches'] // st:4d} launches  {tf:6.1f} TF")
PY
