"""bench.py's N > 1 path end to end on the one-GPU box: two ranks under torch.distributed.run, the
shipped ShardedEncodeDecode per rank, barriers and max-over-ranks timing, the codes all_gather inside
the timed step and the C4 pass at N = 2 (global batch 256).  Both ranks share cuda:0 and gloo carries
the collectives (DCX_BENCH_ONE_DEVICE=1): RCCL refuses two ranks on one device, so the "nccl"
branch itself runs only on the driver's multi-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_device():
    env = dict(os.environ, DCX_BENCH_ONE_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "1"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 64 and d["config"]["parallelism"].startswith("clip-sharded x2")
    assert d["c4"]["global_batch"] == 256 and d["c4"]["n_gpus"] == 2 and d["c4"]["value"] > 0
    # single-GPU sub-records are not repeated at N > 1
    assert d["cpu_baseline"] is None and d["c3"] is None and d["c5"] is None and d["codes_vs_oracle"] is None
