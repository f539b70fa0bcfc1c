"""bench.py's multi-rank path (the driver's SCALE runs launch it as `torch.distributed.run ...
bench.py --gpus N`), rehearsed on a one-GPU box: `bench.py --gpus 2 --backend gloo` spawns two
ranks through torch.distributed.run as a fresh child process, both on cuda:0, at small sizes, for
every workload.  Each run must exit 0 and print ONE valid JSON line whose value counts both ranks'
rows -- so the first 8-GPU run is not the first execution of this path."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SMALL = {
    "c1": ["--c1-rows", "200000"],
    "c2": ["--rows", "2000000", "--no-cpu-baseline"],
    "c3": ["--c3-rows", "500000", "--c3-columns", "8"],
    "c4": ["--c4-rows", "2000000", "--c4-batch", "1000000", "--c4-distinct", "500000"],
    "c5": ["--c5-rows", "200000"],
}


@pytest.mark.parametrize("workload", sorted(SMALL))
def test_bench_two_ranks_gloo(gpu, workload):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--workload", workload] + SMALL[workload]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["steps"] == 2, out
    assert out["scaling"] == "weak"
    if workload == "c4":  # the key-hash exchange's cost is reported beside the step time
        ex = out["exchange"]
        assert ex["exchange_bytes"] > 0 and ex["bytes_received"] > 0, ex
        assert ex["max_exchange_ms"] >= ex["exchange_ms"] > 0, ex
        assert ex["exchange_ms"] >= ex["alltoall_ms"] >= 0 and ex["import_ms"] > 0, ex
