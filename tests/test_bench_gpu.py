"""bench.py contract on one GPU, and a 2-rank rehearsal of the multi-GPU path
(routed set/get over ShardedKV with GpuShard kernels; gloo backend so both ranks
can share the single GPU of a test box -- RCCL runs the same ShardedKV code)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--keys-per-gpu", "1000000", "--batch", "200000", "--steps", "2", "--warmup", "1", "--embed-batch", "8",
         "--embed-seq", "128", "--verify", "2000"]


def _json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_gpu_contract():
    r = subprocess.run([sys.executable, "bench.py", *SMALL], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["integrity_failures"] == 0 and d["value"] > 0
    # config #2 literally (every client stream posts its own slice) beside the fused grid
    assert d["kv_async_ops_per_s"] > 0 and d["kv_async_integrity_failures"] == 0, d.get("kv_async_submission")
    assert d["kv_async_streams"] == {"writer": 32, "reader": 32}


def test_bench_two_rank_rehearsal_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--backend", "gloo", *SMALL, "--search-keys", "2000000"],  # two ranks share one GPU's HBM
                       cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 2 and d["integrity_failures"] == 0
    assert d["kv_ok"] >= 0.999 * d["config"]["global_batch"] * 2  # routed ops of the 2 timed steps succeeded
