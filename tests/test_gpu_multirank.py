"""Multi-process runs on the GPU box: two ranks sharing the GPU (gloo transport with device tensors,
staged through the host), fused trainer + LIE attacker (all-gather path) and plain FedAvg (all-reduce
path); the final checkpoint must equal the single-process GPU run of the same configuration."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import yaml

from attackfl_amd.config import from_dict
from attackfl_amd.fl.engine import FLEngine

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("attackers", [{3: {"mode": "LIE", "round": 2, "args": [0.74]}}, {}])
def test_two_ranks_match_single_process(gpu, tmp_path, attackers):
    d = {
        "server": {"num-round": 3, "clients": 4, "mode": "fedavg", "model": "TransformerModel",
                   "genuine-rate": 1.0, "data-distribution": {"num-data-range": [600, 900]}},
        "learning": {"epoch": 2, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 5000, "test-size": 1000},
        "comm": {"backend": "gloo", "attackers": attackers},
        "engine": {"checkpoint-dir": str(tmp_path / "mp"), "trainer": "auto"},
        "log_path": str(tmp_path / "mp"),
    }
    cfg_path = tmp_path / "config.yaml"
    cfg_path.write_text(yaml.safe_dump(d))
    env = dict(os.environ, PYTHONPATH=ROOT, ATTACKFL_QUIET="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "launch.py"), "--config", str(cfg_path),
           "--device", "cuda:0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    mp = torch.load(tmp_path / "mp" / "TransformerModel.pth", weights_only=True)
    d1 = dict(d, engine=dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp")}), log_path=str(tmp_path / "sp"))
    eng = FLEngine(from_dict(d1), device="cuda", verbose=False)
    eng.run()
    eng.close()
    sp = torch.load(tmp_path / "sp" / "TransformerModel.pth", weights_only=True)
    for k in sp:
        assert torch.allclose(sp[k].cpu(), mp[k].cpu(), atol=1e-5), k


@pytest.mark.parametrize("extra", [[], ["--attackers", "3:Min-Max:2"]])
def test_bench_two_ranks(gpu, tmp_path, extra):
    """bench.py's multi-rank path (the driver's scaling run) end to end: two gloo ranks sharing the GPU."""
    import json

    env = dict(os.environ, PYTHONPATH=ROOT, AFL_BENCH_BACKEND="gloo", AFL_BENCH_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1"] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rounds_ok"] == 2 and out["value"] > 0
    assert out["config"]["parallelism"] == "fl8-clients-over-2-ranks"
