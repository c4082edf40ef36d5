"""The RCCL process-group path and the process-group fallback on the GPU box (the driver's 8-GPU scaling run
takes the same code paths with more ranks; docs/ARCHITECTURE.md lists what only it exercises)."""
import json
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


def test_nccl_transport_world1(gpu, tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, ATTACKFL_QUIET="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run(["timeout", "-k", "10", "150", sys.executable, os.path.join(ROOT, "tools", "nccl_world1_check.py")],
                       env=env, capture_output=True, text=True, timeout=200, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ok"], out


def test_process_group_fallback_world2_matches_single_process_bitwise(gpu, tmp_path):
    """IPC disabled (comm.one-shot-allgather: false): the update blocks travel through the gloo process group
    with host staging; the final checkpoint must equal the single-process run bit for bit."""
    d = {
        "server": {"num-round": 3, "clients": 4, "mode": "fedavg", "model": "TransformerModel", "genuine-rate": 1.0,
                   "data-distribution": {"num-data-range": [300, 600]}},
        "learning": {"epoch": 2, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000},
        "comm": {"attackers": {3: {"mode": "Min-Max", "round": 2}}, "one-shot-allgather": False},
        "engine": {"checkpoint-dir": str(tmp_path / "mp"), "trainer": "auto", "seed": 2,
                   "metrics": str(tmp_path / "mp" / "m.jsonl")},
        "log_path": str(tmp_path / "mp"),
    }
    cfg_path = tmp_path / "config.yaml"
    cfg_path.write_text(yaml.safe_dump(d))
    env = dict(os.environ, PYTHONPATH=ROOT, ATTACKFL_QUIET="1")
    cmd = ["timeout", "-k", "10", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "launch.py"), "--config", str(cfg_path), "--device", "cuda:0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    recs = [json.loads(l) for l in open(tmp_path / "mp" / "m.jsonl")]
    assert sum(x["ok"] for x in recs) == 3
    mp = torch.load(tmp_path / "mp" / "TransformerModel.pth", weights_only=True)
    d1 = dict(d, engine=dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp"), "metrics": ""}),
              log_path=str(tmp_path / "sp"))
    eng = FLEngine(from_dict(d1), device="cuda", verbose=False)
    eng.run()
    eng.close()
    sp = torch.load(tmp_path / "sp" / "TransformerModel.pth", weights_only=True)
    for k in sp:
        assert torch.equal(sp[k].cpu(), mp[k].cpu()), k
