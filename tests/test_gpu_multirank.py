"""Multi-process runs on the GPU box: several ranks sharing the one GPU (gloo process group, the one-shot
IPC all-gather as the update path — stream-ordered, no host staging — replicated validation, speculative
launch at world > 1).  The final checkpoint of a multi-rank run must equal the single-process run of the
same configuration BIT FOR BIT (every kernel on the round path is deterministic and a client's trajectory
does not depend on the rank that trains it), and ``bench.py``'s multi-rank path must report the IPC path."""
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


CASES = {
    # fedavg + a Min-Max attacker (all-gather path, attack math on the owning rank)
    "tf-fedavg-minmax": ("TransformerModel", "fedavg", {5: {"mode": "Min-Max", "round": 2}}),
    # hypernetwork server + Opt-Fang on the RNN (replicated hnet update and hyper validation)
    "rnn-hyper-optfang": ("RNNModel", "hyper", {6: {"mode": "Opt-Fang", "round": 2}}),
    # plain fedavg (no attacker): at world > 1 with IPC it stays on the gather + FedAvg kernel path
    "tf-fedavg": ("TransformerModel", "fedavg", {}),
    # the on-chip CNN trainer needs all 32 workgroups of a client co-resident: ranks sharing the GPU size their
    # launches to CUs / sharers (parallel.launcher.gpu_sharers) instead of spinning on absent workgroups
    "cnn-fedavg": ("CNNModel", "fedavg", {}),
    # robust rules in the early launch at world > 1 (device sizes / attacker flags from the gathered meta):
    # a plain device rule, gmm (filter success read after the wait) and FLTrust (replicated server-model step)
    "tf-krum-minmax": ("TransformerModel", "krum", {5: {"mode": "Min-Max", "round": 2}}),
    "tf-gmm-minmax": ("TransformerModel", "gmm", {5: {"mode": "Min-Max", "round": 2}}),
    "tf-fltrust-minmax": ("TransformerModel", "FLTrust", {5: {"mode": "Min-Max", "round": 2}}),
}


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("case", sorted(CASES))
def test_ranks_sharing_gpu_match_single_process_bitwise(gpu, tmp_path, world, case):
    model, mode, attackers = CASES[case]
    d = {
        "server": {"num-round": 3, "clients": 8, "mode": mode, "model": model, "genuine-rate": 0.5,
                   "data-distribution": {"num-data-range": [300, 600]}},
        "learning": {"epoch": 2, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000},
        "comm": {"attackers": attackers},
        "engine": {"checkpoint-dir": str(tmp_path / "mp"), "trainer": "auto", "seed": 2,
                   "metrics": str(tmp_path / "mp" / "m.jsonl")},
        "log_path": str(tmp_path / "mp"),
    }
    cfg_path = tmp_path / "config.yaml"
    cfg_path.write_text(yaml.safe_dump(d))
    env = dict(os.environ, PYTHONPATH=ROOT, ATTACKFL_QUIET="1")
    cmd = ["timeout", "-k", "10", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "launch.py"), "--config", str(cfg_path), "--device", "cuda:0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    name = f"{model}_hyper_8.pth" if mode == "hyper" else f"{model}.pth"
    mp = torch.load(tmp_path / "mp" / name, weights_only=True)
    recs = [json.loads(l) for l in open(tmp_path / "mp" / "m.jsonl")]
    assert sum(r["ok"] for r in recs) == 3
    assert all(r.get("path") != "fedavg-allreduce" for r in recs)  # IPC gather path, not the all-reduce
    # per-client epoch losses of every rank's clients reach the leader's JSONL through the gathered block
    trained = [l for l in recs[-1]["client_loss"] if l is not None]
    assert len(trained) == 8 - len(attackers) and all(len(l) == 2 and l[0] > 0 for l in trained)
    d1 = dict(d, engine=dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp"), "metrics": ""}),
              log_path=str(tmp_path / "sp"))
    eng = FLEngine(from_dict(d1), device="cuda", verbose=False)
    eng.run()
    eng.close()
    sp = torch.load(tmp_path / "sp" / name, weights_only=True)
    assert list(sp) == list(mp)
    for k in sp:
        assert torch.equal(sp[k].cpu(), mp[k].cpu()), k


@pytest.mark.parametrize("world,extra", [(2, []), (8, []), (8, ["--attackers", "3:LIE:2:0.74"]),
                                         (8, ["--mode", "hyper", "--model", "RNNModel",
                                              "--attackers", "6:Opt-Fang:2"])])
def test_bench_ranks_sharing_gpu(gpu, tmp_path, world, extra):
    """bench.py's multi-rank path (the driver's scaling run): N ranks on the one GPU over the IPC path; the
    JSON line reports it, every timed round succeeded and every round's checkpoint landed."""
    env = dict(os.environ, PYTHONPATH=ROOT, AFL_BENCH_DEVICE="0")
    cmd = ["timeout", "-k", "10", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "4", "--warmup", "2"] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["rounds_ok"] == 4 and out["value"] > 0
    assert out["comm"] == "ipc-one-shot" and out["speculative"] is True
    assert out["ckpt_dropped"] == 0 and out["ckpt_written"] >= 4
    assert out["config"]["parallelism"] == f"fl8-clients-over-{world}-ranks"


def test_classic_launch_on_the_gpu_matches_single_process_bitwise(gpu, tmp_path):
    """The reference-style launch on the GPU box: server.py + 4 x client.py (clients 1-4 -> group ranks 0-3, all on
    the one visible GPU: gloo group + IPC all-gather, each client's co-residency budget a quarter of the CUs); the
    leader client writes the server's checkpoint, which equals the single-process run bit for bit."""
    import datetime
    import time

    import torch.distributed as dist

    port = _port()
    d = {
        "server": {"num-round": 2, "clients": 4, "mode": "fedavg", "model": "TransformerModel",
                   "data-distribution": {"num-data-range": [300, 600]}},
        "learning": {"epoch": 2, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000},
        "comm": {"address": "127.0.0.1", "port": port},
        "engine": {"checkpoint-dir": "ckpt", "trainer": "auto", "seed": 3},
        "log_path": "logs",
    }
    cfg_path = tmp_path / "config.yaml"
    cfg_path.write_text(yaml.safe_dump(d))
    env = dict(os.environ, PYTHONPATH=ROOT, ATTACKFL_QUIET="1")
    srv = subprocess.Popen(["timeout", "-k", "10", "170", sys.executable, os.path.join(ROOT, "server.py"),
                            "--config", str(cfg_path)], env=env, cwd=str(tmp_path), stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    cls = []
    try:
        store = None
        for _ in range(300):
            try:
                store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=5),
                                      use_libuv=False)
                break
            except Exception:
                time.sleep(0.2)
        assert store is not None
        for i in range(4):
            cls.append(subprocess.Popen(["timeout", "-k", "10", "160", sys.executable, os.path.join(ROOT, "client.py"),
                                         "--config", str(cfg_path)], env=env, cwd=str(tmp_path),
                                        stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
            while int(store.add("attackfl/next_rank", 0)) < i + 1:  # registration order = client index
                assert cls[-1].poll() is None, cls[-1].communicate()[1][-3000:]
                time.sleep(0.05)
        out, err = srv.communicate(timeout=180)
        assert srv.returncode == 0, err[-3000:]
        for c in cls:
            o, e = c.communicate(timeout=60)
            assert c.returncode == 0, e[-3000:]
    finally:
        for p in [srv] + cls:
            if p.poll() is None:
                p.kill()
    mp = torch.load(tmp_path / "ckpt" / "TransformerModel.pth", weights_only=True)
    assert open(tmp_path / "logs" / "app.log").read().count("ROC_AUC") == 2
    d1 = dict(d, engine=dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp")}), log_path=str(tmp_path / "sp"))
    d1["comm"] = {}
    eng = FLEngine(from_dict(d1), device="cuda", verbose=False)
    eng.run()
    eng.close()
    sp = torch.load(tmp_path / "sp" / "TransformerModel.pth", weights_only=True)
    assert list(sp) == list(mp)
    for k in sp:
        assert torch.equal(sp[k].cpu(), mp[k].cpu()), k
