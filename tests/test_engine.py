"""Round engine on CPU: every server mode, attacks, retry semantics, checkpoints, resume, and the
multi-process paths (gloo, world size 2-3) for both launch styles."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import yaml

from attackfl_amd.config import from_dict
from attackfl_amd.fl.engine import FLEngine, build_client_table
from attackfl_amd.models import HyperNetwork, ParamLayout, build_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp_path, **kw):
    d = {
        "server": {"num-round": 2, "clients": 4, "mode": "fedavg", "model": "TransformerModel",
                   "data-distribution": {"num-data-range": [150, 260]}},
        "learning": {"epoch": 1, "batch-size": 64},
        "data": {"synthetic": True, "train-size": 1500, "test-size": 400},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "eager", "max-retries": 3},
        "log_path": str(tmp_path),
    }
    for k, v in kw.items():
        sect, key = k.split("__")
        d.setdefault(sect, {})[key.replace("_", "-")] = v
    return d


def _run(tmp_path, **kw):
    cfg = from_dict(_cfg(tmp_path, **kw))
    eng = FLEngine(cfg, device="cpu", verbose=False)
    hist = eng.run()
    eng.close()
    return eng, hist


@pytest.mark.parametrize("mode", ["fedavg", "trimmed_mean", "median", "krum", "shieldfl", "scionfl", "FLTrust",
                                  "fltracer", "byzantine", "hyper"])
def test_modes_complete(tmp_path, mode):
    eng, hist = _run(tmp_path, server__mode=mode)
    assert sum(r["ok"] for r in hist) == 2
    assert all(0.0 <= r["metric"] <= 1.0 for r in hist if r["ok"])
    log = open(os.path.join(tmp_path, "app.log")).read()
    assert "### Application start ###" in log and "Active with 4 client: [0, 1, 2, 3]" in log
    assert log.count("ROC_AUC: ") == 2


def test_checkpoint_format_and_resume(tmp_path):
    eng, _ = _run(tmp_path)
    sd = torch.load(os.path.join(tmp_path, "TransformerModel.pth"), weights_only=True)
    ref = build_model("TransformerModel").state_dict()
    assert list(sd) == list(ref) and all(sd[k].shape == ref[k].shape and sd[k].dtype == torch.float32 for k in sd)
    assert torch.allclose(ParamLayout.for_model("TransformerModel").flatten(sd), eng.global_params)
    # load: True re-reads the checkpoint every round and ships it to the clients
    eng2, hist2 = _run(tmp_path, server__parameters={"load": True})
    assert all(r["ok"] for r in hist2)


def test_hyper_checkpoint_keys(tmp_path):
    eng, _ = _run(tmp_path, server__mode="hyper")
    sd = torch.load(os.path.join(tmp_path, "TransformerModel_hyper_4.pth"), weights_only=True)
    ref = HyperNetwork(build_model("TransformerModel"), 4, 8, 100, False, 2).state_dict()
    assert list(sd) == list(ref)
    assert all(sd[k].shape == ref[k].shape for k in sd)


def test_attack_starts_after_genuine_pool(tmp_path):
    d = _cfg(tmp_path, server__num_round=3, server__clients=5)
    d["comm"] = {"attackers": {4: {"mode": "Min-Max", "round": 1}}}
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    hist = eng.run()
    assert "attack" not in hist[0]          # A-14: empty pool in round 1
    assert "attack" in hist[1] and hist[1]["attack"]["iters"] >= 1


def test_nan_client_triggers_retry(tmp_path):
    cfg = from_dict(_cfg(tmp_path, server__num_round=1))
    eng = FLEngine(cfg, device="cpu", verbose=False)
    eng.local_params[1, 3] = float("nan")    # poisoned client model -> NaN loss -> result False
    rec = eng.run_round()
    assert rec["ok"] is False and eng.rounds_left == 1
    eng.global_params = None
    eng.local_params[1].copy_(eng.local_params[0])
    rec = eng.run_round()
    assert rec["ok"] is True and eng.rounds_left == 0


def test_hyper_detection_runs(tmp_path):
    d = _cfg(tmp_path, server__mode="hyper", server__num_round=19, server__clients=4)
    d["server"]["hyper-detection"] = {"enable": True, "cosine-search": 10, "n_components": 2, "eps": 0.5,
                                      "min_samples": 2}
    d["server"]["data-distribution"] = {"num-data-range": [70, 80]}
    d["server"]["validation"] = False
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    hist = eng.run()
    assert sum(r["ok"] for r in hist) == 19
    assert os.path.exists(os.path.join(tmp_path, "all_embeddings.npy"))


def test_hyper_detection_rolls_back_before_validation(tmp_path):
    """On a removal round the reference removes the flagged clients, rolls the hypernetwork back and only then
    validates (server.py:532-543): the logged metric is test_hyper of the ROLLED-BACK hypernetwork over the
    clients that reported (len(all_model_parameters)), and the removed client is not selected afterwards."""
    d = _cfg(tmp_path, server__mode="hyper", server__num_round=3, server__clients=4)
    d["server"]["hyper-detection"] = {"enable": True, "cosine-search": 10, "n_components": 2, "eps": 0.5,
                                      "min_samples": 2}
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    eng.run_round()
    before = eng.hyper.snapshot()
    eng.detector.step = lambda rnd, sel, embs: [3]           # force a removal this round
    rec = eng.run_round()
    assert rec["removed"] == [3] and eng.selected == [0, 1, 2]
    assert torch.equal(eng.hyper.hnet.arena, before)          # rolled back
    ok, auc = eng.validation.test_hyper(eng.hyper, 4)
    assert rec["ok"] and ok and rec["metric"] == auc
    eng.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _write_cfg(tmp_path, d):
    p = os.path.join(tmp_path, "config.yaml")
    with open(p, "w") as fh:
        yaml.safe_dump(d, fh)
    return p


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["ATTACKFL_QUIET"] = "1"
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


@pytest.mark.parametrize("world", [2, 4])
def test_packed_gloo_matches_single_process(tmp_path, world):
    d = _cfg(tmp_path, server__num_round=2)
    d["comm"] = {"backend": "gloo", "attackers": {3: {"mode": "LIE", "round": 1, "args": [0.5]}}}
    d["server"]["genuine-rate"] = 1.0  # K = 3 genuine models (K = 1 would make LIE's unbiased std NaN)
    d["engine"]["checkpoint-dir"] = str(tmp_path / "mp")
    d["log_path"] = str(tmp_path / "mp")
    cfg_path = _write_cfg(tmp_path, d)
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "launch.py"), "--config", cfg_path,
           "--device", "cpu"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    mp = torch.load(os.path.join(tmp_path, "mp", "TransformerModel.pth"), weights_only=True)
    # same config in one process (4 clients on rank 0)
    d1 = dict(d)
    d1["engine"] = dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp")})
    d1["log_path"] = str(tmp_path / "sp")
    eng = FLEngine(from_dict(d1), device="cpu", verbose=False)
    eng.run()
    sp = torch.load(os.path.join(tmp_path, "sp", "TransformerModel.pth"), weights_only=True)
    # torchrun pins OMP_NUM_THREADS=1, so CPU GEMM reduction order differs slightly from this process
    for k in sp:
        assert torch.allclose(sp[k], mp[k], atol=1e-4), k


def _log_lines(path):
    """app.log messages without the timestamp (``asctime - my_logger - LEVEL - message``)."""
    return [ln.split(" - ", 1)[1] for ln in open(path).read().splitlines() if " - " in ln]


def test_classic_server_and_clients(tmp_path):
    """The reference-style launch (server.py + N x client.py): the N clients are the whole device group (client r
    = rank r - 1; on an 8-GPU node 8 clients are 8 RCCL ranks, tests/test_launcher.py), the server holds the store
    and echoes the leader's app.log; the leader (client 1) writes app.log and the .pth into the server's log_path /
    checkpoint directory.  The result equals the packed launch with one client per rank byte for byte: same
    checkpoint tensors, same app.log messages."""
    import datetime

    import torch.distributed as dist

    d = _cfg(tmp_path, server__num_round=2, server__clients=3)
    port = _free_port()
    d["comm"] = {"backend": "gloo", "address": "127.0.0.1", "port": port}
    d["engine"]["checkpoint-dir"] = "ckpt"   # relative: resolved against the SERVER's working directory
    d["log_path"] = "logs"
    cfg_path = _write_cfg(tmp_path, d)
    env = _env()
    env["OMP_NUM_THREADS"] = "1"
    srv_dir, cli_dir = tmp_path / "srv", tmp_path / "cli"
    srv_dir.mkdir()
    cli_dir.mkdir()
    srv = subprocess.Popen([sys.executable, os.path.join(ROOT, "server.py"), "--device", "cpu", "--config", cfg_path],
                           env=env, cwd=str(srv_dir), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    cls = []
    try:
        store = None
        for _ in range(600):
            try:
                store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=5),
                                      use_libuv=False)
                break
            except Exception:  # (the server is still starting)
                import time
                time.sleep(0.1)
        assert store is not None
        for i in range(3):
            extra = ["--attack", "True", "--attack_mode", "Random", "--attack_round", "2", "--attack_args", "0.01"] \
                if i == 2 else []
            cls.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "client.py"), "--device", "cpu",
                                         "--config", cfg_path] + extra, env=env, cwd=str(cli_dir),
                                        stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
            # registration order = client index: start the next client once this one has registered
            while int(store.add("attackfl/next_rank", 0)) < i + 1:
                assert cls[-1].poll() is None, cls[-1].communicate()[1][-3000:]
                import time
                time.sleep(0.05)
        out, err = srv.communicate(timeout=600)
        assert srv.returncode == 0, err[-3000:]
        for c in cls:
            o, e = c.communicate(timeout=120)
            assert c.returncode == 0, e[-3000:]
    finally:
        for p in [srv] + cls:
            if p.poll() is None:
                p.kill()
    log = srv_dir / "logs" / "app.log"
    assert (srv_dir / "ckpt" / "TransformerModel.pth").exists() and log.exists()
    assert not (cli_dir / "logs").exists() and not (cli_dir / "ckpt").exists()
    assert open(log).read().count("ROC_AUC") == 2
    assert "ROC_AUC" in out  # the server console echoes the leader's log
    # the packed launch, one client per rank (same attacker), in one torchrun world of 3
    dp = dict(d)
    dp["comm"] = {"backend": "gloo", "attackers": {2: {"mode": "Random", "round": 2, "args": [0.01]}}}
    dp["engine"] = dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "mp")})
    dp["log_path"] = str(tmp_path / "mp")
    p2 = os.path.join(tmp_path, "packed.yaml")
    with open(p2, "w") as fh:
        yaml.safe_dump(dp, fh)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "launch.py"),
           "--config", p2, "--device", "cpu"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert _log_lines(log) == _log_lines(tmp_path / "mp" / "app.log")
    a = torch.load(srv_dir / "ckpt" / "TransformerModel.pth", weights_only=True)
    b = torch.load(tmp_path / "mp" / "TransformerModel.pth", weights_only=True)
    assert list(a) == list(b) and all(torch.equal(a[k], b[k]) for k in a)


def test_fault_injection_retries_round(tmp_path):
    # (at training round 1 there is no global model yet, so a poisoned client would keep its NaN model
    # and fail every retry — the reference's persistent-client semantics; inject from round 2 on)
    d = _cfg(tmp_path, server__num_round=3)
    d["engine"]["fault-inject"] = [{"client": 2, "round": 2}]
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    hist = eng.run()
    assert [r["ok"] for r in hist] == [True, False, True, True]   # round 2 retried once
    assert hist[1]["round"] == hist[2]["round"] == 2


@pytest.mark.parametrize("mode", ["fedavg", "hyper"])
def test_save_state_resume_is_exact(tmp_path, mode):
    """4 rounds in one run == 2 rounds, then a fresh engine resuming from the state files for 2 more."""
    full = tmp_path / "full"
    d = _cfg(full, server__num_round=4, server__mode=mode)
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    eng.run()
    name = "TransformerModel_hyper_4.pth" if mode == "hyper" else "TransformerModel.pth"
    ref = torch.load(os.path.join(full, name), weights_only=True)

    part = tmp_path / "part"
    d = _cfg(part, server__num_round=4, server__mode=mode)
    d["engine"]["save-state"] = True
    eng = FLEngine(from_dict(d), device="cpu", verbose=False)
    eng.run(max_rounds=2)
    d2 = _cfg(part, server__num_round=4, server__mode=mode)
    d2["engine"].update({"save-state": True, "resume": True})
    eng2 = FLEngine(from_dict(d2), device="cpu", verbose=False)
    assert eng2.round_no == 3 and eng2.rounds_left == 2
    hist = eng2.run()
    assert [r["round"] for r in hist] == [3, 4]
    got = torch.load(os.path.join(part, name), weights_only=True)
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-6), k


def test_fedavg_allreduce_world2_matches_single_process(tmp_path):
    """fedavg without attackers: the packed world-2 run takes the all_reduce fast path."""
    d = _cfg(tmp_path, server__num_round=2)
    d["comm"] = {"backend": "gloo"}
    d["engine"]["checkpoint-dir"] = str(tmp_path / "mp")
    d["engine"]["metrics"] = str(tmp_path / "mp" / "m.jsonl")
    d["log_path"] = str(tmp_path / "mp")
    cfg_path = _write_cfg(tmp_path, d)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "launch.py"), "--config", cfg_path,
           "--device", "cpu"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"path": "fedavg-allreduce"' in open(tmp_path / "mp" / "m.jsonl").read()
    mp = torch.load(os.path.join(tmp_path, "mp", "TransformerModel.pth"), weights_only=True)
    d1 = dict(d)
    d1["engine"] = dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp"), "metrics": ""})
    d1["log_path"] = str(tmp_path / "sp")
    eng = FLEngine(from_dict(d1), device="cpu", verbose=False)
    eng.run()
    sp = torch.load(os.path.join(tmp_path, "sp", "TransformerModel.pth"), weights_only=True)
    for k in sp:
        assert torch.allclose(sp[k], mp[k], atol=1e-4), k


def test_plan_is_placement_independent():
    """A client's batches depend only on its own seed and size, not on the clients it is packed with."""
    from attackfl_amd.fl.trainers import make_plan
    a = make_plan(1000, [300, 120], 2, [11, 12], "cpu")
    b = make_plan(1000, [120], 2, [12], "cpu")
    c = make_plan(1000, [300, 500, 120], 2, [11, 99, 12], "cpu")
    assert torch.equal(a.client(1), b.client(0)) and torch.equal(a.client(1), c.client(2))
    assert torch.equal(a.client(0), c.client(0))


def test_plan_subset_and_epoch_permutations():
    """Each client visits nd distinct rows; every epoch is a permutation of the same subset."""
    from attackfl_amd.fl.trainers import make_plan
    nd = [700, 333, 1000]
    p = make_plan(1000, nd, 3, [5, 6, 7], "cpu")
    for c, n in enumerate(nd):
        sub = p.order[c, 0, :n]
        assert len(set(sub.tolist())) == n and int(sub.min()) >= 0 and int(sub.max()) < 1000
        for e in range(1, 3):
            ep = p.order[c, e, :n]
            assert torch.equal(ep.sort().values, sub.sort().values) and not torch.equal(ep, sub)


def test_hyper_generate_cache_invalidated_by_every_arena_change():
    """HyperServer.generate_many is memoised per hypernetwork state: train / restore / load_arena drop it."""
    import torch

    from attackfl_amd.fl.hyper_server import HyperServer
    from attackfl_amd.models import build_model

    sd = build_model("TransformerModel", seed=0).state_dict()
    hs = HyperServer(sd, 3, 0.01, 1e9, "cpu", seed=1)
    a = hs.generate_many([0, 2])
    assert hs.generate_many([0, 2]) is a                       # same clients, same state: cached
    assert hs.generate_many([2, 0]) is not a                   # other order: recomputed
    snap = hs.snapshot()
    hs.train([0], {0: a[0] + 0.1})
    b = hs.generate_many([0, 2])
    assert not torch.equal(a, b)                               # trained: new state
    hs.restore(snap)
    assert torch.equal(hs.generate_many([0, 2]), a)            # restored: recomputed from the old state
    hs.load_arena(snap + 0.0)
    assert hs.generate_many([0, 2]) is not a


def test_replicated_detection_and_validation_world2(tmp_path):
    """Validation and hyper-detection are replicated on every rank (no control broadcast): a 2-rank gloo run
    with detection active from round 18 matches the single-process run; only the leader writes the
    embeddings file, app.log and the JSONL (with every client's per-epoch losses)."""
    d = _cfg(tmp_path, server__mode="hyper", server__num_round=19, server__clients=4)
    d["server"]["hyper-detection"] = {"enable": True, "cosine-search": 10, "n_components": 2, "eps": 0.5,
                                      "min_samples": 2}
    d["server"]["data-distribution"] = {"num-data-range": [70, 80]}
    d["comm"] = {"backend": "gloo"}
    d["engine"]["checkpoint-dir"] = str(tmp_path / "mp")
    d["engine"]["metrics"] = str(tmp_path / "mp" / "m.jsonl")
    d["log_path"] = str(tmp_path / "mp")
    cfg_path = _write_cfg(tmp_path, d)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "launch.py"), "--config", cfg_path,
           "--device", "cpu"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    recs = [json.loads(l) for l in open(tmp_path / "mp" / "m.jsonl")]
    assert sum(x["ok"] for x in recs) == 19
    assert all(len(x["client_loss"]) == 4 and all(len(l) == 1 for l in x["client_loss"]) for x in recs)
    assert open(tmp_path / "mp" / "app.log").read().count("ROC_AUC") == 19
    assert os.path.exists(tmp_path / "mp" / "all_embeddings.npy")
    mp = torch.load(os.path.join(tmp_path, "mp", "TransformerModel_hyper_4.pth"), weights_only=True)
    d1 = dict(d)
    d1["engine"] = dict(d["engine"], **{"checkpoint-dir": str(tmp_path / "sp"), "metrics": ""})
    d1["log_path"] = str(tmp_path / "sp")
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # as under torchrun: the same CPU GEMM reduction order over 19 rounds
    try:
        eng = FLEngine(from_dict(d1), device="cpu", verbose=False)
        hist = eng.run()
        eng.close()
    finally:
        torch.set_num_threads(nt)
    assert [x["removed"] for x in hist] == [x["removed"] for x in recs]
    sp = torch.load(os.path.join(tmp_path, "sp", "TransformerModel_hyper_4.pth"), weights_only=True)
    for k in sp:
        assert torch.allclose(sp[k], mp[k], atol=1e-4), (k, (sp[k] - mp[k]).abs().max())


def test_decision_check_covers_ranks_without_selected_clients():
    """the gather path saw decision words only on selected, valid rows, so a rank with no such
    client could diverge unchecked; its first slot row's word is now checked too."""
    import numpy as np
    import pytest as _pytest
    from attackfl_amd.fl.engine import DECISION, FLEngine

    stub = type("S", (), {"round_no": 3})()
    mn = np.zeros((2, DECISION + 1))
    mn[:, 0] = 1.0
    mn[:, DECISION] = 77.0
    FLEngine._check_decisions(stub, mn, np.array([77.0, 77.0]))
    with _pytest.raises(RuntimeError, match="disagree"):
        FLEngine._check_decisions(stub, mn, np.array([77.0, 78.0]))
    mn[1, 0] = 0.0  # an invalid row's word is ignored, the per-rank words are not
    mn[1, DECISION] = 5.0
    FLEngine._check_decisions(stub, mn, np.array([77.0, 77.0]))
