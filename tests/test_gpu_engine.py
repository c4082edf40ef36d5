"""End-to-end rounds on the GPU for every model family: the engine picks the native trainer
(fused kernel for TransformerModel, graph-replayed layer programs for CNN/RNN/HAR) and the native
eval forward; fedavg and hyper modes."""
import os

import pytest
import torch

from attackfl_amd.config import from_dict
from attackfl_amd.fl.engine import EARLY_AGGREGATORS, FLEngine, build_client_table
from launch import parse_attackers

pytestmark = pytest.mark.gpu


def _run(tmp_path, model, data, mode, clients=4, rounds=2):
    d = {
        "server": {"num-round": rounds, "clients": clients, "mode": mode, "model": model, "data-name": data,
                   "data-distribution": {"num-data-range": [300, 500] if data == "ICU" else [40, 60]}},
        "learning": {"epoch": 2, "batch-size": 128 if data == "ICU" else 16},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000, "har-train-size": 256,
                 "har-test-size": 64},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "auto"},
        "log_path": str(tmp_path),
    }
    eng = FLEngine(from_dict(d), device="cuda", verbose=False)
    hist = eng.run()
    kind = eng.trainer.kind
    eng.close()
    return hist, kind


@pytest.mark.parametrize("model,data,kind", [("CNNModel", "ICU", "graph"), ("RNNModel", "ICU", "fused"),
                                             ("TransformerModel", "ICU", "fused"),
                                             ("TransformerClassifier", "HAR", "graph")])
@pytest.mark.parametrize("mode", ["fedavg", "hyper"])
def test_engine_rounds_native(gpu, tmp_path, model, data, kind, mode):
    if data == "HAR" and mode == "hyper":
        pytest.skip("hyper validation is ICU-only in the reference (test_hyper)")
    hist, got_kind = _run(tmp_path, model, data, mode)
    assert got_kind == kind
    assert sum(r["ok"] for r in hist) == 2
    assert all(0.0 <= r["metric"] <= 1.0 for r in hist)
    assert os.path.exists(os.path.join(tmp_path, "app.log"))


def test_async_checkpoint_files(gpu, tmp_path):
    """Background-written checkpoints hold the final global / hypernetwork (reference file names)."""
    import torch

    from attackfl_amd.utils.ckpt import CheckpointWriter

    w = CheckpointWriter()
    src = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
    w.submit("x", src, lambda t: {"t": t.clone()}, str(tmp_path / "x.pth"))
    src.zero_()  # ordered after the copy on the stream: the file keeps the old values
    w.close()
    got = torch.load(tmp_path / "x.pth", weights_only=True)["t"]
    assert torch.equal(got, torch.arange(1 << 20, dtype=torch.float32))

    d = {"server": {"num-round": 2, "clients": 3, "mode": "hyper", "model": "RNNModel", "data-name": "ICU",
                    "data-distribution": {"num-data-range": [200, 300]}},
         "learning": {"epoch": 1, "batch-size": 128},
         "data": {"synthetic": True, "train-size": 2000, "test-size": 500},
         "engine": {"checkpoint-dir": str(tmp_path)}, "log_path": str(tmp_path)}
    eng = FLEngine(from_dict(d), device="cuda", verbose=False)
    eng.run()
    sd_live = eng.hyper.hnet.state_dict()
    eng.close()
    assert eng.ckpt_writer.template_writes >= 1   # the 2nd round's file went through the zip template
    sd = torch.load(tmp_path / "RNNModel_hyper_3.pth", weights_only=True)
    assert list(sd.keys()) == list(sd_live.keys())
    assert all(torch.equal(sd[k], sd_live[k]) for k in sd)
    import zipfile

    with zipfile.ZipFile(tmp_path / "RNNModel_hyper_3.pth") as z:
        assert z.testzip() is None


def test_checkpoint_every_submit_written_in_order(gpu, tmp_path):
    """Submits that outpace the disk wait for a staging slot instead of being dropped: every file is written,
    in order, through the zip template with the GPU CRC (valid zip), and the file ends with the newest state."""
    import zipfile

    import torch

    from attackfl_amd.utils.ckpt import CheckpointWriter

    w = CheckpointWriter()
    src = torch.empty(1 << 22, dtype=torch.float32, device="cuda")
    for v in range(6):
        src.fill_(float(v))
        w.submit("x", src, lambda t: {"t": t}, str(tmp_path / "x.pth"))
    w.flush()
    got = torch.load(tmp_path / "x.pth", weights_only=True)["t"]
    assert bool((got == 5.0).all())
    assert w.written == 6 and w.dropped == 0 and w.template_writes == 5
    with zipfile.ZipFile(tmp_path / "x.pth") as z:
        assert z.testzip() is None   # the patched CRC-32 (computed on the GPU) is right
    w.close()


def test_checkpoint_copy_fenced_against_in_place_update(gpu, tmp_path):
    """The device -> host copy runs on a side stream: after ``fence()`` an in-place update on the compute
    stream (the hypernetwork arena's next Adam step) cannot leak into the checkpoint being written."""
    import torch

    from attackfl_amd.utils.ckpt import CheckpointWriter

    w = CheckpointWriter()
    src = torch.full((1 << 24,), 1.0, dtype=torch.float32, device="cuda")  # 64 MB: a copy of ~1 ms
    w.submit("y", src, lambda t: {"t": t.clone()}, str(tmp_path / "y.pth"))
    w.fence()
    src.fill_(2.0)
    w.flush()
    got = torch.load(tmp_path / "y.pth", weights_only=True)["t"]
    assert bool((got == 1.0).all())
    assert bool((src == 2.0).all())
    w.close()


def test_deferred_checkpoint_copies_the_submitted_state(gpu, tmp_path):
    """``submit(defer=True)`` records the state and issues the copy at ``kick`` (after the next training
    launch in the engine): work enqueued between submit and kick that does not touch the source must not
    delay or change it; ``fence`` kicks a pending copy before an in-place update; a newer deferred submit
    supersedes an older one that was never copied."""
    import torch

    from attackfl_amd.utils.ckpt import CheckpointWriter

    w = CheckpointWriter()
    src = torch.full((1 << 22,), 1.0, dtype=torch.float32, device="cuda")
    path = str(tmp_path / "d.pth")
    w.submit("d", src, lambda t: {"t": t.clone()}, path, defer=True)
    other = torch.zeros_like(src)
    other.add_(3.0)            # unrelated work queued before the copy is issued
    w.kick()
    w.fence()
    src.fill_(2.0)             # the next in-place update, after the fence
    w.flush()
    assert bool((torch.load(path, weights_only=True)["t"] == 1.0).all())
    # superseded deferred submits: only the newest state is written; fence() issues it first
    src.fill_(4.0)
    w.submit("d", src, lambda t: {"t": t.clone()}, path, defer=True)
    dropped = w.dropped
    src2 = torch.full_like(src, 5.0)
    w.submit("d", src2, lambda t: {"t": t.clone()}, path, defer=True)
    assert w.dropped == dropped + 1
    w.fence()
    src2.fill_(6.0)
    w.flush()
    assert bool((torch.load(path, weights_only=True)["t"] == 5.0).all())
    w.close()


@pytest.mark.parametrize("model,attackers,mode", [("TransformerModel", False, "fedavg"),
                                                  ("TransformerModel", True, "fedavg"),
                                                  ("TransformerModel", True, "hyper"), ("RNNModel", True, "hyper"),
                                                  ("CNNModel", False, "fedavg"),
                                                  ("TransformerModel", True, "krum"),
                                                  ("TransformerModel", True, "scionfl"),
                                                  ("TransformerModel", True, "fltracer"),
                                                  ("TransformerModel", False, "shieldfl"),
                                                  ("TransformerModel", True, "trimmed_mean"),
                                                  ("TransformerModel", True, "FLTrust"),
                                                  ("TransformerModel", True, "gmm")])
def test_speculative_launch_matches_serial(gpu, tmp_path, model, attackers, mode):
    """The next round's training enqueued before this round's validation (engine.speculative) gives the
    same rounds bit for bit as the serial schedule — including a round whose validation fails (the retry
    consumes the speculative launch) and one whose training fails (no speculation after it)."""
    import torch

    def run(spec, sub):
        d = {
            "server": {"num-round": 4, "clients": 3, "mode": mode, "model": model, "data-name": "ICU",
                       "data-distribution": {"num-data-range": [300, 500]}},
            "learning": {"epoch": 2, "batch-size": 128},
            "data": {"synthetic": True, "train-size": 4000, "test-size": 1000},
            "engine": {"checkpoint-dir": str(tmp_path / sub), "trainer": "auto", "speculative": spec,
                       "fault-inject": [{"client": 1, "round": 4}], "seed": 3},
            "log_path": str(tmp_path / sub),
        }
        if attackers:  # client 2 runs Min-Max from its 2nd training round (pool drawn before the launch)
            d["server"]["random-seed"] = 11
        cfg = from_dict(d)
        atk = "2:Opt-Fang:2" if mode == "hyper" else "2:Min-Max:2"
        table = build_client_table(cfg, 1, parse_attackers(atk) if attackers else None)
        eng = FLEngine(cfg, device="cuda", table=table, verbose=False)
        assert eng._speculative == spec
        calls = {"n": 0}
        name = "test_hyper" if mode == "hyper" else "test"
        test = getattr(eng.validation, name)

        def flaky(*a):  # the second validation fails once: that round is retried
            calls["n"] += 1
            ok, m = test(*a)
            return (False, m) if calls["n"] == 2 else (ok, m)

        setattr(eng.validation, name, flaky)
        hist = eng.run()
        out = (eng.hyper.hnet.arena if mode == "hyper" else eng.global_params).detach().cpu().clone()
        # (the robust rules run in the early launch too: aggregate + next launch before the host wait)
        assert not spec or mode not in EARLY_AGGREGATORS + ("FLTrust", "gmm") or \
            any(r.get("path") == "early-launch" for r in hist)
        eng.close()
        return [(r["ok"], None if r["metric"] != r["metric"] else r["metric"]) for r in hist], out

    h0, p0 = run(False, "serial")
    h1, p1 = run(True, "spec")
    if not attackers:
        assert [ok for ok, _ in h0] == [True, False, True, False, True, True]
    assert sum(ok for ok, _ in h0) == 4
    # the on-chip trainers, the CNN step program (ordered split-K / conv-gradient / head sums) and the hyper
    # server kernels are bit-reproducible: the speculative schedule must give the serial rounds exactly
    assert h0 == h1
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("mode", ["trimmed_mean", "median", "krum", "shieldfl", "scionfl", "gmm", "FLTrust",
                                  "fltracer", "byzantine"])
@pytest.mark.parametrize("attack", ["Min-Max", "LIE"])
def test_robust_modes_end_to_end(gpu, tmp_path, monkeypatch, mode, attack):
    """Every robust server mode on the native path (fused TransformerModel trainer, device aggregators,
    device validation) with one attacker of 5 from round 2 (reference server.py:286-494).  The rules in
    EARLY_AGGREGATORS run inside the early launch from round 2 on (aggregate + next launch before the host wait):
    the rule itself is captured, on whichever path calls it."""
    d = {
        "server": {"num-round": 3, "clients": 5, "mode": mode, "model": "TransformerModel", "data-name": "ICU",
                   "genuine-rate": 1.0, "data-distribution": {"num-data-range": [300, 500]}},
        "learning": {"epoch": 2, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "auto", "metrics": str(tmp_path / "m.jsonl")},
        "log_path": str(tmp_path),
    }
    cfg = from_dict(d)
    spec = "4:Min-Max:2" if attack == "Min-Max" else "4:LIE:2:0.74"
    eng = FLEngine(cfg, device="cuda", table=build_client_table(cfg, 1, parse_attackers(spec)), verbose=False)
    assert eng.trainer.kind == "fused"
    # every round's device aggregate against the CPU composite of the same rule on the same gathered rows
    from attackfl_amd.agg import AGGREGATORS
    seen = []
    orig_fn = AGGREGATORS.get(mode)

    def capture(U, sizes, attackers=None, seed=0, **kw):
        rows = U.detach().cpu().clone()
        res = orig_fn(U, sizes, attackers=attackers, seed=seed, **kw)
        seen.append((rows, sizes.detach().cpu().clone(), None if attackers is None else attackers.clone(),
                     res.params.detach().cpu().clone(), seed))
        return res

    if orig_fn is not None:
        monkeypatch.setitem(AGGREGATORS, mode, capture)
    if mode == "gmm":  # (the early launch calls the filter without its host read)
        import attackfl_amd.fl.engine as engine_mod
        orig_early = engine_mod.gmm_early

        def capture_early(U, attackers, gmm_rank=None):
            rows = U.detach().cpu().clone()
            params, ok, info = orig_early(U, attackers, gmm_rank)
            seen.append((rows, torch.ones(U.shape[0]), attackers.detach().cpu().clone(), params.detach().cpu().clone(),
                         eng.seed * 13 + len(seen) + 1))
            return params, ok, info

        monkeypatch.setattr(engine_mod, "gmm_early", capture_early)
    fl_seen = []
    if mode == "FLTrust":  # the rows, g_0 and the server model around every device FLTrust aggregate
        orig_fl = eng._fltrust

        def cap_fl(U):
            g0 = (eng.global_params if eng.global_params is not None else eng.fltrust_model).detach().cpu().clone()
            out = orig_fl(U)
            fl_seen.append((U.detach().cpu().clone(), g0, eng.fltrust_model.detach().cpu().clone(),
                            out.detach().cpu().clone()))
            return out

        eng._fltrust = cap_fl
    hist = eng.run()
    eng.close()
    assert [r["ok"] for r in hist] == [True, True, True]
    assert len(seen) == (0 if mode == "FLTrust" else 3)
    if mode in EARLY_AGGREGATORS + ("FLTrust", "gmm"):
        assert any(r.get("path") == "early-launch" for r in hist)  # (the last round never launches early)
    if mode == "FLTrust":
        # the trust / rescale math of server.py:714-740 in fp64 on the captured rows and server delta
        assert len(fl_seen) == 3
        for U, g0, server_new, out in fl_seen:
            d = (U - g0[None, :]).double()
            gd = (server_new - g0).double()
            dn = d.norm(dim=1)
            cos = (d @ gd) / torch.clamp(dn * gd.norm(), min=1e-8)
            trust = cos.clamp_min(0.0)
            w = (gd.norm() / (dn + 1e-6)) * trust / (trust.sum() + 1e-6)
            ref = g0.double() + (w[:, None] * d).sum(0)
            assert (out.double() - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())
            assert bool((trust > 0).any())  # (some clients trusted: the check is not vacuous)
    if mode != "FLTrust":  # (FLTrust trains a server model: its composite would need the CPU trainer)
        for k, (rows, sizes, att, got, seed) in enumerate(seen):
            assert seed == eng.seed * 13 + k + 1
            ref = orig_fn(rows, sizes, attackers=att, seed=seed, gmm_rank=1).params
            tol = 1e-6 if mode in ("median", "trimmed_mean", "krum") else 2e-5
            assert (got - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item()), (mode, k)
    assert all(0.0 <= r["metric"] <= 1.0 for r in hist)
    assert "attack" in hist[1] and "attack" in hist[2]
    if mode == "FLTrust":
        assert len(hist[-1]["trust"]) == 5 and all(t >= 0.0 for t in hist[-1]["trust"])
    assert os.path.exists(os.path.join(tmp_path, "TransformerModel.pth"))


@pytest.mark.parametrize("shape", [(6, 5000), (8, 47693), (37, 100), (3, 7), (5, 257)])
def test_stoch_quant_matches_cpu_mirror(gpu, shape):
    """k_stoch_quant's Bernoulli draws are the counter-based afl_uniform the CPU composite mirrors bit for bit;
    the chunked row min / max (32 partials per row, reduced by the quantisation blocks) at row lengths above and
    below one block, and at a block straddling rows."""
    from attackfl_amd import ops
    from attackfl_amd.ops import composite as C

    U = torch.randn(*shape, generator=torch.Generator().manual_seed(0))
    s_d, lo_d, hi_d = ops.stochastic_quantize(U.to(gpu), 1234)
    s_c, lo_c, hi_c = C.stochastic_quantize(U, 1234)
    assert torch.equal(lo_d.cpu(), lo_c) and torch.equal(hi_d.cpu(), hi_c)
    assert (s_d.cpu() != s_c).sum().item() == 0


def test_hyper_detection_end_to_end(gpu, tmp_path):
    """hyper-detection on the device path (reference server.py:496-536): 19 rounds (detection from round 18),
    embeddings history saved, decisions made on every round."""
    d = {
        "server": {"num-round": 19, "clients": 4, "mode": "hyper", "model": "TransformerModel", "data-name": "ICU",
                   "hyper-detection": {"enable": True, "cosine-search": 10, "n_components": 2, "eps": 0.5,
                                       "min_samples": 2},
                   "data-distribution": {"num-data-range": [200, 300]}},
        "learning": {"epoch": 1, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 3000, "test-size": 500},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "auto"},
        "log_path": str(tmp_path),
    }
    cfg = from_dict(d)
    eng = FLEngine(cfg, device="cuda", table=build_client_table(cfg, 1, parse_attackers("3:Opt-Fang:2")), verbose=False)
    assert not eng._speculative  # detection may roll the hypernetwork back: no speculative launch
    hist = eng.run()
    eng.close()
    assert sum(r["ok"] for r in hist) == 19
    assert os.path.exists(os.path.join(tmp_path, "all_embeddings.npy"))
    assert all(isinstance(r["removed"], list) for r in hist)


def test_hyper_detection_rollback_before_validation_on_device(gpu, tmp_path):
    """GPU twin of test_engine.py's rollback test: a forced removal rolls the hypernetwork back BEFORE
    validation (reference server.py:532-543), so the logged metric equals test_hyper of the rolled-back arena
    bit for bit, and the removed client is not selected afterwards."""
    import torch

    d = {
        "server": {"num-round": 3, "clients": 4, "mode": "hyper", "model": "TransformerModel", "data-name": "ICU",
                   "hyper-detection": {"enable": True, "cosine-search": 10, "n_components": 2, "eps": 0.5,
                                       "min_samples": 2},
                   "data-distribution": {"num-data-range": [200, 300]}},
        "learning": {"epoch": 1, "batch-size": 128},
        "data": {"synthetic": True, "train-size": 3000, "test-size": 500},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "auto"},
        "log_path": str(tmp_path),
    }
    eng = FLEngine(from_dict(d), device="cuda", verbose=False)
    eng.run_round()
    before = eng.hyper.snapshot().clone()
    eng.detector.step = lambda rnd, sel, embs: [3]  # force a removal this round
    rec = eng.run_round()
    assert rec["removed"] == [3] and eng.selected == [0, 1, 2]
    assert torch.equal(eng.hyper.hnet.arena, before)
    ok, auc = eng.validation.test_hyper(eng.hyper, 4)
    assert rec["ok"] and ok and rec["metric"] == auc
    eng.close()
