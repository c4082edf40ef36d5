"""Reference-quirk switches (docs/PARITY.md): ``engine.compat-har-train`` (the reference ``train_HAR`` loop,
``client.py:114-131``: size-1 batches train, a NaN loss does not abort) and ``engine.compat-fedavg-alias``
(A-13: FedAvg averages into the first stored update, which is also the first genuine model attackers can
receive, ``server.py:263-268,763``)."""
import pytest
import torch

from attackfl_amd.config import from_dict
from attackfl_amd.data import DeviceTable, synthetic_har
from attackfl_amd.fl.engine import FLEngine, build_client_table
from attackfl_amd.fl.programs import ProgramRunner, make_program
from attackfl_amd.fl.trainers import EagerTrainer, make_plan
from attackfl_amd.models import ParamLayout, build_model
from launch import parse_attackers


def _har(nd=17, seed=0):
    ds = synthetic_har(64, seed=3)
    table = DeviceTable(ds, "cpu")
    lay = ParamLayout.for_model("TransformerClassifier")
    p = lay.flatten(build_model("TransformerClassifier", seed=seed).state_dict())[None].clone()
    plan = make_plan(table.n, [nd], 1, [7], "cpu")
    return table, p, plan


@pytest.mark.parametrize("kind", ["eager", "program"])
def test_compat_har_trains_size_one_batch(kind):
    """17 rows at batch 16: the default skips the last (size-1) batch, compat trains it."""
    outs = {}
    for compat in (False, True):
        table, p, plan = _har()
        if kind == "eager":
            tr = EagerTrainer("TransformerClassifier", "HAR", table, "cpu")
            tr.compat_har = compat
            oks, _ = tr.train(p, plan, 0.004, 16, [5])
        else:
            r = ProgramRunner(make_program("TransformerClassifier", 1, 16, "cpu", train=True, dropout=False))
            ok, _ = r.train(table, p, plan, 0.004, [5], compat_har=compat)
            oks = ok.tolist()
        assert oks == [True]
        outs[compat] = p.clone()
    # the runs agree up to the 16-row step and then differ by the extra size-1 step
    assert not torch.equal(outs[False], outs[True])


@pytest.mark.parametrize("kind", ["eager", "program"])
def test_compat_har_does_not_abort_on_nan(kind):
    res = {}
    for compat in (False, True):
        table, p, plan = _har(nd=32)
        p[0, 10] = float("nan")
        if kind == "eager":
            tr = EagerTrainer("TransformerClassifier", "HAR", table, "cpu")
            tr.compat_har = compat
            oks, _ = tr.train(p, plan, 0.004, 16, [5])
        else:
            r = ProgramRunner(make_program("TransformerClassifier", 1, 16, "cpu", train=True, dropout=False))
            ok, _ = r.train(table, p, plan, 0.004, [5], compat_har=compat)
            oks = ok.tolist()
        res[compat] = oks[0]
    assert res == {False: False, True: True}


def test_compat_fedavg_alias_puts_aggregate_in_pool(tmp_path):
    def run(compat):
        d = {"server": {"num-round": 2, "clients": 4, "mode": "fedavg", "model": "TransformerModel",
                        "genuine-rate": 1.0, "data-distribution": {"num-data-range": [100, 150]}},
             "learning": {"epoch": 1, "batch-size": 64},
             "data": {"synthetic": True, "train-size": 1000, "test-size": 200},
             "engine": {"checkpoint-dir": str(tmp_path / str(compat)), "trainer": "eager",
                        "compat-fedavg-alias": compat},
             "log_path": str(tmp_path / str(compat))}
        cfg = from_dict(d)
        eng = FLEngine(cfg, device="cpu", verbose=False, table=build_client_table(cfg, 1, parse_attackers("3:LIE:5")))
        eng.run_round()
        return eng

    plain, alias = run(False), run(True)
    assert torch.equal(alias.genuine_pool[0], alias.global_params)
    assert not torch.equal(plain.genuine_pool[0], plain.global_params)
    assert torch.equal(alias.genuine_pool[1:], plain.genuine_pool[1:])
