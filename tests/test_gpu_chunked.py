"""More clients than one persistent launch holds (ops.transformer.chunked / ProgramRunner._train_cnn2): the
on-chip trainers run back-to-back launches of clients that fit, and a client's result is bit-identical to
the one-launch run (placement independence) — reference server.py:58 takes any client count."""
import pytest
import torch

from attackfl_amd.data import DeviceTable, synthetic_icu
from attackfl_amd.fl.trainers import make_plan
from attackfl_amd.models import ParamLayout, build_model

pytestmark = pytest.mark.gpu


def _setup(model, C, nd, gpu):
    ds = synthetic_icu(4000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(gpu)
    lay = ParamLayout.for_model(model)
    params = torch.stack([lay.flatten(build_model(model, seed=i).state_dict()) for i in range(C)]).to(gpu)
    plan = make_plan(rows.shape[0], nd, 2, torch.Generator().manual_seed(9), gpu)
    return rows, params, plan


@pytest.mark.parametrize("model", ["TransformerModel", "RNNModel"])
def test_onchip_chunks_match_one_launch(gpu, model, monkeypatch):
    from attackfl_amd.ops import rnn as R
    from attackfl_amd.ops import transformer as T

    M = T if model == "TransformerModel" else R
    nd = [600, 513, 300, 700]
    rows, params, plan = _setup(model, 4, nd, gpu)
    seeds = [31, 32, 33, 34]
    one = params.clone()
    ok1, l1 = M.train_clients(one, rows, plan.order, plan.nd, 2, 128, 0.004, seeds)
    monkeypatch.setenv("AFL_MAX_CLIENTS_PER_LAUNCH", "2")  # -> 2 launches of 2 clients
    two = params.clone()
    ok2, l2 = M.train_clients(two, rows, plan.order, plan.nd, 2, 128, 0.004, seeds)
    assert ok1.tolist() == ok2.tolist() == [1, 1, 1, 1]
    assert torch.equal(one, two)
    assert torch.equal(l1, l2)


def test_cnn2_chunks_match_one_launch(gpu, monkeypatch):
    from attackfl_amd.fl.trainers import GraphTrainer

    nd = [400, 300, 513]
    _, params, plan = _setup("CNNModel", 3, nd, gpu)
    tab = DeviceTable(synthetic_icu(4000, seed=3), gpu)
    outs = []
    for lim in ("0", "1"):  # one launch of 3 clients, then 3 launches of 1
        monkeypatch.setenv("AFL_MAX_CLIENTS_PER_LAUNCH", lim)
        tr = GraphTrainer("CNNModel", "ICU", tab, gpu)
        p = params.clone()
        ok, losses = tr.train(p, plan, 0.004, 128, [41, 42, 43])
        assert ok == [True, True, True]
        outs.append((p, losses))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
