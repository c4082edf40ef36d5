"""Layer programs (CNN / RNN / HAR classifier) on CPU: the composite ops against the reference
``nn.Module`` math — eval forward, and the hand-written backward against autograd (one SGD step with
dropout off), plus the Adam / size-1-skip / NaN semantics of the step runner."""
import pytest
import torch
import torch.nn.functional as F

from attackfl_amd.data import DeviceTable, synthetic_har, synthetic_icu
from attackfl_amd.fl.programs import ProgramRunner, make_program, step_tables
from attackfl_amd.fl.trainers import Plan, bce_loss
from attackfl_amd.models import ParamLayout, build_model

ICU_MODELS = ["CNNModel", "RNNModel"]


def _params(name, C, seed=0):
    lay = ParamLayout.for_model(name)
    base = lay.flatten(build_model(name, seed=seed).state_dict())
    g = torch.Generator().manual_seed(seed + 1)
    out = base[None].repeat(C, 1)
    out[1:] += 0.01 * torch.randn(C - 1, lay.P, generator=g)
    return out, lay


def _module(name, flat, lay):
    m = build_model(name, seed=0)
    m.load_state_dict(lay.unflatten(flat))
    return m.eval()


def _table(name, n):
    return DeviceTable(synthetic_har(n) if name == "TransformerClassifier" else synthetic_icu(n), "cpu")


@pytest.mark.parametrize("name", ICU_MODELS + ["TransformerClassifier"])
def test_eval_forward_matches_module(name):
    C = 2
    params, lay = _params(name, C)
    n = 5 if name == "TransformerClassifier" else 37
    tab = _table(name, n)
    prog = make_program(name, C, 16 if name != "TransformerClassifier" else 3, "cpu", train=False)
    data = tab.x if name == "TransformerClassifier" else tab.rows
    out = ProgramRunner(prog).predict(params, data)
    for c in range(C):
        m = _module(name, params[c], lay)
        with torch.no_grad():
            if name == "TransformerClassifier":
                ref = m(tab.x[:, None, :])
            else:
                ref = m(tab.rows[:, :7], tab.rows[:, 7:23])[:, 0]
        assert torch.allclose(out[c], ref, atol=2e-5, rtol=1e-4), (name, c, (out[c] - ref).abs().max())


def _ref_grads(name, flat, lay, tab, idx):
    m = _module(name, flat, lay)  # eval mode: dropout off, same as the program's dropout=False
    for p_ in m.parameters():
        p_.grad = None
    if name == "TransformerClassifier":
        x, y = tab.har_batch(idx)
        loss = F.cross_entropy(m(x), y)
    else:
        v, l, y = tab.icu_batch(idx)
        loss = bce_loss(m(v, l), y[:, None])
    loss.backward()
    g = torch.zeros(lay.P)
    named = dict(m.named_parameters())
    for s in lay.slots:
        if s.name in named and named[s.name].grad is not None:
            g[s.offset:s.offset + s.numel] = named[s.name].grad.reshape(-1)
    return g, float(loss)


@pytest.mark.parametrize("name", ICU_MODELS + ["TransformerClassifier"])
def test_backward_matches_autograd(name):
    C = 2
    B = 3 if name == "TransformerClassifier" else 24
    params, lay = _params(name, C)
    tab = _table(name, 40)
    g = torch.Generator().manual_seed(3)
    order = torch.stack([torch.randperm(40, generator=g)[:B] for _ in range(C)])[:, None, :].to(torch.int32)
    plan = Plan(order, torch.tensor([B] * C, dtype=torch.int32), 1)
    prog = make_program(name, C, B, "cpu", train=True, dropout=False)
    before = params.clone()
    sgd = 1e-3
    ok, losses = ProgramRunner(prog).train(tab, params, plan, lr=0.0, seeds=[11, 12], sgd_lr=sgd)
    assert ok.all()
    for c in range(C):
        ref, ref_loss = _ref_grads(name, before[c], lay, tab, order[c, 0].long())
        got = (before[c] - params[c]) / sgd
        assert abs(float(losses[c, 0]) - ref_loss) < 1e-5
        tol = 2e-3 * float(ref.abs().max()) + 1e-6
        assert (got - ref).abs().max() < tol, (name, c, float((got - ref).abs().max()), tol)


def test_step_tables_skip_and_padding():
    order = torch.arange(2 * 1 * 9, dtype=torch.int32).reshape(2, 1, 9)
    idx, bsz, ep, nb, S = step_tables(order, [9, 5], 1, 4, "cpu")
    assert S == 3 and nb.tolist() == [3, 2]
    assert bsz[:, 0].tolist() == [4, 4, 1] and bsz[:, 1].tolist() == [4, 1, 0]   # size-1 batch -> skipped
    assert idx[2, 0, 0] == 8 and (idx[2, 0, 1:] == -1).all()


def _step_tables_loop(order, nd, epochs, B):
    """The per-batch loop form of step_tables (the oracle of the vectorised one)."""
    C = order.shape[0]
    nbat = [max(1, -(-int(n) // B)) for n in nd]
    S = max([epochs * n for n in nbat] + [0])
    idx = torch.full((S, C, B), -1, dtype=torch.int32)
    bsz = torch.zeros(S, C, dtype=torch.int32)
    ep = torch.zeros(S, C, dtype=torch.int32)
    for c in range(C):
        s = 0
        for e in range(epochs):
            for j in range(nbat[c]):
                a, b = j * B, min(int(nd[c]), (j + 1) * B)
                idx[s, c, :b - a] = order[c, e, a:b]
                bsz[s, c] = b - a
                ep[s, c] = e
                s += 1
    return idx, bsz, ep, S


@pytest.mark.parametrize("nd,epochs,B", [([33, 17, 1, 128], 3, 16), ([129, 128, 2], 2, 128), ([5], 1, 8), ([0, 7], 2, 4)])
def test_step_tables_match_loop_form(nd, epochs, B):
    g = torch.Generator().manual_seed(9)
    maxnd = max(max(nd), 1)
    order = torch.stack([torch.stack([torch.randperm(300, generator=g)[:maxnd] for _ in range(epochs)])
                         for _ in nd]).to(torch.int32)
    idx, bsz, ep, nb, S = step_tables(order, nd, epochs, B, "cpu")
    ri, rb, re, rS = _step_tables_loop(order, nd, epochs, B)
    assert S == rS and torch.equal(idx, ri) and torch.equal(bsz, rb) and torch.equal(ep, re)


def test_adam_dropout_training_runs_and_nan_fails():
    name = "CNNModel"
    C, B = 2, 16
    params, lay = _params(name, C)
    tab = _table(name, 64)
    g = torch.Generator().manual_seed(5)
    order = torch.stack([torch.stack([torch.randperm(64, generator=g)[:33] for _ in range(2)]) for _ in range(C)])
    plan = Plan(order.to(torch.int32), torch.tensor([33, 33], dtype=torch.int32), 2)
    params[1, 5] = float("nan")
    before = params.clone()
    ok, losses = ProgramRunner(make_program(name, C, B, "cpu")).train(tab, params, plan, lr=1e-3, seeds=[1, 2])
    assert ok.tolist() == [True, False]
    assert torch.isfinite(losses[0]).all() and (losses[0] > 0).all()
    assert not torch.equal(params[0], before[0])
    # the failed client stops before its first update
    assert torch.equal(torch.nan_to_num(params[1]), torch.nan_to_num(before[1]))


def test_attention_rc_mask_statistics():
    """The row / column-pair attention dropout hash (masks.keep_rc, har.hip attn_mix): keep rate 1 - p, no
    row or column structure (every row's and column's keep rate near 1 - p), independent of the pair hash."""
    import numpy as np

    from attackfl_amd.ops import masks

    rows, cols = np.arange(512)[:, None], np.arange(576)[None, :]
    k = masks.keep_rc(masks.step_key(7, 3), 10, rows, cols, 0.1).numpy()
    assert abs(k.mean() - 0.9) < 0.003
    assert np.abs(k.mean(axis=1) - 0.9).max() < 0.06 and np.abs(k.mean(axis=0) - 0.9).max() < 0.06
    kp = masks.keep(masks.step_key(7, 3), 10, rows, cols, 0.1).numpy()
    agree = (k == kp).mean()
    assert abs(agree - (0.9 * 0.9 + 0.1 * 0.1)) < 0.01  # independent draws


def test_attention_rc_keep_rate_within_3_sigma():
    """Keep rate of the attention dropout draw over >= 1e6 draws (two 16-bit decisions per 32-bit mix, threshold
    round(p * 2^16)) is within 3 sigma of 1 - p, for the whole draw and for each 16-bit half (even / odd columns)."""
    import numpy as np

    from attackfl_amd.ops import masks

    p = 0.1
    rows, cols = np.arange(1024)[:, None], np.arange(1040)[None, :]
    k = np.concatenate([masks.keep_rc(masks.step_key(11, s), 10 + s, rows, cols, p).numpy().ravel()
                        for s in range(2)]).astype(np.float64)
    n = k.size
    assert n >= 2_000_000
    q = 1 - round(p * 65536) / 65536  # the exact keep probability of a 16-bit threshold
    assert abs(q - (1 - p)) < 2 ** -16
    sig = np.sqrt(q * (1 - q) / n)
    assert abs(k.mean() - q) < 3 * sig, (k.mean(), q, sig)
    halves = k.reshape(-1, 2)  # (even, odd) column pairs = low / high halves of one mix
    for h in range(2):
        assert abs(halves[:, h].mean() - q) < 3 * np.sqrt(2) * sig
    # the two halves of one mix are independent decisions
    both = (halves[:, 0] * halves[:, 1]).mean()
    assert abs(both - q * q) < 3 * np.sqrt(q * q * (1 - q * q) / (n / 2))
    # no xor structure from hr ^ hc: the four corners of random (row pair, column pair) rectangles, whose mix
    # inputs xor to zero, are independent draws (all kept: q^4; odd count kept: the binomial parity)
    km = k[: 1024 * 1040].reshape(1024, 1040)
    rs = np.random.RandomState(5)
    i1, i2, j1, j2 = rs.randint(0, 1024, 400000), rs.randint(0, 1024, 400000), rs.randint(0, 1040, 400000), \
        rs.randint(0, 1040, 400000)
    ok = (i1 != i2) & (j1 != j2)
    corners = np.stack([km[i1, j1], km[i1, j2], km[i2, j1], km[i2, j2]])[:, ok]
    m = corners.shape[1]
    all4, par = corners.prod(axis=0).mean(), (corners.sum(axis=0) % 2).mean()
    par_q = 4 * q * (1 - q) ** 3 + 4 * q ** 3 * (1 - q)
    assert abs(all4 - q ** 4) < 4 * np.sqrt(q ** 4 * (1 - q ** 4) / m), all4
    assert abs(par - par_q) < 4 * np.sqrt(par_q * (1 - par_q) / m), par


def test_client_chunks_balanced():
    from attackfl_amd.ops.transformer import client_chunks

    assert client_chunks(8, 85) == [(0, 8)]
    assert client_chunks(128, 85) == [(0, 64), (64, 128)]
    assert client_chunks(16, 8) == [(0, 8), (8, 16)]
    assert client_chunks(17, 8) == [(0, 6), (6, 12), (12, 17)]
    assert client_chunks(0, 8) == []
    for C in range(1, 60):
        for cap in (1, 2, 3, 7, 8):
            parts = client_chunks(C, cap)
            assert parts[0][0] == 0 and parts[-1][1] == C and all(b - a <= cap for a, b in parts)
            assert all(parts[i][1] == parts[i + 1][0] for i in range(len(parts) - 1))
            assert len(parts) == -(-C // cap)


def test_upload_and_prefetch_cpu_paths():
    """ops.layers.upload is a plain copy off the GPU; Validation.prefetch is a no-op there (test() recomputes)."""
    from attackfl_amd.eval import Validation
    from attackfl_amd.ops.layers import upload

    t = torch.arange(5, dtype=torch.int32)
    u = upload(t, "cpu")
    assert torch.equal(u, t)

    class _Log:
        def log_info(self, *a, **k):
            pass

    ds = synthetic_icu(300, seed=2)
    val = Validation("CNNModel", "ICU", _Log(), "cpu", dataset=ds, verbose=False)
    flat = ParamLayout.for_model("CNNModel").flatten(build_model("CNNModel", seed=1).state_dict())
    assert val.prefetch(flat) is False
    ok, auc = val.test(flat)
    assert ok and 0.0 <= auc <= 1.0
