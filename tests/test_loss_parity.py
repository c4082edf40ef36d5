"""BCE gradient parity with the reference's ``nn.BCELoss`` (``client.py:76``) where the sigmoid saturates.

An Opt-Fang round (``src/Utils.py:101-132``: every weight moved by ~0.6 towards -sign(mean)) leaves models
whose outputs round to exactly 0.0 / 1.0 in fp32.  ``nn.BCELoss`` back-propagates
``(p - y) / max(p (1 - p), 1e-12)`` there — finite — while autograd through clamped logs gives
``0 * inf = NaN``; the CPU oracles once did the latter and failed clients (NaN-abort, round retry) that the
reference and the GPU kernels (``tf2.hip`` / ``rnn2.hip`` / ``cnn2.hip`` / ``layers.hip`` use torch's form)
train normally."""
import torch

from attackfl_amd.data import DeviceTable, resolve_dataset
from attackfl_amd.fl.trainers import bce_loss, make_plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import transformer as T


def test_bce_matches_torch_bceloss_including_saturation():
    p = torch.tensor([1.0, 0.0, 0.3, 1.0 - 2 ** -24, 2 ** -30, 0.5], dtype=torch.float32, requires_grad=True)
    y = torch.tensor([0.0, 1.0, 1.0, 0.0, 1.0, 0.0])
    ref = torch.nn.BCELoss()(p, y)
    ref.backward()
    g_ref = p.grad.clone()
    p.grad = None
    got = bce_loss(p, y)
    got.backward()
    assert torch.equal(got, ref) and torch.equal(p.grad, g_ref) and torch.isfinite(p.grad).all()
    # through a saturated sigmoid the gradient w.r.t. the logit is exactly torch's (0 where p*(1-p) == 0)
    z = torch.tensor([40.0, -40.0, 0.3], requires_grad=True)
    bce_loss(torch.sigmoid(z), torch.tensor([0.0, 1.0, 1.0])).backward()
    z2 = z.detach().clone().requires_grad_(True)
    torch.nn.BCELoss()(torch.sigmoid(z2), torch.tensor([0.0, 1.0, 1.0])).backward()
    assert torch.equal(z.grad, z2.grad)


def test_bce_nan_input_gives_nan_loss():
    """NaN outputs still reach the NaN abort (client.py:100-102) instead of raising in a range check."""
    p = torch.tensor([0.5, float("nan")])
    assert torch.isnan(bce_loss(p, torch.tensor([1.0, 0.0])))


def saturated_start(seed: int = 3) -> torch.Tensor:
    """A fedavg aggregate after an Opt-Fang round: every weight moved by ~0.586 against its own sign
    (5 genuine rows + 3 rows of mean - 1.5625 sign(mean), the bisection's last-tried γ)."""
    lay = ParamLayout.for_model("TransformerModel")
    P = lay.flatten(build_model("TransformerModel", seed=seed).state_dict())
    return P - 0.586 * torch.sign(P)


def test_oracle_trains_through_saturated_sigmoid():
    ds = resolve_dataset("ICU", "train", {"synthetic": True, "train-size": 4000}, verbose=False)
    rows = DeviceTable(ds, "cpu").rows
    start = saturated_start()
    lay = ParamLayout.for_model("TransformerModel")
    with torch.no_grad():
        out = T.reference_forward(lay.unflatten(start, clone=True), rows[:2000, :7], rows[:2000, 7:23])
    assert int(((out == 1.0) | (out == 0.0)).sum()) > 0  # the case: outputs saturate exactly in fp32
    plan = make_plan(rows.shape[0], [1000], 2, [5], "cpu")
    p = start[None].clone()
    ok, losses = T.reference_train(p, rows, plan.order, plan.nd, 2, 128, 0.004, [11])
    assert ok.tolist() == [1] and torch.isfinite(p).all() and torch.isfinite(losses).all()
    assert float(losses[0, 1]) < float(losses[0, 0])  # and it learns
