"""CIFAR10 image validation (reference ``src/Validation.py:38-44,69-90,147-175``).

The reference downloads CIFAR10 through torchvision; there is no network here, so the loader is
checked on a hand-written file in the raw ``cifar-10-batches-bin`` record layout and the metrics on
synthetic images.  The reference ships no image model, so a tiny log-softmax CNN is registered for
the test; loss/accuracy are compared against a plain PyTorch fp32 computation of the same formulas.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from attackfl_amd import models
from attackfl_amd.data import DeviceTable, load_cifar10_bin, resolve_dataset, synthetic_cifar10
from attackfl_amd.eval import Validation


class TinyImageNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 4, 3, stride=2, padding=1)
        self.fc = nn.Linear(4 * 16 * 16, 10)

    def forward(self, x):
        return F.log_softmax(self.fc(F.relu(self.conv(x)).flatten(1)), dim=1)


class _Log:
    def __init__(self):
        self.lines = []

    def log_info(self, m):
        self.lines.append(m)


def _reference_metrics(model, ds):
    with torch.no_grad():
        out = model(ds.x)
    loss = F.nll_loss(out, ds.y, reduction="sum").item() / len(ds)
    correct = int((out.argmax(1) == ds.y).sum())
    return loss, correct


def test_cifar_bin_loader_matches_totensor_normalize(tmp_path):
    rs = np.random.RandomState(0)
    rec = rs.randint(0, 256, (5, 3073)).astype(np.uint8)
    rec[:, 0] = np.arange(5)
    rec.tofile(tmp_path / "test_batch.bin")
    ds = load_cifar10_bin(str(tmp_path), "test")
    assert ds.x.shape == (5, 3, 32, 32) and ds.y.tolist() == [0, 1, 2, 3, 4]
    want = (torch.from_numpy(rec[:, 1:].reshape(5, 3, 32, 32).astype(np.float32)) / 255.0 - 0.5) / 0.5
    torch.testing.assert_close(ds.x, want)
    # resolve_dataset finds it under <root>/data/cifar-10-batches-bin
    d = tmp_path / "data" / "cifar-10-batches-bin"
    d.mkdir(parents=True)
    rec.tofile(d / "test_batch.bin")
    ds2 = resolve_dataset("CIFAR10", "test", {"root": str(tmp_path)}, verbose=False)
    torch.testing.assert_close(ds2.x, want)
    # data.synthetic false forces the real records (no pickle path exists for CIFAR10)
    ds3 = resolve_dataset("CIFAR10", "test", {"root": str(tmp_path), "synthetic": False}, verbose=False)
    torch.testing.assert_close(ds3.x, want)


def test_cifar_synthetic_false_without_records_raises(tmp_path):
    import pytest

    with pytest.raises(FileNotFoundError, match="CIFAR10 binary batches"):
        resolve_dataset("CIFAR10", "test", {"root": str(tmp_path), "synthetic": False}, verbose=False)


def test_image_validation_and_hyper_pooling(monkeypatch):
    monkeypatch.setitem(models.MODEL_REGISTRY, "TinyImageNet", TinyImageNet)
    ds = synthetic_cifar10(96, seed=5, split_seed=1)
    assert DeviceTable(ds, "cpu").kind == "IMAGE"
    log = _Log()
    val = Validation("TinyImageNet", "CIFAR10", log, "cpu", dataset=ds, verbose=False)
    net = TinyImageNet()
    flat = val.layout.flatten(net.state_dict())
    ok, acc = val.test(flat)
    loss, correct = _reference_metrics(net, ds)
    assert ok and abs(acc - 100.0 * correct / len(ds)) < 1e-9
    assert f"Average loss: {loss:.4f}, Accuracy: {correct}/{len(ds)}" in log.lines[-1]

    nets = [TinyImageNet() for _ in range(3)]

    class FakeHnet:
        def generate(self, i):
            return val.layout.flatten(nets[i].state_dict())

    ok, acc = val.test_hyper(FakeHnet(), 3)
    stats = [_reference_metrics(m, ds) for m in nets]
    pooled_loss = sum(s[0] for s in stats)  # reference divides the pooled sum by ONE test-set length
    pooled_correct = sum(s[1] for s in stats)
    assert ok and abs(acc - 100.0 * pooled_correct / len(ds)) < 1e-9
    assert f"Average loss: {pooled_loss:.4f}" in log.lines[-1]


def test_image_validation_fails_on_nan(monkeypatch):
    monkeypatch.setitem(models.MODEL_REGISTRY, "TinyImageNet", TinyImageNet)
    ds = synthetic_cifar10(16, seed=2)
    val = Validation("TinyImageNet", "CIFAR10", _Log(), "cpu", dataset=ds, verbose=False)
    flat = val.layout.flatten(TinyImageNet().state_dict())
    flat[:] = float("nan")
    ok, _ = val.test(flat)
    assert not ok


def test_image_eager_training_steps(monkeypatch):
    """CIFAR10 is validation-only in the reference; the eager trainer still takes image batches (NLL on
    the model's log-probabilities) instead of failing inside the forward."""
    from attackfl_amd.fl.trainers import EagerTrainer, make_plan, make_trainer

    monkeypatch.setitem(models.MODEL_REGISTRY, "TinyImageNet", TinyImageNet)
    ds = synthetic_cifar10(64, seed=4)
    table = DeviceTable(ds, "cpu")
    tr = make_trainer("auto", "TinyImageNet", "CIFAR10", table, "cpu")
    assert isinstance(tr, EagerTrainer)
    net = TinyImageNet()
    params = tr.layout.flatten(net.state_dict())[None].clone()
    p0 = params.clone()
    plan = make_plan(64, [48], 2, torch.Generator().manual_seed(0), "cpu")
    oks, losses = tr.train(params, plan, 0.01, 16, [7])
    assert oks == [True] and torch.isfinite(losses).all()
    assert not torch.equal(params, p0)
    # the first epoch's mean loss is the NLL objective (epoch 2 starts from the trained weights)
    assert float(losses[0, 1]) < float(losses[0, 0]) + 1.0
