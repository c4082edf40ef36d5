"""Model state_dict layouts (``.pth`` compatibility) and the config schema."""
import os

import pytest
import torch

from attackfl_amd.config import REFERENCE_DEFAULTS, from_dict, load_config
from attackfl_amd.models import (CNNHyper, HyperNetwork, PackedHyperNet, ParamLayout, build_model, model_layout)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EXPECTED = {
    "CNNModel": (20, 203649),
    "RNNModel": (58, 97665),
    "TransformerModel": (38, 47693),
    "TransformerClassifier": (31, 143174),
}


@pytest.mark.parametrize("name", list(EXPECTED))
def test_layout_counts(name):
    lay = model_layout(name)
    assert (len(lay), lay.P) == EXPECTED[name]


def test_transformer_keys():
    sd = build_model("TransformerModel").state_dict()
    assert tuple(sd["vitals_dense.weight"].shape) == (64, 7)
    assert tuple(sd["labs_dense.weight"].shape) == (64, 16)
    assert tuple(sd["vitals_transformer.attention.in_proj_weight"].shape) == (192, 64)
    assert tuple(sd["labs_transformer.ffn.0.weight"].shape) == (6, 64)
    assert tuple(sd["labs_transformer.ffn.3.weight"].shape) == (64, 6)
    assert tuple(sd["fc1.weight"].shape) == (64, 128)
    assert tuple(sd["output.weight"].shape) == (1, 32)
    assert list(sd)[0] == "vitals_dense.weight" and list(sd)[-1] == "output.bias"


def test_rnn_and_cnn_keys():
    sd = build_model("RNNModel").state_dict()
    assert tuple(sd["vitals_gru1.weight_ih_l0"].shape) == (96, 7)
    assert tuple(sd["labs_gru1.weight_ih_l0_reverse"].shape) == (96, 16)
    assert tuple(sd["labs_gru3.weight_hh_l0"].shape) == (96, 32)
    sd = build_model("CNNModel").state_dict()
    assert tuple(sd["vitals_conv3.weight"].shape) == (128, 64, 3)
    assert tuple(sd["fc1.weight"].shape) == (128, 1024)
    sd = build_model("TransformerClassifier").state_dict()
    assert tuple(sd["pe.pe"].shape) == (1, 600, 64)
    assert tuple(sd["transformer.layers.1.linear1.weight"].shape) == (256, 64)


@pytest.mark.parametrize("name", ["CNNModel", "RNNModel", "TransformerModel"])
def test_icu_forward(name):
    m = build_model(name, seed=0).eval()
    out = m(torch.randn(5, 7), torch.randn(5, 16))
    assert out.shape == (5, 1) and ((out >= 0) & (out <= 1)).all()


def test_har_forward():
    m = build_model("TransformerClassifier", seed=0).eval()
    assert m(torch.randn(2, 1, 561)).shape == (2, 6)


def test_flatten_roundtrip():
    m = build_model("RNNModel", seed=1)
    lay = ParamLayout.from_state_dict(m.state_dict())
    flat = lay.flatten(m.state_dict())
    sd = lay.unflatten(flat)
    for k, v in m.state_dict().items():
        assert torch.equal(sd[k], v)


def test_hypernetwork_packed_equivalence():
    torch.manual_seed(0)
    target = build_model("TransformerModel", seed=0)
    hnet = HyperNetwork(target, 8, 8, 100, False, 2)
    sd = hnet.state_dict()
    assert len(sd) == 121
    assert sum(p.numel() for p in hnet.parameters()) == 4885850
    packed = PackedHyperNet(target.state_dict(), 8)
    packed.load_state_dict(sd)
    psd = packed.state_dict()
    assert list(psd.keys()) == list(sd.keys())
    for k in sd:
        assert torch.equal(psd[k], sd[k]), k
    lay = ParamLayout.from_state_dict(target.state_dict())
    with torch.no_grad():
        for i in (0, 5):
            w, emb = hnet(torch.tensor([i]))
            ref = lay.flatten(w)
            assert torch.allclose(packed.generate(i), ref, atol=1e-5)
            assert torch.allclose(packed.emb[i], emb[0])


def test_cnn_hyper_shapes():
    h = CNNHyper(4, 10, 100, 3)
    w, _ = h(torch.tensor([1]))
    assert tuple(w["fc1.weight"].shape) == (128, 1024) and tuple(w["vitals_conv2.weight"].shape) == (64, 32, 3)


def test_repo_config_matches_reference_defaults():
    cfg = load_config(os.path.join(ROOT, "config.yaml"))
    for sect in ("server", "learning"):
        for k, v in REFERENCE_DEFAULTS[sect].items():
            assert cfg.raw[sect][k] == v, (sect, k)
    assert cfg.raw["rabbit"] == REFERENCE_DEFAULTS["rabbit"]


def test_config_validation():
    with pytest.raises(ValueError):
        from_dict({"server": {"mode": "nope"}})
    with pytest.raises(ValueError):
        from_dict({"server": {"model": "ResNet"}})
    cfg = from_dict({"comm": {"attackers": {2: {"mode": "LIE", "round": 2, "args": [0.74]}}}})
    a = cfg.attackers()[2]
    assert a.mode == "LIE" and a.round == 2 and a.args == [0.74]
    with pytest.raises(ValueError):
        from_dict({"comm": {"attackers": {0: {"mode": "Evil"}}}}).attackers()
