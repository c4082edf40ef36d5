"""Defenses on the flat update matrix vs direct state_dict-level statements of the reference rules."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from attackfl_amd import agg
from attackfl_amd.ops import composite as C


def _U(n=6, p=3000, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(1, p, generator=g) + 0.1 * torch.randn(n, p, generator=g)


def test_fedavg_weighted():
    U = _U()
    sizes = torch.tensor([12000., 13000, 14000, 15000, 12500, 13500])
    out = agg.fedavg(U, sizes).params
    ref = sum(U[i] * sizes[i] for i in range(6)) / sizes.sum()
    assert torch.allclose(out, ref, atol=1e-6)


def test_median_lower_and_trimmed():
    U = _U(8)
    assert torch.equal(agg.median(U).params, torch.median(U, dim=0).values)
    U = _U(20)
    k = int(20 * 0.1)
    s, _ = torch.sort(U, dim=0)
    assert torch.allclose(agg.trimmed_mean(U).params, s[k:20 - k].mean(0))
    with pytest.raises(ValueError):
        agg.trimmed_mean(_U(2), trim_ratio=0.5)


def test_krum_picks_reference_argmin():
    U = _U(7)
    U[3] += 5.0  # outlier
    res = agg.krum(U)
    res.info = agg.host_info(res.info)
    n, f = 7, 0
    vec = U.numpy().astype(np.float64)
    scores = []
    for i in range(n):
        d = sorted(float(np.linalg.norm(vec[i] - vec[j]) ** 2) for j in range(n) if j != i)
        scores.append(sum(d[: n - f - 2]))
    assert res.info["selected"] == int(np.argmin(scores))
    assert torch.equal(res.params, U[res.info["selected"]])


def test_shieldfl_weights():
    U = _U(5)
    res = agg.shieldfl(U)
    res.info = agg.host_info(res.info)
    vecs = [u / (u.norm() + 1e-8) for u in U]
    ref = sum(vecs) / len(vecs)
    cos = torch.tensor([F.cosine_similarity(v.view(1, -1), ref.view(1, -1)).item() for v in vecs])
    w = 1 / (1 - cos + 1e-6)
    w = w / w.sum()
    assert torch.allclose(torch.tensor(res.info["weights"]), w, atol=1e-4)
    assert torch.allclose(res.params, sum(U[i] * w[i] for i in range(5)), atol=1e-5)


def test_scionfl_keeps_least_similar_half():
    U = _U(6)
    res = agg.scionfl(U, torch.full((6,), 100.0), seed=3)
    res.info = agg.host_info(res.info)
    s = res.info["scores"]
    thr = sorted(s, reverse=True)[3]
    assert res.info["kept"] == [i for i, x in enumerate(s) if x > thr]


def test_gmm_low_rank_runs():
    U = _U(8, 2000)
    U[6:] += 1.0
    att = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1])
    res = agg.gmm(U, torch.ones(8), attackers=att)
    assert res.ok and res.params.shape == (2000,)


def test_fltracer_flags_outlier():
    U = _U(10)
    U[4] += 3.0
    res = agg.fltracer(U, torch.ones(10))
    assert 4 in res.info["anomalies"]


def test_byzantine_filter():
    U = _U(5)
    U[2] = -U[2]
    res = agg.byzantine(U)
    res.info = agg.host_info(res.info)
    assert 2 not in res.info["kept"]


def test_composite_roc_auc_matches_sklearn():
    from sklearn.metrics import roc_auc_score

    g = torch.Generator().manual_seed(0)
    y = (torch.rand(3000, generator=g) < 0.2).float()
    s = ((torch.rand(3000, generator=g) + 0.4 * y) * 20).round() / 20
    assert C.roc_auc(s, y) == pytest.approx(roc_auc_score(y.numpy(), s.numpy()), abs=1e-12)
