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
    assert 4 in agg.host_info(res.info)["anomalies"]


def _fltracer_numpy(U, sizes, threshold=2.5):
    """The reference pipeline on the host: PCA(1) scores via eigh, scipy MAD, np.median."""
    import numpy as np
    from scipy.stats import median_abs_deviation

    X = U.double().numpy()
    Xc = X - X.mean(axis=0, keepdims=True)
    ev, V = np.linalg.eigh(Xc @ Xc.T)
    z = V[:, -1] * np.sqrt(max(ev[-1], 0.0))
    scores = np.abs(z - np.median(z)) / (1.4826 * median_abs_deviation(z) + 1e-6)
    bad = scores > threshold
    keep = [i for i in range(len(z)) if not bad[i]] or list(range(len(z)))
    w = sizes.double().numpy()[keep]
    return sorted(np.where(bad)[0].tolist()), (X[keep] * (w / w.sum())[:, None]).sum(axis=0), scores


@pytest.mark.parametrize("n,seed", [(8, 0), (9, 1), (10, 2), (6, 3)])
def test_fltracer_device_form_matches_host_pipeline(n, seed):
    g = torch.Generator().manual_seed(seed)
    U = torch.randn(n, 3000, generator=g)
    U[1] += 2.5 * torch.randn(3000, generator=g)  # one dominant direction
    U[n - 1] *= 4.0
    sizes = torch.randint(50, 200, (n,), generator=g).float()
    res = agg.fltracer(U, sizes)
    bad, ref, scores = _fltracer_numpy(U, sizes)
    assert agg.host_info(res.info)["anomalies"] == bad
    assert torch.allclose(res.info["scores"], torch.from_numpy(scores), rtol=1e-6, atol=1e-6)
    assert torch.allclose(res.params.double(), torch.from_numpy(ref), rtol=1e-5, atol=1e-6)


def _near_degenerate(n, ratio, seed=0, P=2000):
    """fp32 rows whose centred Gram has eigenvalues 1, ratio, 0.25, 0.09 (nearly iid updates: a flat top)."""
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(n, 4, generator=g, dtype=torch.float64)
    A -= A.mean(0)  # orthogonal to the all-ones vector: centring leaves the rows' span alone
    Q, _ = torch.linalg.qr(A)
    B, _ = torch.linalg.qr(torch.randn(P, 4, generator=g, dtype=torch.float64))
    s = torch.tensor([1.0, ratio ** 0.5, 0.5, 0.3], dtype=torch.float64)
    return (Q * s) @ B.T * 10.0 + 0.25


@pytest.mark.parametrize("ratio", [0.9, 0.999, 0.9999])
def test_fltracer_near_degenerate_spectrum_matches_host_pipeline(ratio):
    """PCA(1) by repeated squaring leaked the second eigenvector at (l2/l1)^4096 (66 % at 0.9999);
    the eigen-decomposition matches numpy's eigh for any gap."""
    U = _near_degenerate(9, ratio).float()
    sizes = torch.ones(9)
    res = agg.fltracer(U, sizes)
    bad, ref, scores = _fltracer_numpy(U, sizes)
    assert agg.host_info(res.info)["anomalies"] == bad
    assert torch.allclose(res.info["scores"].double().cpu(), torch.from_numpy(scores), rtol=1e-6, atol=1e-6)
    z = agg._top_pc_scores(U).double().cpu().abs()
    X = U.double().numpy()
    import numpy as np
    Xc = X - X.mean(axis=0, keepdims=True)
    ev, V = np.linalg.eigh(Xc @ Xc.T)
    assert torch.allclose(z, torch.from_numpy(np.abs(V[:, -1]) * np.sqrt(ev[-1])), rtol=1e-6, atol=1e-8)


def test_fltracer_identical_rows_keep_everyone():
    U = torch.ones(5, 100)
    res = agg.fltracer(U, torch.ones(5))
    assert agg.host_info(res.info)["anomalies"] == [] and torch.allclose(res.params, U[0])


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


def _gmm_case(n, seed):
    g = torch.Generator().manual_seed(seed)
    U = torch.randn(n, 3000, generator=g) * 0.1
    U[n - 2:] += 0.4 * torch.randn(3000, generator=g)  # two displaced attackers
    att = torch.zeros(n, dtype=torch.bool)
    att[n - 2:] = True
    return U, att


@pytest.mark.parametrize("n,seed,rank", [(8, 0, None), (10, 1, None), (12, 2, None), (8, 0, 1), (10, 1, 2)])
def test_gmm_filter_em_matches_sklearn_from_the_same_init(n, seed, rank):
    """The mirror's EM (after its deterministic k-means init) equals sklearn's GaussianMixture started from the
    same weights / means / precisions (reference train_gmm_model, src/Utils.py:257-262)."""
    import math as m_
    import numpy as np
    from sklearn.mixture import GaussianMixture

    U, att = _gmm_case(n, seed)
    G = agg._centred_gram(U).numpy()
    keep, thr, kept, ok = agg.gmm_filter_ref(G, att.numpy(), rank=rank)
    assert ok and 0 < kept <= n
    # independent PCA scores (eigh) and the same k-means init
    ev, V = np.linalg.eigh(G)
    r = rank or max(1, min(4, n // 2 - 1))
    Z = V[:, ::-1][:, :r] * np.sqrt(np.maximum(ev[::-1][:r], 1e-30))
    Z = Z / np.abs(Z).max()
    X = np.vstack([Z[~att.numpy()], Z[att.numpy()]])
    c0 = X[0]
    c1 = X[np.argmax(((X - c0) ** 2).sum(1))]
    mu = np.stack([c0, c1])
    for _ in range(10):
        lab = (((X - mu[1]) ** 2).sum(1) < ((X - mu[0]) ** 2).sum(1)).astype(int)
        mu = np.stack([X[lab == k].mean(0) if (lab == k).any() else mu[k] for k in range(2)])
    resp = np.eye(2)[lab]
    nk = resp.sum(0) + 10 * np.finfo(float).eps
    means = resp.T @ X / nk[:, None]
    covs = np.stack([((resp[:, k, None] * (X - means[k])).T @ (X - means[k])) / nk[k] + 1e-6 * np.eye(r)
                     for k in range(2)])
    gm = GaussianMixture(2, covariance_type="full", reg_covar=1e-6, tol=1e-3, max_iter=100,
                         weights_init=nk / nk.sum(), means_init=means,
                         precisions_init=np.linalg.inv(covs)).fit(X)
    md0 = [m_.sqrt((x - gm.means_[0]) @ np.linalg.inv(gm.covariances_[0]) @ (x - gm.means_[0]))
           for x in X[:int((~att).sum())]]
    assert thr == pytest.approx(3 * np.std(md0), rel=1e-4, abs=1e-9)
    lab = gm.predict(Z)
    ref_keep = np.array([m_.sqrt((z - gm.means_[k]) @ np.linalg.inv(gm.covariances_[k]) @ (z - gm.means_[k])) <= thr
                         for z, k in zip(Z, lab)])
    assert (keep == ref_keep).all()


def test_gmm_round_fails_when_nothing_is_kept():
    U = torch.full((6, 100), float("nan"))
    res = agg.gmm(U, torch.ones(6), attackers=torch.zeros(6, dtype=torch.bool))
    assert not res.ok and res.params is None
