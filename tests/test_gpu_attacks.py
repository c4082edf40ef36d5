"""Fused device bisection (K-G5, linalg.hip ``bisect_decide``) vs the generic unrolled device loop and the
CPU reference loop (src/Utils.py:101-204): same tried γ sequence, same decisions, same malicious model."""
import pytest
import torch

from attackfl_amd import attacks
from attackfl_amd.attacks import DistanceEngine
from attackfl_amd.models import ParamLayout, build_model

pytestmark = pytest.mark.gpu


def _G(name, K, scale, seed):
    torch.manual_seed(seed)
    lay = ParamLayout.for_model(name)
    base = lay.flatten(build_model(name, seed=seed).state_dict())
    return lay, base[None] + scale * torch.randn(K, lay.P)


@pytest.mark.parametrize("name", ["TransformerModel", "RNNModel"])
@pytest.mark.parametrize("mode", ["spectral", "flat"])
@pytest.mark.parametrize("fn", [attacks.min_max, attacks.min_sum, attacks.opt_fang])
@pytest.mark.parametrize("scale", [0.02, 0.5])
def test_fused_bisection_matches_generic_and_cpu(gpu, name, mode, fn, scale, monkeypatch):
    lay, G = _G(name, 5, scale, 3)
    eng = DistanceEngine(lay, mode)
    cpu = attacks.host_info(fn(G, G[0], eng).info)
    Gd = G.to(gpu)
    fused = fn(Gd, Gd[0], eng)
    hf = attacks.host_info(fused.info)
    monkeypatch.setattr(attacks, "_bisect_fused", lambda *a, **k: None)  # force the generic device loop
    gen = fn(Gd, Gd[0], eng)
    hg = attacks.host_info(gen.info)
    assert hf["gammas"] == hg["gammas"] == cpu["gammas"]
    assert hf["accepted"] == hg["accepted"] == cpu["accepted"]
    assert hf["gamma"] == cpu["gamma"] and hf["gamma_succ"] == cpu["gamma_succ"]
    assert torch.equal(fused.params, gen.params)


@pytest.mark.parametrize("n,seed,rank", [(8, 0, 0), (10, 1, 0), (12, 2, 0), (5, 3, 0), (8, 0, 1), (12, 2, 2), (6, 4, 4)])
def test_gmm_filter_kernel_matches_host_mirror(gpu, n, seed, rank):
    """agg.hip k_gmm_filter (the whole GMM decision in one launch) vs its fp64 host mirror."""
    from attackfl_amd import agg
    from attackfl_amd.ops import native

    g = torch.Generator().manual_seed(seed)
    U = torch.randn(n, 4000, generator=g) * 0.1
    U[n - 2:] += 0.4 * torch.randn(4000, generator=g)
    att = torch.zeros(n, dtype=torch.bool)
    att[n - 2:] = True
    G = agg._centred_gram(U)
    keep, thr, kept, ok = agg.gmm_filter_ref(G.numpy(), att.numpy(), rank=rank)
    kd, info = native().gmm_filter(G.to(gpu), att.to(gpu, torch.uint8), rank)
    assert kd.bool().cpu().numpy().tolist() == keep.tolist()
    assert info[0].item() == pytest.approx(thr, rel=1e-9, abs=1e-12)
    assert int(info[1].item()) == kept and bool(info[2].item()) == ok
    res = agg.gmm(U.to(gpu), torch.ones(n), attackers=att, gmm_rank=rank)
    assert res.ok == (kept > 0)  # (nothing kept: the round fails)
    if kept:
        assert torch.allclose(res.params.cpu(), U[torch.from_numpy(keep)].mean(0), atol=1e-6)


def test_gram_centred_matches_fp64_reference(gpu):
    from attackfl_amd.ops import native

    g = torch.Generator().manual_seed(5)
    U = torch.randn(9, 47693, generator=g) * 0.01 + 0.5
    C = native().gram_centred(U.to(gpu))[0].cpu()
    X = U.double() - U.double().mean(0, keepdim=True)
    ref = X @ X.t()
    assert torch.allclose(C, ref, rtol=1e-9, atol=1e-9 * ref.abs().max().item())


@pytest.mark.parametrize("n,ratio", [(9, 0.999), (9, 0.9999), (64, 0.99), (5, 0.5)])
def test_fltracer_top_pc_kernel_matches_eigh(gpu, n, ratio):
    """k_top_pc (Jacobi, one wave) gives numpy eigh's first principal-component scores (up to the sign), also
    for a nearly flat spectrum top, and FLTracer's device decisions equal the host pipeline's."""
    import numpy as np
    from test_aggregators import _fltracer_numpy, _near_degenerate

    from attackfl_amd import agg

    U = _near_degenerate(n, ratio, seed=n).float()
    z = agg._top_pc_scores(U.to(gpu)).cpu().abs()
    X = U.double().numpy()
    Xc = X - X.mean(axis=0, keepdims=True)
    ev, V = np.linalg.eigh(Xc @ Xc.T)
    # (the device Gram's fp64 rounding differs from numpy's in the last bits; an eigenvector amplifies that by
    # 1 / gap = 1e4 here — the repeated-squaring form it replaces was off by 2 % at 0.999 and 66 % at 0.9999)
    tol = max(1e-5, 1e-7 / (1.0 - ratio))  # both solvers see a problem conditioned like 1 / gap
    assert torch.allclose(z, torch.from_numpy(np.abs(V[:, -1]) * np.sqrt(ev[-1])), rtol=tol, atol=1e-7)
    sizes = torch.arange(1, n + 1).float()
    res = agg.fltracer(U.to(gpu), sizes.to(gpu))
    bad, ref, scores = _fltracer_numpy(U, sizes)
    assert agg.host_info(res.info)["anomalies"] == bad
    assert torch.allclose(res.info["scores"].double().cpu(), torch.from_numpy(scores), rtol=tol, atol=1e-6)
