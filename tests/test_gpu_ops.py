"""Every native aggregation / attack / metric kernel vs its fp32/fp64 PyTorch composite."""
import pytest
import torch

from attackfl_amd import ops
from attackfl_amd.ops import composite as C
from attackfl_amd.models import ParamLayout
from attackfl_amd.ops import native

pytestmark = pytest.mark.gpu


def _U(n=8, p=47693, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, p, generator=g) * 0.1 + torch.randn(1, p, generator=g)


def test_colstats_lie(gpu):
    U = _U(5)
    m, s = ops.column_mean_std(U.to(gpu))
    mr, sr = C.column_mean_std(U)
    assert torch.allclose(m.cpu(), mr, atol=1e-6) and torch.allclose(s.cpu(), sr, atol=1e-5)
    assert torch.allclose(ops.lie_candidate(U.to(gpu), 0.74).cpu(), C.lie_candidate(U, 0.74), atol=1e-5)
    one = ops.column_mean_std(U[:1].to(gpu))[1]
    assert torch.isnan(one).all()


def test_weighted_rows_fedavg(gpu):
    U = _U(8)
    sizes = torch.tensor([12000., 13000, 15000, 14000, 12500, 12001, 14999, 13333])
    assert torch.allclose(ops.fedavg(U.to(gpu), sizes).cpu(), C.fedavg(U, sizes), atol=1e-6)


@pytest.mark.parametrize("n", [3, 8, 11, 33])
def test_median_trimmed(gpu, n):
    U = _U(n, 5000, seed=n)
    assert torch.equal(ops.coord_median(U.to(gpu)).cpu(), C.coord_median(U))
    k = max(1, int(n * 0.1))
    assert torch.allclose(ops.trimmed_mean(U.to(gpu), k).cpu(), C.trimmed_mean(U, k), atol=1e-5)


def test_pairwise(gpu):
    U = _U(9, 20000)
    d = ops.pairwise_l2(U.to(gpu)).cpu()
    assert torch.allclose(d, C.pairwise_l2(U), rtol=1e-6, atol=1e-6)


def test_row_dots_cosine(gpu):
    U = _U(6, 30000)
    r = U.mean(0)
    assert torch.allclose(ops.cosine_to(U.to(gpu), r.to(gpu)).cpu(), C.cosine_to(U, r), atol=1e-9)
    assert torch.allclose(ops.row_norms(U.to(gpu)).cpu(), C.row_norms(U), rtol=1e-9)


def test_segments_and_coeffs(gpu):
    lay = ParamLayout.for_model("TransformerModel")
    G = _U(4)
    mean, std = C.column_mean_std(G)
    vec = [s for s in lay.slots if len(s.shape) == 1]
    A, B, Cc = ops.attack_coeffs_segments(G.to(gpu), mean.to(gpu), std.to(gpu), vec)
    Ar, Br, Cr = C.attack_coeffs_segments(G, mean, std, vec)
    assert torch.allclose(A.cpu(), Ar, rtol=1e-9) and torch.allclose(B.cpu(), Br, rtol=1e-7, atol=1e-9)
    assert torch.allclose(Cc.cpu(), Cr, rtol=1e-9)
    diffs = G[1:] - G[:1]
    assert torch.allclose(ops.segment_l2_sum(diffs.to(gpu), vec).cpu(), C.segment_l2_sum(diffs, vec), rtol=1e-9)


@pytest.mark.parametrize("shape", [(192, 64), (64, 64), (64, 7), (6, 64), (1, 32), (128, 1024), (96, 32)])
def test_spectral_norm(gpu, shape):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(5, *shape, generator=g)
    got = ops.batched_spectral_norm(X.to(gpu)).cpu()
    ref = C.batched_spectral_norm(X)
    assert torch.allclose(got, ref, rtol=2e-5), (got, ref)


@pytest.mark.parametrize("model", ["RNNModel", "CNNModel", "TransformerModel", "big"])
def test_spectral_norm_slots(gpu, model):
    """One ragged launch over every matrix slot of a model == per-slot fp64 SVD norms."""
    from attackfl_amd.attacks import DistanceEngine
    from attackfl_amd.models import TensorSlot

    if model == "big":  # a slot past the Gram kernel's 128 limit goes to the library, mixed with small ones
        layout = ParamLayout([TensorSlot("a", (200, 150), 0, 30000), TensorSlot("b", (7,), 30000, 7),
                              TensorSlot("c", (96, 7), 30007, 672)])
    else:
        layout = ParamLayout.for_model(model)
    eng = DistanceEngine(layout, "spectral")
    g = torch.Generator().manual_seed(3)
    D = torch.randn(6, layout.P, generator=g) * 0.05
    got = ops.spectral_norm_sum(D.to(gpu), eng.mat_slots).cpu()
    ref = sum(C.batched_spectral_norm(D[:, s.offset:s.offset + s.numel].reshape(6, s.shape[0], -1))
              for s in eng.mat_slots)
    assert torch.allclose(got, ref, rtol=2e-5), (got, ref)
    assert torch.allclose(ops.spectral_norm_sum(D, eng.mat_slots), ref, rtol=1e-12)


@pytest.mark.parametrize("model", ["RNNModel", "TransformerModel", "big"])
def test_spectral_family_matches_materialised_rows(gpu, model):
    """Gram form (k_spec_grams once + k_spec_eval per γ, γ read from device memory) == fp64 SVD norms of
    the materialised rows X_m - γ·dev, for the γs a bisection visits."""
    from attackfl_amd.attacks import DistanceEngine
    from attackfl_amd.models import TensorSlot

    if model == "big":
        layout = ParamLayout([TensorSlot("a", (200, 150), 0, 30000), TensorSlot("b", (7,), 30000, 7),
                              TensorSlot("c", (96, 7), 30007, 672), TensorSlot("d", (16, 3, 5), 30679, 240)])
    else:
        layout = ParamLayout.for_model(model)
    slots = DistanceEngine(layout, "spectral").mat_slots
    g = torch.Generator().manual_seed(5)
    X = torch.randn(4, layout.P, generator=g) * 0.05
    dev = torch.rand(layout.P, generator=g) * 0.01
    fam = ops.SpectralFamily(X.to(gpu), slots, dev.to(gpu))
    for gamma in (50.0, 25.0, 37.5, 0.0, -3.0):
        got = fam(torch.tensor(gamma, dtype=torch.float64, device=gpu)).cpu()
        rows = X - gamma * dev
        ref = sum(C.batched_spectral_norm(rows[:, s.offset:s.offset + s.numel].reshape(4, s.shape[0], -1).double())
                  for s in slots)
        assert torch.allclose(got, ref, rtol=2e-5), (gamma, got, ref)
    assert torch.allclose(fam(None).cpu(), ops.spectral_norm_sum(X.to(gpu), slots).cpu(), rtol=1e-12)


def test_spectral_family_degenerate(gpu):
    from attackfl_amd.models import TensorSlot

    layout = ParamLayout([TensorSlot("a", (16, 16), 0, 256), TensorSlot("b", (5, 40), 256, 200)])
    X = torch.zeros(3, layout.P)
    X[0, :256] = (torch.eye(16) * 2.0).reshape(-1)   # repeated top singular value
    X[2, 0] = 1e-3
    got = ops.spectral_norm_sum(X.to(gpu), layout.slots).cpu()
    assert torch.allclose(got, torch.tensor([2.0, 0.0, 1e-3], dtype=torch.float64), rtol=1e-5), got


def test_spectral_degenerate(gpu):
    X = torch.zeros(3, 16, 16)
    X[0] = torch.eye(16) * 2.0          # repeated top singular value
    X[2, 0, 0] = 1e-3
    got = ops.batched_spectral_norm(X.to(gpu)).cpu()
    assert torch.allclose(got, torch.tensor([2.0, 0.0, 1e-3], dtype=torch.float64), rtol=1e-5)


def test_roc_auc(gpu):
    from sklearn.metrics import roc_auc_score

    g = torch.Generator().manual_seed(0)
    for n in (10, 1000, 5000, 32768, 32769, 80000):  # <= 32768: pair counts, above: rank sums after a sort
        y = (torch.rand(n, generator=g) < 0.3).float()
        s = torch.rand(n, generator=g) + y * 0.3
        s = (s * 50).round() / 50  # many ties
        a = ops.roc_auc(s.to(gpu), y.to(gpu))
        assert abs(a - roc_auc_score(y.numpy(), s.numpy())) < 1e-9


def test_roc_auc_nan_flag_and_degenerate(gpu):
    s = torch.tensor([0.3, float("nan"), 0.9, 0.1])
    y = torch.tensor([0.0, 1.0, 1.0, 0.0])
    assert ops.roc_auc_checked(s.to(gpu), y.to(gpu))[1] is True
    auc, nan = ops.roc_auc_checked(torch.tensor([0.2, 0.2, 0.7]).to(gpu), torch.tensor([1.0, 0.0, 1.0]).to(gpu))
    assert not nan and abs(auc - 0.75) < 1e-12
    import math
    assert math.isnan(ops.roc_auc(torch.rand(50).to(gpu), torch.ones(50).to(gpu)))  # one class only


def test_adam_flat(gpu):
    g = torch.Generator().manual_seed(0)
    p, gr = torch.randn(1000, generator=g), torch.randn(1000, generator=g)
    m, v = torch.zeros(1000), torch.zeros(1000)
    pd, md, vd = p.clone().to(gpu), m.clone().to(gpu), v.clone().to(gpu)
    for step in (1, 2, 3):
        C.adam_step_scaled(p, gr, m, v, step, 1e-3, 0.5)
        ops.adam_step_scaled(pd, gr.to(gpu), md, vd, step, 1e-3, 0.5)
    assert torch.allclose(pd.cpu(), p, atol=1e-6)


def test_hyper_kernels(gpu):
    g = torch.Generator().manual_seed(0)
    P, H = 47693, 100
    W, b, f, u = torch.randn(P, H, generator=g) * 0.1, torch.randn(P, generator=g), torch.randn(H, generator=g), torch.randn(P, generator=g)
    d, df = ops.hyper_delta_vjp(W.to(gpu), b.to(gpu), f.to(gpu), u.to(gpu))
    dr, dfr = C.hyper_delta_vjp(W, b, f, u)
    assert torch.allclose(d.cpu(), dr, atol=1e-4) and torch.allclose(df.cpu(), dfr, rtol=1e-4, atol=1e-2)
    assert torch.allclose(ops.hyper_generate(W.to(gpu), b.to(gpu), f.to(gpu)).cpu(), torch.addmv(b, W, f), atol=1e-4)
    m, v = torch.zeros(P * H + P), torch.zeros(P * H + P)
    Wd, bd, md, vd = W.clone().to(gpu), b.clone().to(gpu), m.clone().to(gpu), v.clone().to(gpu)
    C.hyper_adam_outer(W, b, m, v, dr, f, 1, 1e-3, 0.3)
    ops.hyper_adam_outer(Wd, bd, md, vd, dr.to(gpu), f.to(gpu), 1, 1e-3, 0.3)
    assert torch.allclose(Wd.cpu(), W, atol=1e-6) and torch.allclose(bd.cpu(), b, atol=1e-6)


def test_stoch_quant(gpu):
    U = _U(4, 100000)
    sigma, smin, smax = ops.stochastic_quantize(U.to(gpu), 123)
    assert torch.allclose(smin.cpu(), U.min(1).values) and torch.allclose(smax.cpu(), U.max(1).values)
    probs = (U - U.min(1, keepdim=True).values) / (U.max(1, keepdim=True).values - U.min(1, keepdim=True).values + 1e-6)
    assert abs(sigma.cpu().mean().item() - probs.mean().item()) < 5e-3


@pytest.mark.gpu
@pytest.mark.parametrize("model,clip", [("TransformerModel", 1e9), ("RNNModel", 0.05)])
def test_hyper_server_update_matches_composite(gpu, model, clip):
    """Sync-free native round update (rows / small-net / head-Adam kernels) vs the CPU composite path."""
    from attackfl_amd.fl.hyper_server import HyperServer
    from attackfl_amd.models import build_model

    sd = build_model(model, seed=0).state_dict()
    n = 5
    cpu = HyperServer(sd, n, 0.01, clip, "cpu", seed=3)
    dev = HyperServer(sd, n, 0.01, clip, gpu, seed=3)
    assert dev._native_ok()
    g = torch.Generator().manual_seed(1)
    for rnd in range(2):
        sel = [3, 0, 4, 1] if rnd == 0 else [2, 1]
        # |delta| >= 0.05 everywhere: Adam's first steps are sign-like, so a cancellation-sized delta would
        # amplify fp32 summation-order differences into O(lr) parameter differences
        r = torch.randn(len(sel), cpu.hnet.P, generator=g)
        U = torch.stack([cpu.generate(i) for i in sel]) - 0.1 * torch.sign(r) * (0.5 + r.abs())
        cpu.train(sel, {i: U[k] for k, i in enumerate(sel)})
        Ud = U.to(gpu)
        dev.train(sel, {i: Ud[k] for k, i in enumerate(sel)})
        assert dev.step == cpu.step
        assert abs(dev.last_info["grad_norm"] - cpu.last_info["grad_norm"]) <= 1e-3 * cpu.last_info["grad_norm"]
        assert abs(dev.last_info["clip_scale"] - cpu.last_info["clip_scale"]) <= 1e-3 * cpu.last_info["clip_scale"]
    a, b = dev.hnet.arena.cpu(), cpu.hnet.arena
    # fp32 reduction order differs (per-block partials); Adam amplifies it where clipped grads approach eps
    assert torch.allclose(a, b, rtol=1e-4, atol=2e-4), float((a - b).abs().max())
    feats = ops.hyper_features(dev.hnet.arena, [0, 2, 4], dev.layout_vec()).cpu()
    cpu.hnet.arena.copy_(a)  # same parameters on both sides
    ref = torch.stack([cpu.hnet.features(i)[1] for i in (0, 2, 4)])
    assert torch.allclose(feats, ref, rtol=1e-4, atol=1e-5)
    # the round's START models: native features + one heads sweep (HyperServer.generate_many) vs the torch MLP
    many = dev.generate_many([4, 0, 2, 1]).cpu()
    ref_many = dev.hnet.generate_many([4, 0, 2, 1]).cpu()
    assert torch.allclose(many, ref_many, rtol=1e-4, atol=1e-5), float((many - ref_many).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["TransformerModel", "RNNModel"])
@pytest.mark.parametrize("ngen", [3, 8, 11])
def test_hyper_update_fused_generation(gpu, model, ngen):
    """The next START generated inside the update's last launches (features in the last small-net launch, the
    heads sweep fused with the last head Adam) equals a plain generate_many from the updated arena BITWISE, the
    update itself equals the unfused one bitwise, and a device-disabled update generates from the unchanged arena."""
    from attackfl_amd.fl.hyper_server import HyperServer
    from attackfl_amd.models import build_model

    sd = build_model(model, seed=0).state_dict()
    n = 12
    srv = [HyperServer(sd, n, 0.01, 0.05, gpu, seed=3) for _ in range(2)]
    g = torch.Generator().manual_seed(2)
    sel = [3, 0, 4, 1, 7]
    gen = [(5 * k + 1) % n for k in range(ngen)]
    r = torch.randn(len(sel), srv[0].hnet.P, generator=g).to(gpu)
    U = torch.stack([srv[0].generate(i) for i in sel]) - 0.1 * torch.sign(r) * (0.5 + r.abs())
    on = torch.ones(1, dtype=torch.int32, device=gpu)
    srv[0].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=on, gen_key=gen)
    fused = srv[0].generate_many(gen)  # (memoised by the update)
    srv[1].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=on)
    assert torch.equal(srv[0].hnet.arena, srv[1].hnet.arena)
    assert torch.equal(srv[0].m, srv[1].m) and torch.equal(srv[0].v, srv[1].v)
    plain = srv[1].generate_many(gen)
    assert torch.equal(fused, plain), float((fused - plain).abs().max())
    ref = srv[1].hnet.generate_many(gen)  # torch MLP + GEMM
    assert torch.allclose(plain, ref, rtol=1e-4, atol=1e-5), float((plain - ref).abs().max())
    # a disabled update: arena, moments untouched, START generated from the unchanged hypernetwork
    before = (srv[0].hnet.arena.clone(), srv[0].m.clone(), srv[0].v.clone())
    srv[0].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=torch.zeros_like(on), gen_key=gen)
    assert all(torch.equal(a, b) for a, b in zip((srv[0].hnet.arena, srv[0].m, srv[0].v), before))
    assert torch.equal(srv[0].generate_many(gen), ops.hyper_generate_many(before[0], gen, srv[0].layout_vec()))


@pytest.mark.gpu
def test_make_plan_native_matches_cpu_mirror(gpu):
    from attackfl_amd.fl.trainers import make_plan
    nd, seeds = [15000, 12001, 2, 13999], [17, 2 ** 40 + 3, 99, 2 ** 63 + 5]
    a = make_plan(60000, nd, 5, seeds, gpu)
    b = make_plan(60000, nd, 5, seeds, "cpu")
    assert a.order.is_cuda
    for c, n in enumerate(nd):
        assert torch.equal(a.order[c, :, :n].cpu(), b.order[c, :, :n])


@pytest.mark.parametrize("n", [1, 7, 64, 65, 1000, 4096 * 3 + 5, 4885850])
def test_crc32_matches_zlib(gpu, n):
    """csrc/kernels/crc.hip: zlib-compatible CRC-32 of a device buffer (checkpoint zip records), any length
    (multiple of 4 bytes) — chunk tails, run tails and one full hypernetwork arena."""
    import zlib

    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g)
    got = int(native().crc32(x.cuda()).item()) & 0xFFFFFFFF
    assert got == zlib.crc32(x.numpy().tobytes())


@pytest.mark.parametrize("K,P", [(1, 1000), (2, 47693), (8, 47693), (8, 5), (17, 20000), (40, 3001), (64, 9000)])
def test_pairwise_gram_mfma_matches_fp64(gpu, K, P):
    """k_gram_f64 (centred Gram on fp64 MFMA) against the fp64 difference form; nearby rows (model updates)
    are where the uncentred Gram form would cancel."""
    g = torch.Generator().manual_seed(K * 1000 + P)
    G = torch.randn(1, P, generator=g) * 3.0 + 1e-3 * torch.randn(K, P, generator=g)
    got = native().pairwise_sqdist_gram(G.cuda()).cpu()
    Gd = G.double()
    ref = ((Gd[:, None, :] - Gd[None, :, :]) ** 2).sum(-1)
    assert torch.allclose(got, ref, rtol=1e-9, atol=1e-12 * float(ref.max() + 1))
    assert torch.equal(got, got.t()) and bool((got.diagonal() == 0).all())
    if K <= 64 and K > 1:  # the dispatcher takes this path
        assert torch.equal(ops.pairwise_sqdist(G.cuda()).cpu(), got)


@pytest.mark.parametrize("P", [1, 3, 4, 1001, 203649])
def test_philox_noise_matches_cpu_mirror(gpu, P):
    g = torch.Generator().manual_seed(P)
    own = torch.randn(P, generator=g)
    for seed in (0, 12345678901234):
        got = ops.noise(own.cuda(), 0.3, seed).cpu()
        ref = ops.noise(own, 0.3, seed)
        assert torch.allclose(got, ref, atol=2e-6, rtol=0)
        assert torch.equal(ops.noise(own.cuda(), 0.3, seed).cpu(), got)   # deterministic


@pytest.mark.gpu
def test_weighted_rows_with_success_check(gpu):
    """FedAvg's early-launch aggregate: the weighted sum when every client succeeded, the fallback (previous
    global model) otherwise — decided inside the same pass (agg.hip k_weighted_rows ok / fallback)."""
    from attackfl_amd import ops

    g = torch.Generator().manual_seed(3)
    U = torch.randn(7, 5003, generator=g)
    w = torch.rand(7, generator=g, dtype=torch.float64)
    w = w / w.sum()
    old = torch.randn(5003, generator=g)
    ref = (w[:, None] * U.double()).sum(0).float()
    Ud, wd, oldd = U.to(gpu), w.to(gpu), old.to(gpu)
    ok = torch.ones(7, dtype=torch.int32, device=gpu)
    assert torch.allclose(ops.weighted_rows(Ud, wd, ok, oldd).cpu(), ref, atol=1e-6)
    assert torch.equal(ops.weighted_rows(Ud, wd).cpu(), ops.weighted_rows(Ud, wd, ok, oldd).cpu())
    ok[4] = 0
    assert torch.equal(ops.weighted_rows(Ud, wd, ok, oldd).cpu(), old)
    # CPU composite: same decision
    assert torch.equal(ops.weighted_rows(U, w, ok.cpu(), old), old)
