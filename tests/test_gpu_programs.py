"""GPU numerics of the client-batched layer kernels and the graph-captured step programs, each
against the fp32 PyTorch composite of the same op (CPU), with identical hash dropout masks."""
import pytest
import torch

from attackfl_amd.data import DeviceTable, synthetic_har, synthetic_icu
from attackfl_amd.fl.programs import ProgramRunner, make_program
from attackfl_amd.fl.trainers import Plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import layers as Lx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, rel=2e-2, name=""):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= rel * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def _ctl(C):
    return Lx.StepCtl.create([7 + 3 * c for c in range(C)], DEV), Lx.StepCtl.create([7 + 3 * c for c in range(C)],
                                                                                       "cpu")


@pytest.mark.parametrize("N", [70, 136])  # 136: row-contiguous aligned output -> LDS-staged vector epilogue
@pytest.mark.parametrize("act,gact,p", [(0, 0, 0.0), (1, 0, 0.1), (2, 0, 0.3), (0, 1, 0.1), (0, 2, 0.0)])
def test_bgemm_epilogues(gpu, act, gact, p, N):
    C, M, K = 3, 150, 45
    g = torch.Generator().manual_seed(0)
    A = torch.randn(C, M, K, generator=g)
    W = torch.randn(C, N, K, generator=g)
    bias = torch.randn(C, N, generator=g)
    G = torch.randn(C, M, N, generator=g)
    cg, cc = _ctl(C)
    outs = []
    for dev, ctl in ((DEV, cg), ("cpu", cc)):
        Cm = torch.zeros(C, M, N, device=dev)
        Z = torch.zeros(C, M, N, device=dev)
        Lx.bgemm(A.to(dev), W.to(dev), Cm, bias=bias.to(dev), Z=Z, G=G.to(dev) if gact else None, act=act, gact=gact,
                 ctl=ctl, layer=5, p=p)
        outs.append((Cm, Z))
    _close(outs[0][0], outs[1][0], name="C")
    _close(outs[0][1], outs[1][1], name="Z")
    # dropout masks identical: zeros in the same places
    if p > 0:  # (away from relu's kink, where bf16 rounding may flip the sign)
        z = outs[1][1]
        sure = (torch.relu(z) if act == 1 else (torch.nn.functional.gelu(z) if act == 2 else z)).abs() > 0.5
        assert torch.equal((outs[0][0].cpu() == 0)[sure], (outs[1][0] == 0)[sure])


def test_bgemm_transposed_views_and_splitk(gpu):
    C, M, N, K = 2, 2048, 96, 40
    g = torch.Generator().manual_seed(1)
    dY = torch.randn(C, M, N, generator=g)
    X = torch.randn(C, M, K, generator=g)
    ref = torch.bmm(dY.transpose(1, 2), X)
    for splitk in (1, 6):
        out = torch.zeros(C, N, K, device=DEV)
        Lx.bgemm(dY.to(DEV).transpose(1, 2), X.to(DEV).transpose(1, 2), out, accum=2 if splitk > 1 else 0,
                 splitk=splitk)
        _close(out, ref, name=f"dW splitk={splitk}")
    # dX = dY W with W a strided view into a flat arena
    P = 10000
    flat = torch.randn(C, P, generator=g)
    W = flat[:, 100:100 + N * K].view(C, N, K)
    out = torch.zeros(C, M, K, device=DEV)
    Lx.bgemm(dY.to(DEV), flat.to(DEV)[:, 100:100 + N * K].view(C, N, K).transpose(1, 2), out)
    _close(out, torch.bmm(dY, W), name="dX")


@pytest.mark.parametrize("N,K,trans", [(192, 64, False), (64, 64, False), (256, 64, False), (64, 256, False),
                                       (256, 64, True), (64, 192, True), (128, 64, False)])
def test_tall_skinny_gemm_matches_generic_and_composite(gpu, N, K, trans):
    """k_tsgemm (B staged once per workgroup, A streamed into fragments, float4 epilogue) vs k_bgemm and the
    fp32 composite, every epilogue on: bias, Z, relu, dropout, act'(G), accumulate; M not a multiple of 16."""
    C, M = 3, 1000 + 7
    g = torch.Generator().manual_seed(3)
    A = torch.randn(C, M, K, generator=g)
    flat = torch.randn(C, N * K + 64, generator=g) * 0.2
    W = flat[:, 16:16 + N * K].view(C, K, N).transpose(1, 2) if trans else flat[:, 16:16 + N * K].view(C, N, K)
    bias, G = torch.randn(C, N, generator=g), torch.randn(C, M, N, generator=g)
    C0 = torch.randn(C, M, N, generator=g)
    cg, cc = _ctl(C)
    outs = []
    for dev, ctl, generic in ((DEV, cg, False), (DEV, cg, True), ("cpu", cc, False)):
        Wd = (flat.to(dev)[:, 16:16 + N * K].view(C, K, N).transpose(1, 2) if trans
              else flat.to(dev)[:, 16:16 + N * K].view(C, N, K))
        Cm, Z = C0.clone().to(dev), torch.zeros(C, M, N, device=dev)
        asum = torch.ones(C, K, device=dev)  # accumulates: starts at 1
        Lx.bgemm(A.to(dev), Wd, Cm, bias=bias.to(dev), Z=Z, G=G.to(dev), act=1, gact=1, accum=1, ctl=ctl, layer=4,
                 p=0.1, generic=generic, asum=asum)
        outs.append((Cm, Z, asum))
    for k, name in ((0, "tsgemm"), (1, "bgemm")):
        _close(outs[k][0], outs[2][0], name=name + " C")
        _close(outs[k][1], outs[2][1], name=name + " Z")
        assert torch.allclose(outs[k][2].cpu(), 1 + A.sum(dim=1), rtol=1e-5, atol=1e-3), name + " column sums"
    # the two device kernels share operand rounding (bf16) and accumulate in fp32: near-identical
    assert (outs[0][1] - outs[1][1]).abs().max().item() < 1e-3 * (outs[1][1].abs().max().item() + 1)
    del W


@pytest.mark.parametrize("P,skip", [(1024, (5, 518)), (1003, (0, 0)), (1024, (0, 0))])
@pytest.mark.parametrize("sgd", [0.0, 0.05])
def test_adam_clients_vector_and_scalar_paths(gpu, P, skip, sgd):
    """k_adam_clients: float4 path (P % 4 == 0, a skip range straddling float4 groups) and scalar path vs
    the composite, 3 steps, one inactive client, gradients zeroed on the device as they are consumed."""
    C = 3
    g = torch.Generator().manual_seed(4)
    p0, grads = torch.randn(C, P, generator=g), [torch.randn(C, P, generator=g) for _ in range(3)]
    bsz = torch.tensor([[8, 8, 1]] * 3, dtype=torch.int32)  # client 2: batch of 1 -> inactive
    res = []
    for dev in (DEV, "cpu"):
        ctl = Lx.StepCtl.create([1, 2, 3], dev)
        p, m, v = p0.clone().to(dev), torch.zeros(C, P, device=dev), torch.zeros(C, P, device=dev)
        tcount = torch.zeros(C, dtype=torch.int32, device=dev)
        failed = torch.zeros(C, dtype=torch.int32, device=dev)
        gr = torch.zeros(C, P, device=dev)
        for s in range(3):
            if dev == "cpu":
                gr.copy_(grads[s])
            else:
                gr += grads[s].to(dev)  # zeroed by the previous step's Adam (inactive client accumulates)
            Lx.adam_clients(p, gr, m, v, tcount, bsz.to(dev), ctl, failed, 1e-2, skip, sgd, zero_grads=dev != "cpu")
            Lx.step_end(ctl, tcount, bsz.to(dev), failed)
        res.append(p.cpu())
    assert torch.allclose(res[0][:2], res[1][:2], rtol=1e-5, atol=1e-6)
    assert torch.equal(res[0][2], p0[2])  # inactive client untouched
    if skip[1] > skip[0]:
        assert torch.equal(res[0][:, skip[0]:skip[1]], p0[:, skip[0]:skip[1]])


@pytest.mark.parametrize("stride", [64, 67])  # 67: rows not 16-B aligned -> the scalar-access kernel path
def test_layernorm_fwd_bwd(gpu, stride):
    C, R = 2, 300
    g = torch.Generator().manual_seed(2)
    x, a, dy = (torch.randn(C, R, stride, generator=g)[:, :, :64] for _ in range(3))
    gam, bet = 1 + 0.1 * torch.randn(C, 64, generator=g), 0.1 * torch.randn(C, 64, generator=g)
    cg, cc = _ctl(C)
    res = []
    for dev, ctl in ((DEV, cg), ("cpu", cc)):
        s = torch.zeros(C, R, 64, device=dev)
        y = torch.zeros(C, R, 64, device=dev)
        st = torch.zeros(C, R, 2, device=dev)
        Lx.ln_fwd(x.to(dev), a.to(dev), s, y, st, gam.to(dev), bet.to(dev), ctl, layer_a=3, p_a=0.1, layer_o=4,
                  p_o=0.3)
        dx = torch.zeros(C, R, 64, device=dev)
        da = torch.zeros(C, R, 64, device=dev)
        dg = torch.zeros(C, 64, device=dev)
        db = torch.zeros(C, 64, device=dev)
        Lx.ln_bwd(dy.to(dev), s, st, gam.to(dev), dx, 0, da, dg, db, ctl, layer_a=3, p_a=0.1, layer_o=4, p_o=0.3)
        res.append((y, dx, da, dg, db))
    for i, n in enumerate(["y", "dx", "da", "dgamma", "dbeta"]):
        _close(res[0][i], res[1][i], rel=1e-4, name=n)


def test_gru_pool_conv_ops(gpu):
    C, B = 2, 33
    g = torch.Generator().manual_seed(3)
    gi, bhh = torch.randn(C, B, 96, generator=g), torch.randn(C, 96, generator=g)
    dh = torch.randn(C, B, 64, generator=g)
    res = []
    for dev in (DEV, "cpu"):
        h = torch.zeros(C, B, 64, device=dev)
        Lx.gru_fwd(gi.to(dev), bhh.to(dev), h, 32)
        dgi = torch.zeros(C, B, 96, device=dev)
        dbi, dbh = torch.zeros(C, 96, device=dev), torch.zeros(C, 96, device=dev)
        Lx.gru_bwd(dh.to(dev), 32, gi.to(dev), bhh.to(dev), dgi, dbi, dbh)
        res.append((h, dgi, dbi, dbh))
    for i in range(4):
        _close(res[0][i], res[1][i], rel=1e-4, name=f"gru{i}")
    # conv patches + pooling with dropout
    L, Cin = 7, 32
    x = torch.relu(torch.randn(C, B * L, Cin, generator=g))
    dcols = torch.randn(C, B * L, 3 * Cin, generator=g)
    h3 = torch.relu(torch.randn(C, B * L, 128, generator=g))
    dout = torch.randn(C, B, 1024, generator=g)
    cg, cc = _ctl(C)
    res = []
    for dev, ctl in ((DEV, cg), ("cpu", cc)):
        cols = torch.zeros(C, B * L, 3 * Cin, device=dev)
        Lx.im2col3(x.to(dev), B, L, cols)
        dx = torch.zeros(C, B * L, Cin, device=dev)
        Lx.col2im3(dcols.to(dev), B, L, Cin, x.to(dev), dx)
        cat = torch.zeros(C, B, 1024, device=dev)
        Lx.pool4_fwd(h3.to(dev), B, L, cat, 512, ctl, layer=1, p=0.3)
        dh3 = torch.zeros(C, B * L, 128, device=dev)
        Lx.pool4_bwd(dout.to(dev), 512, h3.to(dev), B, L, dh3, ctl, layer=1, p=0.3)
        res.append((cols, dx, cat, dh3))
    for i, n in enumerate(["im2col", "col2im", "pool", "pool_bwd"]):
        _close(res[0][i], res[1][i], rel=1e-5, name=n)


@pytest.mark.parametrize("L,p", [(50, 0.0), (561, 0.1)])
def test_flash_attention_fwd_bwd(gpu, L, p):
    C, B = 2, 2
    g = torch.Generator().manual_seed(4)
    qkv = torch.randn(C, B * L, 192, generator=g)
    dout = torch.randn(C, B * L, 64, generator=g)
    cg, cc = _ctl(C)
    Lp = Lx.attn_lp(L)
    res = []
    for dev, ctl in ((DEV, cg), ("cpu", cc)):
        o = torch.zeros(C, B * L, 64, device=dev)
        lse = torch.zeros(C * B * 4, Lp, device=dev)
        Lx.attn_fwd(qkv.to(dev), o, lse, B, L, ctl, layer=2, p=p)
        dq = torch.zeros(C, B * L, 192, device=dev)
        Lx.attn_bwd(qkv.to(dev), o, lse, dout.to(dev), dq, B, L, ctl, layer=2, p=p)
        res.append((o, lse[:, :L], dq))
    for i, n in enumerate(["O", "lse", "dqkv"]):
        _close(res[0][i], res[1][i], rel=3e-2, name=n)


def _params(name, C):
    lay = ParamLayout.for_model(name)
    base = lay.flatten(build_model(name, seed=0).state_dict())
    out = base[None].repeat(C, 1)
    out[1:] += 0.01 * torch.randn(C - 1, lay.P, generator=torch.Generator().manual_seed(9))
    return out


@pytest.mark.parametrize("name,B,n", [("CNNModel", 64, 300), ("RNNModel", 64, 300), ("TransformerClassifier", 4, 24)])
def test_program_sgd_step_matches_composite(gpu, name, B, n):
    """One graph-free SGD step with dropout ON: native gradients vs the composite's (same masks)."""
    C = 2
    ds = synthetic_har(n) if name == "TransformerClassifier" else synthetic_icu(n)
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:B] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32), torch.tensor([B] * C, dtype=torch.int32), 1)
    params = _params(name, C)
    res = []
    for dev in (DEV, "cpu"):
        p = params.clone().to(dev)
        ok, losses = ProgramRunner(make_program(name, C, B, dev), use_graph=False).train(
            DeviceTable(ds, dev), p, Plan(plan.order.to(dev), plan.nd, 1), lr=0.0, seeds=[3, 4], sgd_lr=1.0)
        assert ok.all()
        res.append(((params - p.cpu()), losses))
    _close(res[0][0], res[1][0], rel=3e-2, name=f"{name} grads")
    assert torch.allclose(res[0][1], res[1][1], rtol=1e-2)


@pytest.mark.parametrize("name,B,n,E", [("CNNModel", 128, 1000, 2), ("RNNModel", 128, 1000, 2),
                                        ("TransformerClassifier", 16, 80, 1)])
def test_program_graph_adam_training(gpu, name, B, n, E):
    """Multi-step Adam through the captured HIP graph tracks the composite run (losses per epoch)."""
    C = 3
    ds = synthetic_har(n) if name == "TransformerClassifier" else synthetic_icu(n)
    nd = [n // 2, n // 2 - 17, n // 3 + 1]
    order = torch.stack([torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(10 * c + e))[:max(nd)]
                                      for e in range(E)]) for c in range(C)]).to(torch.int32)
    params = _params(name, C)
    res = []
    for dev in (DEV, "cpu"):
        p = params.clone().to(dev)
        ok, losses = ProgramRunner(make_program(name, C, B, dev)).train(
            DeviceTable(ds, dev), p, Plan(order.to(dev), torch.tensor(nd, dtype=torch.int32), E), lr=1e-3,
            seeds=[5, 6, 7])
        assert ok.all()
        res.append((p.cpu(), losses))
    assert torch.allclose(res[0][1], res[1][1], rtol=2e-2, atol=2e-3), (res[0][1], res[1][1])
    assert (res[0][0] - res[1][0]).abs().max() < 0.05


@pytest.mark.parametrize("B,p", [(128, 0.3), (37, 0.0)])
def test_cnn_tower_kernels_match_composite(gpu, B, p):
    """Fused CNN tower fwd / bwd and the one-launch conv weight gradients vs the fp32 composites.
    Each stage runs on the SAME inputs on both sides (the device's activations are copied to the CPU
    buffers first), so bf16 rounding cannot flip a ReLU mask between the two."""
    C = 3
    lay = ParamLayout.for_model("CNNModel")
    g = torch.Generator().manual_seed(4)
    params = torch.stack([lay.flatten(build_model("CNNModel", seed=s).state_dict()) for s in range(C)])
    x = {"vitals": torch.randn(C, B, 7, generator=g), "labs": torch.randn(C, B, 16, generator=g)}
    dcat = torch.randn(C, B, 1024, generator=g) * 0.1
    st = {}
    for dev in (DEV, "cpu"):
        prog = make_program("CNNModel", C, B, dev, train=True)
        P = params.to(dev).contiguous()
        prog.buf("xv", C, B, 7).copy_(x["vitals"])
        prog.buf("xl", C, B, 16).copy_(x["labs"])
        st[dev] = (prog, P, torch.zeros_like(P), Lx.StepCtl.create([7 + 3 * c for c in range(C)], dev))
    tw = {d: st[d][0].towers(st[d][1]) for d in st}
    cat = {d: st[d][0].buf("cat", C, B, 1024) for d in st}
    for d in st:
        Lx.cnn_towers_fwd(tw[d], B, cat[d], st[d][3], p, st[d][0].wimg())
    _close(cat[DEV], cat["cpu"], rel=3e-2, name="cat")
    for tg, tc in zip(tw[DEV], tw["cpu"]):
        for k in ("h1", "h2", "h3"):
            _close(getattr(tg, k), getattr(tc, k), rel=3e-2, name=k)
            getattr(tc, k).copy_(getattr(tg, k).cpu())
    for d in st:
        Lx.cnn_towers_bwd(tw[d], B, dcat.to(d), st[d][3], p, st[d][0].wimg())
    for tg, tc in zip(tw[DEV], tw["cpu"]):
        for k in ("dh3", "dh2", "dh1"):
            _close(getattr(tg, k), getattr(tc, k), rel=3e-2, name=k)
            getattr(tc, k).copy_(getattr(tg, k).cpu())
    for d in st:
        prog, _, grads, _ = st[d]
        jobs = []
        for t, br in zip(tw[d], ("vitals", "labs")):
            for i, (dh, h) in enumerate(zip((t.dh1, t.dh2, t.dh3), (t.x, t.h1, t.h2)), start=1):
                jobs.append((dh, h, prog.w(grads, f"{br}_conv{i}.weight"), prog.w(grads, f"{br}_conv{i}.bias"), t.L))
        Lx.conv_dw(jobs, B)
    prog = st["cpu"][0]
    for br in ("vitals", "labs"):
        for i in (1, 2, 3):
            for kind in ("weight", "bias"):
                name = f"{br}_conv{i}.{kind}"
                _close(prog.w(st[DEV][2], name), prog.w(st["cpu"][2], name), rel=2e-2, name=name)


def test_splitk_gemm_is_deterministic(gpu):
    """Split-K (accum 2) stores each split's partial tile and adds the splits in split order: the same
    bits every run, whatever order the workgroups ran in (it was an atomic accumulation)."""
    C, M, N, K = 3, 4096, 64, 40
    g = torch.Generator().manual_seed(2)
    dY = torch.randn(C, M, N, generator=g).to(DEV)
    X = torch.randn(C, M, K, generator=g).to(DEV)
    outs = []
    for _ in range(3):
        out = torch.zeros(C, N, K, device=DEV)
        Lx.bgemm(dY.transpose(1, 2), X.transpose(1, 2), out, accum=2, splitk=16)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    _close(outs[0], torch.bmm(dY.cpu().transpose(1, 2), X.cpu()), name="splitk")


@pytest.mark.parametrize("name,B,n,E", [("CNNModel", 128, 1000, 2), ("TransformerClassifier", 16, 80, 1),
                                        ("RNNModel", 128, 1000, 2)])
def test_program_training_is_bit_reproducible(gpu, name, B, n, E):
    """Two graph-replayed training runs from the same state give the same parameters bit for bit (split-K
    GEMMs, conv / stem weight gradients, LayerNorm gamma / beta, bias column sums and the CNN head's sums all
    reduce in a fixed order), and so does client 1 trained ALONE vs beside clients 0 and 2
    (placement-independent: the multi-rank claim)."""
    C = 3
    ds = synthetic_har(n) if name == "TransformerClassifier" else synthetic_icu(n)
    nd = [n // 2, n // 2 - 17, n // 3 + 1]
    order = torch.stack([torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(10 * c + e))[:max(nd)]
                                      for e in range(E)]) for c in range(C)]).to(torch.int32)
    params = _params(name, C)
    table = DeviceTable(ds, DEV)
    runs = []
    for _ in range(2):
        p = params.clone().to(DEV)
        ok, losses = ProgramRunner(make_program(name, C, B, DEV)).train(
            table, p, Plan(order.to(DEV), torch.tensor(nd, dtype=torch.int32), E), lr=1e-3, seeds=[5, 6, 7])
        assert ok.all()
        runs.append((p.cpu(), losses.cpu()))
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0] - runs[1][0]).abs().max()
    assert torch.equal(runs[0][1], runs[1][1])
    p1 = params[1:2].clone().to(DEV)
    ok, losses = ProgramRunner(make_program(name, 1, B, DEV)).train(
        table, p1, Plan(order[1:2].contiguous().to(DEV), torch.tensor(nd[1:2], dtype=torch.int32), E), lr=1e-3,
        seeds=[6])
    assert ok.all()
    assert torch.equal(p1.cpu()[0], runs[0][0][1]), (p1.cpu()[0] - runs[0][0][1]).abs().max()


@pytest.mark.parametrize("C,n,E", [(3, 1000, 2), (8, 600, 1)])
def test_cnn2_onchip_trainer_tracks_layer_program(gpu, monkeypatch, C, n, E):
    """The CNNModel on-chip trainer (csrc/kernels/cnn2.hip: one launch per round, 32 workgroups per client)
    follows the graph-replayed layer program (same batches, dropout masks and Adam): per-epoch losses and
    the trained parameters agree to bf16-operand tolerance, and two launches give the same bits."""
    ds = synthetic_icu(n)
    nd = [max(3, n // 2 - 17 * c) for c in range(C)]
    order = torch.stack([torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(10 * c + e))[:max(nd)]
                                      for e in range(E)]) for c in range(C)]).to(torch.int32)
    params = _params("CNNModel", C)
    table = DeviceTable(ds, DEV)
    res = {}
    for mode in ("0", "1", "1b"):
        monkeypatch.setenv("AFL_CNN2", mode[0])
        p = params.clone().to(DEV)
        runner = ProgramRunner(make_program("CNNModel", C, 128, DEV))
        assert runner._onchip_cnn(p, 0.0, None) == (mode[0] == "1")
        ok, losses = runner.train(table, p, Plan(order.to(DEV), torch.tensor(nd, dtype=torch.int32), E), lr=1e-3,
                                  seeds=[5 + c for c in range(C)])
        assert ok.all()
        res[mode] = (p.cpu(), losses)
    assert torch.equal(res["1"][0], res["1b"][0]) and torch.equal(res["1"][1], res["1b"][1])
    assert torch.allclose(res["1"][1], res["0"][1], rtol=2e-2, atol=2e-3), (res["1"][1], res["0"][1])
    assert (res["1"][0] - res["0"][0]).abs().max() < 0.05
    assert (res["1"][0] - params).abs().max() > 1e-3  # it trained


@pytest.mark.parametrize("B,drop", [(128, True), (128, False), (37, True)])
def test_cnn2_sgd_gradients_match_composite(gpu, monkeypatch, B, drop):
    """One raw-SGD step (opt_mode 1: p -= lr g) of the on-chip CNN trainer exposes its gradients.  Per tensor
    they match the GPU layer program (the same bf16 MFMA operands, ``AFL_CNN2=0``) closely and the fp32
    composite (CPU, same batch rows and dropout masks) within bf16 error, judged like the rnn2 trainer's
    test (tests/test_gpu_rnn.py: relative norm error, 12 % vs fp32): the first conv layer's gradient is a
    residual of cancelling terms and collects the rounding of every layer above it."""
    from attackfl_amd.models import ParamLayout

    C, n = 2, 400
    ds = synthetic_icu(n)
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:B] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32), torch.tensor([B] * C, dtype=torch.int32), 1)
    params = _params("CNNModel", C)
    res = []
    for dev, onchip in ((DEV, "1"), (DEV, "0"), ("cpu", "0")):
        monkeypatch.setenv("AFL_CNN2", onchip)
        p = params.clone().to(dev)
        runner = ProgramRunner(make_program("CNNModel", C, B, dev, dropout=drop), use_graph=False)
        if dev == DEV:
            assert bool(runner._onchip_cnn(p, 1.0, None)) == (onchip == "1")
        ok, losses = runner.train(DeviceTable(ds, dev), p, Plan(plan.order.to(dev), plan.nd, 1), lr=0.0, seeds=[3, 4],
                                  sgd_lr=1.0)
        assert ok.all()
        res.append(((params - p.cpu()), losses.cpu()))
    assert torch.allclose(res[0][1], res[2][1], rtol=1e-2)
    lay = ParamLayout.for_model("CNNModel")
    bad = {}
    for s in lay.slots:
        a, c, b = (r[0][:, s.offset:s.offset + s.numel] for r in res)
        vs_layer = ((a - c).norm() / (c.norm() + 1e-12)).item()
        vs_fp32 = ((a - b).norm() / (b.norm() + 1e-12)).item()
        if vs_layer > 0.06 or vs_fp32 > 0.12:
            bad[s.name] = (round(vs_layer, 4), round(vs_fp32, 4))
    assert not bad, bad


@pytest.mark.parametrize("nan_at", ["first", "weights"])
def test_cnn2_nan_loss_fails_only_that_client(gpu, monkeypatch, nan_at):
    """A NaN batch loss aborts the client's round (reference client.py:100-102) on the on-chip CNN trainer: the
    abort is detected after the hand-off and goes out at the next step's start (or at the round's end), the
    other clients of the launch train normally and match their single-client runs."""
    monkeypatch.setenv("AFL_CNN2", "1")
    C, n, B = 3, 600, 64
    ds = synthetic_icu(n)
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:n] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32), torch.tensor([n] * C, dtype=torch.int32), 1)
    params = _params("CNNModel", C)
    from attackfl_amd.models import ParamLayout

    lay = ParamLayout.for_model("CNNModel")
    s = lay.slots[[x.name for x in lay.slots].index("output.bias")]
    params[1, s.offset] = float("nan") if nan_at == "weights" else 1e30  # client 1: NaN loss at step 1
    if nan_at == "first":
        s2 = lay.slots[[x.name for x in lay.slots].index("output.weight")]
        params[1, s2.offset:s2.offset + s2.numel] = float("inf")
    p = params.clone().to(DEV)
    runner = ProgramRunner(make_program("CNNModel", C, B, DEV), use_graph=False)
    assert runner._onchip_cnn(p, 0.0, None)
    ok, losses = runner.train(DeviceTable(ds, DEV), p, Plan(plan.order.to(DEV), plan.nd, 1), lr=1e-3, seeds=[3, 4, 5])
    ok = ok.cpu().tolist()
    assert ok[1] == 0 and ok[0] == 1 and ok[2] == 1, ok
    # the healthy clients are unaffected by the failing one (placement independence)
    for c in (0, 2):
        q = params[c:c + 1].clone().to(DEV)
        r1 = ProgramRunner(make_program("CNNModel", 1, B, DEV), use_graph=False)
        ok1, _ = r1.train(DeviceTable(ds, DEV), q, Plan(plan.order[c:c + 1].to(DEV), plan.nd[c:c + 1], 1), lr=1e-3,
                          seeds=[3 + c])
        assert bool(ok1.all()) and torch.equal(q[0], p[c])



def test_cnn2_eval_many_matches_eager_model(gpu):
    """Fused forward-only CNN eval of C models (cnn2.hip k_cnn2_eval, the validation pass) against torch's fp32
    CNNModel in eval mode: bf16 MFMA convolutions / fc1 -> outputs within 2e-2, mean error far below; n not a
    multiple of the 16-sample tile; an odd arena row stride (padded by the binding)."""
    from attackfl_amd.eval import cnn_eval_many

    ds = synthetic_icu(1000, seed=5)
    n = 333
    lay = ParamLayout.for_model("CNNModel")
    models = [build_model("CNNModel", seed=20 + i).eval() for i in range(3)]
    params = torch.stack([lay.flatten(m.state_dict()) for m in models])
    assert params.shape[1] % 4 != 0  # (203649: the padded-copy path)
    rows = torch.cat([ds.vitals[:n], ds.labs[:n], ds.labels[:n, None]], 1)
    out = cnn_eval_many(params.to(DEV), rows.to(DEV), lay).cpu()
    with torch.no_grad():
        ref = torch.stack([m(rows[:, :7], rows[:, 7:23]).reshape(-1) for m in models])
    assert out.shape == (3, n)
    err = (out - ref).abs()
    assert err.max().item() < 2e-2 and err.mean().item() < 3e-3, (err.max().item(), err.mean().item())
    # one model through Validation's path equals its row of the batched launch
    one = cnn_eval_many(params[1].to(DEV), rows.to(DEV), lay).cpu()
    assert torch.equal(one[0], out[1])


class _NullLog:
    def log_info(self, *a, **k):
        pass


def test_validation_prefetch_equals_direct(gpu):
    """Validation.prefetch (the engine queues the validation forward + AUC ahead of a speculative launch that
    fills the GPU) gives the direct test()'s metric, and falls back to a fresh evaluation when the model tensor
    changed in place after the prefetch."""
    from attackfl_amd.eval import Validation
    from attackfl_amd.data import synthetic_icu

    ds = synthetic_icu(700, seed=9)
    val = Validation("CNNModel", "ICU", _NullLog(), DEV, dataset=ds, verbose=False)
    lay = ParamLayout.for_model("CNNModel")
    flat = lay.flatten(build_model("CNNModel", seed=4).state_dict()).to(DEV)
    direct = val.test(flat)
    assert val.prefetch(flat)
    assert val.test(flat) == direct
    assert val.prefetch(flat)
    flat.mul_(1.5)  # (in place: the prefetched metric is stale)
    again = val.test(flat)
    val2 = Validation("CNNModel", "ICU", _NullLog(), DEV, dataset=ds, verbose=False)
    assert again == val2.test(flat)

def _har_slot_errors(res, lay):
    """Per ParamLayout slot: (relative norm error, max error / the slot's own max) of res[0] vs res[1]."""
    out = {}
    for sl in lay.slots:
        a, b = (r[:, sl.offset:sl.offset + sl.numel] for r in res)
        if float(b.abs().max()) == 0.0 and float(a.abs().max()) == 0.0:
            continue  # (the positional-encoding buffer: no gradient)
        out[sl.name] = (((a - b).norm() / (b.norm() + 1e-12)).item(),
                        ((a - b).abs().max() / (b.abs().max() + 1e-12)).item())
    return out


@pytest.mark.parametrize("B,drop", [(16, True), (24, False)])
def test_har_encoder_sgd_gradients_per_tensor(gpu, B, drop):
    """har.hip (the bf16 TransformerClassifier encoder: stem, q|k|v, flash attention, post / FFN row passes and
    their backward) at the reference shape L = 561, C = 2: one raw-SGD step exposes every gradient, compared
    PER TENSOR with the fp32 composite (CPU) on the same rows and dropout masks — each slot judged against its
    own scale, so a wrong LayerNorm / bias / conv gradient far below in_proj's magnitude cannot hide
    (reference model src/Model.py:418-458)."""
    C, n = 2, 4 * B
    ds = synthetic_har(n)
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:B] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32), torch.tensor([B] * C, dtype=torch.int32), 1)
    params = _params("TransformerClassifier", C)
    res, losses = [], []
    for dev in (DEV, "cpu"):
        p = params.clone().to(dev)
        ok, ls = ProgramRunner(make_program("TransformerClassifier", C, B, dev, dropout=drop), use_graph=False).train(
            DeviceTable(ds, dev), p, Plan(plan.order.to(dev), plan.nd, 1), lr=0.0, seeds=[3, 4], sgd_lr=1.0)
        assert ok.all()
        res.append(params - p.cpu())
        losses.append(ls.cpu())
    assert torch.allclose(losses[0], losses[1], rtol=1e-2), (losses[0], losses[1])
    errs = _har_slot_errors(res, ParamLayout.for_model("TransformerClassifier"))
    print({k: (round(a, 4), round(b, 4)) for k, (a, b) in errs.items()})
    bad = {k: v for k, v in errs.items() if v[0] > HAR_GRAD_NORM_TOL or v[1] > HAR_GRAD_MAX_TOL}
    assert not bad, bad


HAR_GRAD_NORM_TOL, HAR_GRAD_MAX_TOL = 0.10, 0.25


def test_har_encoder_adam_epochs_track_composite(gpu):
    """Three epochs of Adam (9 steps per client, dropout on) through the fused HAR path track the fp32
    composite: per-epoch losses, and per tensor the device-vs-composite deviation stays a small fraction of
    the distance the composite moved."""
    C, B, E, n = 2, 16, 3, 96
    ds = synthetic_har(n)
    nd = [48, 41]
    order = torch.stack([torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(10 * c + e))[:max(nd)]
                                      for e in range(E)]) for c in range(C)]).to(torch.int32)
    params = _params("TransformerClassifier", C)
    res, losses = [], []
    for dev in (DEV, "cpu"):
        p = params.clone().to(dev)
        ok, ls = ProgramRunner(make_program("TransformerClassifier", C, B, dev)).train(
            DeviceTable(ds, dev), p, Plan(order.to(dev), torch.tensor(nd, dtype=torch.int32), E), lr=1e-3,
            seeds=[5, 6])
        assert ok.all()
        res.append(p.cpu())
        losses.append(ls.cpu())
    assert torch.allclose(losses[0], losses[1], rtol=2e-2, atol=2e-3), (losses[0], losses[1])
    lay = ParamLayout.for_model("TransformerClassifier")
    ratios = {}
    for sl in lay.slots:
        a, b, p0 = (t[:, sl.offset:sl.offset + sl.numel] for t in (res[0], res[1], params))
        if sl.name.endswith("in_proj_bias"):
            # the key bias adds q.b_k to every score of a query row: softmax is shift-invariant, so its gradient is
            # exactly zero and Adam (m / sqrt(v)) turns the rounding noise of either side into full-size steps
            keep = torch.ones(sl.numel, dtype=torch.bool)
            keep[64:128] = False
            a, b, p0 = a[:, keep], b[:, keep], p0[:, keep]
        moved = (b - p0).norm().item()
        if moved == 0.0:
            continue
        ratios[sl.name] = round((a - b).norm().item() / moved, 4)
    print(ratios)
    # Adam's per-element normalisation amplifies bf16-operand differences where a gradient is small: a deviation
    # of a few tenths of the distance moved is that noise; a wrong gradient moves the tensor elsewhere (ratio >= 1)
    bad = {k: r for k, r in ratios.items() if r > HAR_ADAM_TOL}
    assert not bad, bad


HAR_ADAM_TOL = 0.4


@pytest.mark.parametrize("nd,B,E", [([700, 513, 300, 129, 0, 1], 128, 3), ([5, 64, 65], 64, 2), ([0, 0], 32, 1)])
def test_native_step_tables_match_tensor_ops(gpu, nd, B, E):
    """plan.hip k_step_tables (the cnn2 round boundary in one launch) equals the tensor-op step tables, and zeroes
    the per-round words it is given."""
    import math

    from attackfl_amd.fl.programs import step_tables, step_tables_native
    from attackfl_amd.fl.trainers import make_plan

    plan = make_plan(2000, [max(n, 1) for n in nd], E, torch.Generator().manual_seed(3), gpu)
    plan = Plan(plan.order, torch.tensor(nd, dtype=torch.int32), E)
    ref = step_tables(plan.order, plan.nd, E, B, gpu)
    S = max([E * max(1, math.ceil(n / B)) for n in nd] + [0])
    assert S == ref[4]
    zi = torch.full((37,), 7, dtype=torch.int32, device=gpu)
    zf = torch.full((5, 3), 2.5, device=gpu)
    got = step_tables_native(plan.order, plan.nd.to(gpu), S, B, zi, zf)
    for a, b in zip(got, ref[:4]):
        assert torch.equal(a.cpu(), b.cpu())
    assert int(zi.abs().sum()) == 0 and float(zf.abs().sum()) == 0.0
