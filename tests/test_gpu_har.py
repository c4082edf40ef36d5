"""bf16 HAR encoder kernels (csrc/kernels/har.hip) against the fp32 composites of the layer program."""
import numpy as np
import pytest
import torch

from attackfl_amd.ops import layers as Lx
from attackfl_amd.ops import native

pytestmark = pytest.mark.gpu


def _ctl(C, dev):
    return Lx.StepCtl.create(list(range(3, 3 + C)), dev)


def _close(a, b, rel, name):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-12
    assert err <= rel * scale, (name, err, scale)


def _headmajor(qkv, B, L, Lp):
    """[C, B*L, 192] fp32 -> [C*B*4, 3, Lp, 16] bf16 (q scaled by log2(e) / 4, as the program stores it)."""
    C = qkv.shape[0]
    x = qkv.reshape(C, B, L, 3, 4, 16).permute(0, 1, 4, 3, 2, 5).clone()  # [C, B, H, 3, L, 16]
    x[:, :, :, 0] *= 0.25 * 1.4426950408889634
    out = torch.zeros(C, B, 4, 3, Lp, 16, dtype=torch.bfloat16, device=qkv.device)
    out[..., :L, :] = x.to(torch.bfloat16)
    return out.reshape(C * B * 4, 3, Lp, 16)


@pytest.mark.parametrize("L,p", [(50, 0.0), (561, 0.1), (200, 0.1)])
def test_har_attention_matches_composite(gpu, L, p):
    C, B = 2, 2
    g = torch.Generator().manual_seed(4)
    qkv = torch.randn(C, B * L, 192, generator=g)
    # bf16-exact inputs, so the composite sees what the kernel reads
    qkv = qkv.to(torch.bfloat16).float()
    dout = torch.randn(C, B * L, 64, generator=g).to(torch.bfloat16).float()
    Lp = (L + 63) // 64 * 64
    nat = native()
    ctl = _ctl(C, gpu)
    hm = _headmajor(qkv.to(gpu), B, L, Lp)
    # the composite sees the q the kernel reads (rounded after the log2(e)/4 scale)
    qr = hm.float().cpu().reshape(C, B, 4, 3, Lp, 16)[..., :L, :][:, :, :, 0] / (0.25 * 1.4426950408889634)
    qkv = qkv.reshape(C, B, L, 3, 4, 16).clone()
    qkv[:, :, :, 0] = qr.permute(0, 1, 3, 2, 4)
    qkv = qkv.reshape(C, B * L, 192)
    o = torch.zeros(C, B * L, 64, dtype=torch.bfloat16, device=gpu)
    lse2 = torch.zeros(C * B * 4, Lp, device=gpu)
    mask = torch.zeros(C * B * 4, nat.har_mask_words(Lp), dtype=torch.int64, device=gpu) if p else None
    nat.har_attn_fwd(hm, o, lse2, B, L, ctl.seeds if p else None, ctl.stepctl if p else None, 2, p, mask)
    cc = _ctl(C, "cpu")
    ref_o, ref_lse = Lx._attn_ref(qkv, B, L, cc, 2, p, "rc")
    _close(o, ref_o, 2e-2, "O")
    _close(lse2[:, :L] * np.log(2.0), ref_lse.reshape(-1, L), 1e-3, "lse")
    # backward: Delta from the kernel's own (bf16) O, as the post pass computes it
    ob = o.float()
    delta = torch.zeros(C * B * 4, Lp, device=gpu)
    dd = (dout.to(gpu) * ob).reshape(C, B, L, 4, 16).sum(-1).permute(0, 1, 3, 2).reshape(C * B * 4, L)
    delta[:, :L] = dd
    dq = torch.zeros_like(hm)
    nat.har_attn_bwd(hm, lse2, dout.to(gpu).to(torch.bfloat16), delta, dq, B, L, ctl.seeds if p else None,
                     ctl.stepctl if p else None, 2, p, mask)
    x = qkv.clone().requires_grad_(True)
    with torch.enable_grad():
        out, _ = Lx._attn_ref(x, B, L, cc, 2, p, "rc")
        (gref,) = torch.autograd.grad(out, x, dout)
    gq = gref.reshape(C, B, L, 3, 4, 16).permute(0, 1, 4, 3, 2, 5).reshape(C * B * 4, 3, L, 16)
    got = dq[:, :, :L].float().cpu()
    errs = {}
    for w, n in enumerate(["dq", "dk", "dv"]):
        e = (got[:, w] - gq[:, w]).abs().max().item() / (gq[:, w].abs().max().item() + 1e-12)
        if e > 3e-2:
            errs[n] = round(e, 4)
    assert not errs, errs


def _decode_keep_words(words, L, Lp):
    """[Lp/16, Lp/64, 4, 4] int64 ballot words of one (client, sample, head) -> bool [L, L] (query, key):
    word (T, c, t, e) bit 16 g + i = keep(query 16 T + i, key 64 c + 16 t + 4 g + e)."""
    w = words.reshape(Lp // 16, Lp // 64, 4, 4).numpy().view(np.uint64)
    bits = ((w[..., None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)  # [T, c, t, e, 64]
    bits = bits.reshape(Lp // 16, Lp // 64, 4, 4, 4, 16)  # [T, c, t, e, g, i]
    keep = bits.transpose(0, 5, 1, 2, 4, 3).reshape(Lp, Lp)  # [(T, i), (c, t, g, e)]
    return keep[:L, :L]


def test_har_attention_keep_words_match_keep_rc(gpu):
    """The forward's stored dropout flags are exactly masks.keep_rc (the draws both backward kernels use)."""
    from attackfl_amd.ops import masks

    C, B, L, p = 2, 2, 200, 0.1
    Lp = (L + 63) // 64 * 64
    nat = native()
    ctl = _ctl(C, gpu)
    qkv = torch.randn(C, B * L, 192, generator=torch.Generator().manual_seed(1))
    hm = _headmajor(qkv.to(gpu), B, L, Lp)
    o = torch.zeros(C, B * L, 64, dtype=torch.bfloat16, device=gpu)
    lse2 = torch.zeros(C * B * 4, Lp, device=gpu)
    mask = torch.zeros(C * B * 4, nat.har_mask_words(Lp), dtype=torch.int64, device=gpu)
    nat.har_attn_fwd(hm, o, lse2, B, L, ctl.seeds, ctl.stepctl, 12, p, mask)
    cc = _ctl(C, "cpu")
    words = mask.cpu()
    for cbh in (0, 5, C * B * 4 - 1):
        c, bh = divmod(cbh, B * 4)
        rows = (bh * L + np.arange(L))[:, None]
        ref = masks.keep_rc(cc.key(c), 12, rows, np.arange(L)[None, :], p).numpy()
        got = _decode_keep_words(words[cbh], L, Lp)
        assert (got == ref).all(), (cbh, int((got != ref).sum()))
        assert abs(got.mean() - 0.9) < 0.01


def test_har_post_keep_bits_match_afl_keep(gpu):
    """The row pass's stored dropout flags (``AflHarPost::kbits``, read back by the post backward instead of
    re-hashing) are exactly the layer library's ``afl_keep`` draws (``masks.keep``) of the three sites."""
    from attackfl_amd.fl.programs import make_program
    from attackfl_amd.models import ParamLayout, build_model
    from attackfl_amd.ops import masks

    C, B, L, p = 2, 2, 50, 0.1
    R = B * L
    nat = native()
    prog = make_program("TransformerClassifier", C, B, gpu)
    lay = ParamLayout.for_model("TransformerClassifier")
    params = torch.stack([lay.flatten(build_model("TransformerClassifier", seed=s).state_dict()) for s in range(C)]).to(gpu)
    g = torch.Generator().manual_seed(5)
    bf = torch.bfloat16
    o = torch.randn(C, R, 64, generator=g).to(gpu, bf)
    x = torch.randn(C, R, 64, generator=g).to(gpu, bf)
    xh1, xh2, y = (torch.zeros(C, R, 64, dtype=bf, device=gpu) for _ in range(3))
    rs = torch.zeros(C, R, 2, device=gpu)
    kb = torch.zeros(C, R, int(nat.har_kbits_per_row), dtype=torch.int32, device=gpu)
    ctl = _ctl(C, gpu)
    nat.har_post(o, x, xh1, xh2, rs, y, params, prog._lw(0), ctl.seeds, ctl.stepctl, 0, p, kb)
    words = kb.cpu().numpy().astype(np.uint32).reshape(C, R, 4, 4)  # [c][row][g][word]
    cc = _ctl(C, "cpu")
    rows = np.arange(R)[:, None]

    def decode(word, ntiles, t0):  # bit 4t + i <-> feature 16 (t0 + t) + 4g + i of the lane (row, g)
        out = np.zeros((R, 16 * (t0 + ntiles)), dtype=bool)
        for gg in range(4):
            w = word[:, gg]
            for t in range(ntiles):
                for i in range(4):
                    out[:, 16 * (t0 + t) + 4 * gg + i] = (w >> np.uint32(4 * t + i)) & np.uint32(1)
        return out[:, 16 * t0:]

    for c in range(C):
        w = words[c]
        d1 = decode(w[:, :, 0] & np.uint32(0xFFFF), 4, 0)
        d2 = decode(w[:, :, 0] >> np.uint32(16), 4, 0)
        df = np.concatenate([decode(w[:, :, 1], 8, 0), decode(w[:, :, 2], 8, 8)], axis=1)
        key = cc.key(c)
        for got, layer, n in ((d1, 1, 64), (df, 2, 256), (d2, 3, 64)):
            ref = masks.keep(key, layer, rows, np.arange(n)[None, :], p).numpy()
            assert (got == ref).all(), (c, layer, int((got != ref).sum()))
            assert abs(got.mean() - 0.9) < 0.03
