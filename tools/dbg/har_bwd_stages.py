"""Debug: one HAR step (dropout on) with the fused backward run stage by stage; prints the NaN count of every
stage's outputs, so the first kernel that produces a NaN is named.

    python tools/dbg/har_bwd_stages.py [--B 4] [--n 24] [--p-off]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from attackfl_amd import ops
from attackfl_amd.data import DeviceTable, synthetic_har
from attackfl_amd.fl.programs import make_program, step_tables
from attackfl_amd.fl.trainers import Plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import layers as Lx
from attackfl_amd.ops.layers import ACT_RELU, StepCtl


def nan(t):
    return int(torch.isnan(t.float()).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--C", type=int, default=2)
    a = ap.parse_args()
    C, B, n = a.C, a.B, a.n
    ds = synthetic_har(n)
    lay = ParamLayout.for_model("TransformerClassifier")
    params = torch.stack([lay.flatten(build_model("TransformerClassifier", seed=s).state_dict()) for s in range(C)])
    P = (lay.P + 15) // 16 * 16
    pp = torch.zeros(C, P)
    pp[:, :lay.P] = params
    params = pp.cuda()
    grads = torch.zeros(C, P, device="cuda")
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:B] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32).cuda(), torch.tensor([B] * C, dtype=torch.int32), 1)
    pg = make_program("TransformerClassifier", C, B, "cuda")
    idx, bsz, ep, nb, S = step_tables(plan.order, plan.nd, plan.epochs, pg.B, "cuda")
    ctl = StepCtl.create([3, 4][:C] if C <= 2 else list(range(C)), "cuda", min_bs=2, nan_abort=True)
    table = DeviceTable(ds, "cuda")
    failed = torch.zeros(C, dtype=torch.int32, device="cuda")
    losses = torch.zeros(C, 1, device="cuda")
    pg.inputs(table, idx, ctl)
    out = pg.forward(params, ctl)
    torch.cuda.synchronize()
    print("forward: logits nan", nan(out), "fused", pg._fused(params))
    dz = pg.buf("dz", *out.shape)
    Lx.ce(out, pg.labels(), bsz, ep, nb, ctl, failed, losses, dz)
    nat = ops.native()
    L = pg.L
    R, Lp, G = B * L, pg._lp(), pg._groups()
    bf = torch.bfloat16
    p = pg.p(0.1)
    seeds, stepctl = ctl.seeds, ctl.stepctl
    dlog, dc1, dpool = pg.buf("dz", C, B, 6), pg.buf("dc1", C, B, 64), pg.buf("dpool", C, B, 64)
    c1 = pg.buf("c1", C, B, 64)
    pg.linear_bwd(dlog, c1, params, grads, "classifier.3.weight", "classifier.3.bias", dc1, G=c1,
                  gact=ACT_RELU, ctl=ctl, layer=30, p=0.3)
    pg.linear_bwd(dc1, pg.buf("pool", C, B, 64), params, grads, "classifier.0.weight", "classifier.0.bias", dpool)
    torch.cuda.synchronize()
    print("head bwd: dpool nan", nan(dpool), "loss", losses.flatten().tolist())
    ws_p = pg.buf("ws_post", C * G * int(nat.har_post_ng))
    ws_q = pg.buf("ws_qkv", C * G * int(nat.har_qkv_ng))
    dres, dout = pg.buf("dres", C, R, 64), pg.buf("doutb", C, R, 64, dtype=bf)
    delta, dqkv = pg.buf("delta", C * B * 4, Lp), pg.buf("dqkvb", C * B * 4, 3, Lp, 16, dtype=bf)
    dxs = [pg.buf("dxA", C, R, 64), pg.buf("dxB", C, R, 64)]
    dy = None
    for i in reversed(range(pg.NL)):
        w = pg._lw(i)
        for nm in ("ob", "xh1_", "xh2_", "rs", "qkvb", "lse2_"):
            key = f"{nm}{i}"
            t = pg._bufs.get(key)
            if t is not None and nan(t):
                print(f"  input {key} nan {nan(t)}")
        nat.har_post_bwd(dy, dpool if dy is None else None, B, L, pg.buf(f"ob{i}", C, R, 64, dtype=bf),
                         pg.buf(f"xh1_{i}", C, R, 64, dtype=bf), pg.buf(f"xh2_{i}", C, R, 64, dtype=bf),
                         pg.buf(f"rs{i}", C, R, 2), dres, dout, delta, ws_p, params, w, seeds, stepctl, 10 * i,
                         p, G, pg._kbits(i))
        torch.cuda.synchronize()
        print(f"layer {i} post_bwd: dres {nan(dres)} dout {nan(dout)} delta {nan(delta)} ws {nan(ws_p)}")
        nat.har_attn_bwd(pg.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf), pg.buf(f"lse2_{i}", C * B * 4, Lp),
                         dout, delta, dqkv, B, L, seeds, stepctl, 10 * i, p, pg._mask(i))
        torch.cuda.synchronize()
        dq = dqkv.view(C * B * 4, 3, Lp, 16)
        print(f"layer {i} attn_bwd: dq {nan(dq[:, 0])} dk {nan(dq[:, 1])} dv {nan(dq[:, 2])} "
              f"(valid rows: dq {nan(dq[:, 0, :L])} dk {nan(dq[:, 1, :L])} dv {nan(dq[:, 2, :L])})")
        if nan(dq[:, 0]):
            rows = torch.isnan(dq[0, 0].float()).any(-1).nonzero().flatten().tolist()
            print("   cbh 0 NaN dq rows:", len(rows), rows[:40])
            per = torch.isnan(dq[:, 0].float()).any(-1).sum(-1).tolist()
            print("   NaN rows per cbh:", per)
            # same buffers, no dropout: does the NaN persist?
            dq2 = torch.zeros_like(dqkv)
            nat.har_attn_bwd(pg.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf), pg.buf(f"lse2_{i}", C * B * 4, Lp),
                             dout, delta, dq2, B, L, None, None, 10 * i, 0.0, None)
            torch.cuda.synchronize()
            print("   no-dropout rerun: dq nan", nan(dq2[:, 0]), "dk", nan(dq2[:, 1]), "dv", nan(dq2[:, 2]))
            dq3 = torch.zeros_like(dqkv)
            nat.har_attn_bwd(pg.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf), pg.buf(f"lse2_{i}", C * B * 4, Lp),
                             dout, delta, dq3, B, L, seeds, stepctl, 10 * i, p, pg._mask(i))
            torch.cuda.synchronize()
            print("   dropout rerun: dq nan", nan(dq3[:, 0]), "same bits as first", torch.equal(dq3.view(torch.int16), dqkv.view(torch.int16)))
            qk = pg.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf).float()
            lse = pg.buf(f"lse2_{i}", C * B * 4, Lp)
            s2 = torch.einsum("bqd,bkd->bqk", qk[:, 0, :L], qk[:, 1, :L])
            print("   max(s - lse2) over valid", (s2 - lse[:, :L, None]).max().item())
            print("   dout absmax", dout.float().abs().max().item(), "delta absmax", delta.abs().max().item())
        if nan(dq[:, 1]) or nan(dq[:, 2]):
            lse = pg.buf(f"lse2_{i}", C * B * 4, Lp)
            qk = pg.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf)
            print("   lse2 valid min/max", lse[:, :L].min().item(), lse[:, :L].max().item(), "pad", lse[:, L:].min().item(),
                  "| qkv pad absmax", qk[:, :, L:].float().abs().max().item(), "| delta pad absmax",
                  delta[:, L:].abs().max().item())
        dx = dxs[i % 2]
        nat.har_qkv_bwd(dqkv, dres, pg.buf(f"hb{i}", C, R, 64, dtype=bf), dx, ws_q, params, w[0], B, L, G)
        torch.cuda.synchronize()
        print(f"layer {i} qkv_bwd: dx {nan(dx)} ws {nan(ws_q)}")
        dy = dx


if __name__ == "__main__":
    main()
