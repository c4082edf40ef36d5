"""Where do the fused-generation update and the plain update differ (regions of the arena / moments)?"""
import torch
from attackfl_amd.fl.hyper_server import HyperServer
from attackfl_amd.models import build_model

gpu = torch.device("cuda", 0)
sd = build_model("TransformerModel", seed=0).state_dict()
n = 12
srv = [HyperServer(sd, n, 0.01, 0.05, gpu, seed=3) for _ in range(3)]
g = torch.Generator().manual_seed(2)
sel = [3, 0, 4, 1, 7]
gen = [1, 6, 11]
r = torch.randn(len(sel), srv[0].hnet.P, generator=g).to(gpu)
U = torch.stack([srv[0].generate(i) for i in sel]) - 0.1 * torch.sign(r) * (0.5 + r.abs())
on = torch.ones(1, dtype=torch.int32, device=gpu)
srv[0].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=on, gen_key=gen)
srv[1].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=on)
srv[2].train(sel, {i: U[k] for k, i in enumerate(sel)}, enable=on)
h = srv[0].hnet
offW, _ = h.slots["W"]
offB, _ = h.slots["b"]
regions = {"small": (0, offW), "W": (offW, offB), "b": (offB, h.arena.numel())}
for name, t in (("arena", lambda s: s.hnet.arena), ("m", lambda s: s.m), ("v", lambda s: s.v)):
    for rn, (a, b) in regions.items():
        x, y, z = t(srv[0])[a:b], t(srv[1])[a:b], t(srv[2])[a:b]
        d = (x != y).nonzero().reshape(-1)
        print(name, rn, "fused!=plain", d.numel(), "first", d[:5].tolist(), "max", float((x - y).abs().max()),
              "| plain!=plain", int((y != z).sum()))
