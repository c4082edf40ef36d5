import sys, os
sys.path.insert(0, os.getcwd())
import torch
from attackfl_amd.fl.hyper_server import HyperServer
from attackfl_amd.models import build_model
from attackfl_amd import ops
for model, clip in (("RNNModel", 1e9),):
    sd = build_model(model, seed=0).state_dict()
    n = 5
    cpu = HyperServer(sd, n, 0.01, clip, "cpu", seed=3)
    dev = HyperServer(sd, n, 0.01, clip, "cuda", seed=3)
    g = torch.Generator().manual_seed(1)
    for i in [3, 0]:
        U = torch.randn(1, cpu.hnet.P, generator=g) * 0.1 + cpu.generate(i)[None]
        cpu.train([i], {i: U[0]})
        Ud = U.to("cuda")
        dev.train([i], {i: Ud[0]})
        a, b = dev.hnet.arena.cpu(), cpu.hnet.arena
        for name, (off, shp) in cpu.hnet.slots.items():
            n_ = 1
            for s in shp: n_ *= s
            d = (a[off:off+n_] - b[off:off+n_]).abs()
            k = int(d.argmax())
            print(i, name, shp, "maxdiff", float(d.max()), "at", k, "gpu", float(a[off+k]), "cpu", float(b[off+k]),
                  "m cpu", float(cpu.m[off+k]), "m gpu", float(dev.m[off+k].cpu()), "ndiff>1e-4", int((d > 1e-4).sum()))
