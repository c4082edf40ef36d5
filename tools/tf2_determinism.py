"""Determinism check of the fused TransformerModel trainers: the same clients trained (a) twice with the
same launch, (b) inside launches of different client counts must give bit-identical parameters (the
multi-rank engine relies on it: a client's result may not depend on which rank or launch trains it).
Diagnostics only; tests/test_gpu_transformer.py holds the assertion."""
import sys

import torch

sys.path.insert(0, ".")
from attackfl_amd.data import synthetic_icu  # noqa: E402
from attackfl_amd.fl.trainers import make_plan  # noqa: E402
from attackfl_amd.models import ParamLayout, build_model  # noqa: E402
from attackfl_amd.ops import transformer as T  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    splits = [int(s) for s in (sys.argv[1:] or ["3", "4"])]
    ds = synthetic_icu(5000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("TransformerModel")
    C = 4
    nd = [700, 650, 900, 801]
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=i).state_dict()) for i in range(C)]).to(dev)
    plan = make_plan(rows.shape[0], nd, 2, torch.Generator().manual_seed(7), dev)
    seeds = [101, 102, 103, 104]
    for split in splits:
        outs = []
        for rep in range(2):
            p = params.clone()
            ok, loss = T.train_clients(p, rows, plan.order, plan.nd, 2, 128, 0.004, seeds, split=split)
            outs.append(p)
        same = [bool(torch.equal(outs[0][c], outs[1][c])) for c in range(C)]
        md = (outs[0] - outs[1]).abs().max().item()
        print(f"split {split}: repeat bit-identical per client={same} maxdiff={md:.3e}", flush=True)
        sub = []
        for lo in (0, 2):
            p = params[lo:lo + 2].clone()
            T.train_clients(p, rows, plan.order[lo:lo + 2].contiguous(), plan.nd[lo:lo + 2], 2, 128, 0.004,
                            seeds[lo:lo + 2], split=split)
            sub.append(p)
        sub = torch.cat(sub)
        same = [bool(torch.equal(outs[0][c], sub[c])) for c in range(C)]
        md = (outs[0] - sub).abs().max().item()
        print(f"split {split}: C=4 vs 2x C=2 bit-identical per client={same} maxdiff={md:.3e}", flush=True)
        for c in range(C):
            d = (outs[0][c] - sub[c]).abs()
            if d.max() > 0:
                worst = sorted(((d[s.offset:s.offset + s.numel].max().item(), s.name) for s in lay.slots), reverse=True)[:4]
                print(f"   client {c}: worst slots {worst}", flush=True)


if __name__ == "__main__":
    main()
