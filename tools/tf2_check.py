"""Numerics + timing check of the fused TransformerModel trainers (split 3 vs the on-chip split 4)
against the fp32 oracle: per-tensor relative error of one raw SGD step, an Adam epoch, and the time
of a bench-sized round.  Diagnostics only (the pytest suite holds the assertions)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from attackfl_amd.data import synthetic_icu  # noqa: E402
from attackfl_amd.fl.trainers import make_plan  # noqa: E402
from attackfl_amd.models import ParamLayout, build_model  # noqa: E402
from attackfl_amd.ops import transformer as T  # noqa: E402


def setup(C, nd, seed=0, n=2000):
    ds = synthetic_icu(n, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1)
    lay = ParamLayout.for_model("TransformerModel")
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=seed + i).state_dict()) for i in range(C)])
    plan = make_plan(rows.shape[0], nd, 1, torch.Generator().manual_seed(7), "cpu")
    return rows, params, plan, lay


def main():
    dev = torch.device("cuda", 0)
    splits = [int(s) for s in (sys.argv[1:] or ["3", "4"])]
    rows, params, plan, lay = setup(2, [128, 100])
    ref = params.clone()
    T.reference_train(ref, rows, plan.order, plan.nd, 1, 128, 1.0, [11, 12], opt_mode=1, max_steps=1)
    for split in splits:
        d = params.clone().to(dev)
        ok, _ = T.train_clients(d, rows.to(dev), plan.order.to(dev), plan.nd, 1, 128, 1.0, [11, 12], opt_mode=1, split=split)
        gd, gr = params - d.cpu(), params - ref
        worst = []
        for s in lay.slots:
            a, b = gd[:, s.offset:s.offset + s.numel], gr[:, s.offset:s.offset + s.numel]
            sc = b.abs().max().item() + 1e-6
            worst.append(((a - b).abs().max().item() / sc, s.name))
        worst.sort(reverse=True)
        print(f"split {split}: ok={ok.tolist()} SGD worst rel err:", [(round(e, 4), n) for e, n in worst[:6]], flush=True)
    nd = [1100, 900]
    rows, params, plan, _ = setup(2, nd, seed=5)
    ref = params.clone()
    _, loss_r = T.reference_train(ref, rows, plan.order, plan.nd, 1, 128, 0.004, [3, 4])
    for split in splits:
        d = params.clone().to(dev)
        ok, loss = T.train_clients(d, rows.to(dev), plan.order.to(dev), plan.nd, 1, 128, 0.004, [3, 4], split=split)
        diff = (d.cpu() - ref).abs().mean().item()
        moved = (ref - params).abs().mean().item()
        print(f"split {split}: ok={ok.tolist()} adam diff/moved={diff / moved:.4f} loss={loss.tolist()} ref={loss_r.tolist()}", flush=True)
    # bench-sized round: 8 clients x 5 epochs x 13500 rows
    ds = synthetic_icu(60000, seed=1)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("TransformerModel")
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=i).state_dict()) for i in range(8)]).to(dev)
    plan = make_plan(60000, [13500] * 8, 5, torch.Generator().manual_seed(1), dev)
    for split in splits:
        for it in range(3):
            p = params.clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ok, loss = T.train_clients(p, rows, plan.order, plan.nd, 5, 128, 0.004, list(range(8)), split=split)
            t1 = time.perf_counter()
        steps = 5 * (13500 // 128 + 1)
        print(f"split {split}: round {1e3 * (t1 - t0):.2f} ms, {1e6 * (t1 - t0) / steps:.2f} us/step, ok={ok.tolist()}, "
              f"loss e0..4={[round(float(x), 4) for x in loss[0]]}", flush=True)


if __name__ == "__main__":
    main()
