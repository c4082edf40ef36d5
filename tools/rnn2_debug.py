"""Diagnostics of the on-chip RNN trainer (rnn2.hip) against the composite program: per-configuration ok
flags, losses and the parameter distance, for SGD / Adam and one / several steps."""
import sys

import torch

sys.path.insert(0, ".")
from attackfl_amd.data import DeviceTable, synthetic_icu  # noqa: E402
from attackfl_amd.fl.programs import ProgramRunner, make_program  # noqa: E402
from attackfl_amd.fl.trainers import make_plan  # noqa: E402
from attackfl_amd.models import ParamLayout, build_model  # noqa: E402
from attackfl_amd.ops import rnn as R  # noqa: E402


def run(nd, E, lr, sgd, split=4):
    gpu = torch.device("cuda", 0)
    ds = synthetic_icu(3000, seed=3)
    lay = ParamLayout.for_model("RNNModel")
    C = len(nd)
    params = torch.stack([lay.flatten(build_model("RNNModel", seed=i).state_dict()) for i in range(C)])
    plan = make_plan(len(ds), nd, E, [101 + i for i in range(C)], "cpu")
    seeds = [5 + i for i in range(C)]
    ref = params.clone()
    ok_r, loss_r = ProgramRunner(make_program("RNNModel", C, 128, "cpu")).train(
        DeviceTable(ds, "cpu"), ref, plan, lr=0.0 if sgd else lr, seeds=seeds, sgd_lr=lr if sgd else 0.0)
    dev = params.clone().to(gpu)
    ok, loss = R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, E, 128, lr, seeds,
                               opt_mode=1 if sgd else 0, split=split)
    d = dev.cpu()
    moved = (ref - params).abs().mean().item()
    print(f"nd={nd} E={E} sgd={sgd} split={split}: ok={ok.tolist()} ref_ok={ok_r.tolist()} loss={loss.tolist()} "
          f"ref_loss={loss_r.tolist()} dist/moved={(d - ref).abs().mean().item() / max(moved, 1e-30):.4f} "
          f"nan={int(torch.isnan(d).sum())}", flush=True)
    if not torch.isfinite(d).all() or (d - ref).abs().mean().item() > 0.2 * moved:
        worst = []
        for s in lay.slots:
            a = d[:, s.offset:s.offset + s.numel]
            b = ref[:, s.offset:s.offset + s.numel]
            m = (b - params[:, s.offset:s.offset + s.numel]).abs().mean().item()
            worst.append(((a - b).abs().mean().item() / max(m, 1e-30), s.name, int(torch.isnan(a).sum())))
        worst.sort(key=lambda t: -t[0] if t[0] == t[0] else -1e30)
        print("   worst slots:", worst[:8], flush=True)




def nan_pattern(nd, E, lr, sgd):
    gpu = torch.device("cuda", 0)
    ds = synthetic_icu(3000, seed=3)
    lay = ParamLayout.for_model("RNNModel")
    C = len(nd)
    params = torch.stack([lay.flatten(build_model("RNNModel", seed=i).state_dict()) for i in range(C)])
    plan = make_plan(len(ds), nd, E, [101 + i for i in range(C)], "cpu")
    dev = params.clone().to(gpu)
    R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, E, 128, lr, [5 + i for i in range(C)],
                    opt_mode=1 if sgd else 0)
    d = dev.cpu()
    for s in lay.slots:
        a = d[:, s.offset:s.offset + s.numel]
        bad = (~torch.isfinite(a)).nonzero().tolist()
        big = (a.abs() > 100).nonzero().tolist()
        if bad or big:
            print(f"  {s.name} shape={tuple(s.shape)} nonfinite={bad[:40]} big={big[:20]}", flush=True)


def trap(nd, E, lr, sgd):
    gpu = torch.device("cuda", 0)
    ds = synthetic_icu(3000, seed=3)
    lay = ParamLayout.for_model("RNNModel")
    C = len(nd)
    params = torch.stack([lay.flatten(build_model("RNNModel", seed=i).state_dict()) for i in range(C)])
    plan = make_plan(len(ds), nd, E, [101 + i for i in range(C)], "cpu")
    dev = params.clone().to(gpu)
    st = torch.zeros(64, dtype=torch.int64, device=gpu)
    R.train_clients_async(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, E, 128, lr,
                          [5 + i for i in range(C)], opt_mode=1 if sgd else 0, stamps=st)
    torch.cuda.synchronize()
    rec = st.cpu()
    print("trap flag", int(rec[0]), "rec", rec[1:10].view(torch.float32).tolist(), flush=True)
    print("nan count", int(torch.isnan(dev).sum()), flush=True)


if __name__ == "__main__":
    nan_pattern([256, 256], 1, 0.5, True)
    nan_pattern([384, 300, 700], 1, 0.004, False)
    run([384, 300], 2, 0.004, False)
