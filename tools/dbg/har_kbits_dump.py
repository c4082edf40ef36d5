"""Debug: one HAR SGD step with dropout on; reports NaNs per program buffer and the keep-bit density.

    python tools/dbg/har_kbits_dump.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from attackfl_amd.data import DeviceTable, synthetic_har
from attackfl_amd.fl.programs import ProgramRunner, make_program
from attackfl_amd.fl.trainers import Plan
from attackfl_amd.models import ParamLayout, build_model


def main():
    C, B, n = 2, 4, 24
    ds = synthetic_har(n)
    lay = ParamLayout.for_model("TransformerClassifier")
    params = torch.stack([lay.flatten(build_model("TransformerClassifier", seed=s).state_dict()) for s in range(C)])
    order = torch.stack([torch.randperm(n, generator=torch.Generator().manual_seed(c))[:B] for c in range(C)])
    plan = Plan(order[:, None, :].to(torch.int32).cuda(), torch.tensor([B] * C, dtype=torch.int32), 1)
    prog = make_program("TransformerClassifier", C, B, "cuda")
    p = params.clone().cuda()
    ok, losses = ProgramRunner(prog, use_graph=False).train(DeviceTable(ds, "cuda"), p, plan, lr=0.0, seeds=[3, 4],
                                                            sgd_lr=1.0)
    torch.cuda.synchronize()
    print("ok", ok.tolist(), "losses", losses.tolist())
    for name, t in sorted(prog._bufs.items()):
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            continue
        if t.dtype in (torch.float32, torch.bfloat16):
            nn = int(torch.isnan(t.float()).sum())
            print(f"{name:12s} {tuple(t.shape)} nan {nn} absmax {t.float().nan_to_num().abs().max().item():.3e}")
        elif t.dtype == torch.int32 and name.startswith("kbits"):
            u = t.view(-1, 4).cpu().numpy().astype("uint32")
            import numpy as np
            bits = np.unpackbits(u[:, :3].copy().view(np.uint8)).mean()
            print(f"{name:12s} {tuple(t.shape)} bit density (words 0-2) {bits:.3f}; word3 nonzero {int((u[:, 3] != 0).sum())}")
    d = (params - p.cpu())
    bad = torch.isnan(d)
    print("SUMMARY", os.environ.get("AFL_NATIVE_SO", "_C.so"), "nan grads", int(bad.sum()))
    for s in lay.slots:
        seg = bad[:, s.offset:s.offset + s.numel]
        if seg.any():
            print("NaN grad:", s.name, int(seg.sum()))


if __name__ == "__main__":
    main()
