"""Micro-benchmark of the flash-attention kernels at the HAR shape (L=561, 4 heads x 16).

    python tools/attn_bench.py [--clients 8] [--batch 64] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from attackfl_amd.ops import layers as Lx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--L", type=int, default=561)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    C, B, L = a.clients, a.batch, a.L
    dev = torch.device("cuda")
    qkv = torch.randn(C, B * L, 192, device=dev)
    o = torch.zeros(C, B * L, 64, device=dev)
    lse = torch.zeros(C * B * 4, Lx.attn_lp(L), device=dev)
    dout = torch.randn(C, B * L, 64, device=dev)
    dq = torch.zeros(C, B * L, 192, device=dev)
    ctl = Lx.StepCtl.create(list(range(C)), dev)
    res = {}
    for p in (0.0, 0.1):
        for name, fn in (("fwd", lambda: Lx.attn_fwd(qkv, o, lse, B, L, ctl, 3, p)),
                         ("bwd", lambda: Lx.attn_bwd(qkv, o, lse, dout, dq, B, L, ctl, 3, p))):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            flops = 4 * C * B * 4 * L * L * 16 * (1 if name == "fwd" else 2.5)
            res[f"{name}_p{p}"] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 2)}
    print(json.dumps({"C": C, "B": B, "L": L, **res}))


if __name__ == "__main__":
    main()
