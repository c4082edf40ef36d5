"""Micro-benchmark of the client-batched GEMM (``Lx.bgemm``) at the HAR TransformerClassifier step
shapes (8 clients x 128 sequences x L=561 rows, d_model 64, FFN 256): forward X.W^T, input gradient
dY.W and weight gradient dY^T.X, each next to the fp32-activation HBM floor (bytes the op must move
at 8 TB/s) and to torch.bmm in bf16 (the library GEMM, operands already bf16, no epilogue).

    python tools/gemm_bench.py [--clients 8] [--rows 71808] [--iters 20]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from attackfl_amd.ops import layers as Lx  # noqa: E402

# (name, kind, N, K): fwd/dx: Y[M,N] = X[M,K] W^T ; dw: G[N,K] = dY[M,N]^T X[M,K]
SHAPES = [("qkv", "fwd", 192, 64), ("out", "fwd", 64, 64), ("lin1", "fwd", 256, 64), ("lin2", "fwd", 64, 256),
          ("lin2.dx", "dx", 256, 64), ("lin1.dx", "dx", 64, 256), ("qkv.dx", "dx", 64, 192), ("out.dx", "dx", 64, 64),
          ("qkv.dw", "dw", 192, 64), ("lin1.dw", "dw", 256, 64), ("lin2.dw", "dw", 64, 256), ("out.dw", "dw", 64, 64)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rows", type=int, default=128 * 561)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C, M = a.clients, a.rows
    dev = torch.device("cuda")
    ctl = Lx.StepCtl.create(list(range(C)), dev)
    out = {"C": C, "M": M}
    tot = {"afl": 0.0, "floor": 0.0}
    for name, kind, N, K in SHAPES:
        W = torch.randn(C, N, K, device=dev) * 0.05
        bias = torch.randn(C, N, device=dev) * 0.05
        if kind == "fwd":
            X = torch.randn(C, M, K, device=dev)
            Y = torch.empty(C, M, N, device=dev)
            relu = name == "lin1"
            fn = lambda: Lx.bgemm(X, W, Y, bias=bias, act=Lx.ACT_RELU if relu else 0, ctl=ctl, layer=2,  # noqa: E731
                                  p=0.1 if relu else 0.0)
            nbytes = 4 * C * M * (K + N)
            Xb, Wb = X.bfloat16(), W.bfloat16()
            lib = lambda: torch.bmm(Xb, Wb.transpose(1, 2))  # noqa: E731
        elif kind == "dx":  # dX[M,K'] = dY[M,N'] W[N',K'] with (N', K') = (K, N) of the forward layer
            dY = torch.randn(C, M, K, device=dev)
            Wf = torch.randn(C, K, N, device=dev) * 0.05
            G = torch.randn(C, M, N, device=dev)
            dX = torch.empty(C, M, N, device=dev)
            gact = Lx.ACT_RELU if name == "lin2.dx" else 0
            fn = lambda: Lx.bgemm(dY, Wf.transpose(1, 2), dX, G=G if gact else None, gact=gact,  # noqa: E731
                                  ctl=ctl, layer=2, p=0.1 if gact else 0.0)
            nbytes = 4 * C * M * (K + N * (2 if gact else 1))
            dYb, Wfb = dY.bfloat16(), Wf.bfloat16()
            lib = lambda: torch.bmm(dYb, Wfb)  # noqa: E731
        else:
            dY = torch.randn(C, M, N, device=dev)
            X = torch.randn(C, M, K, device=dev)
            gW = torch.zeros(C, N, K, device=dev)
            tiles = math.ceil(N / 64) * math.ceil(K / 64) * C
            splitk = max(1, min(M // 256, math.ceil(1024 / tiles)))

            def fn(dY=dY, X=X, gW=gW, splitk=splitk):
                gW.zero_()
                Lx.bgemm(dY.transpose(1, 2), X.transpose(1, 2), gW, accum=2 if splitk > 1 else 0, splitk=splitk)
            nbytes = 4 * C * M * (N + K)
            dYb, Xb = dY.bfloat16(), X.bfloat16()
            lib = lambda: torch.bmm(dYb.transpose(1, 2), Xb)  # noqa: E731
        ms = timeit(fn, a.iters)
        ms_lib = timeit(lib, a.iters)
        floor = nbytes / 8e12 * 1e3
        tot["afl"] += ms
        tot["floor"] += floor
        out[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1), "floor_ms": round(floor, 4),
                     "bmm_bf16_ms": round(ms_lib, 4), "tflops": round(2 * C * M * N * K / ms / 1e9, 1)}
        print(name, json.dumps(out[name]), flush=True)
    out["total"] = {k: round(v, 3) for k, v in tot.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
