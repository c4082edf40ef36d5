"""Per-phase wall-clock breakdown of the fused training kernels (TransformerModel: tf2 / transformer.hip,
RNNModel: rnn2.hip with --model RNNModel), one stamped workgroup.

Runs one client's local round (default 13500 rows, 5 epochs) with the stamps buffer enabled and prints
microseconds per phase per step.  Usage: python tools/phase_profile.py [--rows N] [--clients C]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from attackfl_amd.data import synthetic_icu
from attackfl_amd.fl.trainers import make_plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import rnn as R
from attackfl_amd.ops import transformer as T

NAMES = {0: "F:G1 dense+E1", 1: "F:G2 vproj+E2", 2: "F:G3 oproj+E3 LN1", 3: "F:G4 ffn0+E4", 4: "F:G5 ffn3+E5 LN2/3",
         5: "F:branch tail", 6: "H:fc1+E6", 7: "H:fc2+E7 loss", 8: "H:bwd fc2 dX+E8", 9: "H:dcat+dWf2+dWf1",
         10: "B:E10 LN bwd", 11: "B:A10+G11", 12: "B:E11", 13: "B:G12+dW2", 14: "B:E12 LN1 bwd", 15: "B:G13+dW1",
         16: "B:E13", 17: "B:(none)", 18: "B:G14+dWo", 19: "B:E14+dWv", 20: "B:E15+dWd",
         21: "X:publish+wait d(out)"}
# on-chip trainer (split 4, tf2.hip): branch workgroups (blocks 3c+1, 3c+2) and the head (3c)
NAMES4 = {0: "B:forward", 1: "B:publish+prefetch", 2: "B:wait d(out)", 3: "B:backward",
          4: "B:wait counter (A leaders / B laggards)+abort",
          5: "B:leaders out_proj+v units / laggards small tiles", 6: "B:bar 1 + sums, staging + bar 2",
          7: "B:U3 compact Adam", 8: "B:end barrier", 10: "H:wait branches", 11: "H:fwd+loss+bwd+publish", 12: "H:bar+loss",
          13: "H:dW+Adam", 14: "H:end barrier"}

def block_stride(clients: int, wgs: int, dev) -> int:
    """tf2.hip's role-major block stride: C padded to a multiple of 8 when the padded grid still fits."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    cp = -(-clients // 8) * 8
    return cp if wgs * cp <= cus else clients


# on-chip RNN trainer (rnn2.hip): branch workgroups and the head
NAMES_RNN_B = {0: "B:forward (3 GRU layers + LN)", 1: "B:publish+prefetch", 2: "B:wait d(out)", 3: "B:LN bwd + layer-3 bwd",
               4: "B:barrier A3 + abort", 5: "B:dW3+Adam (+bar B3)", 6: "B:layer-2 bwd (+bar A2)",
               7: "B:dW2+Adam (+bar B2)", 8: "B:layer-1 gate bwd (+bar A1)", 9: "B:dW1 staging (+bar C)",
               10: "B:compact Adam", 11: "B:end barrier"}
NAMES_RNN_H = {0: "H:wait branches", 1: "H:fwd+loss+bwd+publish", 2: "H:tiles+bar+loss", 3: "H:dW+Adam",
               4: "H:end barrier"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=13500)
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--opt-mode", type=int, default=0, help="1 = SGD test mode (no Adam moments)")
    ap.add_argument("--split", type=int, default=0, help="workgroups per client (1, 2, 3); 0 = auto")
    ap.add_argument("--block", type=int, default=0, help="workgroup whose phases are stamped (-1: 0, 1, 2 in turn)")
    ap.add_argument("--model", default="TransformerModel")
    ap.add_argument("--wave", type=int, default=0, help="stamping wave of the workgroup (-1: 0..7 in turn; tf2 only)")
    args = ap.parse_args()
    if args.model == "RNNModel":
        return main_rnn(args)
    dev = torch.device("cuda", 0)
    blocks = [0, 1, 2] if args.block < 0 else [args.block]
    ds = synthetic_icu(60000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("TransformerModel")
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=i).state_dict())
                          for i in range(args.clients)]).to(dev)
    plan = make_plan(rows.shape[0], [args.rows] * args.clients, args.epochs, torch.Generator().manual_seed(0), "cpu")
    order = plan.order.to(dev)
    split = None if args.split <= 0 else args.split
    T.train_clients(params.clone(), rows, order, plan.nd, args.epochs, 128, 0.004, list(range(args.clients)),
                    split=split)
    torch.cuda.synchronize()
    used = split or T.auto_split(args.clients, dev)
    for b in blocks:
        for wv in (range(8) if args.wave < 0 else [args.wave]):
            run(args, dev, rows, order, plan, params, split, used, b, wv)


def run(args, dev, rows, order, plan, params, split, used, block, wave=0):
    names = NAMES4 if used == 4 else NAMES
    stamps = torch.zeros(64, dtype=torch.int64, device=dev)
    # role-major block order: role r of client 0 is block r * CP (the padded stride of the on-chip trainers)
    stamps[63] = block * (block_stride(args.clients, 3, dev) if used == 4 else args.clients)
    stamps[62] = wave
    t0 = time.perf_counter()
    T.train_clients(params.clone(), rows, order, plan.nd, args.epochs, 128, 0.004, list(range(args.clients)),
                    opt_mode=args.opt_mode, stamps=stamps, split=split)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = args.epochs * ((args.rows + 127) // 128)
    st = stamps.cpu().tolist()[:63]
    tot = sum(st)
    out = {"split": used, "block": block, "wave": wave, "opt_mode": args.opt_mode, "clients": args.clients, "wall_ms": wall * 1e3, "steps": steps, "us_per_step_wall": wall * 1e6 / steps,
           "us_per_step_stamped": tot * 0.01 / steps, "phases_us_per_step": {}}
    for i, v in enumerate(st):
        if v:
            out["phases_us_per_step"][f"{i:02d} {names.get(i, '?')}"] = round(v * 0.01 / steps, 3)
    print(json.dumps(out, indent=1))


def main_rnn(args):
    blocks = [0, 1, 2] if args.block < 0 else [args.block]
    dev = torch.device("cuda", 0)
    ds = synthetic_icu(60000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("RNNModel")
    params = torch.stack([lay.flatten(build_model("RNNModel", seed=i).state_dict())
                          for i in range(args.clients)]).to(dev)
    plan = make_plan(rows.shape[0], [args.rows] * args.clients, args.epochs, torch.Generator().manual_seed(0), "cpu")
    order = plan.order.to(dev)
    seeds = list(range(args.clients))
    R.train_clients(params.clone(), rows, order, plan.nd, args.epochs, 128, 0.004, seeds)
    torch.cuda.synchronize()
    steps = args.epochs * ((args.rows + 127) // 128)
    for b, wv in [(b, wv) for b in blocks for wv in (range(8) if args.wave < 0 else [args.wave])]:
        stamps = torch.zeros(64, dtype=torch.int64, device=dev)
        stamps[63] = b * args.clients  # role-major block order: role r of client 0 is block r * C
        stamps[62] = wv
        t0 = time.perf_counter()
        R.train_clients(params.clone(), rows, order, plan.nd, args.epochs, 128, 0.004, seeds, opt_mode=args.opt_mode,
                        stamps=stamps)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        names = NAMES_RNN_H if b == 0 else NAMES_RNN_B
        st = stamps.cpu().tolist()[:63]
        out = {"model": "RNNModel", "block": b, "wave": wv, "clients": args.clients, "wall_ms": wall * 1e3, "steps": steps,
               "us_per_step_wall": wall * 1e6 / steps, "us_per_step_stamped": sum(st) * 0.01 / steps,
               "phases_us_per_step": {f"{i:02d} {names.get(i, '?')}": round(v * 0.01 / steps, 3)
                                      for i, v in enumerate(st) if v}}
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
