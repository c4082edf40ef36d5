"""Which host calls synchronise the device in a steady-state round?  torch.cuda.set_sync_debug_mode("warn") on
the bench configuration, every warning printed with its stack (first occurrence of each call site).

  python tools/dbg/sync_debug.py --mode FLTrust --attackers 7:Min-Max:2
"""
import argparse
import os
import sys
import tempfile
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from attackfl_amd.config import from_dict  # noqa: E402
from attackfl_amd.fl.engine import FLEngine, build_client_table  # noqa: E402
from attackfl_amd.parallel.comm import LoopbackComm  # noqa: E402
from launch import parse_attackers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--attackers", default=None)
    ap.add_argument("--model", default="TransformerModel")
    ap.add_argument("--mode", default="fedavg")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tmp = tempfile.mkdtemp(prefix="afl_syncdbg_")
    cfg = from_dict({
        "server": {"num-round": args.steps + 20, "clients": 8, "mode": args.mode, "model": args.model,
                   "data-name": "ICU", "validation": True, "data-distribution": {"num-data-range": [12000, 15000]}},
        "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 60000, "test-size": 10000},
        "engine": {"trainer": "auto", "checkpoint-dir": tmp, "seed": 1}, "log_path": tmp})
    table = build_client_table(cfg, 1, parse_attackers(args.attackers) if args.attackers else None)
    eng = FLEngine(cfg, comm=LoopbackComm(dev), table=table, device=dev, verbose=False)
    eng.client_selection()
    for _ in range(6):
        eng.run_round()
    torch.cuda.synchronize()
    seen = set()

    def show(message, category, filename, lineno, file=None, line=None):
        st = traceback.extract_stack()[:-2]
        key = tuple((f.filename, f.lineno) for f in st[-6:])
        if key in seen:
            return
        seen.add(key)
        print("SYNC:", message)
        for f in st[-8:]:
            print(f"    {f.filename}:{f.lineno} {f.name}: {f.line}")

    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    for r in range(args.steps):
        print(f"-- round {r}")
        eng.run_round()
    torch.cuda.set_sync_debug_mode(0)
    eng.close()


if __name__ == "__main__":
    main()
