"""Host-side profile of the headline round loop: cProfile over N steady-state rounds of the bench
configuration (the per-round Python work between two training launches).

  python tools/host_profile.py [--steps 100] [--attackers 3:Min-Max:2] > gpurun_out/host_profile.txt
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from attackfl_amd.config import from_dict  # noqa: E402
from attackfl_amd.fl.engine import FLEngine, build_client_table  # noqa: E402
from attackfl_amd.parallel.comm import LoopbackComm  # noqa: E402
from launch import parse_attackers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--attackers", default=None)
    ap.add_argument("--model", default="TransformerModel")
    ap.add_argument("--mode", default="fedavg")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = LoopbackComm(dev)
    tmp = tempfile.mkdtemp(prefix="afl_hostprof_")
    cfg = from_dict({
        "server": {"num-round": args.steps + 20, "clients": 8, "mode": args.mode, "model": args.model,
                   "data-name": "ICU", "validation": True, "data-distribution": {"num-data-range": [12000, 15000]}},
        "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 60000, "test-size": 10000},
        "engine": {"trainer": "auto", "checkpoint-dir": tmp, "seed": 1}, "log_path": tmp})
    table = build_client_table(cfg, 1, parse_attackers(args.attackers) if args.attackers else None)
    eng = FLEngine(cfg, comm=comm, table=table, device=dev, verbose=False)
    eng.client_selection()
    for _ in range(10):
        eng.run_round()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        eng.run_round()
    pr.disable()
    eng.ckpt_writer.flush()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(45)
    print(s.getvalue())
    eng.close()


if __name__ == "__main__":
    main()
