"""Per-round trace of the gmm robust mode on the bench configuration: validation metric and the aggregator's
kept set each round (which rows the GMM filter keeps, attacker = client 7).  Usage: python tools/dbg/gmm_rounds.py"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from attackfl_amd.config import from_dict  # noqa: E402
from attackfl_amd.fl.engine import FLEngine, build_client_table  # noqa: E402
from attackfl_amd.parallel.comm import LoopbackComm  # noqa: E402
from launch import parse_attackers  # noqa: E402
from attackfl_amd import agg  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tmp = tempfile.mkdtemp(prefix="afl_gmm_")
    cfg = from_dict({
        "server": {"num-round": 14, "clients": 8, "mode": "gmm", "model": "TransformerModel", "data-name": "ICU",
                   "validation": True, "data-distribution": {"num-data-range": [12000, 15000]}},
        "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 60000, "test-size": 10000},
        "engine": {"trainer": "auto", "checkpoint-dir": tmp, "seed": 1}, "log_path": tmp})
    table = build_client_table(cfg, 1, parse_attackers("7:Min-Max:2"))
    eng = FLEngine(cfg, comm=LoopbackComm(dev), table=table, device=dev, verbose=False)
    eng.client_selection()
    orig = agg.gmm

    def traced(U, *a, **k):
        res = orig(U, *a, **k)
        kept = res.info.get("kept")
        print("  gmm kept", None if kept is None else kept.int().tolist(), "thr", float(res.info.get("threshold", float("nan"))), flush=True)
        return res
    agg.gmm = traced
    if hasattr(agg, "AGGREGATORS") and "gmm" in agg.AGGREGATORS:
        agg.AGGREGATORS["gmm"] = traced
    for r in range(12):
        rec = eng.run_round()
        print(json.dumps({k: rec[k] for k in rec if k in ("round", "ok", "metric", "auc")}), flush=True)
    print("final metric", eng.validation.last_metric)


if __name__ == "__main__":
    main()
