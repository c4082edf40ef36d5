"""Sensitivity of the gmm robust mode to its PCA rank r (agg.gmm_filter_ref ``rank``): the bench configuration
(TransformerModel / ICU, 8 clients, client 7 = Min-Max attacker), one 12-round trajectory per r in 1..4 with the
host mirror as the aggregator, and at every round the kept sets every other r would have chosen on the same
updates.  Usage: python tools/dbg/gmm_rank_study.py > gpurun_out/gmm_rank_study.jsonl"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from attackfl_amd import agg  # noqa: E402
from attackfl_amd.config import from_dict  # noqa: E402
from attackfl_amd.fl.engine import FLEngine, build_client_table  # noqa: E402
from attackfl_amd.parallel.comm import LoopbackComm  # noqa: E402
from launch import parse_attackers  # noqa: E402


def run(rank: int, rounds: int = 12):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tmp = tempfile.mkdtemp(prefix="afl_gmm_")
    cfg = from_dict({
        "server": {"num-round": rounds + 2, "clients": 8, "mode": "gmm", "model": "TransformerModel", "data-name": "ICU",
                   "validation": True, "data-distribution": {"num-data-range": [12000, 15000]}},
        "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 60000, "test-size": 10000},
        "engine": {"trainer": "auto", "checkpoint-dir": tmp, "seed": 1}, "log_path": tmp})
    table = build_client_table(cfg, 1, parse_attackers("7:Min-Max:2"))
    eng = FLEngine(cfg, comm=LoopbackComm(dev), table=table, device=dev, verbose=False)
    eng.client_selection()
    seen = {}

    def host_gmm(U, sizes=None, attackers=None, seed=0, **_):
        n = U.shape[0]
        att = (attackers.bool() if attackers is not None else torch.zeros(n, dtype=torch.bool)).cpu().numpy()
        G = agg._centred_gram(U).cpu().numpy()
        sets = {}
        for r in (1, 2, 3, 4):
            keep, thr, kept, ok = agg.gmm_filter_ref(G, att, rank=r)
            sets[r] = keep.astype(int).tolist()
        seen["sets"] = sets
        keep = np.asarray(sets[rank], dtype=bool)
        if not keep.any():
            return agg.AggResult(None, False, {"kept": []})
        idx = torch.from_numpy(np.nonzero(keep)[0]).to(U.device)
        return agg.AggResult(agg.mean_of(U[idx]), True, {"kept": np.nonzero(keep)[0].tolist()})

    agg.AGGREGATORS["gmm"] = host_gmm
    for _ in range(rounds):
        rec = eng.run_round()
        print(json.dumps({"rank": rank, "round": rec.get("round"), "ok": rec.get("ok"), "metric": rec.get("metric"),
                          "kept_by_rank": seen.get("sets")}), flush=True)
    print(json.dumps({"rank": rank, "final_metric": eng.validation.last_metric}), flush=True)
    eng.close()


if __name__ == "__main__":
    for r in ([int(a) for a in sys.argv[1:]] or [1, 2, 3, 4]):
        run(r)
