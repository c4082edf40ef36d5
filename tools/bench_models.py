"""Per-model local-training throughput on one GPU: native trainer (fused kernel / graph-replayed layer
programs) vs the eager PyTorch-module trainer (the reference's execution style) on the same plan.

    python tools/bench_models.py [--models CNNModel,RNNModel,TransformerModel,TransformerClassifier]
                                 [--clients 8] [--rows 2048] [--epochs 1] [--eager-clients 1]

Prints one JSON object: ms per optimizer step (all clients together) and rows/s for each trainer.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from attackfl_amd.data import DeviceTable, synthetic_har, synthetic_icu  # noqa: E402
from attackfl_amd.fl.trainers import make_plan, make_trainer  # noqa: E402
from attackfl_amd.models import ParamLayout, build_model  # noqa: E402


def _time(trainer, params, plan, lr, batch, seeds):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ok, _ = trainer.train(params, plan, lr, batch, seeds)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="CNNModel,RNNModel,TransformerModel,TransformerClassifier")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rows", type=int, default=2048)
    ap.add_argument("--har-rows", type=int, default=512)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--eager-clients", type=int, default=1)
    ap.add_argument("--skip-eager", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    out = {"clients": a.clients, "epochs": a.epochs}
    for name in a.models.split(","):
        har = name == "TransformerClassifier"
        rows = a.har_rows if har else a.rows
        batch = 64 if har else 128
        ds = synthetic_har(rows + 64) if har else synthetic_icu(rows + 64)
        table = DeviceTable(ds, dev)
        lay = ParamLayout.for_model(name)
        base = lay.flatten(build_model(name, seed=0).state_dict()).to(dev)
        res = {}
        for kind, C in (("auto", a.clients), ("eager", a.eager_clients)):
            if kind == "eager" and a.skip_eager:
                continue
            tr = make_trainer(kind, name, "HAR" if har else "ICU", table, dev)
            seeds = list(range(C))
            plan = make_plan(table.n, [rows] * C, a.epochs, [100 + s for s in seeds], dev)
            params = base[None].repeat(C, 1).contiguous()
            _time(tr, params.clone(), plan, 1e-3, batch, seeds)  # warm-up (JIT, allocator, graph)
            dt, ok = _time(tr, params, plan, 1e-3, batch, seeds)
            steps = a.epochs * ((rows + batch - 1) // batch)
            res[tr.kind] = {"clients": C, "s": round(dt, 4), "ms_per_step": round(1e3 * dt / steps, 4),
                            "client_rows_per_s": round(C * rows * a.epochs / dt, 1), "ok": all(ok)}
        if "eager" in res:
            nat = [k for k in res if k != "eager"][0]
            res["speedup_rows_per_s"] = round(res[nat]["client_rows_per_s"] / res["eager"]["client_rows_per_s"], 2)
        out[name] = res
        print(json.dumps({name: res}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
