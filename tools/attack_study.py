#!/usr/bin/env python3
"""Post-attack quality study (BASELINE north star: "post-attack test-accuracy"): per-round test
ROC-AUC of TransformerModel/ICU under every reference attack (src/Utils.py:52-214) against FedAvg and the
robust aggregators (server.py:286-494), with 3 attackers of 8 clients from round 2.

Every cell runs with fixed seeds on the GPU (fused bf16 trainer, native aggregation / attack kernels) or on
the CPU (``trainer: oracle`` — the fp32 twin of the fused trainer with the same dropout masks — and the
PyTorch composites), so the two devices follow the same trajectories up to bf16 rounding and their final
AUCs can be compared cell by cell.  One JSON line per cell:

    {"device", "mode", "attack", "rounds", "auc": [per round], "final_auc", "attack_gamma": [...], "seconds"}

    python tools/attack_study.py --device cuda --out study_gpu.jsonl [--cells fedavg:LIE,median:Min-Max]
    python tools/attack_study.py --device cpu --out study_cpu.jsonl --jobs 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = ["fedavg", "median", "trimmed_mean", "krum", "hyper"]
ATTACKS = {"none": None, "LIE": [0.74], "Min-Max": [], "Min-Sum": [], "Opt-Fang": [], "Random": [0.5]}


def cells(spec: str):
    if spec:
        return [tuple(c.split(":", 1)) for c in spec.split(",")]
    return [(m, a) for m in MODES for a in ATTACKS]


def run_cell(mode: str, attack: str, device: str, rounds: int, threads: int = 0, genuine_rate: float = 0.5,
             distance: str = "spectral", seed: int = 7, tau: float = 1.0, attackers: int = 3) -> dict:
    import torch

    if threads:
        torch.set_num_threads(threads)
    from attackfl_amd.config import AttackSpec, from_dict
    from attackfl_amd.fl.engine import FLEngine, build_client_table
    from attackfl_amd.utils.log import set_quiet

    set_quiet(True)
    tmp = tempfile.mkdtemp(prefix="afl_study_")
    d = {
        "server": {"num-round": rounds, "clients": 8, "mode": mode, "model": "TransformerModel", "data-name": "ICU",
                   "genuine-rate": genuine_rate, "random-seed": seed - 6, "data-distribution": {"num-data-range": [800, 1200]}},
        "learning": {"epoch": 2, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 20000, "test-size": 3000},
        "engine": {"checkpoint-dir": tmp, "trainer": "auto" if device.startswith("cuda") else "oracle", "seed": seed,
                   "max-retries": 5, "distance": distance},
        "log_path": tmp,
    }
    cfg = from_dict(d)
    who = range(8 - attackers, 8)
    atk = {} if ATTACKS[attack] is None else {c: AttackSpec(attack, 2, ATTACKS[attack], tau=tau) for c in who}
    eng = FLEngine(cfg, device=device, table=build_client_table(cfg, 1, atk), verbose=False)
    t0 = time.time()
    stalled = False
    try:
        eng.run()
    except RuntimeError:  # max-retries consecutive failed rounds: the attack stopped training progress
        stalled = True
    hist = eng.history
    eng.close()
    ok = [r for r in hist if r["ok"]]
    return {"device": "gpu" if device.startswith("cuda") else "cpu", "mode": mode, "attack": attack,
            "genuine_rate": genuine_rate, "distance": distance, "seed": seed, "tau": tau,
            "attackers": len(atk), "rounds": len(ok), "failed_rounds": len(hist) - len(ok), "stalled": stalled,
            "auc": [round(r["metric"], 5) for r in ok], "final_auc": round(ok[-1]["metric"], 5) if ok else None,
            "attack_gamma": [round(r["attack"]["gamma"], 4) for r in ok if "attack" in r and "gamma" in r["attack"]],
            # last ACCEPTED γ per attacking round (0: every tried γ was rejected)
            "gamma_succ": [round(r["attack"]["gamma_succ"], 4) for r in ok if "gamma_succ" in r.get("attack", {})],
            # every tried γ of the last attacking round (the reference prints each, src/Utils.py:119)
            "gammas_last": next((r["attack"]["gammas"] for r in reversed(hist) if "gammas" in r.get("attack", {})), None),
            "seconds": round(time.time() - t0, 2)}


def _worker(args):
    mode, attack, device, rounds, threads, gr, dist, seed, tau, na = args
    return run_cell(mode, attack, device, rounds, threads, gr, dist, seed, tau, na)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--out", required=True)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--cells", default="", help="mode:attack,... (default: every mode x attack)")
    ap.add_argument("--jobs", type=int, default=1, help="parallel CPU processes")
    ap.add_argument("--genuine-rate", type=float, default=0.5, help="server.genuine-rate (reference default 0.5)")
    ap.add_argument("--distance", default="spectral", choices=["spectral", "flat"])
    ap.add_argument("--tau", type=float, default=1.0, help="bisection stop gap (reference: 1.0)")
    ap.add_argument("--attackers", type=int, default=3, help="attacking clients (the last N of 8)")
    ap.add_argument("--seeds", default="7", help="comma-separated run seeds (engine seed; server random-seed = seed - 6)")
    args = ap.parse_args()
    seeds = [int(x) for x in args.seeds.split(",")]
    todo = [(m, a, sd) for m, a in cells(args.cells) for sd in seeds]
    with open(args.out, "a") as fh:
        if args.jobs > 1 and not args.device.startswith("cuda"):
            import multiprocessing as mp

            threads = max(1, (os.cpu_count() or 8) // args.jobs)
            with mp.get_context("spawn").Pool(args.jobs) as pool:
                for res in pool.imap_unordered(_worker, [(m, a, args.device, args.rounds, threads, args.genuine_rate,
                                                                   args.distance, sd, args.tau, args.attackers)
                                                                  for m, a, sd in todo]):
                    fh.write(json.dumps(res) + "\n")
                    fh.flush()
                    print(res["mode"], res["attack"], res["final_auc"], res["seconds"], flush=True)
        else:
            for m, a, sd in todo:
                res = run_cell(m, a, args.device, args.rounds, 0, args.genuine_rate, args.distance, sd, args.tau,
                               args.attackers)
                fh.write(json.dumps(res) + "\n")
                fh.flush()
                print(res["mode"], res["attack"], res["final_auc"], res["seconds"], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
