#!/usr/bin/env python3
"""Headline benchmark: FL rounds/sec for the whole node (+ test ROC-AUC), TransformerModel/ICU, 8 clients.

Metric and config come from BASELINE.json ("FL rounds/sec (whole node) + test-acc, TransformerModel/ICU,
8 clients"); the workload is the reference ``config.yaml`` learning setup (5 local epochs, batch 128,
Adam lr 0.004, 12000-15000 rows per client per round) with ``mode: fedavg`` and no attacker.  A "step"
is one complete FL round: every client's local training, the update all-gather, FedAvg, server-side
ROC-AUC validation on the 10k-row test set and the ``TransformerModel.pth`` checkpoint write.

The 8 clients are spread over the N ranks (8/N clients per GPU, one process per GPU, RCCL over xGMI):
total work is fixed as N grows, so scaling is *strong*.  Data are synthetic ICU-shaped rows with a
planted signal, weights are random-init (no datasets or checkpoints are downloadable here).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_ROUNDS_PER_S = 0.18  # measured proxy of the reference, whole node, 8 clients
# BASELINE.md proxy rows for the other model families (same workload, 8 clients); HAR: none measured
MODEL_BASELINES = {"TransformerModel": BASELINE_ROUNDS_PER_S, "CNNModel": 0.075, "RNNModel": 0.15}


def shared_gpu_queues(ranks_per_gpu: int) -> int:
    """Hardware queues per process when ``ranks_per_gpu`` processes share one GPU (kept in sync with
    ``attackfl_amd.parallel.launcher.shared_gpu_queues``; bench.py must set it before importing torch)."""
    return 4 if ranks_per_gpu <= 2 else (2 if ranks_per_gpu <= 8 else 1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--model", default="TransformerModel")
    ap.add_argument("--mode", default="fedavg")
    ap.add_argument("--trainer", default="auto")
    ap.add_argument("--attackers", default="", help="idx:mode:round[:arg...] comma-separated (launch.py syntax)")
    ap.add_argument("--data-name", default="ICU")
    ap.add_argument("--profile-rounds", action="store_true", help="print per-phase timings to stderr")
    args = ap.parse_args()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1 and os.environ.get("AFL_BENCH_DEVICE") is not None:
        # several ranks on ONE GPU: cap each process's hardware queues so that all ranks' queues stay mapped
        # (oversubscribed queues are time-sliced: 8 ranks x 4 queues ran at 43 rounds/s, x 2 at 89)
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)  # the runtime default is 4 (never raised here)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(cur, shared_gpu_queues(world_env)))

    import torch
    import torch.distributed as dist

    from attackfl_amd.config import from_dict
    from attackfl_amd.fl.engine import FLEngine, build_client_table
    from attackfl_amd.parallel.comm import LoopbackComm, TorchComm, init_distributed
    from attackfl_amd.utils.log import set_quiet
    from launch import parse_attackers

    set_quiet(True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    if world > 1:
        # one process per GPU over RCCL; the update exchange is the one-shot IPC all-gather over xGMI (verified
        # collectively at the first round, RCCL otherwise).  Test hooks: AFL_BENCH_DEVICE=i puts every rank on
        # GPU i (several ranks sharing one GPU: gloo group, IPC data path), AFL_BENCH_BACKEND forces the group
        # backend, AFL_BENCH_ONE_SHOT=false forces the process-group collectives.
        dev_idx = os.environ.get("AFL_BENCH_DEVICE")
        shared = dev_idx is not None
        backend = os.environ.get("AFL_BENCH_BACKEND") or (
            "nccl" if torch.cuda.is_available() and not shared else "gloo")
        backend, device = init_distributed(backend, device_index=int(dev_idx) if shared else None)
        comm = TorchComm(device, backend, one_shot=os.environ.get("AFL_BENCH_ONE_SHOT", "auto"))
    else:
        device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        if device.type == "cuda":
            torch.cuda.set_device(device)
        comm = LoopbackComm(device)
    rank = comm.rank
    tmp = tempfile.mkdtemp(prefix=f"attackfl_bench_r{rank}_")
    rows = [12000, 15000] if args.data_name == "ICU" else [1000, 1500]  # HAR: 7352-row train set
    cfg = from_dict({
        "server": {"num-round": args.warmup + args.steps + 1, "clients": args.clients, "mode": args.mode,
                   "model": args.model, "data-name": args.data_name, "validation": True,
                   "data-distribution": {"num-data-range": rows}},
        "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
        "data": {"synthetic": True, "train-size": 60000, "test-size": 10000, "har-train-size": 7352,
                 "har-test-size": 2947},
        "engine": {"trainer": args.trainer, "checkpoint-dir": tmp, "seed": 1,
                   "phase-sync": bool(args.profile_rounds)},
        "log_path": tmp,
    })
    attackers = parse_attackers(args.attackers) if args.attackers else None
    table = build_client_table(cfg, comm.world, attackers)
    eng = FLEngine(cfg, comm=comm, table=table, device=device, verbose=False)
    eng.client_selection()

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if comm.world > 1:
            comm.barrier()

    for _ in range(args.warmup):
        eng.run_round()
    gc.freeze()  # as server.py / launch.py: the long-lived objects leave the collector's full scans
    sync()
    t0 = time.perf_counter()
    recs = []
    w0 = eng.ckpt_writer.written
    for _ in range(args.steps):
        recs.append(eng.run_round())
    eng.ckpt_writer.flush()  # every timed round's .pth is on disk before the clock stops
    sync()
    elapsed = time.perf_counter() - t0
    ckpt = {"ckpt_written": eng.ckpt_writer.written - w0, "ckpt_dropped": eng.ckpt_writer.dropped,
            "ckpt_stalls": eng.ckpt_writer.stalls, "ckpt_template_writes": eng.ckpt_writer.template_writes,
            "t_checkpoint_ms": round(1e3 * sum(r.get("t_checkpoint", 0.0) for r in recs) / max(1, len(recs)), 3)}
    if comm.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if os.environ.get("AFL_BENCH_TIMES") and rank == 0:  # per-round host timings of the timed rounds (JSONL)
        with open(os.environ["AFL_BENCH_TIMES"], "w") as f:
            for r in recs:
                f.write(json.dumps({k: v for k, v in r.items() if k.startswith("t_") or k in ("round", "ok")}) + "\n")
    if args.profile_rounds and rank == 0:
        for r in recs:
            print(json.dumps({k: r[k] for k in ("round", "ok", "t_lw_prep", "t_lw_prep_host", "t_lw_prep_upload", "t_lw_launch", "t_lw_attack", "t_lw_wait", "t_lw_post", "t_local",
                                                "t_gather", "t_aggregate", "t_validate", "t_checkpoint", "t_round", "metric")
                              if k in r}), file=sys.stderr)
    value = args.steps / elapsed
    if rank == 0:
        aucs = [r["metric"] for r in recs if r["metric"] == r["metric"]]
        base = MODEL_BASELINES.get(args.model) if (args.data_name == "ICU" and args.clients == 8) else None
        out = {
            "metric": f"FL rounds/sec (whole node) + test-acc, {args.model}/{args.data_name}, {args.clients} clients",
            "value": round(value, 4),
            "unit": "rounds/s",
            "n_gpus": comm.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base, 2) if base else None,
            "dtype": "bf16",
            "data": ("synthetic ICU-shaped rows (planted signal)" if args.data_name == "ICU" else
                     "synthetic HAR-shaped sequences (L=561, 6 classes)") + ", random-init weights",
            "config": {"model": args.model, "global_batch": 128 * args.clients,
                       "seq_len": 1 if args.data_name == "ICU" else 561,
                       "parallelism": f"fl{args.clients}-clients-over-{comm.world}-ranks",
                       "clients": args.clients, "local_epochs": 5, "rows_per_client": f"{rows[0]}-{rows[1]}",
                       "mode": args.mode, "trainer": eng.trainer.kind if eng.trainer else None,
                       "attackers": args.attackers or None},
            ("test_roc_auc" if args.data_name == "ICU" else "test_accuracy"): round(aucs[-1], 4) if aucs else None,
            "rounds_ok": sum(1 for r in recs if r["ok"]),
            "comm": ("loopback" if comm.world == 1 else
                     ("ipc-one-shot" if getattr(comm, "one_shot", False) else comm.backend)
                     + ("+allreduce" if eng.fast_fedavg else "")),
            "speculative": eng._speculative,
            **ckpt,
        }
        print(json.dumps(out), flush=True)
        if out["rounds_ok"] < args.steps:
            # a failed round skips its update and validation: a timing over failed rounds is not the metric
            print(f"[bench] WARNING: only {out['rounds_ok']} of {args.steps} timed rounds succeeded", file=sys.stderr)
    eng.close()
    comm.close()
    if world > 1:
        dist.destroy_process_group()
    return 0 if (rank != 0 or any(r["ok"] for r in recs)) else 3  # no successful round: fail loudly


if __name__ == "__main__":
    sys.exit(main())
