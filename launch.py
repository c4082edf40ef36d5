#!/usr/bin/env python3
"""Packed SPMD launcher: one process per GPU, ``server.clients`` clients spread over the ranks.

    python launch.py [--config config.yaml] [--attackers "3:LIE:2:0.74,5:Min-Max:2"] [--device cuda:0]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 launch.py [...]

Server state (aggregator, hypernetwork, genuine pool) and the validation / detection decisions are
replicated on every rank; rank 0 logs to ``app.log`` and writes the ``.pth`` checkpoints.  Attackers come from ``--attackers`` or the
``comm.attackers`` config map (client index -> {mode, round, args}).
"""
from __future__ import annotations

import argparse
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_attackers(spec: str):
    from attackfl_amd.config import AttackSpec

    out = {}
    for item in filter(None, (s.strip() for s in (spec or "").split(","))):
        parts = item.split(":")
        idx, mode, rnd = int(parts[0]), parts[1], int(parts[2]) if len(parts) > 2 else 1
        out[idx] = AttackSpec(mode, rnd, [float(x) for x in parts[3:]])
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="attackfl_amd packed launcher")
    ap.add_argument("--config", default="config.yaml")
    ap.add_argument("--attackers", default="", help="idx:mode:round[:arg...] comma-separated")
    ap.add_argument("--device", default=None)
    ap.add_argument("--rounds", type=int, default=None, help="override server.num-round")
    args = ap.parse_args(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1 and args.device and args.device.startswith("cuda:"):
        # every rank pinned to one GPU: keep all ranks' hardware queues mapped (see bench.py)
        from bench import shared_gpu_queues

        os.environ["AFL_SHARED_GPU"] = "1"  # (parallel.launcher.gpu_sharers: all local ranks on one GPU)

        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)  # the runtime default is 4 (never raised here)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(cur, shared_gpu_queues(world_env)))

    import torch

    from attackfl_amd.config import load_config
    from attackfl_amd.fl.engine import FLEngine, build_client_table
    from attackfl_amd.parallel.comm import LoopbackComm, TorchComm, init_distributed

    over = {"server": {"num-round": args.rounds}} if args.rounds else None
    cfg = load_config(args.config, over)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dev_index = None
        if args.device and args.device.startswith("cuda"):  # e.g. several gloo ranks sharing one GPU
            dev_index = int(args.device.split(":")[1]) if ":" in args.device else None
        backend = cfg.comm.get("backend", "auto")
        if backend == "auto" and dev_index is not None:
            backend = "gloo"  # ranks pinned to one GPU share it: RCCL refuses duplicate GPUs
        if backend == "auto" and torch.cuda.is_available():
            # one rank per GPU (LOCAL_RANK % GPUs, comm.init_distributed); more local ranks than GPUs share some
            local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            backend = "nccl" if local <= torch.cuda.device_count() else "gloo"
            if backend == "gloo":
                dev_index = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
        backend, device = init_distributed(backend, int(cfg.comm.get("timeout-s", 600)), device_index=dev_index)
        comm = TorchComm(device, backend, one_shot=cfg.comm.get("one-shot-allgather", "auto"))
    else:
        device = torch.device(args.device) if args.device else (torch.device("cuda", 0) if torch.cuda.is_available()
                                                                else torch.device("cpu"))
        comm = LoopbackComm(device)
    attackers = parse_attackers(args.attackers) if args.attackers else None
    table = build_client_table(cfg, comm.world, attackers, int(cfg.comm.get("clients-per-rank", 0)))
    eng = FLEngine(cfg, comm=comm, table=table, device=device)
    gc.freeze()  # engine, models and tables -> permanent generation: no ms-long full GC scans mid-round
    eng.run()
    eng.close()
    comm.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
