#!/usr/bin/env python3
"""FL client — same flags as the reference (reference client.py:19-38):

    python client.py [--device D] [--attack True --attack_mode {Random,Min-Max,Min-Sum,Opt-Fang,LIE}
                      --attack_round R --attack_args F ...]

Registers with the server's rendezvous, receives its client index (registration order r = 1..N), and runs its
rounds inside the SPMD engine as rank r - 1 of the N-client group, on GPU ``(r - 1) % device_count`` unless
``--device`` names one (one FL client per MI355X; ``parallel.launcher.client_device``): local training through the
fused HIP trainer on GPU (eager PyTorch on CPU) or, once ``training_round >= attack_round`` and genuine models have
been received, the attack.  Every client rank holds the replicated server state; client 1 (rank 0) is the leader
that logs ``app.log`` and writes the checkpoints where the server would.
Unlike the reference (``type=bool``, A-9) ``--attack False`` really disables the attack.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _bool(s: str) -> bool:
    if isinstance(s, bool):
        return s
    v = str(s).strip().lower()
    if v in ("1", "true", "t", "yes", "y"):
        return True
    if v in ("0", "false", "f", "no", "n", ""):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {s}")


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="Split learning framework")
    ap.add_argument("--device", type=str, required=False, help="Device of client")
    ap.add_argument("--attack", type=_bool, required=False, default=False,
                    help="Set to True to enable attack mode, False otherwise.")
    ap.add_argument("--attack_mode", type=str, choices=["Random", "Min-Max", "Min-Sum", "Opt-Fang", "LIE"],
                    help="Mode of operation when the attack is enabled (e.g., Random or Min-Max, Min-Sum ...).")
    ap.add_argument("--attack_round", type=int, help="Client attack at round.")
    ap.add_argument("--attack_args", type=float, nargs="+", required=False,
                    help="A list of attack args. Use space to separate values (e.g., 0.1 0.2 0.5).")
    ap.add_argument("--config", type=str, default="config.yaml")
    args = ap.parse_args(argv)
    if args.attack and not args.attack_mode:
        print("Error: --attack_mode is required when --attack is True.")
        sys.exit()
    if args.attack and not args.attack_round:
        print("Error: --attack_round is required when --attack is True.")
        sys.exit()
    return args


def _one_shot(cfg, auto_choice: bool):
    v = str(cfg.comm.get("one-shot-allgather", "auto")).lower()
    return auto_choice if v == "auto" else v in ("true", "1")


def main(argv=None) -> int:
    args = parse_args(argv)
    print(f"Attack: {args.attack}, Mode: {args.attack_mode}")

    import gc

    import torch

    from attackfl_amd.config import AttackSpec, load_config
    from attackfl_amd.fl.engine import FLEngine
    from attackfl_amd.parallel.comm import TorchComm
    from attackfl_amd.parallel.launcher import (apply_leader_paths, client_device, init_group, join_rendezvous,
                                                read_transport, report_done, report_exit, table_from_json)

    cfg = load_config(args.config)
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    attack = AttackSpec(args.attack_mode, args.attack_round, args.attack_args or []) if args.attack else None
    # the device follows the claimed number: client r -> cuda:{(r - 1) % ndev} unless --device names one
    store, rank, world, table, device = join_rendezvous(
        cfg, attack, device_fn=lambda r: torch.device(client_device(args.device, r, ndev)))
    print(f"Using device: {device}")
    try:
        backend, one_shot = read_transport(store, rank)
        backend = backend if cfg.comm.get("backend", "auto") == "auto" else cfg.comm["backend"]
        if rank == 0:
            apply_leader_paths(store, cfg)
        init_group(store, rank, world, backend, int(cfg.comm.get("timeout-s", 600)), device.index)
        comm = TorchComm(device, backend, one_shot=_one_shot(cfg, one_shot))
        eng = FLEngine(cfg, comm=comm, table=table_from_json(table), device=device, leader=rank == 0,
                       verbose=rank == 0)
        gc.freeze()  # engine, models and tables -> permanent generation: no ms-long full GC scans mid-round
        eng.run()
        eng.close()
        comm.close()
        torch.distributed.destroy_process_group()
    except BaseException as e:
        report_done(store, False, f"client {rank + 1}: {type(e).__name__}: {e}")
        report_exit(store)
        raise
    if rank == 0:
        report_done(store, True)
    report_exit(store)
    return 0


if __name__ == "__main__":
    sys.exit(main())
