#!/usr/bin/env python3
"""FL server — same invocation as the reference (``python server.py [--device D]``, reference server.py:36-40).

Reads ``config.yaml`` from the working directory, waits for ``server.clients`` ``client.py`` processes to
register, then runs the rounds: aggregation / defenses / hypernetwork training, validation (ROC-AUC in
``app.log``) and the per-round ``{model}.pth`` / ``{model}_hyper_{clients}.pth`` checkpoints.

Transport: a TCPStore rendezvous at ``comm.address`` (default ``rabbit.address``) replaces the RabbitMQ
broker.  With ``comm.backend: auto`` the server picks the process group from the registered devices: RCCL
when every process owns its own GPU, gloo when several share one (or run on the CPU); on one host the
update all-gather is the one-shot IPC kernel either way (``comm.one-shot-allgather: auto``).  For
one-process-per-GPU packed runs use ``launch.py`` under torchrun.
"""
from __future__ import annotations

import argparse
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _one_shot(cfg, auto_choice: bool):
    v = str(cfg.comm.get("one-shot-allgather", "auto")).lower()
    return auto_choice if v == "auto" else v in ("true", "1")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Federated learning framework with controller.")
    ap.add_argument("--device", type=str, required=False, help="Device of server")
    ap.add_argument("--config", type=str, default="config.yaml")
    args = ap.parse_args(argv)

    import torch

    from attackfl_amd.config import load_config
    from attackfl_amd.fl.engine import FLEngine
    from attackfl_amd.parallel.comm import TorchComm
    from attackfl_amd.parallel.launcher import init_group, read_transport, serve_rendezvous, table_from_json
    from attackfl_amd.utils.log import print_with_color

    cfg = load_config(args.config)
    # (--device cuda = cuda:0; the clients take GPUs 1, 2, ... in registration order: launcher.client_device)
    device = (torch.device(args.device) if args.device and args.device != "cuda" else
              torch.device("cuda", 0) if torch.cuda.is_available() else torch.device(args.device or "cpu"))
    print_with_color(f"Using device: {device}", "green")
    store, world, table = serve_rendezvous(cfg, device=device)
    backend, one_shot = read_transport(store)
    backend = backend if cfg.comm.get("backend", "auto") == "auto" else cfg.comm["backend"]
    init_group(store, 0, world, backend, int(cfg.comm.get("timeout-s", 600)), device.index)
    comm = TorchComm(device, backend, one_shot=_one_shot(cfg, one_shot))
    eng = FLEngine(cfg, comm=comm, table=table_from_json(table), device=device, leader=True)
    gc.freeze()  # engine, models and tables -> permanent generation: no ms-long full GC scans mid-round
    eng.run()
    eng.close()
    torch.distributed.destroy_process_group()
    print_with_color("Ok, ready!", "green")
    return 0


if __name__ == "__main__":
    sys.exit(main())
