#!/usr/bin/env python3
"""FL server — same invocation as the reference (``python server.py [--device D]``, reference server.py:36-40).

Reads ``config.yaml`` from the working directory, waits for ``server.clients`` ``client.py`` processes to
register, then runs the rounds: aggregation / defenses / hypernetwork training, validation (ROC-AUC in
``app.log``) and the per-round ``{model}.pth`` / ``{model}_hyper_{clients}.pth`` checkpoints.

Transport: a TCPStore rendezvous at ``comm.address`` (default ``rabbit.address``) replaces the RabbitMQ
broker.  The registered CLIENTS form the device process group (client r = group rank r - 1), with server state
replicated on every client rank; group rank 0 is the leader that writes ``app.log`` and the checkpoints into this
server's ``log_path`` / checkpoint directory.  This process holds the store and the client table, echoes the
leader's ``app.log`` to its console and exits when the run is done — it computes nothing and needs no GPU, so 8
clients on an 8-GPU node are 8 ranks on 8 distinct GPUs.  With ``comm.backend: auto`` the clients' group is RCCL
when every client owns its own GPU, gloo when several share one (or run on the CPU); on one host the update
all-gather is the one-shot IPC kernel either way (``comm.one-shot-allgather: auto``).  For packed runs (several
clients per process) use ``launch.py`` under torchrun.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Federated learning framework with controller.")
    ap.add_argument("--device", type=str, required=False, help="Device of server")
    ap.add_argument("--config", type=str, default="config.yaml")
    args = ap.parse_args(argv)

    import os as _os

    from attackfl_amd.config import load_config
    from attackfl_amd.parallel.launcher import serve_rendezvous, serve_until_done
    from attackfl_amd.utils.log import print_with_color

    cfg = load_config(args.config)
    # (--device is accepted for the reference's command line; the server computes nothing: every client rank
    # holds the replicated server state and the leader client validates, logs and checkpoints)
    print_with_color(f"Using device: {args.device or 'none (state replicated on the client ranks)'}", "green")
    store, n, _table = serve_rendezvous(cfg)
    ok = serve_until_done(store, _os.path.join(_os.path.abspath(cfg.log_path), "app.log"), n)
    if not ok:
        return 1
    print_with_color("Ok, ready!", "green")
    return 0


if __name__ == "__main__":
    sys.exit(main())
