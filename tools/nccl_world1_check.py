#!/usr/bin/env python3
"""RCCL (torch.distributed "nccl") transport at world 1 on one GPU: the process-group branches of
``TorchComm`` (all_gather_into_tensor, all_reduce, broadcast, barrier with device_ids), the device-side
agreement of the IPC setup (``IpcAllGather._agree`` all-reduces a DEVICE tensor on an nccl group) and the IPC
context at world 1, then two FL rounds of the engine over the nccl comm — FedAvg all-reduce path and the
all-gather path.  An 8-GPU node exercises the same calls with 8 ranks (docs/ARCHITECTURE.md §multi-GPU).
Prints one JSON line; exit code 0 = every check passed."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> int:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    from attackfl_amd.config import from_dict
    from attackfl_amd.fl.engine import FLEngine
    from attackfl_amd.parallel.comm import TorchComm, init_distributed
    from attackfl_amd.parallel.ipc import IpcAllGather

    backend, dev = init_distributed("nccl", 120, rank=0, world_size=1, device_index=0)
    assert backend == "nccl" and dist.get_backend() == "nccl" and dev.type == "cuda"
    comm = TorchComm(dev, "nccl", one_shot=False)
    out = {}
    x = torch.arange(12, dtype=torch.float32, device=dev).reshape(3, 4)
    g = comm.all_gather_rows(x)
    out["all_gather"] = bool(torch.equal(g, x))
    r = comm.all_reduce_(torch.ones(5, device=dev, dtype=torch.float64))
    out["all_reduce"] = r.tolist() == [1.0] * 5
    b = comm.broadcast_(torch.full((2,), 7.0, device=dev))
    out["broadcast"] = b.tolist() == [7.0, 7.0]
    comm.barrier()
    out["barrier"] = True
    ipc = IpcAllGather(dev, 0, 1)
    out["agree_device"] = ipc._agree(True) is True and ipc._agree(False) is False
    ipc.setup(64)
    src = torch.arange(64, dtype=torch.float32, device=dev)
    got = ipc.all_gather(src.reshape(1, 64))
    torch.cuda.synchronize()
    out["ipc_world1"] = bool(torch.equal(got.reshape(-1), src))
    ipc.close()
    for fa in ("true", "false"):
        tmp = tempfile.mkdtemp()
        cfg = from_dict({"server": {"num-round": 2, "clients": 4, "mode": "fedavg", "model": "TransformerModel",
                                    "data-distribution": {"num-data-range": [300, 400]}},
                         "learning": {"epoch": 1, "batch-size": 128},
                         "data": {"synthetic": True, "train-size": 2000, "test-size": 500},
                         "comm": {"fedavg-allreduce": fa},
                         "engine": {"checkpoint-dir": tmp, "trainer": "auto", "metrics": os.path.join(tmp, "m.jsonl")},
                         "log_path": tmp})
        eng = FLEngine(cfg, comm=comm, device=dev, verbose=False)
        hist = eng.run()
        eng.close()
        paths = [h.get("path") for h in hist]
        out[f"engine_fedavg_allreduce_{fa}"] = (all(h["ok"] for h in hist) and len(hist) == 2 and
                                                (("fedavg-allreduce" in paths) == (fa == "true")))
    comm.close()
    dist.destroy_process_group()
    ok = all(out.values())
    print(json.dumps({"ok": ok, **out}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
