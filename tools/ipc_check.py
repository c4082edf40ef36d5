"""Multi-process check of the one-shot IPC all-gather (run under torchrun; every rank may share one
GPU).  Each rank contributes a distinct block; every rank verifies the gathered result against
RCCL/gloo's all-gather semantics for several epochs (exercises both parity buffers) and prints
one JSON line from rank 0 with the mean latency.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/ipc_check.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from attackfl_amd.parallel.comm import TorchComm  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    comm = TorchComm(dev, backend="gloo", one_shot=True)
    assert comm._ipc is not None, "IPC path not enabled"
    rows, cols = 2, 47697
    ok = True
    times = []
    for ep in range(6):
        local = torch.arange(rows * cols, device=dev, dtype=torch.float32).view(rows, cols) * (rank + 1) + ep
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = comm.all_gather_rows(local)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        for r in range(world):
            exp = torch.arange(rows * cols, device=dev, dtype=torch.float32).view(rows, cols) * (r + 1) + ep
            ok &= bool(torch.equal(out[r * rows:(r + 1) * rows], exp))
    flag = torch.tensor([int(ok)])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    comm.close()
    if rank == 0:
        print(json.dumps({"ipc_allgather_ok": bool(flag.item()), "world": world,
                          "mean_ms_after_first": round(1e3 * sum(times[1:]) / max(1, len(times) - 1), 3)}))
    dist.destroy_process_group()
    sys.exit(0 if flag.item() else 1)


if __name__ == "__main__":
    main()
