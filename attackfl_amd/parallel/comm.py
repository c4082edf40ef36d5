"""Collective transport for FL rounds (replaces the reference's RabbitMQ/pika/pickle transport,
``server.py:102-108,187-203``, ``src/RpcClient.py:42-56,174-188``).

One round moves, per rank, a fixed-layout ``[S, W]`` fp32 block (S client slots: flat update row +
[valid, result, size, is_attacker, decision word] + the epoch losses) with ONE all-gather — or, for plain
FedAvg over the process group, ONE all-reduce.  There is no control message: every rank runs the same
deterministic server step on the gathered rows and reaches the same decisions (the decision word checks
that they did, ``FLEngine._check_decisions``).  Backends:

* ``LoopbackComm``  — single process (world 1), zero-copy.
* ``TorchComm``     — ``torch.distributed``: ``nccl`` (= RCCL over xGMI on MI355X) for device
  tensors, ``gloo`` for CPU (and for classic multi-process-per-GPU runs, staging through host).
  On a single node with ``comm.one-shot-allgather`` the RCCL all-gather of small blocks is
  replaced by the IPC one-shot kernel in ``parallel/ipc.py`` (every rank writes its block into
  all peers' buffers over xGMI at once instead of RCCL's ring hops).
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist


class Comm:
    rank: int = 0
    world: int = 1
    backend: str = "loopback"
    device: torch.device = torch.device("cpu")

    def all_gather_rows(self, local: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def check(self) -> None:
        """Raise if an asynchronous exchange the host has synchronised past failed (IPC deadline)."""

    one_shot = False

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def close(self) -> None:
        pass


class LoopbackComm(Comm):
    def __init__(self, device="cpu"):
        self.device = torch.device(device)

    def all_gather_rows(self, local: torch.Tensor) -> torch.Tensor:
        return local

    def broadcast_(self, t, src=0):
        return t

    def all_reduce_(self, t):
        return t


class TorchComm(Comm):
    """``torch.distributed`` process-group transport.

    ``one_shot``: True / False / "auto".  With the IPC path the update all-gather is the one-shot
    kernel (stream-ordered, no host staging even on a gloo group whose ranks share a GPU); "auto"
    enables it for device tensors with world > 1 (setup verifies it collectively and falls back to
    the process group's all-gather on every rank if any rank cannot use it)."""

    def __init__(self, device, backend: Optional[str] = None, pg=None, one_shot=False, ipc_timeout_s: float = 60.0):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.device = torch.device(device)
        self.backend = backend or dist.get_backend()
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.pg = pg
        self._staging = self.backend == "gloo" and self.device.type == "cuda"
        self._ipc = None
        if str(one_shot).lower() in ("true", "auto", "1") and self.device.type == "cuda" and self.world > 1:
            from .ipc import IpcAllGather

            self._ipc = IpcAllGather(self.device, self.rank, self.world, pg, timeout_s=ipc_timeout_s)

    @property
    def one_shot(self) -> bool:
        """True while the IPC one-shot all-gather is (or may still become) the gather path."""
        return self._ipc is not None

    def _to_comm(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if self._staging else t

    def check(self) -> None:
        """Raise if an IPC gather the host has synchronised past timed out (a peer is dead or hung)."""
        if self._ipc is not None:
            self._ipc.check()

    def all_gather_rows(self, local: torch.Tensor) -> torch.Tensor:
        local = local.contiguous()
        if self._ipc is not None and local.is_cuda:
            from .ipc import IpcUnavailable

            try:
                return self._ipc.all_gather(local)
            except IpcUnavailable as e:  # collective decision: every rank falls back together
                from ..utils.log import print_with_color

                if self.rank == 0:
                    print_with_color(f"[comm] one-shot IPC all-gather unavailable ({e}); using {self.backend}",
                                     "yellow")
                self._ipc = None
        src = self._to_comm(local)
        out = torch.empty((self.world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        if hasattr(dist, "all_gather_into_tensor") and self.backend == "nccl":
            dist.all_gather_into_tensor(out, src, group=self.pg)
        else:
            parts = list(out.chunk(self.world, dim=0))
            dist.all_gather(parts, src, group=self.pg)
        return out.to(local.device, non_blocking=True) if self._staging else out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self._staging:
            c = t.cpu()
            dist.broadcast(c, src=src, group=self.pg)
            t.copy_(c)
            return t
        dist.broadcast(t, src=src, group=self.pg)
        return t

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self._staging:
            c = t.cpu()
            dist.all_reduce(c, group=self.pg)
            t.copy_(c)
            return t
        dist.all_reduce(t, group=self.pg)
        return t

    def barrier(self) -> None:
        if self.backend == "nccl" and self.device.type == "cuda":
            dist.barrier(group=self.pg, device_ids=[self.device.index or 0])
        else:
            dist.barrier(group=self.pg)

    def broadcast_object(self, obj, src: int = 0):
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.pg)
        return box[0]

    def close(self) -> None:
        if self._ipc is not None:
            self._ipc.close()
            self._ipc = None


def init_distributed(backend: str = "auto", timeout_s: int = 600, store=None, rank: Optional[int] = None,
                     world_size: Optional[int] = None, device_index: Optional[int] = None):
    """Initialise ``torch.distributed``; returns (backend, device)."""
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl" and torch.cuda.is_available():
        ndev = max(1, torch.cuda.device_count())
        local = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
        if device_index is None and local > ndev:
            # RCCL needs one GPU per rank; wrapping the ordinal would put two ranks on one GPU and fail later
            # with an obscure communicator error
            raise RuntimeError(f"backend 'nccl' with {local} local ranks but {ndev} visible GPU(s): RCCL needs one "
                               "GPU per rank — use comm.backend 'gloo' or 'auto' (gloo + the IPC all-gather)")
        lr = device_index if device_index is not None else int(os.environ.get("LOCAL_RANK", "0"))
        if not 0 <= lr < ndev:
            raise RuntimeError(f"rank's GPU ordinal {lr} is out of range ({ndev} visible)")
        torch.cuda.set_device(lr)
        device = torch.device("cuda", lr)
    elif torch.cuda.is_available() and device_index is not None:
        device = torch.device("cuda", device_index)
    else:
        device = torch.device("cpu")
    kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if store is not None:
        kw.update(store=store, rank=rank, world_size=world_size)
    elif rank is not None:
        kw.update(rank=rank, world_size=world_size)
    if backend == "nccl" and device.type == "cuda":
        kw["device_id"] = device
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    if device.type == "cuda" and dist.get_world_size() > 1 and not os.environ.get("AFL_GPU_SHARERS"):
        from .launcher import sync_gpu_sharers

        sync_gpu_sharers(device)  # processes per physical GPU -> the on-chip trainers' CU budget
    return backend, device
