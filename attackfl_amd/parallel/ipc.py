"""One-shot intra-node all-gather over IPC-mapped peer buffers (``csrc/comm/ipc.cpp`` +
``csrc/kernels/comm.hip``).

RCCL's all-gather walks a ring: world-1 dependent hops, each paying link latency, which dominates
for the FL round's small blocks (one ``[slots, P+4]`` fp32 block per rank: ~190 KB for
TransformerModel).  Here every rank maps every peer's receive buffer once (IPC handles exchanged
through the process group) and writes its block into all of them at once over the point-to-point
xGMI links, then raises an epoch flag per peer.  Opt-in via ``comm.one-shot-allgather``; RCCL
stays the default path and the fallback (any setup error disables IPC with a warning).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..ops import native


class IpcAllGather:
    def __init__(self, device, rank: int, world: int, pg=None, cap: int = 0, max_polls: int = 20_000_000):
        self.device = torch.device(device)
        self.rank, self.world, self.pg = rank, world, pg
        self.max_polls = int(max_polls)
        self._ctx = None
        if cap:
            self._setup(cap)

    def _setup(self, cap: int) -> None:
        """Collective: every rank allocates ``cap`` floats per slot and maps all peers' buffers."""
        if self._ctx is not None:
            self._ctx.close()
        with torch.cuda.device(self.device):
            ctx = native().IpcContext(self.rank, self.world, int(cap))
            handles = [None] * self.world
            dist.all_gather_object(handles, ctx.handle(), group=self.pg)
            ctx.open(handles)
        self._ctx = ctx

    def all_gather(self, local: torch.Tensor) -> Optional[torch.Tensor]:
        """``[rows, ...]`` block per rank -> ``[world * rows, ...]`` (rank-major), or None if the
        block does not fit the mapped buffers (caller falls back to RCCL)."""
        n = local.numel()
        if self._ctx is None or n > self._ctx.capacity():
            self._setup(n)
        flat = local.reshape(-1).float().contiguous()
        out = self._ctx.all_gather(flat, self.max_polls)
        return out.view((self.world * local.shape[0],) + tuple(local.shape[1:])).to(local.dtype)

    def close(self) -> None:
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
