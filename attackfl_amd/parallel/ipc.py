"""One-shot intra-node all-gather over IPC-mapped peer buffers (``csrc/comm/ipc.cpp`` +
``csrc/kernels/comm.hip``).

RCCL's all-gather walks a ring: world-1 dependent hops, each paying link latency, which dominates
for the FL round's small blocks (one ``[slots, W]`` fp32 block per rank: ~190 KB for
TransformerModel).  Here every rank maps every peer's receive buffer once (IPC handles exchanged
through the process group) and writes its block into all of them at once over the point-to-point
xGMI links, then raises an epoch flag per peer.  The whole exchange is stream-ordered (two launches,
no host synchronisation) and returns a view of the receive buffer; ranks may also share one GPU
(several processes per device), which RCCL does not allow.

Setup is collective and verified: after mapping, every rank gathers a known pattern with a short
deadline, checks every row, and the ranks agree (MIN all-reduce) whether the path works — any
failure on any rank (no IPC support, another host, a peer that cannot map, corrupted data) makes
every rank fall back to the process group's own all-gather together.
"""
from __future__ import annotations

import contextlib
import socket
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import ops


def setup_verdict(local_err: str, infos: Sequence[Tuple[str, object, bytes]], rank: int,
                  can_access=None) -> str:
    """This rank's verdict on the IPC path from everyone's ``(host, GPU identity, handle)`` (``""`` = usable):
    a local failure, ranks on several hosts, a peer without an exported buffer, or a peer GPU this GPU cannot
    map.  The identity is physical (``launcher.gpu_key``: the same in every process whatever its device
    ordinals); ``can_access(peer identity)`` answers True / False (hipDeviceCanAccessPeer on this process's
    ordinal of that GPU) or None for a GPU this process cannot see — unknown, left to the open and the
    self-test.  A peer on the same GPU needs no peer access.  Pure host logic — the ranks then AND their
    verdicts (``IpcAllGather._agree``)."""
    if local_err:
        return local_err
    if len({h for h, _, _ in infos}) != 1:
        return "ranks span several hosts"
    if any(len(hd) == 0 for _, _, hd in infos):
        return "a peer could not export its buffer"
    me = infos[rank][1]
    if can_access is not None:
        bad = sorted({str(d) for r, (_, d, _) in enumerate(infos)
                      if r != rank and d != me and can_access(d) is False})
        if bad:
            return f"no peer access from GPU {me} to GPU(s) {bad}"
    return ""


class IpcUnavailable(RuntimeError):
    pass


class IpcAllGather:
    def __init__(self, device, rank: int, world: int, pg=None, timeout_s: float = 60.0):
        self.device = torch.device(device)
        self.rank, self.world, self.pg = rank, world, pg
        self.timeout_s = float(timeout_s)
        self._ctx = None
        self._n = 0

    def _agree(self, ok: bool) -> bool:
        """Collective AND over the process group (gloo: host tensor, nccl: device tensor)."""
        on_dev = dist.get_backend(self.pg) == "nccl"
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.pg)
        return bool(int(t.item()) == 1)

    def _on_device(self):
        return torch.cuda.device(self.device) if self.device.type == "cuda" else contextlib.nullcontext()

    def _can_access(self, peer_key):
        """Peer access from this GPU to the GPU with identity ``peer_key`` (``launcher.gpu_key``): True / False,
        None when this process cannot see that GPU (visibility narrowed per rank)."""
        if self.device.type != "cuda":
            return False
        from .launcher import local_gpu_keys

        idx = local_gpu_keys().get(peer_key)
        if idx is None:
            return None
        try:
            return bool(torch.cuda.can_device_access_peer(self.device.index or 0, int(idx)))
        except Exception:  # noqa: BLE001
            return None

    def setup(self, n: int) -> None:
        """Collective: allocate ``n`` floats per sender slot, map every peer, verify.  Raises
        ``IpcUnavailable`` on every rank if any rank fails (alloc / export, hosts, peer access, open, the
        self-test) — the ranks AND their verdicts, so they all fall back to the process group together."""
        self.close()
        ctx, handle, err = None, b"", ""
        try:
            with self._on_device():
                ctx = ops.native().IpcContext(self.rank, self.world, int(n))
                handle = ctx.handle()
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = f"alloc/export: {e}"
        info = [None] * self.world
        from .launcher import gpu_key

        me = gpu_key(self.device.index or 0) if self.device.type == "cuda" else "cpu"
        dist.all_gather_object(info, (socket.gethostname(), me, handle), group=self.pg)
        err = setup_verdict(err, info, self.rank, self._can_access)
        if not err:
            try:
                with self._on_device():
                    ctx.open([hd for _, _, hd in info])
            except Exception as e:  # noqa: BLE001
                err = f"open: {e}"
        if not err:
            # self-test with the real block size (both parities), short deadline
            try:
                with self._on_device():
                    for ep in range(2):
                        src = torch.arange(n, device=self.device, dtype=torch.float32) + (1000.0 * self.rank + ep)
                        out = ctx.all_gather(src, 5.0)
                        torch.cuda.synchronize(self.device)
                        if ctx.status() != 0:
                            err = f"self-test: no signal from ranks (mask {ctx.status():#x})"
                            break
                        exp = (torch.arange(n, device=self.device, dtype=torch.float32)[None, :]
                               + 1000.0 * torch.arange(self.world, device=self.device, dtype=torch.float32)[:, None]
                               + ep)
                        if not torch.equal(out, exp):
                            err = "self-test: gathered data differ"
                            break
            except Exception as e:  # noqa: BLE001
                err = f"self-test: {e}"
        if not self._agree(not err):
            if ctx is not None:
                ctx.close()
            raise IpcUnavailable(err or "a peer failed the IPC setup")
        self._ctx, self._n = ctx, int(n)

    def all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """``[rows, cols]`` block per rank -> ``[world * rows, cols]`` (rank-major), enqueued on the current
        stream.  The result is a view of the receive buffer: consume it on this stream before the call
        after next (which reuses its parity)."""
        flat = local.reshape(-1)
        if flat.dtype != torch.float32 or not flat.is_contiguous():
            flat = flat.float().contiguous()
        n = flat.numel()
        if self._ctx is None or n != self._n:
            self.setup(n)
        out = self._ctx.all_gather(flat, self.timeout_s)           # [world, n], row stride = capacity
        if out.is_contiguous():
            return out.view((self.world * local.shape[0],) + tuple(local.shape[1:]))
        return out.contiguous().view((self.world * local.shape[0],) + tuple(local.shape[1:]))

    def check(self) -> None:
        """Raise if a wait the host has synchronised past missed its deadline."""
        if self._ctx is not None:
            st = self._ctx.status()
            if st:
                raise RuntimeError(f"IPC all-gather: no signal within {self.timeout_s:.0f} s from ranks "
                                   f"{[r for r in range(self.world) if st >> r & 1]} (peer dead or hung)")

    def close(self) -> None:
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
            self._n = 0
