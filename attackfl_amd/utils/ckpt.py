"""Background checkpoint writer.

The reference saves the model synchronously at the end of every successful round
(``server.py:551-553`` ``torch.save(...)``).  Serialising a hypernetwork of tens of MB costs tens of
milliseconds of CPU per round, which at GPU round rates is a large share of the round.  Here the leader
copies the tensors device→pinned host on the current stream (an async DMA, ordered after the kernels
that produced them), and one background thread waits for the copy and writes the file atomically
(``.tmp`` + ``os.replace``), so a reader never sees a half-written checkpoint.

One write is in flight at a time: ``submit`` first waits for the previous write (its pinned buffer is
reused), ``flush`` waits for the last one (called before the file is read and at shutdown).
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Callable, Dict, Optional

import torch


class CheckpointWriter:
    def __init__(self, asynchronous: bool = True):
        self.asynchronous = asynchronous
        self._pool: Optional[ThreadPoolExecutor] = None
        self._pending: Optional[Future] = None
        self._bufs: Dict[str, torch.Tensor] = {}
        self._lock = threading.Lock()

    def _host(self, key: str, src: torch.Tensor) -> torch.Tensor:
        """Pinned host staging buffer for ``src`` (reused across rounds)."""
        buf = self._bufs.get(key)
        if buf is None or buf.shape != src.shape or buf.dtype != src.dtype:
            buf = torch.empty(src.shape, dtype=src.dtype, pin_memory=src.is_cuda)
            self._bufs[key] = buf
        return buf

    def submit(self, key: str, src: torch.Tensor, build: Callable[[torch.Tensor], object], path: str) -> None:
        """Save ``build(host copy of src)`` to ``path``.  ``src`` may be overwritten right after return."""
        self.flush()
        src = src.detach()
        if not src.is_cuda or not self.asynchronous:
            _atomic_save(build(src.cpu() if src.is_cuda else src.clone()), path)
            return
        host = self._host(key, src)
        host.copy_(src, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="afl-ckpt")

        def job():
            ev.synchronize()
            _atomic_save(build(host), path)

        self._pending = self._pool.submit(job)

    def flush(self) -> None:
        p, self._pending = self._pending, None
        if p is not None:
            p.result()  # re-raises a write error in the caller

    def close(self) -> None:
        self.flush()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)
