"""Background checkpoint writer.

The reference saves the model synchronously at the end of every successful round
(``server.py:551-553`` ``torch.save(...)``).  Serialising a hypernetwork of tens of MB costs tens of
milliseconds of CPU per round, which at GPU round rates is longer than a round.  Here the leader copies
the tensors device -> pinned host on the current stream (an async DMA, ordered after the kernels that
produced them), and one background thread waits for the copy and writes the file atomically (``.tmp`` +
``os.replace``), so a reader never sees a half-written checkpoint.

The device -> host copy runs on a side stream (``fence`` makes the compute stream wait for it before a
submitted tensor is overwritten in place): on the compute stream the copy of a hypernetwork arena (tens of
MB, a blit kernel) sat in front of the next round's training launch.

Deferred copies (``submit(..., defer=True)`` + ``kick``): the copy is a blit kernel that holds CUs for
the ~0.35 ms of a 20 MB arena; issued at the end of a round it delayed the next round's small preparation
kernels by as much.  A deferred submit only records an event on the compute stream (the state to save);
``kick`` — called by the engine right after the next training launch, whose few workgroups leave the
chip idle — issues the side-stream copy ordered after that event.  ``fence`` / ``flush`` / ``close``
kick first, so a deferred copy can never miss its source.

Latest-wins coalescing: two pinned staging slots per key; a ``submit`` that arrives while a write is in
flight replaces any write that has not started yet (only the newest state matters), so a round never
waits for the disk.  The file therefore always holds a complete checkpoint of a finished round, at most
one write behind while rounds outpace the disk, and ``flush`` (called before the file is read and at
shutdown) writes the newest one.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Optional, Tuple

import torch


class CheckpointWriter:
    def __init__(self, asynchronous: bool = True):
        self.asynchronous = asynchronous
        self._bufs: Dict[Tuple[str, int], torch.Tensor] = {}
        self._cv = threading.Condition()
        self._pending = None          # (key, slot, build, path, event) not yet started
        self._writing: Optional[Tuple[str, int]] = None
        self._err: Optional[BaseException] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self.dropped = 0               # superseded writes (diagnostics)
        self._stream = None            # side stream of the device -> host copies
        self._copied = None            # event: the last copy has read its source
        self._deferred = None          # (key, src, build, path, event on the compute stream) not copied yet

    def _host(self, key: str, slot: int, src: torch.Tensor) -> torch.Tensor:
        """Pinned host staging buffer for ``src`` (reused across rounds)."""
        buf = self._bufs.get((key, slot))
        if buf is None or buf.shape != src.shape or buf.dtype != src.dtype:
            buf = torch.empty(src.shape, dtype=src.dtype, pin_memory=src.is_cuda)
            self._bufs[(key, slot)] = buf
        return buf

    def submit(self, key: str, src: torch.Tensor, build: Callable[[torch.Tensor], object], path: str,
               defer: bool = False) -> None:
        """Save ``build(host copy of src)`` to ``path``.  ``src`` may be overwritten right after return
        (with ``defer``: only after ``fence`` or ``kick``; the copy is taken of the state as of this call)."""
        src = src.detach()
        if not src.is_cuda or not self.asynchronous:
            self.flush()
            _atomic_save(build(src.cpu() if src.is_cuda else src.clone()), path)
            return
        if defer:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(src.device))
            if self._deferred is not None:
                self.dropped += 1              # superseded before its copy was issued
            self._deferred = (key, src, build, path, ev)
            return
        self._deferred = None
        self._copy(key, src, build, path, None)

    def kick(self) -> None:
        """Issue the deferred copy, if any (side stream, ordered after the state it saves)."""
        d, self._deferred = self._deferred, None
        if d is not None:
            self._copy(*d)

    def _copy(self, key, src, build, path, after: Optional[torch.cuda.Event]) -> None:
        with self._cv:
            self._raise()
            if self._pending is not None:      # superseded before it started
                self._pending = None
                self.dropped += 1
            slot = 1 if self._writing == (key, 0) else 0
        host = self._host(key, slot, src)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=src.device)
        if after is not None:
            self._stream.wait_event(after)                                  # src as of the deferred submit
        else:
            self._stream.wait_stream(torch.cuda.current_stream(src.device))  # src as produced so far
        with torch.cuda.stream(self._stream):
            host.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        src.record_stream(self._stream)  # the allocator keeps src's memory until the copy has run
        self._copied = ev
        with self._cv:
            self._pending = (key, slot, build, path, ev)
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name="afl-ckpt", daemon=True)
                self._thread.start()
            self._cv.notify_all()

    def fence(self) -> None:
        """Make the current stream wait (on the device, no host sync) until the last submitted copy has
        read its source: call before overwriting a submitted tensor in place."""
        self.kick()
        if self._copied is not None:
            torch.cuda.current_stream().wait_event(self._copied)

    def _run(self) -> None:
        while True:
            with self._cv:
                while self._pending is None and not self._stop:
                    self._cv.wait()
                if self._pending is None:
                    return
                key, slot, build, path, ev = self._pending
                self._pending = None
                self._writing = (key, slot)
            try:
                ev.synchronize()
                _atomic_save(build(self._bufs[(key, slot)]), path)
            except BaseException as e:  # noqa: BLE001 - re-raised in the caller
                with self._cv:
                    self._err = e
            with self._cv:
                self._writing = None
                self._cv.notify_all()

    def _raise(self) -> None:
        if self._err is not None:
            e, self._err = self._err, None
            raise e

    def flush(self) -> None:
        """Wait until the newest submitted checkpoint is on disk (re-raises a write error)."""
        self.kick()
        with self._cv:
            while self._pending is not None or self._writing is not None:
                self._cv.wait()
            self._raise()

    def close(self) -> None:
        self.flush()
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        if self._thread is not None:
            self._thread.join()
            self._thread = None


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)
