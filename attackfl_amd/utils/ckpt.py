"""Background checkpoint writer.

The reference saves the model synchronously at the end of every successful round
(``server.py:551-553`` ``torch.save(...)``).  Serialising a hypernetwork of tens of MB costs tens of
milliseconds of CPU per round (``torch.save`` of the 19.5 MB TransformerModel hypernetwork: ~24 ms, of
which ~12 ms is its CRC-32), which at GPU round rates is longer than a round.  Here:

* the device -> pinned-host copy runs on a side stream, ordered after the kernels that produced the state
  (``fence`` makes the compute stream wait for it before a submitted tensor is overwritten in place); on
  the compute stream the copy of a hypernetwork arena sat in front of the next round's training launch;
* **deferred copies** (``submit(..., defer=True)`` + ``kick``): the copy is a blit kernel that holds CUs
  for the ~0.35 ms of a 20 MB arena; a deferred submit only records an event on the compute stream (the
  state to save) and ``kick`` — called by the engine right after the next training launch — issues the
  side-stream copy ordered after that event.  ``fence`` / ``flush`` / ``close`` kick first;
* **zip-template writes**: the first write of a key runs ``torch.save`` once into memory and, when the
  result holds exactly one storage whose bytes are the staging buffer, keeps the archive as a template
  (prefix, storage bytes, suffix).  Every later write emits prefix + the new storage bytes + suffix with
  the storage record's CRC-32 patched in (local header and central directory), and that CRC is computed
  on the GPU next to the copy (``csrc/kernels/crc.hip``; the first write cross-checks it against zlib).
  The file holds the same records as ``torch.save`` of the same state dict (only the per-save
  ``.data/serialization_id`` is the template's), so ``torch.load(weights_only=True)`` and any zip tool
  (CRCs included) read it;
* **every submitted checkpoint is written, in order**: each key has a ring of staging slots; a submit
  that finds them all queued or being written waits for the writer (back-pressure, counted in
  ``stalls``) instead of dropping a round's file.  ``dropped`` counts deferred states that were
  superseded before their copy was issued (the engine never does that; kept for diagnostics).

A background thread waits for each copy's event and writes the file atomically (``.tmp`` +
``os.replace``), so a reader never sees a half-written checkpoint.
"""
from __future__ import annotations

import collections
import io
import os
import struct
import threading
import zlib
from typing import Callable, Dict, Optional, Tuple

import torch

SLOTS = 3  # staging buffers per key: one being copied, one queued, one being written


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """zlib's crc32_combine: CRC of A || B from crc(A), crc(B) and len(B) (GF(2) polynomial arithmetic)."""
    def multmodp(a: int, b: int) -> int:
        p, m = 0, 1 << 31
        while m:
            if a & m:
                p ^= b
                if (a & (m - 1)) == 0:
                    break
            m >>= 1
            b = (b >> 1) ^ 0xEDB88320 if b & 1 else b >> 1
        return p

    x, e, r = 1 << 30, len2 * 8, 1 << 31  # x^1; exponent; x^0
    while e:
        if e & 1:
            r = multmodp(x, r)
        x = multmodp(x, x)
        e >>= 1
    return multmodp(r, crc1) ^ crc2 if len2 else crc1


class ZipTemplate:
    """``torch.save`` archive of a state dict whose tensors all view ONE storage, split around that
    storage's bytes so later states are written without re-serialising."""

    def __init__(self, blob: bytes, storage_bytes: int):
        eocd = blob.rfind(b"PK\x05\x06")
        if eocd < 0:
            raise ValueError("no end-of-central-directory record")
        n_entries, cd_size, cd_off = struct.unpack_from("<HII", blob, eocd + 10)
        if cd_off == 0xFFFFFFFF or n_entries == 0xFFFF:
            raise ValueError("zip64 archive")
        hits = []
        pos = cd_off
        for _ in range(n_entries):
            if blob[pos:pos + 4] != b"PK\x01\x02":
                raise ValueError("bad central directory entry")
            method, = struct.unpack_from("<H", blob, pos + 10)
            csize, usize = struct.unpack_from("<II", blob, pos + 20)
            nlen, xlen, clen = struct.unpack_from("<HHH", blob, pos + 28)
            loc, = struct.unpack_from("<I", blob, pos + 42)
            name = blob[pos + 46:pos + 46 + nlen].decode("utf-8", "replace")
            parts = name.split("/")
            if len(parts) >= 2 and parts[-2] == "data" and parts[-1].isdigit():
                hits.append((pos, loc, method, csize, usize))
            pos += 46 + nlen + xlen + clen
        if len(hits) != 1:
            raise ValueError(f"{len(hits)} storage records (need exactly one)")
        cd_pos, loc, method, csize, usize = hits[0]
        if method != 0 or csize != usize or usize != storage_bytes:
            raise ValueError("storage record is compressed or has the wrong size")
        if blob[loc:loc + 4] != b"PK\x03\x04":
            raise ValueError("bad local header")
        nlen, xlen = struct.unpack_from("<HH", blob, loc + 26)
        data = loc + 30 + nlen + xlen
        self.prefix = bytearray(blob[:data])
        self.suffix = bytearray(blob[data + usize:])
        self.crc_local = loc + 14                      # in prefix
        self.crc_cd = cd_pos + 16 - (data + usize)     # in suffix
        self.data_off = data
        self.size = usize

    def write(self, path: str, payload: memoryview, crc: int) -> None:
        struct.pack_into("<I", self.prefix, self.crc_local, crc)
        struct.pack_into("<I", self.suffix, self.crc_cd, crc)
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            for part in (memoryview(self.prefix), payload, memoryview(self.suffix)):
                while len(part):
                    n = os.write(fd, part)
                    part = part[n:]
        finally:
            os.close(fd)


class _Slot:
    __slots__ = ("host", "crc", "busy")

    def __init__(self, host: torch.Tensor, crc: Optional[torch.Tensor]):
        self.host = host
        self.crc = crc
        self.busy = False


class CheckpointWriter:
    def __init__(self, asynchronous: bool = True, fast: bool = True):
        self.asynchronous = asynchronous
        self.fast = fast
        self._slots: Dict[str, list] = {}
        self._tails: Dict[str, Tuple[torch.Tensor, int]] = {}  # key -> (constant host tail, its crc)
        self._tmpl: Dict[str, Optional[ZipTemplate]] = {}
        self._cv = threading.Condition()
        self._queue: collections.deque = collections.deque()  # (key, slot, build, path, event) in submit order
        self._writing = 0
        self._err: Optional[BaseException] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self.dropped = 0               # deferred states superseded before their copy was issued
        self.stalls = 0                # submits that waited for a free staging slot
        self.written = 0               # files written
        self.template_writes = 0       # of which through the zip template
        self._stream = None            # side stream of the device -> host copies
        self._copied = None            # event: the last copy has read its source
        self._deferred = None          # (key, src, build, path, tail, event on the compute stream) not copied yet

    # ---- staging ---------------------------------------------------------------------------------
    def _slot(self, key: str, src: torch.Tensor, tail: Optional[torch.Tensor]) -> _Slot:
        """A free pinned staging slot for ``key`` (waits for the writer when all are in use)."""
        n = src.numel() + (tail.numel() if tail is not None else 0)
        ring = self._slots.get(key)
        if ring is None or ring[0].host.numel() != n or ring[0].host.dtype != src.dtype:
            with self._cv:
                while self._writing or any(s.busy for s in (ring or [])):
                    self._cv.wait()
            ring = []
            for _ in range(SLOTS):
                host = torch.empty(n, dtype=src.dtype, pin_memory=True)
                if tail is not None:
                    host[src.numel():].copy_(tail.reshape(-1))
                crc = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                ring.append(_Slot(host, crc))
            self._slots[key] = ring
            if tail is not None:
                tb = tail.reshape(-1).contiguous().numpy().tobytes()
                self._tails[key] = (tail, zlib.crc32(tb), len(tb))
            else:
                self._tails.pop(key, None)
            self._tmpl.pop(key, None)
        with self._cv:
            while True:
                self._raise()
                for s in ring:
                    if not s.busy:
                        s.busy = True
                        return s
                self.stalls += 1
                self._cv.wait()

    def submit(self, key: str, src: torch.Tensor, build: Callable[[torch.Tensor], object], path: str,
               defer: bool = False, tail: Optional[torch.Tensor] = None) -> None:
        """Save ``build(host staging buffer)`` to ``path``.  The staging buffer holds ``src`` followed by the
        constant host tensor ``tail`` (if given), so ``build`` can return views of ONE storage (which makes the
        zip-template path apply).  ``src`` may be overwritten right after return (with ``defer``: only after
        ``fence`` or ``kick``; the copy is taken of the state as of this call)."""
        src = src.detach()
        if not src.is_cuda or not self.asynchronous:
            self.flush()
            host = src.cpu() if src.is_cuda else src.clone()
            if tail is not None:
                host = torch.cat([host.reshape(-1), tail.reshape(-1).to(host.dtype)])
            _atomic_save(build(host), path)
            self.written += 1
            return
        if defer:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(src.device))
            if self._deferred is not None:
                self.dropped += 1              # superseded before its copy was issued
            self._deferred = (key, src, build, path, tail, ev)
            return
        self.kick()                            # an older deferred state goes out first (files stay in order)
        self._copy(key, src, build, path, tail, None)

    def kick(self) -> None:
        """Issue the deferred copy, if any (side stream, ordered after the state it saves)."""
        d, self._deferred = self._deferred, None
        if d is not None:
            self._copy(*d)

    def _copy(self, key, src, build, path, tail, after: Optional[torch.cuda.Event]) -> None:
        slot = self._slot(key, src, tail)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=src.device)
        if after is not None:
            self._stream.wait_event(after)                                  # src as of the deferred submit
        else:
            self._stream.wait_stream(torch.cuda.current_stream(src.device))  # src as produced so far
        with torch.cuda.stream(self._stream):
            slot.host[:src.numel()].copy_(src.reshape(-1), non_blocking=True)
            if self.fast and src.dtype == torch.float32 and src.numel() > 0:
                from ..ops import native

                slot.crc.copy_(native().crc32(src.reshape(-1)), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        src.record_stream(self._stream)  # the allocator keeps src's memory until the copy has run
        if after is None:
            # an immediate submit promises that src may be overwritten right after return: the caller's stream
            # waits (on the device) for the copy AND the CRC pass — without it a write queued behind the submit
            # could land between the two, and the GPU CRC then disagreed with the staged bytes (the template
            # path was dropped for the key: tests/test_gpu_engine.py::test_checkpoint_every_submit_written_in_order)
            torch.cuda.current_stream(src.device).wait_event(ev)
        self._copied = ev
        with self._cv:
            self._queue.append((key, slot, build, path, ev))
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

    # ---- writer thread -----------------------------------------------------------------------------
    def _write(self, key: str, slot: _Slot, build, path: str) -> None:
        tmp = path + ".tmp"
        tmpl = self._tmpl.get(key, False)
        gpu_crc = slot.crc is not None and self.fast and slot.host.dtype == torch.float32
        n_src = slot.host.numel() - (self._tails[key][0].numel() if key in self._tails else 0)
        if tmpl is False and self.fast:
            # first write of this key: serialise once, keep the archive as a template when it has the
            # single-storage form, and cross-check the GPU CRC against zlib on these very bytes
            buf = io.BytesIO()
            torch.save(build(slot.host), buf)
            blob = buf.getvalue()
            try:
                t = ZipTemplate(blob, slot.host.numel() * slot.host.element_size())
                if blob[t.data_off:t.data_off + t.size] != slot.host.numpy().tobytes():
                    raise ValueError("storage bytes are not the staging buffer")
                if gpu_crc and self._crc(key, slot, n_src) != zlib.crc32(memoryview(slot.host.numpy()).cast("B")):
                    raise ValueError("GPU CRC-32 disagrees with zlib")
                self._tmpl[key] = t
            except ValueError as e:
                from .log import print_with_color

                print_with_color(f"[ckpt] {os.path.basename(path)}: torch.save path ({e})", "yellow")
                self._tmpl[key] = None
            with open(tmp, "wb") as fh:
                fh.write(blob)
        elif tmpl and gpu_crc:
            tmpl.write(tmp, memoryview(slot.host.numpy()).cast("B"), self._crc(key, slot, n_src))
            self.template_writes += 1
        else:
            torch.save(build(slot.host), tmp)
        os.replace(tmp, path)
        self.written += 1

    def _crc(self, key: str, slot: _Slot, n_src: int) -> int:
        c = int(slot.crc.item()) & 0xFFFFFFFF
        if key in self._tails:
            _, tcrc, tlen = self._tails[key]
            c = crc32_combine(c, tcrc, tlen)
        return c

    def _run(self) -> None:
        while True:
            with self._cv:
                while not self._queue and not self._stop:
                    self._cv.wait()
                if not self._queue:
                    return
                key, slot, build, path, ev = self._queue.popleft()
                self._writing += 1
            try:
                ev.synchronize()
                self._write(key, slot, build, path)
            except BaseException as e:  # noqa: BLE001 - re-raised in the caller
                with self._cv:
                    self._err = e
            with self._cv:
                slot.busy = False
                self._writing -= 1
                self._cv.notify_all()

    def _raise(self) -> None:
        if self._err is not None:
            e, self._err = self._err, None
            raise e

    def flush(self) -> None:
        """Wait until every submitted checkpoint is on disk (re-raises a write error)."""
        self.kick()
        with self._cv:
            while self._queue or self._writing:
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
