"""Phase tracing: roctx ranges around every round phase (local training, attack, all-gather,
aggregation, detection, validation, checkpoint), visible in ``rocprofv3 --marker-trace`` timelines
next to the kernels, plus wall-clock phase timers for the JSONL metrics.

The reference has no tracing at all.  Ranges go straight to ROCm's ``libroctx64``
through ctypes (no torch dependency); when the library is absent or tracing is off every call is a
no-op.  Enable with ``engine.trace: true`` or ``ATTACKFL_TRACE=1``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, Optional

_LIB = None
_ENABLED = os.environ.get("ATTACKFL_TRACE", "0") == "1"


def _lib():
    global _LIB
    if _LIB is None:
        _LIB = False
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        for name in (os.path.join(rocm, "lib", "libroctx64.so"), "libroctx64.so", "libroctx64.so.4"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _LIB = lib
                break
            except (OSError, AttributeError):
                continue
    return _LIB or None


def enable(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = bool(flag)


def enabled() -> bool:
    return _ENABLED and _lib() is not None


def push(name: str) -> None:
    if _ENABLED:
        lib = _lib()
        if lib is not None:
            lib.roctxRangePushA(name.encode())


def pop() -> None:
    if _ENABLED:
        lib = _lib()
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if _ENABLED:
        lib = _lib()
        if lib is not None:
            lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str, timers: Optional[Dict[str, float]] = None):  # noqa: A001 - roctx vocabulary
    """``with trace.range("fl/local", timers):`` — roctx range + wall-clock seconds into ``timers``."""
    push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if timers is not None:
            timers[name] = timers.get(name, 0.0) + time.perf_counter() - t0
        pop()
