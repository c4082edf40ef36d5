"""Logging: ``app.log`` writer, coloured console output and JSONL round metrics.

Parity target: reference ``src/Log.py:4-44`` (logger named ``my_logger``, DEBUG level,
``%(asctime)s - %(name)s - %(levelname)s - %(message)s`` file format, ANSI colour helper).
The JSONL metrics stream is new: one record per round with per-phase timings.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any, Dict, Optional

ANSI = {
    "header": "\033[95m",
    "blue": "\033[94m",
    "green": "\033[92m",
    "yellow": "\033[93m",
    "red": "\033[91m",
    "end": "\033[0m",
}

_QUIET = os.environ.get("ATTACKFL_QUIET", "0") == "1"


def set_quiet(flag: bool) -> None:
    """Silence coloured console chatter (bench runs, tests)."""
    global _QUIET
    _QUIET = bool(flag)


def print_with_color(text: str, color: str) -> None:
    if _QUIET:
        return
    code = ANSI.get(str(color).lower(), ANSI["end"])
    sys.stdout.write(f"{code}{text}{ANSI['end']}\n")
    sys.stdout.flush()


class Logger:
    """File logger writing the same line format as the reference ``app.log``."""

    NAME = "my_logger"
    FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"

    def __init__(self, log_path: str):
        d = os.path.dirname(os.path.abspath(log_path))
        os.makedirs(d, exist_ok=True)
        self.path = log_path
        self.logger = logging.getLogger(self.NAME)
        self.logger.setLevel(logging.DEBUG)
        self.logger.propagate = False
        # one handler per file, even when several engines are built in one process (tests)
        for h in self.logger.handlers:
            if isinstance(h, logging.FileHandler) and os.path.abspath(h.baseFilename) == os.path.abspath(log_path):
                self._handler = h
                break
        else:
            h = logging.FileHandler(log_path)
            h.setLevel(logging.DEBUG)
            h.setFormatter(logging.Formatter(self.FORMAT))
            self.logger.addHandler(h)
            self._handler = h

    def log_info(self, message: str) -> None:
        self.logger.info(message)

    def log_warning(self, message: str) -> None:
        self.logger.warning(message)

    def log_error(self, message: str) -> None:
        self.logger.error(message)

    def close(self) -> None:
        try:
            self.logger.removeHandler(self._handler)
            self._handler.close()
        except Exception:
            pass


class NullLogger:
    """Logger stand-in for non-leader ranks."""

    def log_info(self, message: str) -> None:  # noqa: D401
        pass

    log_warning = log_info
    log_error = log_info

    def close(self) -> None:
        pass


class MetricsWriter:
    """Append-only JSONL metrics (one object per line)."""

    def __init__(self, path: Optional[str]):
        self.path = path
        self._fh = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def write(self, record: Dict[str, Any]) -> None:
        if self._fh is None:
            return
        rec = {"ts": time.time()}
        rec.update(record)
        self._fh.write(json.dumps(rec, default=_json_default) + "\n")

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None


def _json_default(o):
    try:
        import numpy as np

        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
    except Exception:
        pass
    try:
        import torch

        if isinstance(o, torch.Tensor):
            return o.detach().cpu().tolist()
    except Exception:
        pass
    return str(o)
