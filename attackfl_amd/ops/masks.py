"""Bit-exact host mirror of the device dropout hash (``afl_keep`` in ``csrc/common.h``).

Every native dropout site draws its keep-mask from a stateless hash of
``(step key, layer id, row, column)`` with ``step key = hash32(client seed, step)``; the backward
kernels regenerate the same mask instead of storing it.  The composite (CPU) ops use this module so
the oracle applies exactly the masks the GPU applied.  (Bitwise parity with torch's Philox dropout
stream is impossible by construction; only the distribution matches.)
"""
from __future__ import annotations

import math

import numpy as np
import torch

M32 = 0xFFFFFFFF


def hash32(a: int, b: int) -> int:
    """``afl_hash32`` (lowbias32-style avalanche of two 32-bit words)."""
    a &= M32
    b &= M32
    x = ((a * 0x9E3779B1) & M32) ^ ((b + 0x7F4A7C15 + ((a << 6) & M32) + (a >> 2)) & M32)
    x ^= x >> 16
    x = (x * 0x21F0AAAD) & M32
    x ^= x >> 15
    x = (x * 0x735A2D97) & M32
    x ^= x >> 15
    return x


def step_key(seed: int, step: int) -> int:
    return hash32(int(seed), int(step))


def thr16(p: float) -> int:
    """Keep threshold on a 16-bit uniform: keep iff u16 >= round(p * 65536) (``std::lround``)."""
    return int(math.floor(p * 65536.0 + 0.5))


def keep(key: int, layer: int, rows, cols, p: float) -> torch.Tensor:
    """Keep-mask for broadcastable integer ``rows`` / ``cols`` index arrays -> bool tensor."""
    r = np.asarray(rows, dtype=np.uint64)
    col = np.asarray(cols, dtype=np.uint64)
    m = np.uint64(M32)
    c = col >> np.uint64(1)
    x = (np.uint64(key) ^ ((np.uint64(layer) * np.uint64(0x9E3779B9)) & m) ^ ((r * np.uint64(0x85EBCA6B)) & m)
         ^ ((c * np.uint64(0xC2B2AE35)) & m))
    x &= m
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & m
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & m
    x ^= x >> np.uint64(16)
    u16 = (x >> ((col & np.uint64(1)) << np.uint64(4))) & np.uint64(0xFFFF)
    return torch.from_numpy(np.ascontiguousarray(u16 >= np.uint64(thr16(p))))


def keep_grid(key: int, layer: int, n_rows: int, n_cols: int, p: float) -> torch.Tensor:
    """[n_rows, n_cols] keep-mask of a row-major tensor."""
    return keep(key, layer, np.arange(n_rows)[:, None], np.arange(n_cols)[None, :], p)


def scale_grid(seeds, step: int, layer: int, n_rows: int, n_cols: int, p: float) -> torch.Tensor:
    """Per-client dropout multipliers ``mask / (1 - p)`` -> float32 [C, n_rows, n_cols]."""
    out = torch.empty(len(seeds), n_rows, n_cols)
    for ci, s in enumerate(seeds):
        out[ci] = keep_grid(step_key(int(s), step), layer, n_rows, n_cols, p).float() / (1.0 - p)
    return out


def _hash4(key: int, layer: int, r, c) -> np.ndarray:
    """``afl_hash4`` on broadcastable uint64 arrays (32-bit arithmetic) -> uint64 array of 32-bit values."""
    m = np.uint64(M32)
    r = np.asarray(r, dtype=np.uint64)
    c = np.asarray(c, dtype=np.uint64)
    x = (np.uint64(key & M32) ^ ((np.uint64(layer & M32) * np.uint64(0x9E3779B9)) & m)
         ^ ((r * np.uint64(0x85EBCA6B)) & m) ^ ((c * np.uint64(0xC2B2AE35)) & m))
    x &= m
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & m
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & m
    x ^= x >> np.uint64(16)
    return x


def keep_rc(key: int, layer: int, rows, cols, p: float) -> torch.Tensor:
    """Attention-probability dropout of the bf16 HAR kernels (``har.hip`` ``attn_keep``): a strong hash per
    ROW and one per column PAIR, combined by xor and one multiply-xorshift round; the 32-bit result gives the
    16-bit uniforms of the pair's two columns.  The per-row and per-column hashes are computed once per
    workgroup (registers / an LDS table), so a probability costs half a 2-round mix instead of half a full
    hash4 — the attention kernels are VALU-bound and the full hash was most of their work."""
    m = np.uint64(M32)
    r = np.asarray(rows, dtype=np.uint64)
    col = np.asarray(cols, dtype=np.uint64)
    hr = _hash4(key, layer, r, M32)
    hc = _hash4(key ^ 0xA5A5A5A5, layer, 0, col >> np.uint64(1))
    x = (hr ^ hc) & m
    x = (x * np.uint64(0x7FEB352D)) & m
    x ^= x >> np.uint64(16)
    u16 = (x >> ((col & np.uint64(1)) << np.uint64(4))) & np.uint64(0xFFFF)
    return torch.from_numpy(np.ascontiguousarray(u16 >= np.uint64(thr16(p))))
