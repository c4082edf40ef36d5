"""Op dispatch: HIP kernels for device tensors, PyTorch composites for CPU tensors.

Rule: a CUDA (ROCm) tensor ALWAYS goes to the native gfx950 kernel in ``attackfl_amd/_C.so``;
if that extension is missing on a GPU box the call raises (no silent eager fallback).  CPU
tensors run the composites in ``ops/composite.py``, which double as the numerical oracles in
the test-suite.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple, Optional

import torch

from . import composite

_NATIVE = None


def native():
    """Return the loaded native extension or raise with build instructions."""
    global _NATIVE
    if _NATIVE is None:
        try:
            variant = os.environ.get("AFL_NATIVE_SO")  # A/B builds (tools/ab_native.sh): another in-tree .so
            if variant:
                import importlib.machinery
                import importlib.util

                loader = importlib.machinery.ExtensionFileLoader("attackfl_amd._C", variant)
                spec = importlib.util.spec_from_file_location("attackfl_amd._C", variant, loader=loader)
                _C = importlib.util.module_from_spec(spec)
                loader.exec_module(_C)
            else:
                from .. import _C  # noqa: F401

            _NATIVE = _C
        except Exception as e:  # pragma: no cover - depends on build state
            _NATIVE = e
    if isinstance(_NATIVE, Exception):
        raise RuntimeError("attackfl_amd native extension (_C.so) is not built/loadable; run "
                           "`python -m attackfl_amd._build`: " + repr(_NATIVE))
    return _NATIVE


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def _dev(t: torch.Tensor) -> bool:
    return t.is_cuda


def _tiles(slots, P: int, tile: int = 4096):
    """Split [0, P) into tiles that never cross a slot boundary -> int32 [T, 3] (seg, start, end)."""
    rows = []
    for si, s in enumerate(slots):
        a, b = s.offset, s.offset + s.numel
        while a < b:
            e = min(b, a + tile)
            rows.append((si, a, e))
            a = e
    return torch.tensor(rows, dtype=torch.int32)


_TILE_CACHE = {}


def _tile_table(slots, P: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    key = (tuple((s.offset, s.numel) for s in slots), P, str(device))
    if key not in _TILE_CACHE:
        t = _tiles(slots, P)
        # segment -> [first tile, last tile) ranges for the deterministic second pass
        seg_first = torch.zeros(len(slots) + 1, dtype=torch.int32)
        for i in range(t.shape[0]):
            seg_first[int(t[i, 0]) + 1] = i + 1
        for si in range(1, len(slots) + 1):
            seg_first[si] = max(int(seg_first[si]), int(seg_first[si - 1]))
        _TILE_CACHE[key] = (t.to(device), seg_first.to(device))
    return _TILE_CACHE[key]


class _WholeSlot:
    def __init__(self, P):
        self.offset, self.numel, self.shape = 0, P, (P,)


# ---------------------------------------------------------------- column statistics / attacks
def column_mean_std(G: torch.Tensor):
    if _dev(G):
        out = native().colstats(G.contiguous(), 0, 0.0)
        return out[0], out[1]
    return composite.column_mean_std(G)


def lie_candidate(G: torch.Tensor, z: float) -> torch.Tensor:
    if _dev(G):
        return native().colstats(G.contiguous(), 1, float(z))[2]
    return composite.lie_candidate(G, z)


def pairwise_sqdist(G: torch.Tensor) -> torch.Tensor:
    """[K, K] fp64 squared L2 distances between rows.  Device: the centred Gram matrix on fp64 MFMA for
    K <= 64 (``k_gram_f64``), the fp64 difference loop beyond."""
    if _dev(G):
        if G.shape[0] <= 64:
            return native().pairwise_sqdist_gram(G.contiguous())
        return native().pairwise_sqdist(G.contiguous())
    return composite.pairwise_l2(G) ** 2


def pairwise_l2(G: torch.Tensor) -> torch.Tensor:
    if _dev(G):
        return pairwise_sqdist(G).clamp_min(0.0).sqrt()
    return composite.pairwise_l2(G)


def noise(own: torch.Tensor, sigma: float, seed: int) -> torch.Tensor:
    """``own + sigma * N(0, 1)`` from Philox4x32-10 keyed by ``seed`` (Random attack); the CPU mirror draws
    the same uniforms."""
    if _dev(own):
        return native().noise_philox(own.contiguous(), float(sigma),
                                     (int(seed) & 0xFFFFFFFFFFFFFFFF) - (1 << 64) if (int(seed) & (1 << 63))
                                     else int(seed) & 0xFFFFFFFFFFFFFFFF)
    return composite.noise(own, sigma, seed)


def segment_l2_sum(diffs: torch.Tensor, slots) -> torch.Tensor:
    if _dev(diffs):
        tiles, segf = _tile_table(slots, diffs.shape[1], diffs.device)
        sq = native().segment_sqsum(diffs.contiguous(), tiles, segf, len(slots))  # [M, S] fp64
        return sq.clamp_min(0.0).sqrt().sum(dim=1)
    return composite.segment_l2_sum(diffs, slots)


def batched_spectral_norm(mats: torch.Tensor) -> torch.Tensor:
    if _dev(mats):
        return native().spectral_norm(mats.contiguous())
    return composite.batched_spectral_norm(mats)


_SPEC_CACHE = {}


def _spectral_table(slots, device):
    """(tab [S', 4] int32 for slots with min(r, c) <= 128, max n, scratch floats per row, big slots)."""
    key = (tuple((s.offset, s.numel, s.shape[0]) for s in slots), str(device))
    if key not in _SPEC_CACHE:
        rows, big, scr, max_n = [], [], 0, 0
        for s in slots:
            r = int(s.shape[0])
            c = s.numel // r
            n = min(r, c)
            if n > 128:
                big.append(s)
                continue
            n8 = (n + 7) & ~7
            rows.append((s.offset, r, c, scr))
            scr += n8 * n8
            max_n = max(max_n, n)
        tab = torch.tensor(rows, dtype=torch.int32).reshape(-1, 4).to(device)
        _SPEC_CACHE[key] = (tab, max_n, scr, big)
    return _SPEC_CACHE[key]


_GRAM_CACHE = {}
_GRAM_NMAX = 64
_GRAM_LDS_FLOATS = 40 * 1024  # X and D of one slot staged whole in LDS (160 KB)


def _gram_table(slots, device):
    """Gram-form slots (n = min(r, c) <= 64, X and D fit in LDS): (tab [S', 4] int32 {offset, r, c, arena
    offset}, sumq, max LDS floats, the remaining slots)."""
    key = (tuple((s.offset, s.numel, s.shape[0]) for s in slots), str(device))
    if key not in _GRAM_CACHE:
        rows, rest, sumq, lds = [], [], 0, 0
        for s in slots:
            r = int(s.shape[0])
            c = s.numel // r
            n, k = min(r, c), max(r, c)
            need = 2 * n * (k + 1)
            if n > _GRAM_NMAX or need > _GRAM_LDS_FLOATS:
                rest.append(s)
                continue
            n16 = (n + 15) & ~15
            rows.append((s.offset, r, c, sumq))
            sumq += n16 * n16
            lds = max(lds, need)
        tab = torch.tensor(rows, dtype=torch.int32).reshape(-1, 4).to(device)
        _GRAM_CACHE[key] = (tab, sumq, lds, rest)
    return _GRAM_CACHE[key]


class SpectralFamily:
    """sum over matrix slots of ||X[m, slot] - γ·dev[slot]||_2 for every row m, for any γ (device).

    Reference: the per-tensor ord-2 norms of src/Utils.py:47 inside the bisections of src/Utils.py:101-204.
    The n x n Grams of X, X D^T + D X^T and D D^T are formed ONCE (``k_spec_grams``); each γ then costs one
    small launch (``k_spec_eval``: A - γS + γ²C, squarings on fp64 MFMA, Rayleigh quotient) that reads γ from
    device memory.  Slots outside the Gram form (n > 64) fall back to materialised rows per γ."""

    def __init__(self, X: torch.Tensor, slots, dev: Optional[torch.Tensor] = None):
        self.X = X.contiguous()
        self.dev = dev.contiguous() if dev is not None else None
        self.slots = slots
        self.tab, self.sumq, lds, self.rest = _gram_table(slots, X.device)
        self.arena = None
        if self.tab.shape[0] and X.shape[0]:
            self.arena = native().spec_grams(self.X, self.dev, self.tab, lds, self.sumq)

    def __call__(self, gamma=None) -> torch.Tensor:
        M = self.X.shape[0]
        out = torch.zeros(M, dtype=torch.float64, device=self.X.device)
        if M == 0:
            return out
        g = None
        if gamma is not None and self.dev is not None:
            g = gamma if torch.is_tensor(gamma) else torch.tensor(float(gamma), dtype=torch.float64)
            g = g.to(device=self.X.device, dtype=torch.float64).reshape(())
        if self.arena is not None:
            out += native().spec_eval(self.arena, self.tab, self.sumq, M, g).sum(dim=1)
        if self.rest:
            rows = self.X if g is None else self.X - (g * self.dev.double()).float()[None, :]
            out += _spectral_slots_direct(rows, self.rest)
        return out


def _spectral_slots_direct(diffs: torch.Tensor, slots) -> torch.Tensor:
    diffs = diffs.contiguous()
    tab, max_n, scr, big = _spectral_table(slots, diffs.device)
    out = torch.zeros(diffs.shape[0], dtype=torch.float64, device=diffs.device)
    if tab.shape[0]:
        out += native().spectral_norm_slots(diffs, tab, max_n, scr).sum(dim=1)
    for s in big:
        mats = diffs[:, s.offset:s.offset + s.numel].reshape(diffs.shape[0], s.shape[0], -1)
        out += native().spectral_norm(mats.contiguous())
    return out


def spectral_norm_sum(diffs: torch.Tensor, slots) -> torch.Tensor:
    """sum over matrix slots of ||diffs[m, slot]||_2 (slot viewed as [shape[0], -1]) -> [M] fp64.

    Device: the Gram form (two launches for every (row, slot) pair, reference src/Utils.py:47 per-tensor
    norm); slots with n > 64 through the direct ragged launch."""
    if _dev(diffs):
        return SpectralFamily(diffs, slots)()
    out = torch.zeros(diffs.shape[0], dtype=torch.float64, device=diffs.device)
    for s in slots:
        mats = diffs[:, s.offset:s.offset + s.numel].reshape(diffs.shape[0], s.shape[0], -1)
        out += composite.batched_spectral_norm(mats)
    return out


def attack_coeffs(G: torch.Tensor, mean: torch.Tensor, dev: torch.Tensor):
    if _dev(G):
        A, B, C = attack_coeffs_segments(G, mean, dev, [_WholeSlot(G.shape[1])])
        return A[:, 0], B[:, 0], C[0]
    return composite.attack_coeffs(G, mean, dev)


def attack_coeffs_segments(G: torch.Tensor, mean: torch.Tensor, dev: torch.Tensor, slots):
    if _dev(G):
        tiles, segf = _tile_table(slots, G.shape[1], G.device)
        A, B, C = native().attack_coeffs(G.contiguous(), mean.contiguous(), dev.contiguous(), tiles, segf, len(slots))
        return A, B, C
    return composite.attack_coeffs_segments(G, mean, dev, slots)


# ---------------------------------------------------------------- aggregation
def weighted_rows(U: torch.Tensor, w: torch.Tensor, ok: Optional[torch.Tensor] = None,
                  fallback: Optional[torch.Tensor] = None) -> torch.Tensor:
    """sum_i w_i U_i; with ``ok`` / ``fallback``: ``fallback`` unless every ``ok`` > 0 (one pass on the device)."""
    if _dev(U):
        if ok is not None:
            return native().weighted_rows(U.contiguous(), w.to(device=U.device, dtype=torch.float64).contiguous(),
                                          ok.to(torch.int32).contiguous(), fallback.contiguous())
        return native().weighted_rows(U.contiguous(), w.to(device=U.device, dtype=torch.float64).contiguous())
    out = composite.weighted_rows(U, w)
    return out if ok is None else torch.where((ok > 0).all(), out, fallback)


def fedavg(U: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
    s = sizes.to(torch.float64)
    if _dev(U):
        return weighted_rows(U, s / s.sum())
    return composite.fedavg(U, sizes)


def coord_median(U: torch.Tensor) -> torch.Tensor:
    if _dev(U):
        return native().coord_select(U.contiguous(), 0, 0)
    return composite.coord_median(U)


def trimmed_mean(U: torch.Tensor, trim_k: int) -> torch.Tensor:
    if _dev(U):
        return native().coord_select(U.contiguous(), 1, int(trim_k))
    return composite.trimmed_mean(U, trim_k)


def row_norms(U: torch.Tensor) -> torch.Tensor:
    if _dev(U):
        return native().row_dots(U.contiguous(), U.new_zeros(0), 0)[:, 0].clamp_min(0).sqrt()
    return composite.row_norms(U)


def cosine_to(U: torch.Tensor, ref: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    if _dev(U):
        d = native().row_dots(U.contiguous(), ref.contiguous(), 1)  # [N, 3]: <u,u>, <u,r>, <r,r>
        den = torch.clamp(d[:, 0].sqrt() * d[:, 2].sqrt(), min=eps)
        return d[:, 1] / den
    return composite.cosine_to(U, ref, eps)


def stochastic_quantize(U: torch.Tensor, seed: int):
    if _dev(U):
        sigma, smin, smax = native().stoch_quant(U.contiguous(), int(seed) & 0x7FFFFFFFFFFFFFFF)
        return sigma, smin, smax
    return composite.stochastic_quantize(U, int(seed) & 0x7FFFFFFFFFFFFFFF)  # (the kernel's uniforms)


# ---------------------------------------------------------------- optimizer
def adam_step(p, g, m, v, step: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8) -> None:
    if _dev(p):
        native().adam_flat(p, g, m, v, int(step), float(lr), float(beta1), float(beta2), float(eps), 1.0)
        return
    composite.adam_step(p, g, m, v, step, lr, beta1, beta2, eps)


# ---------------------------------------------------------------- metrics
def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    if _dev(scores):
        return float(native().roc_auc(scores.reshape(-1).float().contiguous(), labels.reshape(-1).float().contiguous()))
    return composite.roc_auc(scores, labels)


def roc_auc_checked(scores: torch.Tensor, labels: torch.Tensor):
    """(ROC-AUC, any NaN score) with ONE host synchronisation on the device path."""
    if _dev(scores):
        r = native().roc_auc_dev(scores.reshape(-1).float().contiguous(), labels.reshape(-1).float().contiguous())
        auc, nan = r.cpu().tolist()
        return auc, nan > 0.5
    nan = bool(torch.isnan(scores).any())
    return (float("nan") if nan else composite.roc_auc(scores, labels)), nan


def adam_step_scaled(p, g, m, v, step: int, lr: float, scale: float, beta1=0.9, beta2=0.999, eps=1e-8) -> None:
    if _dev(p):
        native().adam_flat(p, g, m, v, int(step), float(lr), float(beta1), float(beta2), float(eps), float(scale))
        return
    composite.adam_step_scaled(p, g, m, v, step, lr, scale, beta1, beta2, eps)


# ---------------------------------------------------------------- hypernetwork
def hyper_delta_vjp(W: torch.Tensor, b: torch.Tensor, feat: torch.Tensor, u: torch.Tensor):
    if _dev(W):
        out = native().hyper_delta_vjp(W, b, feat.contiguous(), u.contiguous())
        return out[0], out[1]
    return composite.hyper_delta_vjp(W, b, feat, u)


def hyper_adam_outer(W, b, m_wb, v_wb, delta, feat, step: int, lr: float, scale: float) -> None:
    if _dev(W):
        native().hyper_adam_outer(W, b, m_wb, v_wb, delta.contiguous(), feat.contiguous(), int(step), float(lr),
                                  0.9, 0.999, 1e-8, float(scale))
        return
    composite.hyper_adam_outer(W, b, m_wb, v_wb, delta, feat, step, lr, scale)


def hyper_server_update(arena, m, v, U, urows, clients, layout, step0: int, lr: float, clip: float,
                        beta1=0.9, beta2=0.999, eps=1e-8, enable: Optional[torch.Tensor] = None, gen=()):
    """Sequential pFedHN server update of a whole round on the device (no host sync) -> (info [n, 2],
    generated [len(gen), P]).  ``enable``: optional device int32 word; 0 leaves arena / moments untouched (decided
    on the device).  ``gen``: clients whose models the updated hypernetwork generates inside the update's last
    launches (the next START; <= 32)."""
    info, out = native().hyper_server_update(arena, m, v, U.contiguous(), [int(r) for r in urows],
                                             [int(c) for c in clients], [int(x) for x in layout], int(step0),
                                             float(lr), float(clip), float(beta1), float(beta2), float(eps), enable,
                                             [int(c) for c in gen])
    return info, out


def hyper_features(arena, clients, layout) -> torch.Tensor:
    return native().hyper_features(arena, [int(c) for c in clients], [int(x) for x in layout])


def hyper_generate_many(arena, clients, layout) -> torch.Tensor:
    """Models [n, P] of ``clients`` generated from the packed hypernetwork arena (device; the same per-row
    arithmetic as the generation fused into ``hyper_server_update``)."""
    return native().hyper_generate_many(arena, [int(c) for c in clients], [int(x) for x in layout])


def hyper_generate(W: torch.Tensor, b: torch.Tensor, feat: torch.Tensor) -> torch.Tensor:
    if _dev(W):
        return native().hyper_generate(W, b, feat.contiguous())
    return torch.addmv(b, W, feat)
