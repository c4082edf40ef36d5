"""Plain-PyTorch composites of every native op.

These are the CPU implementations *and* the numerical oracles that the HIP kernels in
``csrc/kernels`` are tested against (fp32/fp64 PyTorch references of the same op).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch


# ---------------------------------------------------------------- loss
class _BCE(torch.autograd.Function):
    """``nn.BCELoss`` (mean) forward AND backward, minus the [0, 1] input-range check.

    Forward: ``-(y·max(log p, -100) + (1-y)·max(log1p(-p), -100))``, mean.  Backward: torch's
    ``(p - y) / max(p (1 - p), 1e-12)`` per element over N — finite where the sigmoid saturates to exactly
    0 or 1 in fp32.  Autograd through the clamped logs instead gives ``0 · inf = NaN`` there (the derivative
    of the clamped branch is 0, of the log ∓inf), a NaN gradient the reference (``client.py:76`` BCELoss)
    never produces: after an Opt-Fang round that turned a healthy reference client into a NaN-loss failure.
    A NaN input still yields a NaN loss (the NaN abort test, ``client.py:100-102``)."""

    @staticmethod
    def forward(ctx, p, y):
        ctx.save_for_backward(p, y)
        lv = -(y * torch.clamp(torch.log(p), min=-100.0) + (1 - y) * torch.clamp(torch.log1p(-p), min=-100.0))
        return lv.mean()

    @staticmethod
    def backward(ctx, g):
        p, y = ctx.saved_tensors
        gp = g * (p - y) / torch.clamp((1 - p) * p, min=1e-12) / p.numel()
        return gp, None


def bce_loss(p: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Mean BCE of probabilities ``p`` against targets ``y`` with ``nn.BCELoss``'s gradient (``_BCE``)."""
    return _BCE.apply(p, y.to(p.dtype).expand_as(p))


# ---------------------------------------------------------------- column statistics / attacks
def column_mean_std(G: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    mean = G.mean(dim=0)
    std = G.std(dim=0) if G.shape[0] > 1 else torch.full_like(mean, float("nan"))
    return mean, std


def lie_candidate(G: torch.Tensor, z: float) -> torch.Tensor:
    mean, std = column_mean_std(G)
    return mean + z * std


def pairwise_l2(G: torch.Tensor) -> torch.Tensor:
    Gd = G.double()
    sq = (Gd * Gd).sum(dim=1)
    gram = Gd @ Gd.t()
    d2 = (sq[:, None] + sq[None, :] - 2.0 * gram).clamp_min(0.0)
    d2.fill_diagonal_(0.0)
    return d2.sqrt()


def gram(G: torch.Tensor) -> torch.Tensor:
    Gd = G.double()
    return Gd @ Gd.t()


def segment_l2_sum(diffs: torch.Tensor, slots) -> torch.Tensor:
    out = torch.zeros(diffs.shape[0], dtype=torch.float64, device=diffs.device)
    for s in slots:
        seg = diffs[:, s.offset:s.offset + s.numel].double()
        out += torch.linalg.vector_norm(seg, dim=1)
    return out


def batched_spectral_norm(mats: torch.Tensor) -> torch.Tensor:
    return torch.linalg.matrix_norm(mats.double(), ord=2).to(torch.float64)


def attack_coeffs(G: torch.Tensor, mean: torch.Tensor, dev: torch.Tensor):
    Gd, md, dd = G.double(), mean.double(), dev.double()
    r = md[None, :] - Gd
    A = (r * r).sum(dim=1)
    B = (r * dd[None, :]).sum(dim=1)
    C = (dd * dd).sum()
    return A, B, C


def attack_coeffs_segments(G: torch.Tensor, mean: torch.Tensor, dev: torch.Tensor, slots):
    K = G.shape[0]
    S = len(slots)
    A = torch.zeros(K, S, dtype=torch.float64, device=G.device)
    B = torch.zeros(K, S, dtype=torch.float64, device=G.device)
    C = torch.zeros(S, dtype=torch.float64, device=G.device)
    for i, s in enumerate(slots):
        sl = slice(s.offset, s.offset + s.numel)
        a, b, c = attack_coeffs(G[:, sl], mean[sl], dev[sl])
        A[:, i], B[:, i], C[i] = a, b, c
    return A, B, C


# ---------------------------------------------------------------- aggregation
def weighted_rows(U: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """sum_i w_i U_i  (w already normalised by the caller)."""
    return (w.to(U.dtype)[:, None] * U).sum(dim=0)


def fedavg(U: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
    s = sizes.to(torch.float64)
    return ((s[:, None] * U.double()).sum(dim=0) / s.sum()).to(U.dtype)


def coord_median(U: torch.Tensor) -> torch.Tensor:
    return torch.median(U, dim=0).values


def trimmed_mean(U: torch.Tensor, trim_k: int) -> torch.Tensor:
    n = U.shape[0]
    s, _ = torch.sort(U, dim=0)
    return s[trim_k:n - trim_k].mean(dim=0)


def row_norms(U: torch.Tensor) -> torch.Tensor:
    return torch.linalg.vector_norm(U.double(), dim=1)


def cosine_to(U: torch.Tensor, ref: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    Ud, rd = U.double(), ref.double()
    num = Ud @ rd
    den = torch.clamp(torch.linalg.vector_norm(Ud, dim=1) * torch.linalg.vector_norm(rd), min=eps)
    return num / den


def _mix64(z):
    """``afl_mix64`` (csrc/common.h, splitmix64 finaliser) on a numpy uint64 array."""
    import numpy as np

    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def afl_uniform(seed: int, n: int) -> torch.Tensor:
    """The [n] fp32 uniforms ``afl_uniform(seed, 0..n-1)`` of the device kernels (bit-identical)."""
    import numpy as np

    ctr = np.arange(n, dtype=np.uint64)
    x = _mix64(np.uint64(int(seed) & 0xFFFFFFFFFFFFFFFF) ^ _mix64(ctr)) >> np.uint64(40)
    return torch.from_numpy((x.astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32))


def stochastic_quantize(U: torch.Tensor, seed=None):
    """ScionFL 1-bit quantisation per row: returns (sigma [N,P] {0,1}, smin [N], smax [N]).  ``seed`` (int):
    the device kernel's counter-based uniforms ``afl_uniform(seed, row * P + col)`` — the same bits as
    ``k_stoch_quant``; a ``torch.Generator`` or None draws with torch instead."""
    smin = U.min(dim=1).values
    smax = U.max(dim=1).values
    probs = (U - smin[:, None]) / (smax - smin + 1e-6)[:, None]
    if isinstance(seed, int):
        u = afl_uniform(seed, U.numel()).reshape(U.shape).to(U.device)
    elif seed is not None:
        u = torch.rand(U.shape, generator=seed, device=U.device, dtype=U.dtype)
    else:
        u = torch.rand_like(U)
    sigma = (u < probs).to(U.dtype)
    return sigma, smin, smax


# ---------------------------------------------------------------- optimizer
def adam_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
              beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8) -> None:
    """In-place Adam (torch.optim.Adam default, non-foreach math)."""
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


# ---------------------------------------------------------------- metrics
def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """ROC-AUC with sklearn's tie handling (trapezoid over distinct thresholds)."""
    s = scores.reshape(-1).double()
    y = labels.reshape(-1).double()
    order = torch.argsort(s, descending=True, stable=True)
    s, y = s[order], y[order]
    tps = torch.cumsum(y, 0)
    fps = torch.cumsum(1 - y, 0)
    # keep the last index of every run of equal scores
    last = torch.ones_like(s, dtype=torch.bool)
    last[:-1] = s[1:] != s[:-1]
    tps, fps = tps[last], fps[last]
    P, N = tps[-1], fps[-1]
    if P <= 0 or N <= 0:
        return float("nan")
    tpr = torch.cat([tps.new_zeros(1), tps / P])
    fpr = torch.cat([fps.new_zeros(1), fps / N])
    return float(torch.trapz(tpr, fpr).item())


def adam_step_scaled(p, g, m, v, step: int, lr: float, scale: float, beta1=0.9, beta2=0.999, eps=1e-8) -> None:
    adam_step(p, g * scale, m, v, step, lr, beta1, beta2, eps)


# ---------------------------------------------------------------- hypernetwork
def hyper_delta_vjp(W: torch.Tensor, b: torch.Tensor, feat: torch.Tensor, u: torch.Tensor):
    """delta = W f + b - u  and  W^T delta (one pass over W in the native kernel)."""
    delta = torch.addmv(b, W, feat) - u
    return delta, W.t() @ delta


def hyper_adam_outer(W, b, m_wb, v_wb, delta, feat, step: int, lr: float, scale: float, beta1=0.9, beta2=0.999,
                     eps=1e-8) -> None:
    """Adam on the packed heads with grad(W) = scale·δ⊗f, grad(b) = scale·δ (never materialised natively)."""
    P, H = W.shape
    gW = torch.outer(delta, feat) * scale
    adam_step(W.view(-1), gW.view(-1), m_wb[:P * H], v_wb[:P * H], step, lr, beta1, beta2, eps)
    adam_step(b, delta * scale, m_wb[P * H:P * H + P], v_wb[P * H:P * H + P], step, lr, beta1, beta2, eps)


# ---------------------------------------------------------------- Philox noise (Random attack, K-G10)
_PHILOX_M0, _PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
_PHILOX_W0, _PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
_M32 = 0xFFFFFFFF


def philox4x32(counter_lo, seed: int):
    """Philox4x32-10 of counters (lo, hi, 0, 0) for a uint64 numpy array ``counter_lo`` -> 4 uint32 arrays
    (the exact integers ``k_noise_philox`` draws; ``agg.hip``)."""
    import numpy as np

    g = counter_lo.astype(np.uint64)
    c0, c1 = g & np.uint64(_M32), g >> np.uint64(32)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0, k1 = seed & _M32, (seed >> 32) & _M32
    for _ in range(10):
        p0 = c0 * np.uint64(_PHILOX_M0)
        p1 = c2 * np.uint64(_PHILOX_M1)
        h0, l0 = p0 >> np.uint64(32), p0 & np.uint64(_M32)
        h1, l1 = p1 >> np.uint64(32), p1 & np.uint64(_M32)
        c0, c1, c2, c3 = h1 ^ c1 ^ np.uint64(k0), l1, h0 ^ c3 ^ np.uint64(k1), l0
        k0, k1 = (k0 + _PHILOX_W0) & _M32, (k1 + _PHILOX_W1) & _M32
    return c0, c1, c2, c3


def philox_normal(n: int, seed: int):
    """N(0, 1) draws of ``k_noise_philox``: Box-Muller on (x + 1) * 2^-32 uniforms in fp64 -> [n] float64."""
    import numpy as np

    groups = (n + 3) // 4
    c0, c1, c2, c3 = philox4x32(np.arange(groups, dtype=np.uint64), seed)
    u = [(c.astype(np.float64) + 1.0) * 2.0 ** -32 for c in (c0, c1, c2, c3)]
    r0, r1 = np.sqrt(-2.0 * np.log(u[0])), np.sqrt(-2.0 * np.log(u[2]))
    t0, t1 = 2.0 * np.pi * u[1], 2.0 * np.pi * u[3]
    z = np.stack([r0 * np.cos(t0), r0 * np.sin(t0), r1 * np.cos(t1), r1 * np.sin(t1)], axis=1).reshape(-1)
    return z[:n]


def noise(own: torch.Tensor, sigma: float, seed: int) -> torch.Tensor:
    z = torch.from_numpy(philox_normal(own.numel(), int(seed) & 0xFFFFFFFFFFFFFFFF)).to(torch.float32)
    return own + float(sigma) * z.reshape(own.shape).to(own.device)
