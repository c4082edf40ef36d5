"""Client-batched layer ops: HIP kernels (``csrc/kernels/layers.hip``, ``attention.hip``) for device
tensors, PyTorch composites for CPU tensors.

All ops write into caller-provided outputs (the step programs preallocate and graph-capture them).
Tensors are ``[C clients, rows, cols]``; weights are strided views into the flat ``[C, P]`` arena,
so ``W.transpose(1, 2)`` is free.  The composites are the fp32 numerical oracles of the kernels and
regenerate the same hash dropout masks (``ops/masks.py``); the native path uses bf16 MFMA operands
with fp32 accumulation.

Dropout convention: ``ctl`` carries the per-client seeds and the device step counter; a site is
identified by ``(layer id, row, column)`` of the tensor it masks.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import masks
from . import native as _native

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2


def upload(t: torch.Tensor, device) -> torch.Tensor:
    """Small host tensor -> ``device`` without blocking the host behind queued GPU work: pinned staging and a
    non-blocking copy (the caching host allocator keeps the staging block until the copy has run).  A pageable
    ``.to(device)`` waits for the stream, which held a speculative next-round launch of the layer-program /
    cnn2 path behind the round's running training kernel (the GPU then idled while the host enqueued it)."""
    device = torch.device(device)
    if device.type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


@dataclass
class StepCtl:
    """Per-client dropout seeds (int32 [C]) + the device step counter (int32 [1])."""

    seeds: torch.Tensor
    stepctl: torch.Tensor

    @classmethod
    def create(cls, seeds, device, min_bs: int = 2, nan_abort: bool = True) -> "StepCtl":
        """``stepctl = [step, min_bs, nan_abort]``: steps with fewer than ``min_bs`` rows are skipped (ICU:
        2, A-21) and a NaN loss aborts the client (ICU); the reference ``train_HAR`` does neither (1, False)."""
        s = torch.tensor([int(x) & masks.M32 for x in seeds], dtype=torch.int64)
        s = torch.where(s >= 2 ** 31, s - 2 ** 32, s).to(torch.int32)
        ctl = torch.tensor([0, int(min_bs), 1 if nan_abort else 0], dtype=torch.int32)
        return cls(upload(s, device), upload(ctl, device))

    # composite helpers
    def step(self) -> int:
        return int(self.stepctl[0])

    @property
    def min_bs(self) -> int:
        return int(self.stepctl[1])

    @property
    def nan_abort(self) -> bool:
        return bool(int(self.stepctl[2]))

    def key(self, c: int) -> int:
        return masks.step_key(int(self.seeds[c]) & masks.M32, self.step())


def _nat(t: torch.Tensor) -> bool:
    return t.is_cuda


def _dargs(ctl: Optional[StepCtl], p: float):
    if p <= 0.0 or ctl is None:
        return None, None
    return ctl.seeds, ctl.stepctl


def _scale(ctl: StepCtl, c: int, layer: int, rows, cols, p: float) -> torch.Tensor:
    return masks.keep(ctl.key(c), layer, rows, cols, p).float() / (1.0 - p)


def _act(v, act):
    return F.relu(v) if act == ACT_RELU else (F.gelu(v) if act == ACT_GELU else v)


def _actd(g, gact):
    if gact == ACT_RELU:
        return (g > 0).float()
    if gact == ACT_GELU:
        cdf = 0.5 * (1.0 + torch.erf(g * 0.7071067811865476))
        return cdf + g * 0.3989422804014327 * torch.exp(-0.5 * g * g)
    return torch.ones_like(g)


def _rc(M, N):
    return np.arange(M)[:, None], np.arange(N)[None, :]


# ------------------------------------------------------------------------------------------ GEMM
def bgemm(A, B, C, bias=None, Z=None, G=None, act=0, gact=0, accum=0, splitk=1, alpha=1.0,
          ctl: Optional[StepCtl] = None, layer: int = 0, p: float = 0.0, generic: bool = False, asum=None) -> None:
    """``C (op)= epi(alpha * A @ B^T)``; A [C,M,K], B [C,N,K], C [C,M,N].

    Epilogue order: +bias -> (Z := pre-activation) -> act -> dropout(layer, m, n) -> *act'(G).
    accum: 0 store, 1 add, 2 atomic add (required when splitk > 1).  On the device, K <= 256 / N <= 256
    shapes with aligned row-major operands take the tall-skinny kernel (k_tsgemm); ``generic`` forces the
    64x64-tile kernel (k_bgemm) — the tests compare the two.  ``asum [C, K]`` (optional) accumulates the
    column sums of A — for ``dX = dY W`` that is the bias gradient, taken from the A rows the GEMM streams
    anyway (fused in k_tsgemm, a separate column-sum pass otherwise)."""
    if _nat(A):
        s, sc = _dargs(ctl, p)
        _native().bgemm(A, B, C, bias, Z, G, act, gact, accum, splitk, alpha, s, sc, layer, p, int(generic), asum)
        return
    if asum is not None:
        asum.add_(A.sum(dim=1))
    v = alpha * torch.bmm(A, B.transpose(1, 2))
    if bias is not None:
        v = v + bias[:, None, :]
    if Z is not None:
        Z.copy_(v)
    v = _act(v, act)
    if p > 0.0:
        r, c = _rc(v.shape[1], v.shape[2])
        v = v * torch.stack([_scale(ctl, ci, layer, r, c, p) for ci in range(v.shape[0])])
    if G is not None:
        v = v * _actd(G, gact)
    if accum == 0:
        C.copy_(v)
    else:
        C.add_(v)


def colsum(Y, out) -> None:
    """``out [C, N] += Y.sum(rows)`` (atomic accumulation on device: zero ``out`` first)."""
    if _nat(Y):
        _native().colsum(Y, out)
        return
    out.add_(Y.sum(dim=1))


# ------------------------------------------------------------------------------------- batches
def gather_icu(rows, idx, ctl: StepCtl, mask: bool, vit, lab, y) -> None:
    """Rows ``idx[step]`` ([S, C, B], -1 = padding) of the ICU table -> vitals/labs/labels."""
    if _nat(rows):
        _native().gather_icu(rows, idx, ctl.stepctl, int(mask), vit, lab, y)
        return
    ix = idx[ctl.step()].long()
    r = torch.where((ix >= 0)[..., None], rows[ix.clamp_min(0)], torch.zeros((), dtype=rows.dtype))
    feat = r[..., :23]
    if mask:
        feat = torch.where(feat == -2.0, torch.zeros_like(feat), feat)
    vit.copy_(feat[..., :7].reshape(vit.shape))
    lab.copy_(feat[..., 7:23].reshape(lab.shape))
    y.copy_(r[..., 23].reshape(y.shape))


def gather_har(x, yl, idx, ctl: StepCtl, ox, oy) -> None:
    if _nat(x):
        _native().gather_har(x, yl, idx, ctl.stepctl, ox, oy)
        return
    ix = idx[ctl.step()].long()
    ok = ix >= 0
    ox.copy_(torch.where(ok[..., None], x[ix.clamp_min(0)], torch.zeros((), dtype=x.dtype)).reshape(ox.shape))
    oy.copy_(torch.where(ok, yl[ix.clamp_min(0)], torch.zeros((), dtype=yl.dtype)).reshape(oy.shape))


# ---------------------------------------------------------------------------------- conv k=3
def _im2col(x, B, L):
    C, _, Cin = x.shape
    xp = F.pad(x.reshape(C, B, L, Cin), (0, 0, 1, 1))
    cols = torch.stack([xp[:, :, j:j + L, :] for j in range(3)], dim=-1)  # [C, B, L, Cin, 3]
    return cols.reshape(C, B * L, Cin * 3)


def im2col3(x, B: int, L: int, out) -> None:
    """Conv1d(k=3, pad=1) patches of channels-last ``x [C, B*L, Cin]`` -> ``out [C, B*L, 3*Cin]``
    (column ``ci*3 + j`` = input position ``l + j - 1``: PyTorch's ``[Cout][Cin][3]`` weight order)."""
    if _nat(x):
        _native().im2col3(x, B, L, out)
        return
    out.copy_(_im2col(x, B, L).reshape(out.shape))


def col2im3(dcols, B: int, L: int, Cin: int, relu_src, dx) -> None:
    """Adjoint of ``im2col3`` (optionally times relu'(relu_src))."""
    if _nat(dcols):
        _native().col2im3(dcols, B, L, Cin, relu_src, dx)
        return
    C = dcols.shape[0]
    x = torch.zeros(C, B * L, Cin, requires_grad=True)
    with torch.enable_grad():
        (g,) = torch.autograd.grad(_im2col(x, B, L), x, dcols.reshape(C, B * L, 3 * Cin))
    if relu_src is not None:
        g = g * (relu_src > 0).float()
    dx.copy_(g.reshape(dx.shape))


# --------------------------------------------------------------------- fused CNNModel towers
@dataclass
class CnnTower:
    """One Conv1d tower of CNNModel (vitals or labs) and its step buffers.

    ``x [C, B, L]`` input; weights as arena views ``W1 [C,32,3] b1 [C,32] W2 [C,64,96] b2 W3 [C,128,192] b3``;
    saved activations ``h1..h3 [C, B*L, 32|64|128]`` and their gradients ``dh1..dh3``; the tower's pooled
    output fills concat columns ``[col0, col0 + 512)`` with dropout site ``layer``."""

    x: torch.Tensor
    W1: torch.Tensor
    b1: torch.Tensor
    W2: torch.Tensor
    b2: torch.Tensor
    W3: torch.Tensor
    b3: torch.Tensor
    h1: torch.Tensor
    h2: torch.Tensor
    h3: torch.Tensor
    dh1: torch.Tensor
    dh2: torch.Tensor
    dh3: torch.Tensor
    L: int
    col0: int
    layer: int

    def tensors(self):
        return [self.x, self.W1, self.b1, self.W2, self.b2, self.W3, self.b3, self.h1, self.h2, self.h3, self.dh1,
                self.dh2, self.dh3]

    def meta(self):
        return [self.L, self.col0, self.layer]


def cnn_wimg_buffer(C: int, device) -> torch.Tensor:
    """Scratch for the towers' per-step bf16 weight images (built by the forward, read by the backward)."""
    return torch.zeros(int(_native().cnn_wimg_size(C)), dtype=torch.int16, device=device)


def cnn_towers_fwd(towers, B: int, cat, ctl: Optional[StepCtl] = None, p: float = 0.0, wimg=None,
                   head=()) -> None:
    """conv1..conv3 (+bias, ReLU) -> AdaptiveAvgPool1d(4) -> dropout into ``cat`` for both towers
    (on device: ``cnn.hip:k_cnn_wimg`` + ``k_cnn_fwd``; ``wimg`` from ``cnn_wimg_buffer``; ``head`` =
    optional ``[fc2.weight, fc3.weight]`` views whose bf16 images ``cnn_head`` then reads)."""
    if _nat(cat):
        s, sc = _dargs(ctl, p)
        _native().cnn_towers_fwd(towers[0].tensors(), towers[1].tensors(), towers[0].meta(), towers[1].meta(), B,
                                 cat, s, sc, p, wimg, list(head))
        return
    for tw in towers:
        C = tw.x.shape[0]
        h = tw.x.reshape(C, B * tw.L, 1)
        for W, b, out in ((tw.W1, tw.b1, tw.h1), (tw.W2, tw.b2, tw.h2), (tw.W3, tw.b3, tw.h3)):
            v = torch.bmm(_im2col(h, B, tw.L), W.reshape(C, W.shape[1], -1).transpose(1, 2)) + b[:, None, :]
            out.copy_(F.relu(v).reshape(out.shape))
            h = out.reshape(C, B * tw.L, -1)
        pool4_fwd(h, B, tw.L, cat, tw.col0, ctl, tw.layer, p)


def cnn_towers_bwd(towers, B: int, dcat, ctl: Optional[StepCtl] = None, p: float = 0.0, wimg=None) -> None:
    """pool'/dropout'/ReLU' -> dh3; dh2 = col2im(dh3 . W3) * relu'(h2); dh1 = col2im(dh2 . W2) * relu'(h1)
    (device: reads the weight images the same step's ``cnn_towers_fwd`` built in ``wimg``)."""
    if _nat(dcat):
        s, sc = _dargs(ctl, p)
        _native().cnn_towers_bwd(towers[0].tensors(), towers[1].tensors(), towers[0].meta(), towers[1].meta(), B,
                                 dcat, s, sc, p, wimg)
        return
    for tw in towers:
        C, L = tw.x.shape[0], tw.L
        h3 = tw.h3.reshape(C, B * L, 128)
        pool4_bwd(dcat, tw.col0, h3, B, L, tw.dh3.reshape(C, B * L, 128), ctl, tw.layer, p)
        for W, hprev, dcur, dprev, cin in ((tw.W3, tw.h2, tw.dh3, tw.dh2, 64), (tw.W2, tw.h1, tw.dh2, tw.dh1, 32)):
            dcols = torch.bmm(dcur.reshape(C, B * L, -1), W.reshape(C, W.shape[1], -1))
            col2im3(dcols, B, L, cin, hprev.reshape(C, B * L, cin), dprev.reshape(C, B * L, cin))


def conv_dw(jobs, B: int, splitk: int = 4) -> None:
    """Conv weight / bias gradients of several (dh, h_prev, gW, gb, L) jobs, ACCUMULATED into gW / gb
    (the step's zeroed gradient arena): ``gW += dh^T . im2col(h_prev)``, ``gb += colsum(dh)``."""
    if _nat(jobs[0][0]):
        _native().conv_dw([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs], [j[3] for j in jobs],
                          [int(j[4]) for j in jobs], int(B), int(splitk))
        return
    for dh, hp, gW, gb, L in jobs:
        C, Cout, K = gW.shape
        cols = _im2col(hp.reshape(C, B * L, K // 3), B, L)
        d = dh.reshape(C, B * L, Cout)
        gW.add_(torch.bmm(d.transpose(1, 2), cols))
        gb.add_(d.sum(dim=1))


def cnn_head(z1, y, w, g, d1, bsz, epoch, nb, ctl: StepCtl, failed, losses, z=None, wimg=None) -> None:
    """CNNModel head in one launch per step: ``f1 = ReLU(z1 + b1)`` from the fc1 pre-activation (the
    device kernel zeroes ``z1`` after reading it: the next split-K fc1 accumulates into it), ``fc2 ->
    ReLU -> fc3 -> ReLU -> output``, the sigmoid-BCE of ``bce`` (same masking / NaN abort / epoch losses),
    and the backward: gradients of fc2 / fc3 / output and the fc1 bias (``g = [gW2, gb2, gW3, gb3, gWo,
    gbo, gb1]``, stored) and ``d1`` = d(fc1 pre-activation).  ``w = [W2, b2, W3, b3, Wo, bo, b1]``; on
    device the fc2 / fc3 weights come from the bf16 images the towers' forward built in ``wimg``."""
    W2, b2, W3, b3, Wo, bo, b1 = w
    if _nat(z1):
        _native().cnn_head(z1, y, list(w), list(g), d1, z, bsz, epoch, nb, ctl.stepctl, failed, losses, wimg)
        return
    f1 = F.relu(z1 + b1[:, None, :])
    f2 = F.relu(torch.bmm(f1, W2.transpose(1, 2)) + b2[:, None, :])
    f3 = F.relu(torch.bmm(f2, W3.transpose(1, 2)) + b3[:, None, :])
    zz = torch.bmm(f3, Wo.reshape(Wo.shape[0], 1, 32).transpose(1, 2)) + bo.reshape(-1, 1, 1)
    if z is not None:
        z.copy_(zz.reshape(z.shape))
    dz = torch.zeros_like(zz)
    bce(zz, y, bsz, epoch, nb, ctl, failed, losses, dz)
    gW2, gb2, gW3, gb3, gWo, gbo, gb1 = g
    gWo.copy_(torch.bmm(dz.transpose(1, 2), f3).reshape(gWo.shape))
    gbo.copy_(dz.sum(dim=1).reshape(gbo.shape))
    d3 = torch.bmm(dz, Wo.reshape(Wo.shape[0], 1, 32)) * (f3 > 0).float()
    gW3.copy_(torch.bmm(d3.transpose(1, 2), f2))
    gb3.copy_(d3.sum(dim=1))
    d2 = torch.bmm(d3, W3) * (f2 > 0).float()
    gW2.copy_(torch.bmm(d2.transpose(1, 2), f1))
    gb2.copy_(d2.sum(dim=1))
    dd1 = torch.bmm(d2, W2) * (f1 > 0).float()
    gb1.copy_(dd1.sum(dim=1))
    d1.copy_(dd1.reshape(d1.shape))


# --------------------------------------------------------------------- AdaptiveAvgPool1d(4)
def _pool4(h, B, L):
    C, _, Ch = h.shape
    return F.adaptive_avg_pool1d(h.reshape(C * B, L, Ch).transpose(1, 2), 4).reshape(C, B, Ch * 4)


def pool4_fwd(h, B: int, L: int, out, col0: int, ctl=None, layer=0, p=0.0) -> None:
    """``out[:, b, col0 + ch*4 + p] = dropout(mean over bin p of h[:, b*L + l, ch])``."""
    if _nat(h):
        s, sc = _dargs(ctl, p)
        _native().pool4_fwd(h, B, L, out, col0, s, sc, layer, p)
        return
    v = _pool4(h, B, L)
    if p > 0.0:
        r, c = _rc(B, v.shape[2])
        v = v * torch.stack([_scale(ctl, ci, layer, r, c + col0, p) for ci in range(v.shape[0])])
    out[:, :, col0:col0 + v.shape[2]] = v


def pool4_bwd(dout, col0: int, h, B: int, L: int, dh, ctl=None, layer=0, p=0.0) -> None:
    """Adjoint of ``pool4_fwd`` times relu'(h)."""
    if _nat(h):
        s, sc = _dargs(ctl, p)
        _native().pool4_bwd(dout, col0, h, B, L, dh, s, sc, layer, p)
        return
    C, _, Ch = h.shape
    g = dout[:, :, col0:col0 + Ch * 4]
    if p > 0.0:
        r, c = _rc(B, Ch * 4)
        g = g * torch.stack([_scale(ctl, ci, layer, r, c + col0, p) for ci in range(C)])
    x = h.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        (d,) = torch.autograd.grad(_pool4(x, B, L), x, g.contiguous())
    dh.copy_((d * (h > 0).float()).reshape(dh.shape))


# ------------------------------------------------------------------------------- LayerNorm(64)
def ln_fwd(x, a, s, y, stats, gamma, beta, ctl=None, layer_a=0, p_a=0.0, layer_o=0, p_o=0.0) -> None:
    """``y = dropout_o(LN(x + dropout_a(a)) * gamma + beta)``; stores the pre-norm sum in ``s`` (optional)
    and (mean, rstd) per row in ``stats [C, rows, 2]``."""
    if _nat(x):
        sd, sc = _dargs(ctl, max(p_a, p_o))
        _native().ln_fwd(x, a, s, y, stats, gamma, beta, sd, sc, layer_a, p_a, layer_o, p_o)
        return
    C, R, _ = x.shape
    v = x.clone()
    if a is not None:
        av = a
        if p_a > 0.0:
            r, c = _rc(R, 64)
            av = a * torch.stack([_scale(ctl, ci, layer_a, r, c, p_a) for ci in range(C)])
        v = v + av
    if s is not None:
        s.copy_(v.reshape(s.shape))
    mean = v.mean(-1, keepdim=True)
    var = ((v - mean) ** 2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + 1e-5)
    out = (v - mean) * rstd * gamma[:, None, :] + beta[:, None, :]
    if p_o > 0.0:
        r, c = _rc(R, 64)
        out = out * torch.stack([_scale(ctl, ci, layer_o, r, c, p_o) for ci in range(C)])
    y.copy_(out)
    stats.copy_(torch.cat([mean, rstd], dim=-1).reshape(stats.shape))


def ln_bwd(dy, s, stats, gamma, dx, dx_accum, da, dgamma, dbeta, ctl=None, layer_a=0, p_a=0.0, layer_o=0,
           p_o=0.0) -> None:
    """Backward of ``ln_fwd``: dx (= d pre-norm sum; stored or accumulated), optional ``da =
    dropout_a'(dx)``, and ``dgamma``/``dbeta`` accumulated (zero them first)."""
    if _nat(dy):
        sd, sc = _dargs(ctl, max(p_a, p_o))
        _native().ln_bwd(dy, s, stats, gamma, dx, int(dx_accum), da, dgamma, dbeta, sd, sc, layer_a, p_a, layer_o,
                         p_o)
        return
    C, R, _ = dy.shape
    g = dy
    if p_o > 0.0:
        r, c = _rc(R, 64)
        g = dy * torch.stack([_scale(ctl, ci, layer_o, r, c, p_o) for ci in range(C)])
    sv = s.detach().clone().requires_grad_(True)
    gm = gamma.detach().clone().requires_grad_(True)
    bt = torch.zeros_like(gm, requires_grad=True)
    with torch.enable_grad():
        out = torch.stack([F.layer_norm(sv[ci], (64,), gm[ci], bt[ci], 1e-5) for ci in range(C)])
        ds, dgm, dbt = torch.autograd.grad(out, (sv, gm, bt), g.contiguous())
    if dx_accum:
        dx.add_(ds)
    else:
        dx.copy_(ds)
    if da is not None:
        v = ds
        if p_a > 0.0:
            r, c = _rc(R, 64)
            v = ds * torch.stack([_scale(ctl, ci, layer_a, r, c, p_a) for ci in range(C)])
        da.copy_(v)
    dgamma.add_(dgm)
    dbeta.add_(dbt)


# ------------------------------------------------------------------------------------- GRU cell
def _gru(gi, bhh):
    r = torch.sigmoid(gi[..., :32] + bhh[:, None, :32])
    z = torch.sigmoid(gi[..., 32:64] + bhh[:, None, 32:64])
    n = torch.tanh(gi[..., 64:] + r * bhh[:, None, 64:])
    return (1 - z) * n


def gru_fwd(gi, bhh, h, col0: int) -> None:
    """One GRU direction at seq_len 1 with h0 = 0: ``h[:, :, col0:col0+32] = (1 - z) * n``."""
    if _nat(gi):
        _native().gru_fwd(gi, bhh, h, col0)
        return
    h[:, :, col0:col0 + 32] = _gru(gi, bhh)


def gru_bwd(dh, col0: int, gi, bhh, dgi, dbih, dbhh) -> None:
    """dgi (= d(x W_ih^T + b_ih)), and the bias gradients (stored)."""
    if _nat(gi):
        _native().gru_bwd(dh, col0, gi, bhh, dgi, dbih, dbhh)
        return
    g = gi.detach().clone().requires_grad_(True)
    b = bhh.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        dg, db = torch.autograd.grad(_gru(g, b), (g, b), dh[:, :, col0:col0 + 32].contiguous())
    dgi.copy_(dg)
    dbih.copy_(dg.sum(1))
    dbhh.copy_(db)


# ------------------------------------------------------------------------------------- losses
def _active(bsz, failed, s: int, c: int, min_bs: int = 2):
    bs = int(bsz[s, c]) if s < bsz.shape[0] else 0
    return bs >= max(min_bs, 1) and int(failed[c]) == 0, bs


def bce(z, y, bsz, epoch, nb, ctl: StepCtl, failed, losses, dz) -> None:
    """Mean BCE on sigmoid(z) over the step's real rows, gradient, NaN abort (client.py:95-103)."""
    if _nat(z):
        _native().bce(z, y, bsz, epoch, nb, ctl.stepctl, failed, losses, dz)
        return
    s = ctl.step()
    dz.zero_()
    C, B = y.shape[0], y.shape[1]
    zz, yy, dd = z.reshape(C, B), y.reshape(C, B), dz.reshape(C, B)
    for c in range(C):
        act, bs = _active(bsz, failed, s, c, ctl.min_bs)
        if not act:
            continue
        p = torch.sigmoid(zz[c, :bs])
        t = yy[c, :bs]
        lv = -(t * torch.clamp(torch.log(p), min=-100.0) + (1 - t) * torch.clamp(torch.log1p(-p), min=-100.0))
        loss = lv.mean()
        if bool(torch.isnan(loss)) and ctl.nan_abort:
            failed[c] = 1
            continue
        losses[c, int(epoch[s, c])] += loss / int(nb[c])
        w = p * (1 - p)
        dd[c, :bs] = (p - t) / torch.clamp(w, min=1e-12) * w / bs


def ce(logits, y, bsz, epoch, nb, ctl: StepCtl, failed, losses, dz) -> None:
    """Mean softmax cross-entropy (``nn.CrossEntropyLoss``) + gradient + NaN abort."""
    if _nat(logits):
        _native().ce(logits, y, bsz, epoch, nb, ctl.stepctl, failed, losses, dz)
        return
    s = ctl.step()
    dz.zero_()
    for c in range(logits.shape[0]):
        act, bs = _active(bsz, failed, s, c, ctl.min_bs)
        if not act:
            continue
        x = logits[c, :bs]
        loss = F.cross_entropy(x, y[c, :bs])
        if bool(torch.isnan(loss)) and ctl.nan_abort:
            failed[c] = 1
            continue
        losses[c, int(epoch[s, c])] += loss / int(nb[c])
        dz[c, :bs] = (torch.softmax(x, -1) - F.one_hot(y[c, :bs], x.shape[-1]).float()) / bs


# ---------------------------------------------------------------------------------- optimizer
def adam_clients(p, g, m, v, tcount, bsz, ctl: StepCtl, failed, lr: float, skip=(0, 0), sgd_lr: float = 0.0,
                 zero_grads: bool = False) -> None:
    """``torch.optim.Adam(lr)`` step (β 0.9/0.999, eps 1e-8) of every client active this step;
    ``skip`` = [lo, hi) of non-trainable entries (buffers); ``sgd_lr > 0`` = plain SGD (test hook);
    ``zero_grads``: zero each consumed gradient entry (the next step then needs no zero-fill launch;
    inactive clients' entries are left alone — they never step again)."""
    if _nat(p):
        _native().adam_clients(p, g, m, v, tcount, bsz, ctl.stepctl, failed, float(lr), int(skip[0]), int(skip[1]),
                               float(sgd_lr), int(zero_grads))
        return
    s = ctl.step()
    keep = torch.ones(p.shape[1], dtype=torch.bool)
    keep[skip[0]:skip[1]] = False
    for c in range(p.shape[0]):
        act, _ = _active(bsz, failed, s, c, ctl.min_bs)
        if not act:
            continue
        gi = g[c][keep]
        if sgd_lr > 0:
            p[c][keep] -= sgd_lr * gi
            continue
        t = int(tcount[c]) + 1
        mi = m[c][keep] + 0.1 * (gi - m[c][keep])
        vi = 0.999 * v[c][keep] + 0.001 * gi * gi
        m[c][keep] = mi
        v[c][keep] = vi
        bc1, bc2 = 1 - 0.9 ** t, 1 - 0.999 ** t
        p[c][keep] -= (lr / bc1) * mi / (vi.sqrt() / (bc2 ** 0.5) + 1e-8)


def step_end(ctl: StepCtl, tcount, bsz, failed) -> None:
    """Advance the device step counter and every active client's Adam step count."""
    if _nat(tcount):
        _native().step_end(ctl.stepctl, tcount, bsz, failed)
        return
    s = ctl.step()
    for c in range(tcount.shape[0]):
        if _active(bsz, failed, s, c, ctl.min_bs)[0]:
            tcount[c] += 1
    ctl.stepctl[0] += 1


# ------------------------------------------------------------------------ HAR stem / pooling
def conv_pe_fwd(x, params, w_off: int, b_off: int, pe_off: int, h) -> None:
    """Conv1d(1->64, k3, p1) over ``x [C, B, L]`` + positional encoding -> ``h [C, B*L, 64]``."""
    if _nat(x):
        _native().conv_pe_fwd(x, params, w_off, b_off, pe_off, h)
        return
    C, B, L = x.shape
    w = params[:, w_off:w_off + 192].reshape(C, 64, 1, 3)
    b = params[:, b_off:b_off + 64]
    pe = params[:, pe_off:pe_off + L * 64].reshape(C, L, 64)
    for c in range(C):
        o = F.conv1d(x[c][:, None, :], w[c], b[c], padding=1).transpose(1, 2) + pe[c][None]
        h[c] = o.reshape(B * L, 64)


def conv_pe_bwd(x, dh, grads, w_off: int, b_off: int) -> None:
    """Accumulate the conv weight/bias gradients into the flat ``grads [C, P]``."""
    if _nat(x):
        _native().conv_pe_bwd(x, dh, grads, w_off, b_off)
        return
    C, B, L = x.shape
    for c in range(C):
        w = torch.zeros(64, 1, 3, requires_grad=True)
        b = torch.zeros(64, requires_grad=True)
        with torch.enable_grad():
            o = F.conv1d(x[c][:, None, :], w, b, padding=1).transpose(1, 2)
            dw, db = torch.autograd.grad(o, (w, b), dh[c].reshape(B, L, 64))
        grads[c, w_off:w_off + 192] += dw.reshape(-1)
        grads[c, b_off:b_off + 64] += db


def mean_rows_fwd(h, B: int, L: int, out) -> None:
    if _nat(h):
        _native().mean_rows_fwd(h, B, L, out)
        return
    out.copy_(h.reshape(h.shape[0], B, L, 64).mean(2).reshape(out.shape))


def mean_rows_bwd(dout, B: int, L: int, dh) -> None:
    if _nat(dout):
        _native().mean_rows_bwd(dout, B, L, dh)
        return
    C = dout.shape[0]
    dh.copy_((dout.reshape(C, B, 1, 64) / L).expand(C, B, L, 64).reshape(dh.shape))


# ---------------------------------------------------------------------------------- attention
def attn_lp(L: int) -> int:
    return (L + 31) // 32 * 32


def _attn_ref(qkv, B, L, ctl, layer, p, scheme: str = "pair"):
    """Composite SDPA (4 heads x 16, scale 1/4, dropout on the probabilities) -> (O, lse).  ``scheme``: the
    probability-dropout hash — "pair" (``afl_keep``, attention.hip) or "rc" (``masks.keep_rc``, har.hip)."""
    C = qkv.shape[0]
    q, k, v = qkv.reshape(C, B, L, 3, 4, 16).permute(3, 0, 1, 4, 2, 5)  # each [C, B, H, L, 16]
    s = torch.matmul(q, k.transpose(-1, -2)) * 0.25
    lse = torch.logsumexp(s, dim=-1)
    pr = torch.softmax(s, dim=-1)
    if p > 0.0:
        rows = (np.arange(B * 4)[:, None] * L + np.arange(L)[None, :]).reshape(B, 4, L, 1)
        cols = np.arange(L).reshape(1, 1, 1, L)
        keepfn = masks.keep_rc if scheme == "rc" else masks.keep
        pr = pr * torch.stack([keepfn(ctl.key(ci), layer, rows, cols, p).float() / (1.0 - p) for ci in range(C)])
    o = torch.matmul(pr, v)  # [C, B, H, L, 16]
    return o.permute(0, 1, 3, 2, 4).reshape(C, B * L, 64), lse


def attn_fwd(qkv, o, lse, B: int, L: int, ctl=None, layer=0, p=0.0, scheme: str = "pair") -> None:
    """Multi-head self-attention of ``qkv [C, B*L, 192]`` -> ``o [C, B*L, 64]``, ``lse [C*B*4, Lp]``.
    ``scheme`` (composite only): the dropout hash of the kernel being mirrored (``_attn_ref``)."""
    if _nat(qkv):
        if scheme != "pair" and p > 0.0:
            raise ValueError("attention.hip draws its dropout with the 'pair' scheme")
        s, sc = _dargs(ctl, p)
        _native().attn_fwd(qkv, o, lse, B, L, s, sc, layer, p)
        return
    out, ls = _attn_ref(qkv, B, L, ctl, layer, p, scheme)
    o.copy_(out)
    Lp = attn_lp(L)
    lv = lse.view(-1, Lp)
    lv.fill_(float("inf"))
    lv[:, :L] = ls.reshape(-1, L)


def attn_bwd(qkv, o, lse, dout, dqkv, B: int, L: int, ctl=None, layer=0, p=0.0, scheme: str = "pair") -> None:
    if _nat(qkv):
        if scheme != "pair" and p > 0.0:
            raise ValueError("attention.hip draws its dropout with the 'pair' scheme")
        s, sc = _dargs(ctl, p)
        _native().attn_bwd(qkv, o, lse, dout, dqkv, B, L, s, sc, layer, p)
        return
    x = qkv.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        out, _ = _attn_ref(x, B, L, ctl, layer, p, scheme)
        (g,) = torch.autograd.grad(out, x, dout)
    dqkv.copy_(g)
