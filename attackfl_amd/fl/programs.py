"""Explicit client-batched training programs (forward + hand-written backward + Adam) for the models
without a whole-step fused kernel: ``CNNModel`` / ``RNNModel`` (ICU) and ``TransformerClassifier`` (HAR).

A program is a fixed sequence of layer ops (``attackfl_amd/ops/layers.py``) over ALL of a rank's
clients at once — tensors are ``[C, rows, cols]`` and weights are views into the flat ``[C, P]``
parameter arena, so one launch serves every client.  Everything that changes per optimizer step
(batch rows, batch size, epoch, dropout key, Adam step) lives in device tensors indexed by a device
step counter, so on a GPU the whole step is captured ONCE into a HIP graph and replayed per step
(no per-step host work, no host/device syncs).  On CPU the same program runs the composite ops —
the fp32 oracle the GPU path is tested against.

Semantics mirror the reference trainers (``client.py:66-131``): fresh Adam per round, BCE (ICU) /
cross-entropy (HAR) mean loss, size-1 batches skipped (A-21), NaN loss aborts the client's round (for HAR
``engine.compat-har-train`` restores the reference ``train_HAR`` loop: no skip, no abort).
Model math mirrors ``src/Model.py:27-88`` (CNN), ``91-163`` (RNN), ``418-458`` (HAR classifier).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Sequence, Tuple

import torch

from ..models import ParamLayout
from ..ops import layers as Lx
from ..ops.layers import ACT_RELU, StepCtl

VIT, LAB = 7, 16


class _Program:
    """Shared machinery: parameter views, buffer pool, weight-gradient GEMM helper."""

    model_name = ""
    loss = "bce"
    fused_loss = False  # True: backward_loss() computes the loss itself (the runner skips its loss kernel)

    def __init__(self, C: int, B: int, device, train: bool = True, dropout: bool = True):
        self.layout = ParamLayout.for_model(self.model_name)
        self.P = self.layout.P
        self.slot = {s.name: s for s in self.layout.slots}
        self.C, self.B, self.device, self.train = C, B, torch.device(device), train
        self.drop_on = train and dropout  # dropout=False: deterministic training (gradient tests)
        self._bufs: Dict[str, torch.Tensor] = {}

    # -- buffers -------------------------------------------------------------------------------
    def p(self, prob: float) -> float:
        return prob if self.drop_on else 0.0

    def buf(self, name: str, *shape, dtype=torch.float32) -> torch.Tensor:
        t = self._bufs.get(name)
        if t is None:
            t = torch.zeros(*shape, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t

    def w(self, flat: torch.Tensor, name: str, as2d: Tuple[int, int] = None) -> torch.Tensor:
        """View of parameter ``name`` across clients: 2-D weights -> [C, N, K], vectors -> [C, N]."""
        s = self.slot[name]
        v = flat[:, s.offset:s.offset + s.numel]
        if as2d is not None:
            return v.view(flat.shape[0], *as2d)
        if len(s.shape) == 1:
            return v
        if len(s.shape) == 2:
            return v.view(flat.shape[0], *s.shape)
        return v.view(flat.shape[0], s.shape[0], -1)

    def dw(self, dY: torch.Tensor, X: torch.Tensor, gW: torch.Tensor) -> None:
        """``gW [C, N, K] = dY^T X`` over the rows (split-K — ordered per-split partials, deterministic — when
        the tile grid alone would leave the GPU idle; ``grads`` is zeroed at the start of every step)."""
        M, N, K = dY.shape[1], dY.shape[2], X.shape[2]
        # per-client tile count only: the split count (and with it the deterministic split-K summation order)
        # must not depend on how many clients share the launch — a client's gradients are then the same bits
        # whichever rank / packing trains it (128 splits x tiles per client ~ 1024 workgroups at 8 clients)
        tiles = math.ceil(N / 64) * math.ceil(K / 64)
        splitk = max(1, min(M // 256, math.ceil(128 / tiles))) if dY.is_cuda else 1
        Lx.bgemm(dY.transpose(1, 2), X.transpose(1, 2), gW, accum=2 if splitk > 1 else 0, splitk=splitk)

    def linear(self, X, params, wname, bname, out, act=0, ctl=None, layer=0, p=0.0):
        Lx.bgemm(X, self.w(params, wname), out, bias=self.w(params, bname), act=act, ctl=ctl, layer=layer,
                 p=self.p(p))

    def linear_bwd(self, dY, X, params, grads, wname, bname, dX=None, G=None, gact=0, accum=0, ctl=None, layer=0,
                   p=0.0):
        """Weight/bias grads of ``Y = X W^T + b`` and (optionally) ``dX = dY W`` with a fused
        dropout'/act' epilogue for the layer that produced X."""
        self.dw(dY, X, self.w(grads, wname))
        if dX is not None:  # the bias gradient rides on the dX GEMM's pass over dY
            Lx.bgemm(dY, self.w(params, wname).transpose(1, 2), dX, G=G, gact=gact, accum=accum, ctl=ctl, layer=layer,
                     p=self.p(p), asum=self.w(grads, bname))
        else:
            Lx.colsum(dY, self.w(grads, bname))

    # -- interface -----------------------------------------------------------------------------
    def inputs(self, table, idx, ctl):  # pragma: no cover - abstract
        raise NotImplementedError

    def set_inputs(self, data: torch.Tensor) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def forward(self, params, ctl):  # -> output buffer
        raise NotImplementedError

    def backward(self, params, grads, ctl):
        raise NotImplementedError

    def skip_range(self) -> Tuple[int, int]:
        return (0, 0)


# ============================================================================================ ICU
class _ICUProgram(_Program):
    mask_inputs = False

    def inputs(self, table, idx, ctl):
        C, B = self.C, self.B
        Lx.gather_icu(table.rows, idx, ctl, self.mask_inputs, self.buf("xv", C, B, VIT), self.buf("xl", C, B, LAB),
                      self.buf("y", C, B))

    def set_inputs(self, rows: torch.Tensor) -> None:
        """Eval: the same ``rows [B, 24]`` for every client (zero-padded to B)."""
        n = rows.shape[0]
        feat = rows[:, :23]
        if self.mask_inputs:
            feat = torch.where(feat == -2.0, torch.zeros_like(feat), feat)
        xv, xl = self.buf("xv", self.C, self.B, VIT), self.buf("xl", self.C, self.B, LAB)
        xv.zero_()
        xl.zero_()
        xv[:, :n] = feat[None, :, :VIT]
        xl[:, :n] = feat[None, :, VIT:23]

    def labels(self):
        return self.buf("y", self.C, self.B)


class CNNProgram(_ICUProgram):
    """CNNModel: both Conv1d towers (conv1..3 + ReLU + pool + dropout) in one fused launch each way
    (``Lx.cnn_towers_fwd/bwd``, ``csrc/kernels/cnn.hip``), every conv weight gradient in one more
    (``Lx.conv_dw``), MLP head as MFMA GEMMs with fused epilogues."""

    model_name = "CNNModel"
    CH = (1, 32, 64, 128)

    def wimg(self):
        if self.device.type != "cuda":
            return None
        if "wimg" not in self._bufs:
            self._bufs["wimg"] = Lx.cnn_wimg_buffer(self.C, self.device)
        return self._bufs["wimg"]

    def towers(self, params):
        C, B = self.C, self.B
        out = []
        for bi, (br, L) in enumerate((("vitals", VIT), ("labs", LAB))):
            h = [self.buf(f"{br}_h{i}", C, B * L, self.CH[i]) for i in (1, 2, 3)]
            dh = [self.buf(f"{br}_dh{i}", C, B * L, self.CH[i]) for i in (1, 2, 3)] if self.train else h
            out.append(Lx.CnnTower(self.buf("xv" if bi == 0 else "xl", C, B, L),
                                   self.w(params, f"{br}_conv1.weight"), self.w(params, f"{br}_conv1.bias"),
                                   self.w(params, f"{br}_conv2.weight"), self.w(params, f"{br}_conv2.bias"),
                                   self.w(params, f"{br}_conv3.weight"), self.w(params, f"{br}_conv3.bias"),
                                   h[0], h[1], h[2], dh[0], dh[1], dh[2], L, 512 * bi, bi))
        return out

    fused_loss = True

    def forward(self, params, ctl):
        """Training: towers + the fc1 pre-activation (split-K; the head kernel inside ``backward_loss`` adds
        the bias and the ReLU); eval: the full forward -> z."""
        C, B = self.C, self.B
        cat = self.buf("cat", C, B, 1024)
        head = [self.w(params, "fc2.weight"), self.w(params, "fc3.weight")] if self.train else []
        Lx.cnn_towers_fwd(self.towers(params), B, cat, ctl, self.p(0.3), self.wimg(), head)
        if self.train:
            # device: split-K accumulation into z1, which the head kernel zeroes after reading it
            Lx.bgemm(cat, self.w(params, "fc1.weight"), self.buf("z1", C, B, 128), accum=2 if cat.is_cuda else 0,
                     splitk=8 if cat.is_cuda else 1)
            return None
        f1, f2, f3 = self.buf("f1", C, B, 128), self.buf("f2", C, B, 64), self.buf("f3", C, B, 32)
        z = self.buf("z", C, B, 1)
        self.linear(cat, params, "fc1.weight", "fc1.bias", f1, act=ACT_RELU)
        self.linear(f1, params, "fc2.weight", "fc2.bias", f2, act=ACT_RELU)
        self.linear(f2, params, "fc3.weight", "fc3.bias", f3, act=ACT_RELU)
        self.linear(f3, params, "output.weight", "output.bias", z)
        return z

    def backward_loss(self, params, grads, ctl, loss_ctx):
        C, B = self.C, self.B
        bsz, ep, nb, failed, losses = loss_ctx
        d1, cat, dcat = self.buf("d1", C, B, 128), self.buf("cat", C, B, 1024), self.buf("dcat", C, B, 1024)
        names = ("fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias", "output.weight", "output.bias")
        Lx.cnn_head(self.buf("z1", C, B, 128), self.labels(), [self.w(params, n) for n in names + ("fc1.bias",)],
                    [self.w(grads, n) for n in names] + [self.w(grads, "fc1.bias")], d1, bsz, ep, nb, ctl, failed,
                    losses, wimg=self.wimg())
        self.dw(d1, cat, self.w(grads, "fc1.weight"))
        Lx.bgemm(d1, self.w(params, "fc1.weight").transpose(1, 2), dcat)
        tw = self.towers(params)
        Lx.cnn_towers_bwd(tw, B, dcat, ctl, self.p(0.3), self.wimg())
        jobs = []
        for t, br in zip(tw, ("vitals", "labs")):
            hp = (t.x, t.h1, t.h2)
            for i, (dh, h) in enumerate(zip((t.dh1, t.dh2, t.dh3), hp), start=1):
                jobs.append((dh, h, self.w(grads, f"{br}_conv{i}.weight"), self.w(grads, f"{br}_conv{i}.bias"), t.L))
        Lx.conv_dw(jobs, B)


class RNNProgram(_ICUProgram):
    """RNNModel: 3 stacked bi-GRU layers per branch at seq_len 1 (h0 = 0), LayerNorm + dropout, MLP."""

    model_name = "RNNModel"
    mask_inputs = True
    DIRS = ("", "_reverse")

    def forward(self, params, ctl):
        C, B = self.C, self.B
        cat = self.buf("cat", C, B, 128)
        for bi, (br, din) in enumerate((("vitals", VIT), ("labs", LAB))):
            x = self.buf("xv" if bi == 0 else "xl", C, B, din)
            for i in (1, 2, 3):
                h = self.buf(f"{br}_h{i}", C, B, 64)
                for d, suf in enumerate(self.DIRS):
                    gi = self.buf(f"{br}_gi{i}{d}", C, B, 96)
                    pre = f"{br}_gru{i}."
                    Lx.bgemm(x, self.w(params, pre + "weight_ih_l0" + suf), gi,
                             bias=self.w(params, pre + "bias_ih_l0" + suf))
                    Lx.gru_fwd(gi, self.w(params, pre + "bias_hh_l0" + suf), h, 32 * d)
                x = h
            Lx.ln_fwd(x, None, None, cat[:, :, 64 * bi:64 * bi + 64], self.buf(f"{br}_st", C, B, 2),
                      self.w(params, f"{br}_ln.weight"), self.w(params, f"{br}_ln.bias"), ctl,
                      layer_o=bi, p_o=self.p(0.3))
        f1, f2, z = self.buf("f1", C, B, 32), self.buf("f2", C, B, 16), self.buf("z", C, B, 1)
        self.linear(cat, params, "fc1.weight", "fc1.bias", f1, act=ACT_RELU)
        self.linear(f1, params, "fc2.weight", "fc2.bias", f2, act=ACT_RELU)
        self.linear(f2, params, "output.weight", "output.bias", z)
        return z

    def backward(self, params, grads, ctl):
        C, B = self.C, self.B
        f1, f2 = self.buf("f1", C, B, 32), self.buf("f2", C, B, 16)
        dz, d2, d1 = self.buf("dz", C, B, 1), self.buf("d2", C, B, 16), self.buf("d1", C, B, 32)
        dcat = self.buf("dcat", C, B, 128)
        self.linear_bwd(dz, f2, params, grads, "output.weight", "output.bias", d2, G=f2, gact=ACT_RELU)
        self.linear_bwd(d2, f1, params, grads, "fc2.weight", "fc2.bias", d1, G=f1, gact=ACT_RELU)
        self.linear_bwd(d1, self.buf("cat", C, B, 128), params, grads, "fc1.weight", "fc1.bias", dcat)
        for bi, (br, din) in enumerate((("vitals", VIT), ("labs", LAB))):
            dh = self.buf(f"{br}_dh3", C, B, 64)
            Lx.ln_bwd(dcat[:, :, 64 * bi:64 * bi + 64], self.buf(f"{br}_h3", C, B, 64), self.buf(f"{br}_st", C, B, 2),
                      self.w(params, f"{br}_ln.weight"), dh, 0, None, self.w(grads, f"{br}_ln.weight"),
                      self.w(grads, f"{br}_ln.bias"), ctl, layer_o=bi, p_o=self.p(0.3))
            for i in (3, 2, 1):
                x = self.buf("xv" if bi == 0 else "xl", C, B, din) if i == 1 else self.buf(f"{br}_h{i - 1}", C, B, 64)
                dprev = self.buf(f"{br}_dh{i - 1}", C, B, 64) if i > 1 else None
                for d, suf in enumerate(self.DIRS):
                    pre = f"{br}_gru{i}."
                    dgi = self.buf(f"{br}_dgi{d}", C, B, 96)
                    Lx.gru_bwd(dh, 32 * d, self.buf(f"{br}_gi{i}{d}", C, B, 96),
                               self.w(params, pre + "bias_hh_l0" + suf), dgi,
                               self.w(grads, pre + "bias_ih_l0" + suf), self.w(grads, pre + "bias_hh_l0" + suf))
                    self.dw(dgi, x, self.w(grads, pre + "weight_ih_l0" + suf))
                    if dprev is not None:
                        Lx.bgemm(dgi, self.w(params, pre + "weight_ih_l0" + suf).transpose(1, 2), dprev,
                                 accum=1 if d else 0)
                if dprev is not None:
                    dh = dprev


# ============================================================================================ HAR
class HARProgram(_Program):
    """TransformerClassifier: Conv1d(1->64)+PE stem, 2 post-norm encoder layers (flash attention,
    fused residual+dropout+LayerNorm, ReLU FFN), mean over L, MLP classifier; cross-entropy."""

    model_name = "TransformerClassifier"
    loss = "ce"
    L = 561
    NL = 2

    def lyr(self, i, name):
        return f"transformer.layers.{i}.{name}"

    def inputs(self, table, idx, ctl):
        C, B = self.C, self.B
        Lx.gather_har(table.x, table.y, idx, ctl, self.buf("x", C, B, self.L),
                      self.buf("y", C, B, dtype=torch.long))

    def set_inputs(self, x: torch.Tensor) -> None:
        n = x.shape[0]
        xb = self.buf("x", self.C, self.B, self.L)
        xb.zero_()
        xb[:, :n] = x.reshape(n, -1)[None]

    def labels(self):
        return self.buf("y", self.C, self.B, dtype=torch.long)

    def skip_range(self):
        s = self.slot["pe.pe"]
        return (s.offset, s.offset + s.numel)

    # ---- device path: the bf16 encoder of csrc/kernels/har.hip (five launches per layer) --------------
    def _fused(self, params) -> bool:
        return params.is_cuda and os.environ.get("AFL_HAR_FUSED", "1") != "0"

    def _scheme(self, params) -> str:
        """Attention dropout hash of this path: the CPU composite mirrors the bf16 device kernels ("rc");
        the device layer-library fallback (AFL_HAR_FUSED=0) has attention.hip's "pair" draws."""
        return "pair" if params.is_cuda else "rc"

    def _lw(self, i) -> list:
        """Flat offsets of layer i's parameters (AflHarLayerW order)."""
        names = ["self_attn.in_proj_weight", "self_attn.in_proj_bias", "self_attn.out_proj.weight",
                 "self_attn.out_proj.bias", "norm1.weight", "norm1.bias", "linear1.weight", "linear1.bias",
                 "linear2.weight", "linear2.bias", "norm2.weight", "norm2.bias"]
        return [self.slot[self.lyr(i, n)].offset for n in names]

    def _lp(self) -> int:
        return (self.L + 63) // 64 * 64

    def _groups(self) -> int:
        """Workgroups per client of the backward row passes (8 clients: one per CU).  Fixed, NOT a function of
        the client count: the weight-gradient partials are summed in workgroup order, so a client's gradients
        are the same bits whichever clients share the launch (placement independence)."""
        return 32

    def _mask(self, i) -> torch.Tensor:
        """Layer i's attention-dropout keep words: written by the forward kernel, read by both backward kernels."""
        from .. import ops

        return self.buf(f"amask{i}", self.C * self.B * 4, int(ops.native().har_mask_words(self._lp())),
                        dtype=torch.int64)

    def _kbits(self, i) -> torch.Tensor:
        """Layer i's row-pass dropout keep bits (out_proj, FFN, linear2): written by ``har_post``, read by
        ``har_post_bwd`` (64 B per row instead of 24 hashes per lane and row in the backward)."""
        from .. import ops

        return self.buf(f"kbits{i}", self.C, self.B * self.L, int(ops.native().har_kbits_per_row), dtype=torch.int32)

    def _post_seg(self, i) -> torch.Tensor:
        key = f"_seg_post{i}"
        if key not in self._bufs:
            o = self._lw(i)
            # partial layout (har.hip G_*): Wo | W1 | W2 | bo g1 be1 b1(256) b2 g2 be2
            segs = [(0, o[2], 4096), (4096, o[6], 16384), (20480, o[8], 16384), (36864, o[3], 64), (36928, o[4], 64),
                    (36992, o[5], 64), (37056, o[7], 256), (37312, o[9], 64), (37376, o[10], 64), (37440, o[11], 64)]
            self._bufs[key] = torch.tensor(segs, dtype=torch.int32, device=self.device)
        return self._bufs[key]

    def _qkv_seg(self, i) -> torch.Tensor:
        key = f"_seg_qkv{i}"
        if key not in self._bufs:
            o = self._lw(i)
            self._bufs[key] = torch.tensor([(0, o[0], 192 * 64), (192 * 64, o[1], 192)], dtype=torch.int32,
                                           device=self.device)
        return self._bufs[key]

    def _forward_fused(self, params, ctl):
        from .. import ops

        nat = ops.native()
        C, B, L = self.C, self.B, self.L
        R, Lp = B * L, self._lp()
        bf = torch.bfloat16
        p = self.p(0.1)
        seeds, stepctl = (ctl.seeds, ctl.stepctl) if (ctl is not None and p > 0.0) else (None, None)
        h = self.buf("hb0", C, R, 64, dtype=bf)
        nat.har_stem(self.buf("x", C, B, L), params, self.slot["conv.weight"].offset, self.slot["conv.bias"].offset,
                     self.slot["pe.pe"].offset, h)
        for i in range(self.NL):
            w = self._lw(i)
            qkv = self.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf)  # padding rows stay zero
            nat.har_qkv(h, params, w[0], w[1], qkv, B, L, 0.25 * 1.4426950408889634)  # 1/sqrt(16) * log2(e)
            o, lse2 = self.buf(f"ob{i}", C, R, 64, dtype=bf), self.buf(f"lse2_{i}", C * B * 4, Lp)
            nat.har_attn_fwd(qkv, o, lse2, B, L, seeds, stepctl, 10 * i, p, self._mask(i) if seeds is not None else None)
            y = self.buf(f"hb{i + 1}", C, R, 64, dtype=bf)
            nat.har_post(o, h, self.buf(f"xh1_{i}", C, R, 64, dtype=bf), self.buf(f"xh2_{i}", C, R, 64, dtype=bf),
                         self.buf(f"rs{i}", C, R, 2), y, params, w, seeds, stepctl, 10 * i, p,
                         self._kbits(i) if seeds is not None else None)
            h = y
        pooled, c1, logits = self.buf("pool", C, B, 64), self.buf("c1", C, B, 64), self.buf("logits", C, B, 6)
        nat.har_pool(h, B, L, pooled)
        self.linear(pooled, params, "classifier.0.weight", "classifier.0.bias", c1, act=ACT_RELU, ctl=ctl, layer=30,
                    p=0.3)
        self.linear(c1, params, "classifier.3.weight", "classifier.3.bias", logits)
        return logits

    def _backward_fused(self, params, grads, ctl):
        from .. import ops

        nat = ops.native()
        C, B, L = self.C, self.B, self.L
        R, Lp, G = B * L, self._lp(), self._groups()
        bf = torch.bfloat16
        p = self.p(0.1)
        seeds, stepctl = (ctl.seeds, ctl.stepctl) if (ctl is not None and p > 0.0) else (None, None)
        dlog, dc1, dpool = self.buf("dz", C, B, 6), self.buf("dc1", C, B, 64), self.buf("dpool", C, B, 64)
        c1 = self.buf("c1", C, B, 64)
        self.linear_bwd(dlog, c1, params, grads, "classifier.3.weight", "classifier.3.bias", dc1, G=c1,
                        gact=ACT_RELU, ctl=ctl, layer=30, p=0.3)
        self.linear_bwd(dc1, self.buf("pool", C, B, 64), params, grads, "classifier.0.weight", "classifier.0.bias",
                        dpool)
        ws_p = self.buf("ws_post", C * G * int(nat.har_post_ng))
        # the q|k|v backward runs two workgroups per CU (two waves per SIMD): twice the partials, same fixed order
        GQ = int(os.environ.get("AFL_HAR_QKV_G", 2 * G))
        ws_q = self.buf("ws_qkv", C * GQ * int(nat.har_qkv_ng))
        dres, dout = self.buf("dres", C, R, 64), self.buf("doutb", C, R, 64, dtype=bf)
        delta, dqkv = self.buf("delta", C * B * 4, Lp), self.buf("dqkvb", C * B * 4, 3, Lp, 16, dtype=bf)
        dxs = [self.buf("dxA", C, R, 64), self.buf("dxB", C, R, 64)]
        dy = None
        for i in reversed(range(self.NL)):
            w = self._lw(i)
            nat.har_post_bwd(dy, dpool if dy is None else None, B, L, self.buf(f"ob{i}", C, R, 64, dtype=bf),
                             self.buf(f"xh1_{i}", C, R, 64, dtype=bf), self.buf(f"xh2_{i}", C, R, 64, dtype=bf),
                             self.buf(f"rs{i}", C, R, 2), dres, dout, delta, ws_p, params, w, seeds, stepctl, 10 * i,
                             p, G, self._kbits(i) if seeds is not None else None)
            nat.har_reduce(ws_p, G, int(nat.har_post_ng), self._post_seg(i), grads)
            nat.har_attn_bwd(self.buf(f"qkvb{i}", C * B * 4, 3, Lp, 16, dtype=bf), self.buf(f"lse2_{i}", C * B * 4, Lp),
                             dout, delta, dqkv, B, L, seeds, stepctl, 10 * i, p,
                             self._mask(i) if seeds is not None else None)
            dx = dxs[i % 2]
            nat.har_qkv_bwd(dqkv, dres, self.buf(f"hb{i}", C, R, 64, dtype=bf), dx, ws_q, params, w[0], B, L, GQ)
            nat.har_reduce(ws_q, GQ, int(nat.har_qkv_ng), self._qkv_seg(i), grads)
            dy = dx
        Lx.conv_pe_bwd(self.buf("x", C, B, L), dy, grads, self.slot["conv.weight"].offset,
                       self.slot["conv.bias"].offset)

    def forward(self, params, ctl):
        if self._fused(params):
            return self._forward_fused(params, ctl)
        C, B, L = self.C, self.B, self.L
        R = B * L
        h = self.buf("h0", C, R, 64)
        Lx.conv_pe_fwd(self.buf("x", C, B, L), params, self.slot["conv.weight"].offset, self.slot["conv.bias"].offset,
                       self.slot["pe.pe"].offset, h)
        for i in range(self.NL):
            qkv, o, a = self.buf(f"qkv{i}", C, R, 192), self.buf(f"o{i}", C, R, 64), self.buf(f"a{i}", C, R, 64)
            lse = self.buf(f"lse{i}", C * B * 4, Lx.attn_lp(L))
            self.linear(h, params, self.lyr(i, "self_attn.in_proj_weight"), self.lyr(i, "self_attn.in_proj_bias"), qkv)
            Lx.attn_fwd(qkv, o, lse, B, L, ctl, layer=10 * i, p=self.p(0.1), scheme=self._scheme(params))
            self.linear(o, params, self.lyr(i, "self_attn.out_proj.weight"), self.lyr(i, "self_attn.out_proj.bias"), a)
            s1, h1 = self.buf(f"s1_{i}", C, R, 64), self.buf(f"h1_{i}", C, R, 64)
            Lx.ln_fwd(h, a, s1, h1, self.buf(f"st1_{i}", C, R, 2), self.w(params, self.lyr(i, "norm1.weight")),
                      self.w(params, self.lyr(i, "norm1.bias")), ctl, layer_a=10 * i + 1, p_a=self.p(0.1))
            f, f2 = self.buf(f"f{i}", C, R, 256), self.buf(f"f2_{i}", C, R, 64)
            self.linear(h1, params, self.lyr(i, "linear1.weight"), self.lyr(i, "linear1.bias"), f, act=ACT_RELU,
                        ctl=ctl, layer=10 * i + 2, p=0.1)
            self.linear(f, params, self.lyr(i, "linear2.weight"), self.lyr(i, "linear2.bias"), f2)
            s2, h2 = self.buf(f"s2_{i}", C, R, 64), self.buf(f"h{i + 1}", C, R, 64)
            Lx.ln_fwd(h1, f2, s2, h2, self.buf(f"st2_{i}", C, R, 2), self.w(params, self.lyr(i, "norm2.weight")),
                      self.w(params, self.lyr(i, "norm2.bias")), ctl, layer_a=10 * i + 3, p_a=self.p(0.1))
            h = h2
        pooled, c1, logits = self.buf("pool", C, B, 64), self.buf("c1", C, B, 64), self.buf("logits", C, B, 6)
        Lx.mean_rows_fwd(h, B, L, pooled)
        self.linear(pooled, params, "classifier.0.weight", "classifier.0.bias", c1, act=ACT_RELU, ctl=ctl, layer=30,
                    p=0.3)
        self.linear(c1, params, "classifier.3.weight", "classifier.3.bias", logits)
        return logits

    def backward(self, params, grads, ctl):
        if self._fused(params):
            return self._backward_fused(params, grads, ctl)
        C, B, L = self.C, self.B, self.L
        R = B * L
        dlog, dc1, dpool = self.buf("dz", C, B, 6), self.buf("dc1", C, B, 64), self.buf("dpool", C, B, 64)
        c1 = self.buf("c1", C, B, 64)
        self.linear_bwd(dlog, c1, params, grads, "classifier.3.weight", "classifier.3.bias", dc1, G=c1,
                        gact=ACT_RELU, ctl=ctl, layer=30, p=0.3)
        self.linear_bwd(dc1, self.buf("pool", C, B, 64), params, grads, "classifier.0.weight", "classifier.0.bias",
                        dpool)
        dh = self.buf("dhA", C, R, 64)
        Lx.mean_rows_bwd(dpool, B, L, dh)
        other = self.buf("dhB", C, R, 64)
        for i in reversed(range(self.NL)):
            hin = self.buf(f"h{i}" if i else "h0", C, R, 64)
            h1 = self.buf(f"h1_{i}", C, R, 64)
            dh1, df2, df = self.buf("dh1", C, R, 64), self.buf("df2", C, R, 64), self.buf("df", C, R, 256)
            Lx.ln_bwd(dh, self.buf(f"s2_{i}", C, R, 64), self.buf(f"st2_{i}", C, R, 2),
                      self.w(params, self.lyr(i, "norm2.weight")), dh1, 0, df2,
                      self.w(grads, self.lyr(i, "norm2.weight")), self.w(grads, self.lyr(i, "norm2.bias")), ctl,
                      layer_a=10 * i + 3, p_a=self.p(0.1))
            self.linear_bwd(df2, self.buf(f"f{i}", C, R, 256), params, grads, self.lyr(i, "linear2.weight"),
                            self.lyr(i, "linear2.bias"), df, G=self.buf(f"f{i}", C, R, 256), gact=ACT_RELU, ctl=ctl,
                            layer=10 * i + 2, p=0.1)
            self.linear_bwd(df, h1, params, grads, self.lyr(i, "linear1.weight"), self.lyr(i, "linear1.bias"), dh1,
                            accum=1)
            da, do, dqkv = self.buf("da", C, R, 64), self.buf("do", C, R, 64), self.buf("dqkv", C, R, 192)
            Lx.ln_bwd(dh1, self.buf(f"s1_{i}", C, R, 64), self.buf(f"st1_{i}", C, R, 2),
                      self.w(params, self.lyr(i, "norm1.weight")), other, 0, da,
                      self.w(grads, self.lyr(i, "norm1.weight")), self.w(grads, self.lyr(i, "norm1.bias")), ctl,
                      layer_a=10 * i + 1, p_a=self.p(0.1))
            self.linear_bwd(da, self.buf(f"o{i}", C, R, 64), params, grads, self.lyr(i, "self_attn.out_proj.weight"),
                            self.lyr(i, "self_attn.out_proj.bias"), do)
            Lx.attn_bwd(self.buf(f"qkv{i}", C, R, 192), self.buf(f"o{i}", C, R, 64),
                        self.buf(f"lse{i}", C * B * 4, Lx.attn_lp(L)), do, dqkv, B, L, ctl, layer=10 * i, p=self.p(0.1),
                        scheme=self._scheme(params))
            self.linear_bwd(dqkv, hin, params, grads, self.lyr(i, "self_attn.in_proj_weight"),
                            self.lyr(i, "self_attn.in_proj_bias"), other, accum=1)
            dh, other = other, dh
        Lx.conv_pe_bwd(self.buf("x", C, B, L), dh, grads, self.slot["conv.weight"].offset,
                       self.slot["conv.bias"].offset)


PROGRAMS = {"CNNModel": CNNProgram, "RNNModel": RNNProgram, "TransformerClassifier": HARProgram}
CNN2_TIMEOUT = "cnn2 trainer: a cross-workgroup wait timed out (workgroups not co-resident?)"


# ================================================================================== step tables
def step_tables_native(order: torch.Tensor, nd_dev: torch.Tensor, S: int, B: int, zero_i=None, zero_f=None):
    """``step_tables`` on the GPU in ONE launch (``plan.hip`` ``k_step_tables``), which also zero-fills the given
    per-round int32 / fp32 tensors: (idx, bsz, ep, nb).  ``S`` = max over clients of epochs x batches."""
    from .. import ops

    zi = [zero_i] if zero_i is not None else []
    zf = [zero_f] if zero_f is not None else []
    return tuple(ops.native().step_tables(order.contiguous(), nd_dev, int(B), int(S), zi, zf))


def step_tables(order: torch.Tensor, nd: Sequence[int], epochs: int, B: int, device):
    """Per-step batch tables from a ``Plan``: ``idx [S, C, B]`` (-1 = padding), ``bsz [S, C]``,
    ``epoch [S, C]``, ``nb [C]`` (batches per epoch, the loss divisor).  Client c's s-th step is its
    s-th batch in (epoch, batch) order; steps past its last batch have ``bsz = 0``.

    Built for all clients at once with a dozen tensor ops on the plan's device (one gather into the plan):
    on a GPU these run between two rounds' training launches, where the earlier per-client loop (~15 small
    kernels per client) cost ~1 ms of back-to-back dispatch per round; a per-batch Python loop of slice copies
    cost ~30 ms.  ``tests/test_programs.py`` pins this against that loop."""
    C = order.shape[0]
    nd = [int(x) for x in nd]
    nbat = [max(1, math.ceil(n / B)) for n in nd]
    S = max([epochs * n for n in nbat] + [0])
    dev = order.device
    dvc = torch.device(device)
    nb_t = Lx.upload(torch.tensor(nbat, dtype=torch.int32), dvc)
    if S == 0 or C == 0:
        return (torch.full((S, C, B), -1, dtype=torch.int32, device=dvc), torch.zeros(S, C, dtype=torch.int32, device=dvc),
                torch.zeros(S, C, dtype=torch.int32, device=dvc), nb_t, S)
    small = Lx.upload(torch.tensor([nbat, nd], dtype=torch.int64), dev)     # [2, C]: batches per epoch, rows
    nbc, ndc = small[0][None, :], small[1][None, :]
    st = torch.arange(S, device=dev)[:, None]                                 # [S, 1]
    valid = st < nbc * epochs                                                  # [S, C]
    e, j = st // nbc, st % nbc
    bsz = torch.where(valid, (ndc - j * B).clamp(min=0, max=B), 0).to(torch.int32)
    ep = torch.where(valid, e, 0).to(torch.int32)
    maxnd = order.shape[2]
    if maxnd == 0:
        idx = torch.full((S, C, B), -1, dtype=torch.int32, device=dev)
    else:
        pos = j[:, :, None] * B + torch.arange(B, device=dev)                 # [S, C, B] row within the epoch
        ok = (pos < ndc[:, :, None]) & valid[:, :, None]
        cc = torch.arange(C, device=dev)[None, :, None]
        lin = (cc * epochs + e.clamp(max=epochs - 1)[:, :, None]) * maxnd + pos.clamp(max=maxnd - 1)
        vals = order.reshape(-1)[lin.reshape(-1)].reshape(S, C, B)
        idx = torch.where(ok, vals.to(torch.int32), -1).to(torch.int32)
    return (idx.to(dvc).contiguous(), bsz.to(dvc).contiguous(), ep.to(dvc).contiguous(), nb_t, S)


class ProgramRunner:
    """Runs a program's optimizer steps for one round: eager on CPU, HIP-graph replay on GPU."""

    def __init__(self, prog: _Program, use_graph: bool = True):
        self.prog = prog
        # AFL_SYNC_CHECK=1 (synchronise + check after every native launch) cannot run inside a capture
        self.use_graph = use_graph and prog.device.type == "cuda" and os.environ.get("AFL_SYNC_CHECK") != "1"
        self._live = None

    def train(self, table, params: torch.Tensor, plan, lr: float, seeds: Sequence[int], sgd_lr: float = 0.0,
              max_steps: int = None, sync: bool = True, compat_har: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """Train ``params [C, P]`` in place.  Returns (ok [C] bool, losses [C, E]) on the host, or with
        ``sync=False`` the device (failed-count [C] int32, losses [C, E]) without synchronising.
        ``compat_har``: the reference ``train_HAR`` loop (``client.py:114-131``) — size-1 batches train,
        a NaN loss does not abort the client."""
        pg = self.prog
        dev = pg.device
        C, P = params.shape
        ctl = StepCtl.create(seeds, dev, min_bs=1 if compat_har else 2, nan_abort=not compat_har)
        if self._onchip_cnn(params, sgd_lr, max_steps):
            # sgd_lr > 0: the gradient-test mode (one plain SGD step p -= sgd_lr g exposes the raw gradients)
            return self._train_cnn2(table, params, plan, sgd_lr if sgd_lr > 0.0 else lr, ctl, sync,
                                    opt_mode=1 if sgd_lr > 0.0 else 0)
        idx, bsz, ep, nb, S = step_tables(plan.order, plan.nd, plan.epochs, pg.B, dev)
        if max_steps is not None:
            S = min(S, max_steps)
        out_params = params
        if params.is_cuda and P % 16:
            # train in a copy whose client rows start 64-byte aligned (P is odd for every model here, so every
            # client's weight views but client 0's were 4-byte aligned only: the GEMM operand loads fell back to
            # scalar).  The padding columns get zero gradients, so Adam leaves them at zero.
            Pp = (P + 15) // 16 * 16
            params = torch.zeros(C, Pp, device=dev)
            params[:, :P].copy_(out_params)
            P = Pp
        grads = torch.zeros(C, P, device=dev)
        m = torch.zeros(C, P, device=dev)
        v = torch.zeros(C, P, device=dev)
        tcount = torch.zeros(C, dtype=torch.int32, device=dev)
        failed = torch.zeros(C, dtype=torch.int32, device=dev)
        losses = torch.zeros(C, plan.epochs, device=dev)
        skip = pg.skip_range()

        on_dev = params.is_cuda

        def step():
            pg.inputs(table, idx, ctl)
            out = pg.forward(params, ctl)
            if pg.fused_loss:
                if not on_dev:
                    grads.zero_()
                pg.backward_loss(params, grads, ctl, (bsz, ep, nb, failed, losses))
                Lx.adam_clients(params, grads, m, v, tcount, bsz, ctl, failed, lr, skip, sgd_lr, zero_grads=on_dev)
                Lx.step_end(ctl, tcount, bsz, failed)
                return
            dz = pg.buf("dz", *out.shape)
            if pg.loss == "bce":
                Lx.bce(out, pg.labels(), bsz, ep, nb, ctl, failed, losses, dz)
            else:
                Lx.ce(out, pg.labels(), bsz, ep, nb, ctl, failed, losses, dz)
            if not on_dev:  # on the device Adam zeroes each gradient entry it consumes
                grads.zero_()
            pg.backward(params, grads, ctl)
            Lx.adam_clients(params, grads, m, v, tcount, bsz, ctl, failed, lr, skip, sgd_lr, zero_grads=on_dev)
            Lx.step_end(ctl, tcount, bsz, failed)

        if S == 0:
            return (torch.ones(C, dtype=torch.bool), losses.double().cpu()) if sync else (failed, losses)
        step()  # eager first step: allocates every buffer and sets kernel attributes before capture
        if S > 1:
            if self.use_graph:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    step()
                # capture recorded without executing; the counter still points at step 1
                for _ in range(S - 1):
                    g.replay()
                self._live = (g, grads, m, v, tcount, params)  # replays may still run when sync=False
            else:
                for _ in range(S - 1):
                    step()
        if params is not out_params:  # (stream-ordered behind the replays)
            out_params.copy_(params[:, :out_params.shape[1]])
        if not sync:
            return failed, losses
        return (failed == 0).cpu(), losses.double().cpu()

    # ---- CNNModel on-chip trainer (csrc/kernels/cnn2.hip) ------------------------------------------------
    cnn2_stamps = None  # optional int64 [C, 25, 64, 8] per-phase wall-clock stamps (tools/cnn2_phases.py)

    def _onchip_cnn(self, params: torch.Tensor, sgd_lr: float, max_steps) -> bool:
        """One persistent launch per round instead of a graph replay per step: CNNModel on a GPU (Adam, or the
        raw-SGD gradient-test mode; step caps stay on the layer program), all 32 workgroups of every client
        co-resident (one per CU).  ``AFL_CNN2=0`` forces the layer program."""
        pg = self.prog
        if pg.model_name != "CNNModel" or not params.is_cuda or not pg.train or max_steps is not None:
            return False
        if os.environ.get("AFL_CNN2", "1") == "0" or pg.B > 128 or pg.B < 2 or params.dtype != torch.float32:
            return False  # (the kernel needs 2 <= B <= 128: hipErrorInvalidValue otherwise)
        from .. import ops
        from ..parallel.launcher import gpu_sharers

        nat = ops.native()
        # every workgroup of a launch must be resident at once; processes sharing the GPU run their own persistent
        # launches on the same CUs, so a launch may count on only its share of them.  More clients than that run
        # in back-to-back launches of clients that fit (_train_cnn2), never on the layer program.
        cus = torch.cuda.get_device_properties(params.device).multi_processor_count // gpu_sharers()
        return int(nat.cnn2_wgs_per_client()) <= cus

    def cnn2_capacity(self, device) -> int:
        """Clients per cnn2 launch: every workgroup co-resident on this process's share of the CUs
        (``AFL_MAX_CLIENTS_PER_LAUNCH`` caps it further: the chunking tests)."""
        from .. import ops
        from ..parallel.launcher import gpu_sharers

        cus = torch.cuda.get_device_properties(device).multi_processor_count // gpu_sharers()
        cap = max(1, cus // int(ops.native().cnn2_wgs_per_client()))
        lim = int(os.environ.get("AFL_MAX_CLIENTS_PER_LAUNCH", "0") or 0)
        return min(cap, lim) if lim > 0 else cap

    def _train_cnn2(self, table, params, plan, lr, ctl, sync, opt_mode: int = 0):
        from .. import ops

        nat = ops.native()
        pg = self.prog
        C = params.shape[0]
        dev = params.device
        if getattr(self, "_cnn2_ws", None) is None or self._cnn2_ws.numel() < C * int(nat.cnn2_ws_bytes()):
            self._cnn2_ws = torch.empty(C * int(nat.cnn2_ws_bytes()), dtype=torch.uint8, device=dev)
        ws = self._cnn2_ws
        # the round boundary in one launch: step tables + zeroed failed flags (int32 [C] | the first chunk's cross-
        # workgroup counters) and losses
        ncw = C * int(nat.cnn2_ctr_words())
        zi = torch.empty(C + ncw, dtype=torch.int32, device=dev)
        failed = zi[:C]
        losses = torch.empty(C, plan.epochs, device=dev)
        nd_dev = plan.nd_dev if plan.nd_dev is not None and plan.nd_dev.device == dev else \
            Lx.upload(torch.as_tensor(plan.nd, dtype=torch.int32), dev)
        nbat = [max(1, math.ceil(int(n) / pg.B)) for n in plan.nd]
        S = max([plan.epochs * n for n in nbat] + [0])
        idx, bsz, ep, nb = step_tables_native(plan.order, nd_dev, S, pg.B, zi, losses)
        if S > 0:
            offs = [s.offset for s in pg.layout.slots]
            pc = params if params.is_contiguous() else params.contiguous()
            live = []
            # back-to-back launches of at most `cap` clients (balanced), each a full persistent round: a client's
            # result does not depend on which launch or how many clients train it (placement independence)
            from ..ops.transformer import client_chunks

            for a, b in client_chunks(C, self.cnn2_capacity(dev)):
                cc = zi[C:C + (b - a) * int(nat.cnn2_ctr_words())]  # (zeroed by the step-table launch)
                if a > 0:  # (later chunks: counters left by the previous chunk's launch)
                    cc.zero_()
                whole = (a, b) == (0, C)
                ti = idx if whole else idx[:, a:b].contiguous()
                tb = bsz if whole else bsz[:, a:b].contiguous()
                te = ep if whole else ep[:, a:b].contiguous()
                nat.cnn2_train(pc[a:b], offs, table.rows, ti, tb, te, nb[a:b], ctl.seeds[a:b], pg.p(0.3), 2, True,
                               float(lr), failed[a:b], losses[a:b], ws, cc, self.cnn2_stamps if whole else None,
                               int(opt_mode))
                live.append((ti, tb, te))
            if pc is not params:
                params.copy_(pc)
            self._live = (ws, zi, idx, bsz, ep, nb, ctl, params, pc, live)  # launches may still run (sync=False)
        if not sync:
            return failed, losses  # failed: 1 = NaN loss, 2 = a cross-workgroup wait timed out (GraphTrainer raises)
        fh = failed.cpu()
        if bool((fh == 2).any()):
            raise RuntimeError(CNN2_TIMEOUT)
        return (fh == 0), losses.double().cpu()

    @torch.no_grad()
    def predict(self, params: torch.Tensor, data: torch.Tensor) -> torch.Tensor:
        """Eval forward of ``params [C, P]`` on ``data`` (ICU rows [N, 24] or HAR x [N, 561]) in chunks
        of the program's batch -> [C, N] probabilities (ICU) or [C, N, 6] logits (HAR)."""
        pg = self.prog
        outs = []
        for a in range(0, data.shape[0], pg.B):
            chunk = data[a:a + pg.B]
            pg.set_inputs(chunk)
            out = pg.forward(params, None)
            n = chunk.shape[0]
            outs.append(torch.sigmoid(out[:, :n, 0]) if pg.loss == "bce" else out[:, :n].clone())
        return torch.cat(outs, dim=1)


def make_program(model_name: str, C: int, B: int, device, train: bool = True, dropout: bool = True) -> _Program:
    if model_name not in PROGRAMS:
        raise ValueError(f"no layer program for {model_name}")
    return PROGRAMS[model_name](C, B, device, train, dropout)
