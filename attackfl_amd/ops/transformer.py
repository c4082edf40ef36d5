"""Fused TransformerModel/ICU training and evaluation (HIP kernels in ``csrc/kernels/tf2.hip``, the on-chip
trainer, and ``csrc/kernels/transformer.hip``, the global-workspace fallback and the eval kernels).

``train_clients`` runs ONE persistent kernel launch that trains every row of ``params [C, P]`` for all
local epochs: by default the on-chip trainer (split 4: head | vitals | labs workgroups, 3 per client), in
back-to-back launches of the clients that fit when C exceeds one launch's co-residency budget
(``auto_split``, ``chunked``); splits 1 / 2 / 3 are the global-workspace kernels (``transformer.hip``).  ``reference_train`` is the
plain PyTorch fp32 oracle of exactly the same computation — same batches, same hash-generated dropout masks,
Adam (or the SGD test mode) — used by the numerics tests to check the kernels.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import native
from .rnn import _dev_i32, _on

NPARAM = 47693
M32 = 0xFFFFFFFF


# ------------------------------------------------------------------------------- device entry points
def auto_split(C: int, dev) -> int:
    """Trainer variant for C clients, the first whose workgroups all fit on the device at once (one per CU):
    4 = the on-chip trainer (``tf2.hip``: head | vitals | labs workgroups), in chunks of clients that fit when
    C is larger (``onchip_capacity``).  The global-workspace kernels of ``transformer.hip`` (split 3 / 2 / 1) are
    explicit choices (the tests' cross-checks) or the fallback below 3 CUs per process.  (A row-split variant —
    each branch over two 4-wave workgroups, 5 per client — was built and measured slower in round 5, 91.5 vs
    103.6 rounds/s, ``profiles/ab_tf2_r5_row_split.log``, and removed.)"""
    from ..parallel.launcher import gpu_sharers

    # (processes sharing the GPU run their own persistent launches on the same CUs: count only this one's share)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count // gpu_sharers()
    # more clients than fit run split 4 in back-to-back launches (train_clients_async), not the slower kernels
    return 4 if cus >= 3 else 1


def client_chunks(C: int, cap: int) -> List[Tuple[int, int]]:
    """[a, b) client ranges of at most ``cap`` clients, as few launches as possible, balanced."""
    if C <= 0:
        return []
    n = -(-C // max(1, cap))
    size = -(-C // n)
    return [(a, min(C, a + size)) for a in range(0, C, size)]


def onchip_capacity(dev, wgs_per_client: int = 3) -> int:
    """Clients per on-chip launch (tf2 / rnn2: 3 co-resident workgroups each) on this process's share of the
    CUs; ``AFL_MAX_CLIENTS_PER_LAUNCH`` caps it (tests).  More clients run in back-to-back launches."""
    from ..parallel.launcher import gpu_sharers

    cus = torch.cuda.get_device_properties(dev).multi_processor_count // gpu_sharers()
    cap = max(1, cus // wgs_per_client)
    lim = int(os.environ.get("AFL_MAX_CLIENTS_PER_LAUNCH", "0") or 0)
    return min(cap, lim) if lim > 0 else cap


def chunked(launch, C: int, cap: int, params, order, nd_t, seeds_t):
    """Run ``launch(params, order, nd, seeds, first) -> (ok, losses)`` over client chunks of at most ``cap``
    clients, back to back on the current stream (``first``: the chunk that takes the diagnostic stamps, if any);
    the per-chunk device results are concatenated (no host sync)."""
    parts = client_chunks(C, cap)
    if len(parts) <= 1:
        return launch(params, order, nd_t, seeds_t, True)
    oks, losses = [], []
    for i, (a, b) in enumerate(parts):
        ok, ls = launch(params[a:b], order[a:b], nd_t[a:b], seeds_t[a:b], i == 0)
        oks.append(ok)
        losses.append(ls)
    return torch.cat(oks), torch.cat(losses)


def device_seed(s: int) -> int:
    """The int32 the kernel receives for client seed ``s`` (a device int32 tensor of these values may be
    passed as ``seeds`` directly)."""
    return int(s) & 0x7FFFFFFF


def train_clients_async(params: torch.Tensor, rows: torch.Tensor, order: torch.Tensor, nd, epochs: int, batch: int,
                        lr: float, seeds: Sequence[int], opt_mode: int = 0, stamps: torch.Tensor = None,
                        split: int = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Enqueue the training launch on the current stream and return (ok [C] int32, losses [C, E]) as
    DEVICE tensors without synchronising (see ``finish``); arguments as ``train_clients``."""
    dev = params.device
    C = params.shape[0]
    if split is None:  # (AFL_TF_SPLIT: A/B override of the automatic choice)
        split = int(os.environ.get("AFL_TF_SPLIT", "0") or 0) or (auto_split(C, dev) if C > 0 else 1)
    nd_t = _dev_i32(nd, dev)
    seeds_t = seeds if _on(seeds, dev) else torch.tensor([device_seed(s) for s in seeds], dtype=torch.int32, device=dev)
    kt = None
    if split == 4:
        kt = adam_step_table(float(lr), int(epochs) * -(-int(order.shape[2]) // int(batch)), dev)
    rows_c, order_c = rows.contiguous(), order.contiguous()

    def launch(p, o, n, s, first=True):
        return native().tf_train(p, rows_c, o, n, s, int(epochs), int(batch), float(lr), int(opt_mode),
                                 stamps if first else None, int(split), kt)
    if split == 4:  # (a stamped run stamps its first chunk only)
        return chunked(launch, C, onchip_capacity(dev, 3), params, order_c, nd_t, seeds_t)
    return launch(params, order_c, nd_t, seeds_t)


_KT_CACHE: Dict[tuple, torch.Tensor] = {}


def adam_step_table(lr: float, steps: int, dev) -> torch.Tensor:
    """[n >= steps, 2] fp32 device table of torch.optim.Adam's per-step scalars, computed in double like
    torch does on the host: (lr / (1 - beta1^t), 1 / sqrt(1 - beta2^t)) for t = 1..n.  Cached per (lr,
    device) and grown in powers of two, so a round never uploads it again."""
    key = (lr, str(dev))
    t = _KT_CACHE.get(key)
    if t is None or t.shape[0] < steps:
        n = 1 << max(10, (max(steps, 1) - 1).bit_length())
        tt = np.arange(1, n + 1, dtype=np.float64)
        tab = np.stack([lr / (1.0 - 0.9 ** tt), 1.0 / np.sqrt(1.0 - 0.999 ** tt)], axis=1).astype(np.float32)
        t = _KT_CACHE[key] = torch.from_numpy(tab).to(dev)
    return t


def finish(ok: torch.Tensor, losses: torch.Tensor, what: str = "fused trainer") -> Tuple[torch.Tensor, torch.Tensor]:
    """Synchronise on a launch from ``train_clients_async`` -> host (ok, losses); a negative ok means a
    cross-workgroup hand-off timed out."""
    ok = ok.cpu()
    if bool((ok < 0).any()):
        raise RuntimeError(f"{what}: a cross-workgroup hand-off timed out (workgroups not co-resident?)")
    return ok, losses.cpu()


def train_clients(params: torch.Tensor, rows: torch.Tensor, order: torch.Tensor, nd, epochs: int, batch: int,
                  lr: float, seeds: Sequence[int], opt_mode: int = 0, stamps: torch.Tensor = None,
                  split: int = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Train all clients in place. Returns (ok [C] int32 on host, losses [C, E] fp32 on host).

    ``split``: workgroups per client — 1 (whole model in one workgroup), 2 (vitals branch + head |
    labs branch) or 3 (head | vitals | labs); the workgroups of a client hand activations and
    gradients to each other every step.  4 = the on-chip trainer (``tf2.hip``, 3 workgroups per client,
    nothing of the model in global memory during the round).  Default: ``auto_split``.
    ``stamps``: optional device int64 [>=64] buffer receiving per-phase wall time (10 ns ticks) of
    workgroup ``stamps[63]`` of the first launch, summed over all steps (diagnostics)."""
    return finish(*train_clients_async(params, rows, order, nd, epochs, batch, lr, seeds, opt_mode, stamps, split))


def eval_forward(params: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """Sigmoid outputs of TransformerModel (eval mode) for every row of ``rows [N, 24]``."""
    return native().tf_eval(params.contiguous(), rows.contiguous())


# ------------------------------------------------------------------------------- hash dropout (host mirror)
def _u32(x):
    return np.asarray(x, dtype=np.uint64) & M32


def hash32(a: int, b: int) -> int:
    a &= M32
    b &= M32
    x = ((a * 0x9E3779B1) & M32) ^ ((b + 0x7F4A7C15 + ((a << 6) & M32) + (a >> 2)) & M32)
    x ^= x >> 16
    x = (x * 0x21F0AAAD) & M32
    x ^= x >> 15
    x = (x * 0x735A2D97) & M32
    x ^= x >> 15
    return x


def keep_mask(key: int, layer: int, n_rows: int, n_cols: int, p: float) -> torch.Tensor:
    """Vectorised mirror of ``tf::keep`` -> bool [n_rows, n_cols] (one hash per column pair)."""
    r = np.arange(n_rows, dtype=np.uint64)[:, None]
    col = np.arange(n_cols, dtype=np.uint64)[None, :]
    c = col >> np.uint64(1)
    x = (np.uint64(key) ^ ((np.uint64(layer) * np.uint64(0x9E3779B9)) & np.uint64(M32))
         ^ ((r * np.uint64(0x85EBCA6B)) & np.uint64(M32)) ^ ((c * np.uint64(0xC2B2AE35)) & np.uint64(M32)))
    x &= np.uint64(M32)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(M32)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    u16 = (x >> ((col & np.uint64(1)) << np.uint64(4))) & np.uint64(0xFFFF)
    thr = {0.1: 6554, 0.3: 19661}[p]
    return torch.from_numpy(u16 >= np.uint64(thr))


# ------------------------------------------------------------------------------- fp32 oracle
def _views(p: torch.Tensor) -> Dict[str, torch.Tensor]:
    from ..models import ParamLayout

    lay = ParamLayout.for_model("TransformerModel")
    return lay.unflatten(p, clone=False)


def reference_forward(sd: Dict[str, torch.Tensor], xv: torch.Tensor, xl: torch.Tensor, masks=None) -> torch.Tensor:
    """Functional TransformerModel forward with explicit dropout masks (None = eval)."""
    outs = []
    for bi, (br, x) in enumerate((("vitals", xv), ("labs", xl))):
        pre = f"{br}_transformer."
        h0 = F.gelu(F.linear(x, sd[f"{br}_dense.weight"], sd[f"{br}_dense.bias"]))
        W = sd[pre + "attention.in_proj_weight"]
        b = sd[pre + "attention.in_proj_bias"]
        v = F.linear(h0, W[128:], b[128:])
        if masks is not None:
            v = v * masks[(bi, "att")].repeat_interleave(16, dim=1) / 0.9
        o = F.linear(v, sd[pre + "attention.out_proj.weight"], sd[pre + "attention.out_proj.bias"])
        if masks is not None:
            o = o * masks[(bi, "d1")] / 0.9
        x1 = F.layer_norm(h0 + o, (64,), sd[pre + "attention_norm.weight"], sd[pre + "attention_norm.bias"], 1e-5)
        f = F.gelu(F.linear(x1, sd[pre + "ffn.0.weight"], sd[pre + "ffn.0.bias"]))
        if masks is not None:
            f = f * masks[(bi, "df")] / 0.9
        f3 = F.linear(f, sd[pre + "ffn.3.weight"], sd[pre + "ffn.3.bias"])
        if masks is not None:
            f3 = f3 * masks[(bi, "d2")] / 0.9
        x2 = F.layer_norm(x1 + f3, (64,), sd[pre + "ffn_norm.weight"], sd[pre + "ffn_norm.bias"], 1e-5)
        outs.append(F.layer_norm(x2, (64,), sd[f"{br}_bn.weight"], sd[f"{br}_bn.bias"], 1e-5))
    h = torch.cat(outs, dim=1)
    h = F.gelu(F.linear(h, sd["fc1.weight"], sd["fc1.bias"]))
    if masks is not None:
        h = h * masks["head"] / 0.7
    h = F.gelu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return torch.sigmoid(F.linear(h, sd["output.weight"], sd["output.bias"]))


def step_masks(seed: int, step: int, n: int) -> dict:
    key = hash32(seed, step)
    m = {}
    for bi in (0, 1):
        m[(bi, "att")] = keep_mask(key, 8 * bi + 0, n, 4, 0.1).float()
        m[(bi, "d1")] = keep_mask(key, 8 * bi + 1, n, 64, 0.1).float()
        m[(bi, "df")] = keep_mask(key, 8 * bi + 2, n, 6, 0.1).float()
        m[(bi, "d2")] = keep_mask(key, 8 * bi + 3, n, 64, 0.1).float()
    m["head"] = keep_mask(key, 16, n, 64, 0.3).float()
    return m


def reference_train(params: torch.Tensor, rows: torch.Tensor, order: torch.Tensor, nd, epochs: int, batch: int,
                    lr: float, seeds: Sequence[int], opt_mode: int = 0, max_steps: int = -1):
    """fp32 PyTorch oracle of ``train_clients`` (CPU).  Returns (ok [C], losses [C, E])."""
    from .composite import adam_step, bce_loss

    C = params.shape[0]
    oks, losses = [], torch.zeros(C, epochs)
    skip = ("in_proj_weight", "in_proj_bias")
    for ci in range(C):
        p = params[ci].clone()
        sd = _views(p)
        train_keys = [k for k in sd]
        m = {k: torch.zeros_like(v) for k, v in sd.items()}
        vv = {k: torch.zeros_like(v) for k, v in sd.items()}
        n = int(nd[ci])
        step = 0
        ok = True
        nbt = max(1, (n + batch - 1) // batch)
        for e in range(epochs):
            tot = 0.0
            for b0 in range(0, n, batch):
                Bn = min(batch, n - b0)
                if Bn == 1:
                    continue
                if 0 <= max_steps <= step:
                    break
                step += 1
                idx = order[ci, e, b0:b0 + Bn].long()
                r = rows[idx]
                leaf = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
                out = reference_forward(leaf, r[:, :7], r[:, 7:23], step_masks(int(seeds[ci]) & 0x7FFFFFFF, step, Bn))
                y = r[:, 23:24]
                loss = bce_loss(out, y)  # (nn.BCELoss forward and backward, as the kernel)
                if torch.isnan(loss):
                    ok = False
                    break
                tot += float(loss.detach())
                loss.backward()
                with torch.no_grad():
                    for k in train_keys:
                        g = leaf[k].grad
                        if g is None:
                            continue
                        if k.endswith(skip):
                            # q/k rows get exactly zero gradient at seq_len 1 (only v rows train)
                            g = g.clone()
                            g[:128] = 0
                        if opt_mode == 1:
                            sd[k].sub_(lr * g)
                        elif k.endswith(skip):
                            sl = slice(128, 192)
                            adam_step(sd[k][sl], g[sl], m[k][sl], vv[k][sl], step, lr)
                        else:
                            adam_step(sd[k], g, m[k], vv[k], step, lr)
            if not ok:
                break
            losses[ci, e] = tot / nbt
        params[ci].copy_(p)
        oks.append(ok)
    return torch.tensor(oks, dtype=torch.int32), losses
