"""pFedHN-style hypernetwork aggregator (reference ``Server.train_hyper``, ``server.py:637-678``).

For every selected client, sequentially: ``W_i = hnet(i)``; ``δ = W_i - w_client``; VJP of
``W_i`` w.r.t. all hnet parameters with cotangent δ; global-norm clip to ``clip-grad-norm``;
one Adam step (lr ``hyper-lr``).  The hnet is held packed (``PackedHyperNet``): all per-key
heads form one ``[P, H]`` matrix, so

* ``W_i = W·f + b`` is one GEMV and ``δ`` comes out of the same pass,
* ``∂L/∂f = Wᵀδ`` is accumulated in that same pass (``ops.hyper_delta_vjp``),
* the head gradient ``δ ⊗ f`` is never materialised: its norm is ``||δ||·||f||`` and the
  Adam update of the ``P·H`` head weights computes each gradient element on the fly
  (``ops.hyper_adam_outer``, one streaming pass),
* the tiny embedding/MLP part (≈ 20 k params) is back-propagated with plain tensor ops and
  updated by the flat Adam kernel.

Every rank holds an identical replica (deterministic kernels), so ``hnet(rank's clients)`` is
computed locally and no scatter is needed.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Optional, Dict, Sequence

import torch

from .. import ops
from ..models import PackedHyperNet

# diagnostic A/B switch: generate_many through the torch MLP (7 small launches) instead of the native features
_TORCH_GEN = bool(os.environ.get("AFL_HYPER_TORCH_GEN"))


class HyperServer:
    def __init__(self, target_sd: "OrderedDict[str, torch.Tensor]", n_clients: int, hyper_lr: float, clip: float,
                 device, seed: int = 0, embedding_dim: int = 8, hidden_dim: int = 100, n_hidden: int = 2):
        g = torch.Generator().manual_seed(int(seed) + 0x5EED)
        self.hnet = PackedHyperNet(target_sd, n_clients, embedding_dim, hidden_dim, n_hidden, device=device,
                                   generator=g)
        self.device = torch.device(device)
        self.lr = float(hyper_lr)
        self.clip = float(clip)
        self.m = torch.zeros_like(self.hnet.arena)
        self.v = torch.zeros_like(self.hnet.arena)
        self.step = 0
        off_W, _ = self.hnet.slots["W"]
        self.n_small = off_W                      # emb + MLP region [0, off_W)
        self._last_info: Dict[str, float] = {}
        self._info_dev = None                     # device [2] (grad norm, clip scale) of the last update
        self._gen_cache = None                    # (client tuple, [n, P]) generated from the current arena

    @property
    def last_info(self) -> Dict[str, float]:
        """Grad norm / clip scale of the last client update; read lazily, so the device path enqueues a
        whole round's update without a host synchronisation (the engine reads it after validation)."""
        if self._info_dev is not None:
            last = self._info_dev.double().cpu()
            self._info_dev = None
            self._last_info = {"grad_norm": float(last[0]), "clip_scale": float(last[1])}
        return self._last_info

    # ------------------------------------------------------------------------------------------
    def generate(self, i: int) -> torch.Tensor:
        return self.hnet.generate(i)

    def generate_many(self, idxs) -> torch.Tensor:
        """``hnet.generate_many`` memoised until the arena next changes (``train`` / ``restore`` /
        ``load_arena``): a round's validation and the next round's START generate the same clients'
        models from the same hypernetwork state.  The result is shared: callers must not modify it."""
        key = tuple(int(i) for i in idxs)
        c = self._gen_cache
        if c is not None and c[0] == key:
            return c[1]
        if self._native_ok() and not _TORCH_GEN:
            # MLP features of every client in one native launch, then one sweep over the packed heads for all of
            # them (the same arithmetic as the generation fused into the update; was a library GEMM, and before
            # that the torch MLP: 7 small launches issued one by one on the round boundary)
            out = ops.hyper_generate_many(self.hnet.arena, key, self.layout_vec())
        else:
            out = self.hnet.generate_many(key)
        self._gen_cache = (key, out)
        return out

    def load_arena(self, arena: torch.Tensor) -> None:
        with torch.no_grad():
            self.hnet.arena.copy_(arena)
        self._gen_cache = None

    def embedding(self, i: int) -> torch.Tensor:
        return self.hnet.emb[i].detach().clone()

    def snapshot(self) -> torch.Tensor:
        return self.hnet.arena.clone()

    def restore(self, snap: torch.Tensor) -> None:
        self.hnet.arena.copy_(snap)
        self._gen_cache = None

    # ------------------------------------------------------------------------------------------
    def _mlp_backward(self, i: int, acts, dfeat: torch.Tensor) -> torch.Tensor:
        """Grads of emb + MLP into a flat [n_small] buffer (same layout as the arena prefix)."""
        h = self.hnet
        g = torch.zeros(self.n_small, dtype=torch.float32, device=self.device)

        def gslot(name):
            off, shp = h.slots[name]
            n = 1
            for s in shp:
                n *= s
            return g[off:off + n].view(shp)

        dz = dfeat
        L = h.n_hidden + 1
        for li in reversed(range(L)):
            Wm, _ = h.mlp(li)
            a_in = acts[li]
            gslot(f"mlp{li}.W").copy_(torch.outer(dz, a_in))
            gslot(f"mlp{li}.b").copy_(dz)
            da = Wm.t() @ dz
            if li > 0:
                dz = da * (acts[li] > 0).to(da.dtype)
            else:
                gslot("emb")[i].copy_(da)
        return g

    def layout_vec(self):
        """Arena offsets for the native kernels: [emb, w_0, b_0, ..., L, E, H, n_nodes, offW, offB, P]."""
        h = self.hnet
        L = h.n_hidden + 1
        lay = [h.slots["emb"][0]]
        for li in range(L):
            lay += [h.slots[f"mlp{li}.W"][0], h.slots[f"mlp{li}.b"][0]]
        lay += [L, h.E, h.H, h.n_nodes, h.slots["W"][0], h.slots["b"][0], h.P]
        return [int(x) for x in lay]

    def _native_ok(self) -> bool:
        h = self.hnet
        if not (self.device.type == "cuda" and h.H % 4 == 0 and h.slots["W"][0] % 4 == 0 and h.H <= 127
                and h.E <= 128 and h.n_hidden + 1 <= 8):
            return False
        return h.slots["W"][0] - h.slots["emb"][0] <= ops.native().hyper_small_capacity()

    def train(self, selected: Sequence[int], updates: Dict[int, torch.Tensor],
              enable: Optional[torch.Tensor] = None, gen_key: Optional[Sequence[int]] = None) -> None:
        """One round of the sequential server update over ``selected`` (client order kept).

        On GPU the whole round is enqueued by ``ops.hyper_server_update`` (three launches per client,
        no host synchronisation, ``last_info`` read lazily); on CPU the composite path below is the oracle.
        ``enable`` (GPU only): device int32 word decided on the device — 0 leaves the hypernetwork and its
        moments untouched (the caller then rolls ``step`` back).  ``gen_key`` (GPU only): the clients of the next
        ``generate_many``; their models come out of the update's own last launches (the features in the last
        small-net launch, the heads sweep fused with the last head Adam) and are memoised for that call."""
        h = self.hnet
        selected = list(selected)
        if not selected:
            return
        self._gen_cache = None
        if self._native_ok():
            rows = [updates[i] for i in selected]
            # the engine hands rows of one gathered matrix; stack only when they are not already views of it
            base = rows[0]._base if rows[0]._base is not None else None
            if base is not None and base.dim() == 2 and all(r._base is base for r in rows) and base.is_contiguous():
                U = base
                urows = [(r.storage_offset() - base.storage_offset()) // base.shape[1] for r in rows]
            else:
                U = torch.stack([r.contiguous() for r in rows])
                urows = list(range(len(rows)))
            gen = tuple(int(i) for i in gen_key) if gen_key is not None and not _TORCH_GEN else ()
            if len(gen) > 32:
                gen = ()
            info, out = ops.hyper_server_update(h.arena, self.m, self.v, U, urows, selected, self.layout_vec(),
                                                self.step, self.lr, self.clip, enable=enable, gen=gen)
            self.step += len(selected)
            self._info_dev = info[-1]  # no host sync here (see last_info)
            if gen:
                self._gen_cache = (gen, out)
            return
        if enable is not None:
            raise RuntimeError("a device-decided hypernetwork update needs the native server kernels")
        for i in selected:
            emb, feat, acts = h.features(i)
            delta, dfeat = ops.hyper_delta_vjp(h.W, h.b, feat, updates[i])   # δ = W f + b - u ; Wᵀδ
            g_small = self._mlp_backward(i, acts, dfeat)
            dd = float(torch.dot(delta.double(), delta.double()).item())
            ff = float(torch.dot(feat.double(), feat.double()).item())
            total_sq = dd * ff + dd + float(torch.dot(g_small.double(), g_small.double()).item())
            total = total_sq ** 0.5
            scale = 1.0
            if self.clip > 0:
                coef = self.clip / (total + 1e-6)
                if coef < 1.0:
                    scale = coef
            self.step += 1
            small = slice(0, self.n_small)
            ops.adam_step_scaled(h.arena[small], g_small, self.m[small], self.v[small], self.step, self.lr, scale)
            offW, _ = h.slots["W"]
            ops.hyper_adam_outer(h.W, h.b, self.m[offW:], self.v[offW:], delta, feat, self.step, self.lr, scale)
            self._info_dev = None
            self._last_info = {"grad_norm": total, "clip_scale": scale}
