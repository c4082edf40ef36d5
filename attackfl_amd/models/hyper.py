"""Hypernetworks (pFedHN-style per-client weight generators).

``HyperNetwork`` keeps the reference module structure so that ``{model}_hyper_{N}.pth``
checkpoints have identical keys (reference ``src/Model.py:251-304``):
``target_model.*``, ``embeddings.weight [N, emb]``, ``mlp.{0,2,4}.{weight,bias}``,
``hyper_layers.<key with '.'->'__'>.{weight [numel, hidden], bias [numel]}``.

The server does not run this module on its hot path.  ``PackedHyperNet`` holds the same
parameters with all per-key heads concatenated into ONE ``[P, hidden]`` matrix (plus a
``[P]`` bias) so that generating a client's weights is a single GEMV and the VJP of a
client update is a single outer product; see ``attackfl_amd/fl/hyper_server.py`` and
``ops/hyper.py``.  ``CNNHyper`` (reference ``src/Model.py:309-416``, dormant there) is provided
for completeness.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
from torch.nn.utils import spectral_norm


def _lin(i: int, o: int, sn: bool) -> nn.Module:
    layer = nn.Linear(i, o)
    return spectral_norm(layer) if sn else layer


class HyperNetwork(nn.Module):
    def __init__(self, target_model: nn.Module, n_nodes: int, embedding_dim: int, hidden_dim: int = 100,
                 spec_norm: bool = False, n_hidden: int = 2):
        super().__init__()
        self.target_model = target_model
        self.embeddings = nn.Embedding(num_embeddings=n_nodes, embedding_dim=embedding_dim)
        layers: List[nn.Module] = [_lin(embedding_dim, hidden_dim, spec_norm)]
        for _ in range(n_hidden):
            layers += [nn.ReLU(inplace=True), _lin(hidden_dim, hidden_dim, spec_norm)]
        self.mlp = nn.Sequential(*layers)
        heads = nn.ModuleDict()
        for name, p in target_model.state_dict().items():
            heads[name.replace(".", "__")] = _lin(hidden_dim, p.numel(), spec_norm)
        self.hyper_layers = heads
        self._shapes = OrderedDict((k, tuple(v.shape)) for k, v in target_model.state_dict().items())

    def forward(self, idx: torch.Tensor) -> Tuple["OrderedDict[str, torch.Tensor]", torch.Tensor]:
        emd = self.embeddings(idx)
        feat = self.mlp(emd)
        out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for safe, layer in self.hyper_layers.items():
            name = safe.replace("__", ".")
            w = layer(feat)
            out[name] = w.view(-1) if "bias" in name else w.view(self._shapes[name])
        return out, emd


class CNNHyper(nn.Module):
    """Hard-coded hypernetwork for ``CNNModel`` (reference ``src/Model.py:309-416``)."""

    _SPEC = [
        ("vitals_conv1.weight", (32, 1, 3)), ("vitals_conv1.bias", (32,)),
        ("vitals_conv2.weight", (64, 32, 3)), ("vitals_conv2.bias", (64,)),
        ("vitals_conv3.weight", (128, 64, 3)), ("vitals_conv3.bias", (128,)),
        ("labs_conv1.weight", (32, 1, 3)), ("labs_conv1.bias", (32,)),
        ("labs_conv2.weight", (64, 32, 3)), ("labs_conv2.bias", (64,)),
        ("labs_conv3.weight", (128, 64, 3)), ("labs_conv3.bias", (128,)),
        ("fc1.weight", (128, 1024)), ("fc1.bias", (128,)),
        ("fc2.weight", (64, 128)), ("fc2.bias", (64,)),
        ("fc3.weight", (32, 64)), ("fc3.bias", (32,)),
        ("output.weight", (1, 32)), ("output.bias", (1,)),
    ]

    def __init__(self, n_nodes: int, embedding_dim: int, hidden_dim: int, n_hidden: int, spec_norm: bool = False):
        super().__init__()
        self.embeddings = nn.Embedding(num_embeddings=n_nodes, embedding_dim=embedding_dim)
        layers: List[nn.Module] = [_lin(embedding_dim, hidden_dim, spec_norm)]
        for _ in range(n_hidden):
            layers += [nn.ReLU(inplace=True), _lin(hidden_dim, hidden_dim, spec_norm)]
        self.mlp = nn.Sequential(*layers)
        for key, shape in self._SPEC:
            attr = key.replace(".weight", "_weights").replace(".bias", "_bias")
            n = 1
            for s in shape:
                n *= s
            setattr(self, attr, _lin(hidden_dim, n, spec_norm))

    def forward(self, idx: torch.Tensor):
        emd = self.embeddings(idx)
        feat = self.mlp(emd)
        out = OrderedDict()
        for key, shape in self._SPEC:
            attr = key.replace(".weight", "_weights").replace(".bias", "_bias")
            out[key] = getattr(self, attr)(feat).view(*shape) if len(shape) > 1 else getattr(self, attr)(feat).view(-1)
        return out, emd


class PackedHyperNet:
    """HyperNetwork parameters in packed, device-resident form.

    Parameters (all fp32, on ``device``):
      ``emb``   [N, E]      embeddings
      ``mlp``   list of (W [H, in], b [H]) for the 3 MLP layers (ReLU between)
      ``W``     [P, H]      all heads, rows ordered as the target state_dict flattening
      ``b``     [P]         all head biases
    ``flat()`` returns every trainable tensor as one contiguous fp32 arena (Adam runs on it).
    """

    def __init__(self, target_sd: "OrderedDict[str, torch.Tensor]", n_nodes: int, embedding_dim: int = 8,
                 hidden_dim: int = 100, n_hidden: int = 2, device="cpu", generator: torch.Generator = None):
        self.target_sd = OrderedDict((k, v.detach().clone().float().cpu()) for k, v in target_sd.items())
        self.n_nodes = n_nodes
        self.E = embedding_dim
        self.H = hidden_dim
        self.n_hidden = n_hidden
        self.keys = list(self.target_sd.keys())
        self.shapes = [tuple(v.shape) for v in self.target_sd.values()]
        self.numels = [v.numel() for v in self.target_sd.values()]
        self.P = sum(self.numels)
        self.device = torch.device(device)
        # arena layout: emb | mlp0.W | mlp0.b | ... | W | b
        sizes = [("emb", (n_nodes, embedding_dim))]
        dims = [embedding_dim] + [hidden_dim] * (n_hidden + 1)
        for i in range(n_hidden + 1):
            sizes.append((f"mlp{i}.W", (dims[i + 1], dims[i])))
            sizes.append((f"mlp{i}.b", (dims[i + 1],)))
        sizes.append(("W", (self.P, hidden_dim)))
        sizes.append(("b", (self.P,)))
        total = 0
        self.slots: Dict[str, Tuple[int, Tuple[int, ...]]] = OrderedDict()
        for name, shp in sizes:
            n = 1
            for s in shp:
                n *= s
            self.slots[name] = (total, shp)
            total += n
        self.numel = total
        self.arena = torch.zeros(total, dtype=torch.float32, device=self.device)
        self.init_from_module(HyperNetwork(_FrozenTarget(self.target_sd), n_nodes, embedding_dim, hidden_dim,
                                           False, n_hidden) if generator is None else
                              _seeded_hnet(self.target_sd, n_nodes, embedding_dim, hidden_dim, n_hidden, generator))

    # -- views -----------------------------------------------------------------
    def view(self, name: str) -> torch.Tensor:
        off, shp = self.slots[name]
        n = 1
        for s in shp:
            n *= s
        return self.arena[off:off + n].view(shp)

    @property
    def emb(self) -> torch.Tensor:
        return self.view("emb")

    @property
    def W(self) -> torch.Tensor:
        return self.view("W")

    @property
    def b(self) -> torch.Tensor:
        return self.view("b")

    def mlp(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.view(f"mlp{i}.W"), self.view(f"mlp{i}.b")

    # -- conversion to / from the reference module state_dict --------------------
    def init_from_module(self, hnet: HyperNetwork) -> None:
        self.load_state_dict(hnet.state_dict(), strict=False)

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        return self.state_dict_of(self.arena.detach().cpu())

    def target_tail(self) -> torch.Tensor:
        """The (constant) target model flattened in state_dict order: appended behind a host copy of the arena
        it lets ``state_dict_of`` return views of ONE storage (the checkpoint writer's zip-template path)."""
        return torch.cat([t.reshape(-1) for t in self.target_sd.values()])

    def state_dict_of(self, arena: torch.Tensor, clone: bool = True) -> "OrderedDict[str, torch.Tensor]":
        """Reference ``HyperNetwork`` state_dict built from a host copy of the arena (views when
        ``clone`` is False: the caller owns ``arena`` until the dict is consumed).  If ``arena`` also holds
        ``target_tail()`` behind the arena, the ``target_model.*`` entries are views of it too."""
        def v(name):
            off, shp = self.slots[name]
            n = 1
            for x in shp:
                n *= x
            t = arena[off:off + n].view(shp)
            return t.clone() if clone else t

        with_tail = not clone and arena.numel() == self.numel + self.P
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        toff = self.numel
        for k, t in self.target_sd.items():
            if with_tail:
                sd[f"target_model.{k}"] = arena[toff:toff + t.numel()].view(t.shape)
                toff += t.numel()
            else:
                sd[f"target_model.{k}"] = t.clone()
        sd["embeddings.weight"] = v("emb")
        for i in range(self.n_hidden + 1):
            sd[f"mlp.{2 * i}.weight"] = v(f"mlp{i}.W")
            sd[f"mlp.{2 * i}.bias"] = v(f"mlp{i}.b")
        W, b = v("W"), v("b")
        off = 0
        for k, n in zip(self.keys, self.numels):
            safe = k.replace(".", "__")
            sd[f"hyper_layers.{safe}.weight"] = W[off:off + n]
            sd[f"hyper_layers.{safe}.bias"] = b[off:off + n]
            off += n
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        with torch.no_grad():
            for k in self.keys:
                tk = f"target_model.{k}"
                if tk in sd:
                    self.target_sd[k] = sd[tk].detach().float().cpu().clone()
            self.emb.copy_(sd["embeddings.weight"].to(self.device))
            for i in range(self.n_hidden + 1):
                Wm, bm = self.mlp(i)
                Wm.copy_(sd[f"mlp.{2 * i}.weight"].to(self.device))
                bm.copy_(sd[f"mlp.{2 * i}.bias"].to(self.device))
            off = 0
            for k, n in zip(self.keys, self.numels):
                safe = k.replace(".", "__")
                self.W[off:off + n].copy_(sd[f"hyper_layers.{safe}.weight"].to(self.device))
                self.b[off:off + n].copy_(sd[f"hyper_layers.{safe}.bias"].to(self.device))
                off += n

    def clone_arena(self) -> torch.Tensor:
        return self.arena.clone()

    # -- forward in plain torch (composite oracle) --------------------------------
    def features(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor, List[torch.Tensor]]:
        """Return (emb [E], feat [H], pre-activations list) for client ``idx``."""
        h = self.emb[idx]
        pre: List[torch.Tensor] = []
        acts = [h]
        for i in range(self.n_hidden + 1):
            Wm, bm = self.mlp(i)
            z = Wm @ h + bm
            pre.append(z)
            h = torch.relu(z) if i < self.n_hidden else z
            acts.append(h)
        return self.emb[idx], h, acts

    def features_many(self, idxs) -> torch.Tensor:
        """MLP features [n, H] of several clients, batched through every layer."""
        key = tuple(int(i) for i in idxs)
        cache = self.__dict__.setdefault("_idx_dev", {})
        ix = cache.get(key)
        if ix is None:
            # (built once per client set: a pageable host -> device copy synchronises the stream, i.e. would
            # make the host wait for the training launch enqueued before it)
            if len(cache) > 256:
                cache.clear()
            ix = cache[key] = torch.as_tensor(list(key), dtype=torch.long, device=self.emb.device)
        h = self.emb[ix]
        for i in range(self.n_hidden + 1):
            Wm, bm = self.mlp(i)
            h = torch.addmm(bm[None, :], h, Wm.t())
            if i < self.n_hidden:
                h = torch.relu(h)
        return h

    def generate_many(self, idxs) -> torch.Tensor:
        """Flat target weights [n, P] of several clients (one GEMM over the packed heads)."""
        return torch.addmm(self.b[None, :], self.features_many(idxs), self.W.t())

    def generate(self, idx: int) -> torch.Tensor:
        """Flat target weights [P] for client ``idx`` (one GEMV over the packed heads)."""
        _, feat, _ = self.features(idx)
        from .. import ops

        return ops.hyper_generate(self.W, self.b, feat)


class _FrozenTarget(nn.Module):
    """Parameter-free stand-in whose ``state_dict()`` reports the target shapes."""

    def __init__(self, sd):
        super().__init__()
        self._sd = sd

    def state_dict(self, *a, **k):  # noqa: D401
        return OrderedDict((kk, vv) for kk, vv in self._sd.items())


def _seeded_hnet(target_sd, n_nodes, E, H, n_hidden, gen: torch.Generator) -> HyperNetwork:
    """Build the reference module with a seeded default-init (nn.Linear kaiming-uniform)."""
    state = torch.random.get_rng_state()
    try:
        torch.manual_seed(int(torch.randint(0, 2 ** 31 - 1, (1,), generator=gen).item()))
        return HyperNetwork(_FrozenTarget(target_sd), n_nodes, E, H, False, n_hidden)
    finally:
        torch.random.set_rng_state(state)
