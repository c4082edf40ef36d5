"""Model registry and the flat parameter layout.

Models are selected by class-name string exactly like the reference
(``getattr(src.Model, name)()``, ``server.py:139-140``, ``src/RpcClient.py:74-75``).

Every model update in this framework travels and is aggregated as ONE flat fp32 row of
length ``P`` (state_dict order).  ``ParamLayout`` maps that row back to named tensors so that
per-tensor semantics (reference ``compute_distance``'s per-key spectral norms, ``.pth`` export)
are preserved while all bulk math runs on contiguous ``[N, P]`` matrices.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from .har import HAR_CLASSES, HAR_LEN, PositionalEncoding, TransformerClassifier
from .hyper import CNNHyper, HyperNetwork, PackedHyperNet
from .icu import CNNModel, RNNModel, TransformerBlock, TransformerModel

MODEL_REGISTRY = {
    "CNNModel": CNNModel,
    "RNNModel": RNNModel,
    "TransformerModel": TransformerModel,
    "TransformerClassifier": TransformerClassifier,
}


def build_model(name: str, seed: Optional[int] = None) -> nn.Module:
    if name not in MODEL_REGISTRY:
        raise ValueError(f"Model name '{name}' is not valid.")
    if seed is None:
        return MODEL_REGISTRY[name]()
    state = torch.random.get_rng_state()
    try:
        torch.manual_seed(int(seed))
        return MODEL_REGISTRY[name]()
    finally:
        torch.random.set_rng_state(state)


@dataclass(frozen=True)
class TensorSlot:
    name: str
    shape: Tuple[int, ...]
    offset: int
    numel: int
    is_long: bool = False


class ParamLayout:
    """Ordered (name, shape, offset) table for a model's state_dict."""

    def __init__(self, slots: List[TensorSlot]):
        self.slots = slots
        self.P = sum(s.numel for s in slots)
        self.index = {s.name: i for i, s in enumerate(slots)}

    @classmethod
    def from_state_dict(cls, sd: "OrderedDict[str, torch.Tensor]") -> "ParamLayout":
        slots = []
        off = 0
        for k, v in sd.items():
            n = v.numel()
            slots.append(TensorSlot(k, tuple(v.shape), off, n, v.dtype in (torch.long, torch.int64, torch.int32)))
            off += n
        return cls(slots)

    @classmethod
    def for_model(cls, name: str) -> "ParamLayout":
        return cls.from_state_dict(build_model(name, seed=0).state_dict())

    def __len__(self) -> int:
        return len(self.slots)

    def keys(self) -> List[str]:
        return [s.name for s in self.slots]

    def flatten(self, sd: Dict[str, torch.Tensor], device=None, dtype=torch.float32) -> torch.Tensor:
        dev = device if device is not None else next(iter(sd.values())).device
        out = torch.empty(self.P, dtype=dtype, device=dev)
        for s in self.slots:
            out[s.offset:s.offset + s.numel].copy_(sd[s.name].reshape(-1))
        return out

    def unflatten(self, flat: torch.Tensor, clone: bool = True) -> "OrderedDict[str, torch.Tensor]":
        """Flat row -> state_dict.  ``clone=False`` returns views (zero-copy)."""
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for s in self.slots:
            t = flat[s.offset:s.offset + s.numel].view(s.shape)
            if s.is_long:
                t = t.round().long()
            elif clone:
                t = t.clone()
            sd[s.name] = t
        return sd

    def matrix_slots(self) -> List[TensorSlot]:
        return [s for s in self.slots if len(s.shape) == 2]

    def vector_slots(self) -> List[TensorSlot]:
        return [s for s in self.slots if len(s.shape) == 1]

    def higher_slots(self) -> List[TensorSlot]:
        return [s for s in self.slots if len(s.shape) >= 3]


def model_layout(name: str) -> ParamLayout:
    return ParamLayout.for_model(name)


__all__ = [
    "CNNModel", "RNNModel", "TransformerBlock", "TransformerModel", "TransformerClassifier", "PositionalEncoding",
    "HyperNetwork", "CNNHyper", "PackedHyperNet", "MODEL_REGISTRY", "build_model", "ParamLayout", "TensorSlot",
    "model_layout", "HAR_LEN", "HAR_CLASSES",
]
