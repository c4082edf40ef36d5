"""Fused RNNModel/ICU local training (``csrc/kernels/rnn2.hip``, on-chip; ``rnn.hip`` as split 3): one
launch trains all of a rank's clients for all their local epochs, three co-resident workgroups per client
(head | vitals | labs).

Dropout masks follow the layer-program convention (``fl/programs.py``), so the composite
``RNNProgram`` on CPU is the exact-semantics oracle of this kernel (tests/test_gpu_rnn.py).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch

from . import native
from .masks import M32

NPARAM = 97665


def fits(C: int, dev) -> bool:
    """The on-chip trainer can train C clients: a launch's 3 workgroups per client must be resident at once
    (one per CU, next to the persistent launches of any other process sharing the GPU,
    ``parallel.launcher.gpu_sharers``); more clients than one launch holds run in back-to-back launches
    (``transformer.chunked``), so any C >= 1 fits once one client does."""
    from .transformer import onchip_capacity

    return C >= 0 and onchip_capacity(dev, 3) >= 1


def _seeds(seeds, dev) -> torch.Tensor:
    s = torch.tensor([int(x) & M32 for x in seeds], dtype=torch.int64)
    return torch.where(s >= 2 ** 31, s - 2 ** 32, s).to(torch.int32).to(dev)


def device_seed(s: int) -> int:
    """The int32 the kernel receives for client seed ``s`` (low 32 bits, two's complement)."""
    s = int(s) & M32
    return s - 2 ** 32 if s >= 2 ** 31 else s


def _on(t, dev) -> bool:
    return torch.is_tensor(t) and t.device == dev and t.dtype == torch.int32


def _dev_i32(nd, dev) -> torch.Tensor:
    """``nd`` as a device int32 tensor (passed through when the engine already staged it there)."""
    if _on(nd, dev):
        return nd
    return torch.as_tensor(list(nd) if not torch.is_tensor(nd) else nd.tolist(), dtype=torch.int32, device=dev)


def train_clients_async(params: torch.Tensor, rows: torch.Tensor, order: torch.Tensor, nd, epochs: int, batch: int,
                        lr: float, seeds: Sequence[int], opt_mode: int = 0, split: int = 4,
                        stamps: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Enqueue the launch; returns DEVICE (ok [C] int32, losses [C, E]) without synchronising.

    ``split`` 4 = the on-chip trainer (``rnn2.hip``: weights, optimizer state and activations in registers /
    LDS for the whole round), 3 = the global-workspace kernel (``rnn.hip``).  ``stamps``: device int64 [64]
    per-phase timers of workgroup ``stamps[63]`` (split 4 only; tools/phase_profile.py)."""
    from .transformer import adam_step_table

    dev = params.device
    nd_t = _dev_i32(nd, dev)
    seeds_t = seeds if _on(seeds, dev) else _seeds(seeds, dev)
    from .transformer import chunked, onchip_capacity

    kt = None
    if split == 4:
        kt = adam_step_table(float(lr), int(epochs) * -(-int(order.shape[2]) // int(batch)), dev)
    rows_c, order_c = rows.contiguous(), order.contiguous()

    def launch(p, o, n, s, first=True):
        return native().rnn_train(p, rows_c, o, n, s, int(epochs), int(batch), float(lr), int(opt_mode), int(split),
                                  kt, stamps if first else None)
    # (clients beyond one launch's co-residency budget: back-to-back launches; a stamped run stamps the first)
    return chunked(launch, params.shape[0], onchip_capacity(dev, 3), params, order_c, nd_t, seeds_t)


def train_clients(params: torch.Tensor, rows: torch.Tensor, order: torch.Tensor, nd, epochs: int, batch: int,
                  lr: float, seeds: Sequence[int], opt_mode: int = 0, split: int = 4,
                  stamps: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Train ``params [C, 97665]`` in place.  Returns (ok [C] int32, losses [C, E]) on the host."""
    from .transformer import finish

    return finish(*train_clients_async(params, rows, order, nd, epochs, batch, lr, seeds, opt_mode, split, stamps),
                  what="fused RNN trainer")


def eval_many(params: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """Sigmoid outputs of C RNNModels (``params [C, 97665]``, eval mode) over ``rows [n, 24]`` -> ``[C, n]``:
    one launch (``rnn2.hip`` ``k_rnn2_eval``)."""
    p = params if params.dim() == 2 else params[None]
    return native().rnn_eval_many(p.contiguous(), rows.contiguous())
