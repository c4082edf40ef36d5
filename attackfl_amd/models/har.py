"""HAR sequence classifier (x[B,1,561] -> 6 classes).

Composite form of reference ``src/Model.py:418-458`` (``PositionalEncoding`` with the
``pe`` buffer in the state_dict, max_len 600; ``TransformerClassifier`` with a Conv1d stem,
two post-norm ``nn.TransformerEncoderLayer`` (d 64, 4 heads, ff 256, ReLU, seq-first),
mean-pool and an MLP head).  The L=561 attention is the only real attention workload of the
testbed; the HIP flash-attention path lives in ``attackfl_amd/ops/attention.py``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

HAR_LEN = 561
HAR_CLASSES = 6
PE_MAX_LEN = 600


class PositionalEncoding(nn.Module):
    def __init__(self, d_model: int, max_len: int = PE_MAX_LEN):
        super().__init__()
        pos = torch.arange(max_len, dtype=torch.float32)[:, None]
        inv = torch.exp(torch.arange(0, d_model, 2, dtype=torch.float32) * (-math.log(10000.0) / d_model))
        table = torch.zeros(max_len, d_model)
        table[:, 0::2] = torch.sin(pos * inv)
        table[:, 1::2] = torch.cos(pos * inv)
        self.register_buffer("pe", table[None])  # [1, max_len, d_model]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.size(1) > self.pe.size(1):
            raise ValueError(f"sequence length {x.size(1)} exceeds the positional-encoding cap {self.pe.size(1)}")
        return x + self.pe[:, : x.size(1), :]


class TransformerClassifier(nn.Module):
    def __init__(self, d_model: int = 64, nhead: int = 4, num_layers: int = 2, num_classes: int = HAR_CLASSES):
        super().__init__()
        self.conv = nn.Conv1d(1, d_model, kernel_size=3, padding=1)
        self.pe = PositionalEncoding(d_model)
        layer = nn.TransformerEncoderLayer(d_model=d_model, nhead=nhead, dim_feedforward=256, dropout=0.1)
        self.transformer = nn.TransformerEncoder(layer, num_layers=num_layers, enable_nested_tensor=False)
        self.classifier = nn.Sequential(nn.Linear(d_model, 64), nn.ReLU(), nn.Dropout(0.3),
                                        nn.Linear(64, num_classes))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.conv(x).permute(0, 2, 1)          # [B, L, d]
        h = self.pe(h).permute(1, 0, 2)            # [L, B, d] (seq-first encoder)
        h = self.transformer(h).mean(dim=0)        # [B, d]
        return self.classifier(h)
