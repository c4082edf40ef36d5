"""ICU tabular models (vitals[7] + labs[16] -> mortality probability).

These ``nn.Module`` definitions are the *composite* (eager PyTorch) form: they define the
parameter names/shapes used by ``.pth`` checkpoints and serve as the CPU oracle for the fused
HIP training kernels in ``attackfl_amd/ops``.  Parameter names, shapes, initialisation and
forward semantics follow the reference:

* ``CNNModel``          — reference ``src/Model.py:27-88``
* ``RNNModel``          — reference ``src/Model.py:91-163`` (bi-GRU, PyTorch (r,z,n) gate order)
* ``TransformerBlock``  — reference ``src/Model.py:166-191``
* ``TransformerModel``  — reference ``src/Model.py:194-246`` (seq_len 1 attention, A-22)
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

VITALS_DIM = 7
LABS_DIM = 16
MASK_VALUE = -2.0


class CNNModel(nn.Module):
    """Two Conv1d towers (1->32->64->128, k=3, pad=1, ReLU) + AdaptiveAvgPool1d(4) + MLP head."""

    def __init__(self):
        super().__init__()
        for br in ("vitals", "labs"):
            setattr(self, f"{br}_conv1", nn.Conv1d(1, 32, kernel_size=3, padding=1))
            setattr(self, f"{br}_conv2", nn.Conv1d(32, 64, kernel_size=3, padding=1))
            setattr(self, f"{br}_conv3", nn.Conv1d(64, 128, kernel_size=3, padding=1))
            setattr(self, f"{br}_pool", nn.AdaptiveAvgPool1d(4))
            setattr(self, f"{br}_dropout", nn.Dropout(0.3))
        self.fc1 = nn.Linear(128 * 2 * 4, 128)
        self.fc2 = nn.Linear(128, 64)
        self.fc3 = nn.Linear(64, 32)
        self.output = nn.Linear(32, 1)

    def _tower(self, br: str, x: torch.Tensor) -> torch.Tensor:
        x = x.unsqueeze(1)
        x = F.relu(getattr(self, f"{br}_conv1")(x))
        x = F.relu(getattr(self, f"{br}_conv2")(x))
        x = F.relu(getattr(self, f"{br}_conv3")(x))
        x = getattr(self, f"{br}_pool")(x)
        x = x.reshape(x.shape[0], -1)
        return getattr(self, f"{br}_dropout")(x)

    def forward(self, vitals: torch.Tensor, labs: torch.Tensor) -> torch.Tensor:
        h = torch.cat([self._tower("vitals", vitals), self._tower("labs", labs)], dim=1)
        h = F.relu(self.fc1(h))
        h = F.relu(self.fc2(h))
        h = F.relu(self.fc3(h))
        return torch.sigmoid(self.output(h))


class RNNModel(nn.Module):
    """Three stacked bidirectional GRUs per branch, LayerNorm, dropout, MLP head."""

    def __init__(self, vitals_input_dim: int = VITALS_DIM, labs_input_dim: int = LABS_DIM, hidden_dim: int = 32,
                 dropout_rate: float = 0.3):
        super().__init__()
        self.mask_value = MASK_VALUE
        self.hidden_dim = hidden_dim
        for br, din in (("vitals", vitals_input_dim), ("labs", labs_input_dim)):
            setattr(self, f"{br}_gru1", nn.GRU(din, hidden_dim, batch_first=True, bidirectional=True))
            setattr(self, f"{br}_gru2", nn.GRU(2 * hidden_dim, hidden_dim, batch_first=True, bidirectional=True))
            setattr(self, f"{br}_gru3", nn.GRU(2 * hidden_dim, hidden_dim, batch_first=True, bidirectional=True))
            setattr(self, f"{br}_ln", nn.LayerNorm(2 * hidden_dim))
            setattr(self, f"{br}_dropout", nn.Dropout(dropout_rate))
        self.fc1 = nn.Linear(4 * hidden_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim // 2)
        self.output = nn.Linear(hidden_dim // 2, 1)

    def _branch(self, br: str, x: torch.Tensor) -> torch.Tensor:
        x = torch.where(x == self.mask_value, torch.zeros_like(x), x)
        if x.dim() == 2:
            x = x.unsqueeze(1)
        for i in (1, 2, 3):
            x, _ = getattr(self, f"{br}_gru{i}")(x)
        x = x[:, -1, :]
        x = getattr(self, f"{br}_ln")(x)
        return getattr(self, f"{br}_dropout")(x)

    def forward(self, vitals: torch.Tensor, labs: torch.Tensor) -> torch.Tensor:
        h = torch.cat([self._branch("vitals", vitals), self._branch("labs", labs)], dim=1)
        h = F.relu(self.fc1(h))
        h = F.relu(self.fc2(h))
        return torch.sigmoid(self.output(h))


class TransformerBlock(nn.Module):
    """Post-LN block: MHA + residual + LN, FFN(GELU) + residual + LN."""

    def __init__(self, input_dim: int, num_heads: int, ff_dim: int, dropout_rate: float = 0.1):
        super().__init__()
        self.attention = nn.MultiheadAttention(embed_dim=input_dim, num_heads=num_heads, dropout=dropout_rate,
                                               batch_first=True)
        self.attention_norm = nn.LayerNorm(input_dim)
        self.dropout1 = nn.Dropout(dropout_rate)
        self.ffn = nn.Sequential(nn.Linear(input_dim, ff_dim), nn.GELU(), nn.Dropout(dropout_rate),
                                 nn.Linear(ff_dim, input_dim))
        self.ffn_norm = nn.LayerNorm(input_dim)
        self.dropout2 = nn.Dropout(dropout_rate)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        a, _ = self.attention(x, x, x, need_weights=False)
        x = self.attention_norm(x + self.dropout1(a))
        return self.ffn_norm(x + self.dropout2(self.ffn(x)))


class _NoParamPool(nn.Sequential):
    """AdaptiveAvgPool1d(1) -> AdaptiveMaxPool1d(1); constructed but unused (reference A-22)."""

    def __init__(self):
        super().__init__(nn.AdaptiveAvgPool1d(1), nn.AdaptiveMaxPool1d(1))


class TransformerModel(nn.Module):
    """Two Linear->GELU->TransformerBlock(seq_len 1)->LayerNorm branches + GELU MLP head."""

    def __init__(self, vitals_input_dim: int = VITALS_DIM, labs_input_dim: int = LABS_DIM, num_heads: int = 4,
                 ff_dim: int = 6):
        super().__init__()
        for br, din in (("vitals", vitals_input_dim), ("labs", labs_input_dim)):
            setattr(self, f"{br}_dense", nn.Linear(din, 64))
            setattr(self, f"{br}_transformer", TransformerBlock(64, num_heads, ff_dim))
            setattr(self, f"{br}_pool", _NoParamPool())
            setattr(self, f"{br}_bn", nn.LayerNorm(64))
        self.fc1 = nn.Linear(128, 64)
        self.dropout = nn.Dropout(0.3)
        self.fc2 = nn.Linear(64, 32)
        self.output = nn.Linear(32, 1)

    def _branch(self, br: str, x: torch.Tensor) -> torch.Tensor:
        x = F.gelu(getattr(self, f"{br}_dense")(x)).unsqueeze(1)
        x = getattr(self, f"{br}_transformer")(x).squeeze(1)
        return getattr(self, f"{br}_bn")(x)

    def forward(self, vitals: torch.Tensor, labs: torch.Tensor) -> torch.Tensor:
        h = torch.cat([self._branch("vitals", vitals), self._branch("labs", labs)], dim=1)
        h = self.dropout(F.gelu(self.fc1(h)))
        h = F.gelu(self.fc2(h))
        return torch.sigmoid(self.output(h))
