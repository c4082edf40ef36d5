"""Datasets: ICU tabular rows and HAR sequences.

* ``ICUData`` — same attributes as the reference dataset class (reference ``src/Model.py:9-24``,
  duplicate ``src/Utils.py:13-27``): float32 ``vitals [N,7]``, ``labs [N,16]``, ``labels [N]``.
* ``load_pickled_dataset`` — reads the reference's gzip-pickled datasets through a
  *restricted* unpickler (only dataset classes, numpy/pandas-free tensor rebuilds; torch
  storages are decoded with ``torch.load(weights_only=True)``).  Nothing from the file can run
  arbitrary code.
* ``synthetic_icu`` / ``synthetic_har`` — deterministic synthetic data with a planted signal
  (the reference's pickles are not shipped: ``.MISSING_LARGE_BLOBS``), including ``-2.0``
  missing-value markers that ``RNNModel`` masks.
* ``ImageData`` / ``load_cifar10_bin`` / ``synthetic_cifar10`` — the reference's CIFAR10 test path
  (``src/Validation.py:38-44``: ``ToTensor`` + ``Normalize(0.5, 0.5)``) read from the raw-byte
  ``cifar-10-batches-bin`` layout (no pickles, no download), or synthetic images of that shape.
* ``DeviceTable`` — the whole train set resident on device as one ``[N, 24]`` fp32 row table
  (vitals | labs | label), from which fused trainers gather batches by index.
"""
from __future__ import annotations

import gzip
import io
import os
import pickle
from typing import Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset, TensorDataset

from ..utils.log import print_with_color

VITALS_DIM = 7
LABS_DIM = 16
ROW_DIM = VITALS_DIM + LABS_DIM + 1


class ICUData(Dataset):
    """ICU rows: (vitals[7], labs[16], label) float32 triples."""

    def __init__(self, dataframe=None, vitals_cols=None, labs_cols=None, label_col=None, *, vitals=None, labs=None,
                 labels=None):
        if dataframe is not None:
            vitals = dataframe[vitals_cols].values
            labs = dataframe[labs_cols].values
            labels = dataframe[label_col].values
        self.vitals = torch.as_tensor(np.asarray(vitals), dtype=torch.float32)
        self.labs = torch.as_tensor(np.asarray(labs), dtype=torch.float32)
        self.labels = torch.as_tensor(np.asarray(labels), dtype=torch.float32)

    def __len__(self) -> int:
        return len(self.labels)

    def __getitem__(self, idx):
        return self.vitals[idx], self.labs[idx], self.labels[idx]


class HARData(Dataset):
    """HAR rows: (x[1, 561], y) with integer class labels 0..5."""

    def __init__(self, x, y):
        self.x = torch.as_tensor(x, dtype=torch.float32)
        if self.x.dim() == 2:
            self.x = self.x[:, None, :]
        self.y = torch.as_tensor(y, dtype=torch.long)

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, idx):
        return self.x[idx], self.y[idx]


# ----------------------------------------------------------------------------------------------
# restricted unpickler for the reference pickles
# ----------------------------------------------------------------------------------------------

def _load_storage_bytes(b: bytes):
    return torch.load(io.BytesIO(b), weights_only=True)


_ALLOWED = {
    ("src.Model", "ICUData"): ICUData,
    ("src.Utils", "ICUData"): ICUData,
    ("__main__", "ICUData"): ICUData,
    ("attackfl_amd.data", "ICUData"): ICUData,
    ("torch.utils.data.dataset", "TensorDataset"): TensorDataset,
    ("torch.utils.data.dataset", "Subset"): torch.utils.data.Subset,
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch._utils", "_rebuild_parameter"): torch._utils._rebuild_parameter,
    ("torch.storage", "_load_from_bytes"): _load_storage_bytes,
    ("collections", "OrderedDict"): __import__("collections").OrderedDict,
    ("torch", "FloatStorage"): torch.FloatStorage,
    ("torch", "LongStorage"): torch.LongStorage,
    ("torch", "IntStorage"): torch.IntStorage,
    ("torch", "DoubleStorage"): torch.DoubleStorage,
    ("torch", "float32"): torch.float32,
    ("torch", "int64"): torch.int64,
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        key = (module, name)
        if key in _ALLOWED:
            return _ALLOWED[key]
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a dataset pickle")


def load_pickled_dataset(path: str):
    """Load a (gzip) pickled dataset with the restricted unpickler above."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        obj = _SafeUnpickler(fh).load()
    if isinstance(obj, ICUData) and not isinstance(obj.vitals, torch.Tensor):
        obj = ICUData(vitals=obj.vitals, labs=obj.labs, labels=obj.labels)
    return obj


# ----------------------------------------------------------------------------------------------
# synthetic data with a planted signal
# ----------------------------------------------------------------------------------------------

def _icu_generator(seed: int):
    rs = np.random.RandomState(seed)
    w_v = rs.normal(0, 1.0, VITALS_DIM)
    w_l = rs.normal(0, 0.7, LABS_DIM)
    w_q = rs.normal(0, 0.4, 4)
    return w_v, w_l, w_q


def synthetic_icu(n: int, seed: int = 1234, split_seed: int = 0, missing_rate: float = 0.05) -> ICUData:
    """Deterministic ICU-shaped rows.  ``seed`` fixes the ground-truth model, ``split_seed`` the rows."""
    w_v, w_l, w_q = _icu_generator(seed)
    rs = np.random.RandomState(seed * 7919 + split_seed + 1)
    vit = rs.normal(0, 1, (n, VITALS_DIM)).astype(np.float32)
    lab = rs.normal(0, 1, (n, LABS_DIM)).astype(np.float32)
    logit = vit @ w_v + lab @ w_l + w_q[0] * vit[:, 0] * lab[:, 0] + w_q[1] * np.tanh(vit[:, 1] * 2) \
        + w_q[2] * lab[:, 3] ** 2 - 1.0
    p = 1.0 / (1.0 + np.exp(-logit))
    y = (rs.uniform(0, 1, n) < p).astype(np.float32)
    # missing values are recorded as -2.0 (RNNModel masks them)
    if missing_rate > 0:
        vit[rs.uniform(0, 1, vit.shape) < missing_rate] = -2.0
        lab[rs.uniform(0, 1, lab.shape) < missing_rate] = -2.0
    return ICUData(vitals=vit, labs=lab, labels=y)


def synthetic_har(n: int, seed: int = 1234, split_seed: int = 0, length: int = 561, classes: int = 6) -> HARData:
    rs = np.random.RandomState(seed)
    protos = rs.normal(0, 1, (classes, length)).astype(np.float32)
    rs2 = np.random.RandomState(seed * 31 + split_seed + 7)
    y = rs2.randint(0, classes, n)
    x = protos[y] * 0.5 + rs2.normal(0, 1, (n, length)).astype(np.float32)
    return HARData(x, y)


class ImageData(Dataset):
    """``x [N, 3, 32, 32]`` fp32 (already normalised to [-1, 1]), ``y [N]`` int64 class labels."""

    def __init__(self, x, y):
        self.x = torch.as_tensor(x, dtype=torch.float32)
        self.y = torch.as_tensor(y, dtype=torch.long)

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]


CIFAR_FILES = {"train": [f"data_batch_{i}.bin" for i in range(1, 6)], "test": ["test_batch.bin"]}


def load_cifar10_bin(root: str, split: str = "test") -> ImageData:
    """CIFAR-10 binary batches: records of 1 label byte + 3072 pixel bytes (R, G, B planes, 32x32).

    Pixels map through ``ToTensor`` (/255) then ``Normalize((0.5,)*3, (0.5,)*3)`` exactly like the
    reference's ``transform_test`` (``src/Validation.py:39-42``).
    """
    recs = []
    for name in CIFAR_FILES[split]:
        raw = np.fromfile(os.path.join(root, name), dtype=np.uint8)
        if raw.size % 3073:
            raise ValueError(f"{name}: size {raw.size} is not a multiple of the 3073-byte CIFAR record")
        recs.append(raw.reshape(-1, 3073))
    r = np.concatenate(recs, 0)
    x = (r[:, 1:].reshape(-1, 3, 32, 32).astype(np.float32) / 255.0 - 0.5) / 0.5
    return ImageData(x, r[:, 0].astype(np.int64))


def synthetic_cifar10(n: int, seed: int = 1234, split_seed: int = 0, classes: int = 10) -> ImageData:
    rs = np.random.RandomState(seed)
    protos = rs.uniform(-1, 1, (classes, 3, 32, 32)).astype(np.float32)
    rs2 = np.random.RandomState(seed * 31 + split_seed + 11)
    y = rs2.randint(0, classes, n)
    x = np.clip(protos[y] * 0.6 + rs2.normal(0, 0.4, (n, 3, 32, 32)).astype(np.float32), -1, 1)
    return ImageData(x, y)


# ----------------------------------------------------------------------------------------------
# dataset resolution (reference file locations, or synthetic)
# ----------------------------------------------------------------------------------------------

REF_PATHS = {
    # reference client/server read these (A-3: train in CWD, test under data/)
    ("ICU", "train"): ["train_dataset.pkl.gz", "data/train_dataset.pkl.gz"],
    ("ICU", "test"): ["data/test_dataset.pkl.gz", "test_dataset.pkl.gz"],
    ("HAR", "train"): ["data/icu_har_train_ds.pkl.gz"],
    ("HAR", "test"): ["data/icu_har_test_ds.pkl.gz"],
}


def resolve_dataset(data_name: str, split: str, data_cfg: Optional[dict] = None, verbose: bool = True):
    cfg = dict(data_cfg or {})
    mode = str(cfg.get("synthetic", "auto")).lower()
    root = cfg.get("root", ".")
    if mode in ("auto", "false", "0", "no"):
        for rel in REF_PATHS.get((data_name, split), []):
            p = os.path.join(root, rel)
            if os.path.exists(p):
                if verbose:
                    print_with_color(f"Loading {data_name}/{split} from {p}", "green")
                return load_pickled_dataset(p)
        if mode in ("false", "0", "no") and (data_name, split) in REF_PATHS:
            raise FileNotFoundError(f"no {data_name}/{split} pickle under {root} and data.synthetic is false")
    if data_name == "CIFAR10" and mode in ("auto", "false", "0", "no"):
        d = os.path.join(root, "data", "cifar-10-batches-bin")
        if all(os.path.exists(os.path.join(d, f)) for f in CIFAR_FILES[split]):
            if verbose:
                print_with_color(f"Loading CIFAR10/{split} from {d}", "green")
            return load_cifar10_bin(d, split)
        if mode in ("false", "0", "no"):
            raise FileNotFoundError(f"no CIFAR10 binary batches under {d} and data.synthetic is false")
    seed = int(cfg.get("seed", 1234))
    split_seed = 0 if split == "train" else 1
    if data_name == "ICU":
        n = int(cfg.get("train-size" if split == "train" else "test-size", 60000 if split == "train" else 10000))
        return synthetic_icu(n, seed=seed, split_seed=split_seed)
    if data_name == "HAR":
        n = int(cfg.get("har-train-size" if split == "train" else "har-test-size", 2048 if split == "train" else 512))
        return synthetic_har(n, seed=seed, split_seed=split_seed)
    if data_name == "CIFAR10":
        n = int(cfg.get("cifar-train-size" if split == "train" else "cifar-test-size", 2048 if split == "train" else 512))
        return synthetic_cifar10(n, seed=seed, split_seed=split_seed)
    raise ValueError(f"Data name '{data_name}' is not valid.")


class DeviceTable:
    """Dataset resident on one device as a single row table.

    ICU: ``rows [N, 24]`` = vitals(7) | labs(16) | label(1); HAR: ``x [N, 561]``, ``y [N]``.
    """

    def __init__(self, ds, device):
        self.device = torch.device(device)
        if isinstance(ds, ICUData):
            self.kind = "ICU"
            self.rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], dim=1).contiguous().to(self.device)
            self.n = self.rows.shape[0]
        elif isinstance(ds, HARData):
            self.kind = "HAR"
            self.x = ds.x.reshape(len(ds), -1).contiguous().to(self.device)
            self.y = ds.y.to(self.device)
            self.n = self.x.shape[0]
        elif isinstance(ds, ImageData):
            self.kind = "IMAGE"
            self.x = ds.x.contiguous().to(self.device)
            self.y = ds.y.to(self.device)
            self.n = self.x.shape[0]
        elif isinstance(ds, TensorDataset):
            self.kind = "HAR"
            x, y = ds.tensors[0], ds.tensors[1]
            self.x = x.reshape(len(x), -1).float().contiguous().to(self.device)
            self.y = y.long().to(self.device)
            self.n = self.x.shape[0]
        else:
            raise TypeError(f"unsupported dataset type {type(ds)}")

    def icu_batch(self, idx: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        r = self.rows.index_select(0, idx)
        return r[:, :VITALS_DIM], r[:, VITALS_DIM:VITALS_DIM + LABS_DIM], r[:, -1]

    def image_batch(self, idx: torch.Tensor):
        return self.x.index_select(0, idx), self.y.index_select(0, idx)

    def har_batch(self, idx: torch.Tensor):
        return self.x.index_select(0, idx)[:, None, :], self.y.index_select(0, idx)
