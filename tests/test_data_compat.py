"""Reference-data compatibility (reference ``src/Utils.py:13-27``, ``src/Model.py:9-24``,
``src/RpcClient.py:157-166``, ``src/Validation.py:32-37``): the reference ships its ICU sets as gzip
pickles of an ``ICUData`` object defined in ``src.Model`` / ``src.Utils`` (the blobs themselves are not
in the snapshot, ``.MISSING_LARGE_BLOBS``).  A helper process here defines a class of that module path
and shape, pickles instances of it at the reference's file locations (A-3: train set in the CWD, test
set under ``data/``), and the framework must

* load them through its restricted unpickler (``attackfl_amd.data.load_pickled_dataset``) with the same
  tensors,
* train and validate rounds on them (``data.synthetic: false`` — no silent synthetic fallback),
* refuse a pickle that names any other global (``os.system``) without running it.
"""
import gzip
import os
import pickle
import subprocess
import sys
import textwrap

import pytest
import torch

from attackfl_amd.config import from_dict
from attackfl_amd.data import ICUData, load_pickled_dataset
from attackfl_amd.fl.engine import FLEngine

REF_CLASS = textwrap.dedent('''
    import torch
    from torch.utils.data import Dataset


    class ICUData(Dataset):
        def __init__(self, dataframe, vitals_cols, labs_cols, label_col):
            self.vitals = torch.tensor(dataframe[vitals_cols].values, dtype=torch.float32)
            self.labs = torch.tensor(dataframe[labs_cols].values, dtype=torch.float32)
            self.labels = torch.tensor(dataframe[label_col].values, dtype=torch.float32)

        def __len__(self):
            return len(self.labels)

        def __getitem__(self, idx):
            return self.vitals[idx], self.labs[idx], self.labels[idx]
''')

MAKER = textwrap.dedent('''
    import gzip, os, pickle, sys
    import numpy as np, pandas as pd
    sys.path.insert(0, sys.argv[1])
    import src.Model, src.Utils

    def make(mod, n, seed, path):
        rs = np.random.RandomState(seed)
        cols = [f"v{i}" for i in range(7)] + [f"l{i}" for i in range(16)]
        df = pd.DataFrame(rs.normal(0, 1, (n, 23)).astype(np.float32), columns=cols)
        logit = df[cols[:7]].values.sum(1) - df[cols[7:]].values[:, :4].sum(1)
        df["y"] = (rs.uniform(0, 1, n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
        df.loc[rs.uniform(0, 1, n) < 0.05, "v3"] = -2.0
        d = mod.ICUData(df, cols[:7], cols[7:], "y")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with gzip.open(path, "wb") as fh:
            pickle.dump(d, fh)

    root = sys.argv[1]
    make(src.Utils, 3000, 1, os.path.join(root, "train_dataset.pkl.gz"))       # RpcClient.py:161 (CWD)
    make(src.Model, 800, 2, os.path.join(root, "data", "test_dataset.pkl.gz"))  # Validation.py:33
''')


@pytest.fixture(scope="module")
def ref_root(tmp_path_factory):
    root = tmp_path_factory.mktemp("refdata")
    (root / "src").mkdir()
    (root / "src" / "__init__.py").write_text("")
    (root / "src" / "Model.py").write_text(REF_CLASS)
    (root / "src" / "Utils.py").write_text(REF_CLASS)
    r = subprocess.run([sys.executable, "-c", MAKER, str(root)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return root


def test_reference_pickles_load(ref_root):
    tr = load_pickled_dataset(str(ref_root / "train_dataset.pkl.gz"))
    te = load_pickled_dataset(str(ref_root / "data" / "test_dataset.pkl.gz"))
    assert isinstance(tr, ICUData) and isinstance(te, ICUData)
    assert tr.vitals.shape == (3000, 7) and tr.labs.shape == (3000, 16) and tr.labels.shape == (3000,)
    assert te.vitals.dtype == torch.float32 and len(te) == 800
    assert bool((tr.vitals == -2.0).any())  # missing-value markers survive
    assert set(tr.labels.unique().tolist()) <= {0.0, 1.0}


def _cfg(root, out, device_trainer="eager"):
    return from_dict({
        "server": {"num-round": 2, "clients": 3, "mode": "fedavg", "model": "TransformerModel",
                   "data-distribution": {"num-data-range": [300, 400]}},
        "learning": {"epoch": 1, "batch-size": 64},
        "data": {"synthetic": False, "root": str(root)},
        "engine": {"checkpoint-dir": str(out), "trainer": device_trainer},
        "log_path": str(out),
    })


def test_rounds_train_on_reference_pickles(ref_root, tmp_path):
    eng = FLEngine(_cfg(ref_root, tmp_path), device="cpu", verbose=False)
    assert eng.train_table.n == 3000 and eng.validation.table.n == 800
    hist = eng.run()
    eng.close()
    assert [r["ok"] for r in hist] == [True, True]
    assert all(0.0 <= r["metric"] <= 1.0 for r in hist)


def test_missing_reference_pickle_is_an_error_not_synthetic(tmp_path):
    with pytest.raises(FileNotFoundError):
        FLEngine(_cfg(tmp_path / "empty", tmp_path), device="cpu", verbose=False)


class _Evil:
    def __init__(self, marker):
        self.marker = marker

    def __reduce__(self):
        return (os.system, (f"touch {self.marker}",))


def test_hostile_pickle_is_refused(tmp_path):
    marker = tmp_path / "pwned"
    path = tmp_path / "train_dataset.pkl.gz"
    with gzip.open(path, "wb") as fh:
        pickle.dump(_Evil(str(marker)), fh)
    with pytest.raises(pickle.UnpicklingError, match="refusing"):
        load_pickled_dataset(str(path))
    assert not marker.exists()


def test_hostile_global_inside_dataset_is_refused(tmp_path):
    """A dataset-shaped pickle that smuggles another global in an attribute is refused as a whole."""
    marker = tmp_path / "pwned2"
    d = ICUData(vitals=torch.zeros(2, 7), labs=torch.zeros(2, 16), labels=torch.zeros(2))
    d.extra = _Evil(str(marker))
    path = tmp_path / "x.pkl"
    path.write_bytes(pickle.dumps(d))
    with pytest.raises(pickle.UnpicklingError):
        load_pickled_dataset(str(path))
    assert not marker.exists()


@pytest.mark.gpu
def test_gpu_rounds_on_reference_pickles(gpu, ref_root, tmp_path):
    """The native path (fused trainer, device validation) on the reference-format data."""
    eng = FLEngine(_cfg(ref_root, tmp_path, "auto"), device="cuda", verbose=False)
    assert eng.trainer.kind == "fused"
    hist = eng.run()
    eng.close()
    assert [r["ok"] for r in hist] == [True, True]
    assert all(0.5 < r["metric"] <= 1.0 for r in hist)
