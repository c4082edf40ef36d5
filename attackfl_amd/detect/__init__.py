"""Hypernetwork embedding anomaly detection (reference ``server.py:496-536``,
helpers ``src/Utils.py:391-436``).

A client is removed only if BOTH tests flag it (from round 18 on):
* ``cosine_anomaly`` — current embedding's cosine to the mean of the normalised history falls
  below mu - 2 sigma of the history's own cosines;
* ``dbscan_outliers`` — DBSCAN on the PCA(n_components) projection of embedding deltas r-1 -> r.
Both run on the host over <= N x 8 numbers; the embeddings are read from the packed hypernet.
The per-client history deque has maxlen 5 (reference hard-codes it; ``cosine-search`` is
ignored, A-12).
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Sequence

import numpy as np

from ..utils.log import print_with_color

HISTORY_LEN = 5
START_ROUND = 18


def _quiet(*_a, **_k):
    return None


def cosine_anomaly(previous: np.ndarray, current: np.ndarray, log=print_with_color) -> bool:
    hist = np.asarray(previous, dtype=np.float64)
    if hist.size == 0:
        return False
    hist_n = hist / np.linalg.norm(hist, axis=1, keepdims=True)
    cur = current / np.linalg.norm(current, axis=1, keepdims=True)
    mean_n = hist_n.mean(axis=0)
    cs = float(np.dot(cur, mean_n).reshape(-1)[0] / (np.linalg.norm(cur) * np.linalg.norm(mean_n)))
    hist_cs = np.sum(hist * mean_n, axis=1) / (np.linalg.norm(hist, axis=1) * np.linalg.norm(mean_n))
    mu = float(np.mean(hist_cs))
    sigma = max(float(np.std(hist_cs)), 1e-6)
    flag = cs < mu - 2 * sigma
    if flag:
        log("Anomalies detection !!!", "yellow")
    return bool(flag)


def dbscan_outliers(before: Sequence[np.ndarray], after: Sequence[np.ndarray], selected: Sequence[int],
                    n_components: int = 3, eps: float = 0.008, min_samples: int = 3, log=print_with_color) -> List[int]:
    from sklearn.cluster import DBSCAN
    from sklearn.decomposition import PCA

    a = np.array([after[c] for c in selected])
    b = np.array([before[c] for c in selected])
    delta = (a - b).reshape(len(selected), -1)
    k = min(n_components, delta.shape[0], delta.shape[1])
    proj = PCA(n_components=k).fit_transform(delta)
    labels = DBSCAN(eps=eps, min_samples=min_samples).fit(proj).labels_
    out = [selected[i] for i in np.where(labels == -1)[0]]
    log(f"DBSCAN outliers: {out}", "yellow")
    return out


class HyperDetector:
    def __init__(self, n_clients: int, n_components: int = 3, eps: float = 0.007, min_samples: int = 3,
                 save_path: str = "all_embeddings.npy", verbose: bool = True):
        self.hist: List[deque] = [deque(maxlen=HISTORY_LEN) for _ in range(n_clients)]
        self.n_components = n_components
        self.eps = eps
        self.min_samples = min_samples
        self.save_path = save_path
        self.log = print_with_color if verbose else _quiet

    def step(self, round_no: int, selected: Sequence[int], embeddings: Dict[int, np.ndarray]) -> List[int]:
        """Feed this round's embeddings ([1, E] each); return the clients to remove."""
        flagged = []
        for i in selected:
            cur = np.asarray(embeddings[i], dtype=np.float32).reshape(1, -1)
            prev = np.vstack(self.hist[i]) if self.hist[i] else np.empty((0, cur.shape[1]))
            if round_no >= START_ROUND and cosine_anomaly(prev, cur, self.log):
                flagged.append(i)
            self.hist[i].append(cur)
        if self.save_path:
            arr = np.empty(len(self.hist), dtype=object)
            for j, dq in enumerate(self.hist):
                arr[j] = list(dq)
            np.save(self.save_path, arr, allow_pickle=True)
        if round_no < START_ROUND:
            return []
        outs = dbscan_outliers([h[-2] for h in self.hist], [h[-1] for h in self.hist], list(selected),
                               self.n_components, self.eps, self.min_samples, self.log)
        return sorted(set(flagged) & set(outs))
