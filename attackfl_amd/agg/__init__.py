"""Server aggregation rules / robust defenses on the gathered update matrix ``U [N, P]``.

Each rule returns ``AggResult(params [P] | None, ok, info)``.  Rows are in client-index order;
``sizes [N]`` are the clients' reported sample counts; ``attackers [N]`` the oracle attacker flags
(only GMM uses them, as the reference does).  Reference sites:

* fedavg        ``server.py:751-775``      size-weighted mean (fp64 accumulation)
* trimmed_mean  ``src/Utils.py:267-302``   coordinate-wise, trim int(0.1·N) per side
* median        ``src/Utils.py:344-357``   coordinate-wise lower median (``torch.median``)
* krum          ``server.py:373-389``, ``src/Utils.py:326-342``  f = int(N·0.0) (A-11)
* shieldfl      ``server.py:306-350``      cosine-to-mean inverse-deviation weights
* gmm           ``server.py:352-372``, ``src/Utils.py:250-323``  (crashes in the reference, A-8;
  here: 2-component GMM in the rank-(N-1) principal subspace = low-rank Mahalanobis)
* scionfl       ``server.py:436-492``, ``src/Utils.py:371-387``  1-bit stochastic quantisation +
  norm clip + cosine filter + FedAvg of the kept originals
* fltracer      ``src/Utils.py:359-369`` (dormant in the reference)  PCA(1) + MAD z-score
* byzantine     ``src/Utils.py:218-248`` (dead code in the reference) cosine ≥ 0.9 to model 0
FLTrust and the hypernetwork live in ``fl/server.py`` (they need training).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import math

import numpy as np
import torch

from .. import ops


@dataclass
class AggResult:
    params: Optional[torch.Tensor]
    ok: bool = True
    info: Dict = field(default_factory=dict)


def fedavg(U: torch.Tensor, sizes: torch.Tensor, **_) -> AggResult:
    if U.shape[0] == 0:
        return AggResult(None, True, {"n": 0})
    return AggResult(ops.fedavg(U, sizes), True, {"n": int(U.shape[0])})


def mean_of(U: torch.Tensor) -> torch.Tensor:
    w = torch.full((U.shape[0],), 1.0 / U.shape[0], dtype=torch.float64, device=U.device)
    return ops.weighted_rows(U, w)


def host_info(info: Dict) -> Dict:
    """An aggregator's info with device values read back (the engine calls it where the host waits anyway,
    after validation): bool masks become index lists, 0-d tensors numbers, vectors lists."""
    out = {}
    for k, v in info.items():
        if torch.is_tensor(v):
            v = v.cpu()
            if v.dtype == torch.bool:
                v = torch.nonzero(v).reshape(-1).tolist() if v.dim() else bool(v)
            elif v.dim() == 0:
                v = int(v) if not v.is_floating_point() else float(v)
            else:
                v = v.tolist()
        out[k] = v
    return out


def _device_weights(sizes: torch.Tensor, device) -> torch.Tensor:
    """Host sizes -> a device fp64 vector without a synchronising pageable copy."""
    s = sizes.to(torch.float64)
    if torch.device(device).type == "cuda" and s.device.type == "cpu":
        s = s.pin_memory().to(device, non_blocking=True)
    return s.to(device)


def _masked_mean(U: torch.Tensor, keep: torch.Tensor, w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weighted mean over the rows where ``keep`` (all rows when none is kept), on the device."""
    keep = torch.where(keep.any(), keep, torch.ones_like(keep))
    w = keep.double() if w is None else keep.double() * w
    return ops.weighted_rows(U, w / w.sum())


def trimmed_mean(U: torch.Tensor, sizes=None, trim_ratio: float = 0.1, **_) -> AggResult:
    n = U.shape[0]
    k = int(n * trim_ratio)
    if 2 * k >= n:
        raise ValueError("Too few clients for the chosen trim_ratio.")
    return AggResult(ops.trimmed_mean(U, k), True, {"trim_k": k})


def median(U: torch.Tensor, sizes=None, **_) -> AggResult:
    return AggResult(ops.coord_median(U), True, {})


def krum(U: torch.Tensor, sizes=None, f_rate: float = 0.0, **_) -> AggResult:
    """Krum without a host read: fp64 Gram distances, each row's own distance pushed to +inf, a row sort,
    the n-f-2 smallest summed and the argmin (first minimum, like ``np.argmin``) selected on the device."""
    n = U.shape[0]
    f = int(n * f_rate)
    m = max(n - f - 2, 0)
    d2 = ops.pairwise_sqdist(U).double()
    d2 = d2 + torch.diag(torch.full((n,), float("inf"), dtype=torch.float64, device=d2.device))
    scores = torch.sort(d2, dim=1).values[:, :m].sum(dim=1)
    sel = torch.argmin(scores)
    return AggResult(U.index_select(0, sel.reshape(1))[0], True, {"selected": sel, "f": f, "scores": scores})


def shieldfl(U: torch.Tensor, sizes=None, **_) -> AggResult:
    norms = ops.row_norms(U).to(U.device)
    Un = U / (norms.to(U.dtype)[:, None] + 1e-8)
    ref = mean_of(Un)
    cos = ops.cosine_to(Un, ref, eps=1e-8).float()
    dev = 1.0 - cos
    w = 1.0 / (dev + 1e-6)
    w = w / w.sum()
    return AggResult(ops.weighted_rows(U, w.double()), True, {"weights": w, "cos": cos})


def _centred_gram(U: torch.Tensor) -> torch.Tensor:
    """n x n Gram of the rows centred on their mean (fp64).  On the device: the fp64-MFMA Gram pass of
    ``agg.hip`` (rows centred on row 0, then double-centred) instead of a generic fp64 GEMM with M = N = n and
    K = P (~50 k), a shape the library GEMM handles poorly."""
    if U.is_cuda and 1 <= U.shape[0] <= 64:
        return ops.native().gram_centred(U.to(torch.float32).contiguous())[0]
    X = U.double()
    Xc = X - X.mean(dim=0, keepdim=True)
    return Xc @ Xc.t()


def _gmm_chol(S, r):
    Lc = np.zeros((4, 4))
    for i in range(r):
        for j in range(i + 1):
            s = S[i][j]
            for k in range(j):
                s -= Lc[i][k] * Lc[j][k]
            if i == j:
                if not s > 0.0:
                    return None
                Lc[i][i] = math.sqrt(s)
            else:
                Lc[i][j] = s / Lc[j][j]
    return Lc


def _gmm_md2(Lc, r, x, mu):
    y = [0.0] * r
    s = 0.0
    for i in range(r):
        v = x[i] - mu[i]
        for k in range(i):
            v -= Lc[i][k] * y[k]
        y[i] = v / Lc[i][i]
        s += y[i] * y[i]
    return s


def gmm_filter_ref(G: np.ndarray, att: np.ndarray, rank: Optional[int] = None):
    """Host mirror of ``agg.hip`` ``k_gmm_filter`` (same algorithm and operation order, fp64): returns
    (keep [n] bool, threshold, kept, ok).  See the kernel for the algorithm and its reference mapping.
    ``rank`` > 0 sets the PCA rank r = min(rank, 4, n); None / 0: r = max(1, min(4, n // 2 - 1)) (the
    sensitivity study: profiles/gmm_rank_study_r6.md)."""
    n = G.shape[0]
    A = [list(map(float, row)) for row in G]
    V = [[1.0 if i == j else 0.0 for j in range(n)] for i in range(n)]
    for _ in range(12):
        for p in range(n - 1):
            for q in range(p + 1, n):
                apq = A[p][q]
                if abs(apq) < 1e-300:
                    continue
                th = (A[q][q] - A[p][p]) / (2.0 * apq)
                t = (1.0 if th >= 0.0 else -1.0) / (abs(th) + math.sqrt(th * th + 1.0))
                c = 1.0 / math.sqrt(t * t + 1.0)
                sn = t * c
                for k in range(n):
                    akp, akq = A[k][p], A[k][q]
                    A[k][p] = c * akp - sn * akq
                    A[k][q] = sn * akp + c * akq
                for k in range(n):
                    apk, aqk = A[p][k], A[q][k]
                    A[p][k] = c * apk - sn * aqk
                    A[q][k] = sn * apk + c * aqk
                for k in range(n):
                    vkp, vkq = V[k][p], V[k][q]
                    V[k][p] = c * vkp - sn * vkq
                    V[k][q] = sn * vkp + c * vkq
    order = sorted(range(n), key=lambda i: -A[i][i])  # stable: ties keep index order (as the insertion sort)
    ev = [A[i][i] for i in order]
    r = min(int(rank), 4, n) if rank else max(1, min(4, n // 2 - 1))
    Z = [[V[i][order[k]] * math.sqrt(max(ev[k], 1e-30)) for k in range(r)] for i in range(n)]
    zmax = max(1e-30, max(abs(z) for row in Z for z in row))
    Z = [[z / zmax for z in row] for row in Z]
    idx = [i for i in range(n) if not att[i]]
    nb = len(idx)
    idx += [i for i in range(n) if att[i]]
    X = [Z[i] for i in idx]
    m = len(X)
    K = 2 if m >= 2 else 1
    mu = [list(X[0]), list(X[0])]
    resp = [[1.0, 0.0] for _ in range(m)]
    if K == 2:
        far, best = 0, -1.0
        for i in range(m):
            d = sum((X[i][k] - X[0][k]) * (X[i][k] - X[0][k]) for k in range(r))
            if d > best:
                best, far = d, i
        mu[1] = list(X[far])
        for _ in range(10):
            s = [[0.0] * r, [0.0] * r]
            cnt = [0.0, 0.0]
            for i in range(m):
                d0 = d1 = 0.0
                for k in range(r):
                    d0 += (X[i][k] - mu[0][k]) * (X[i][k] - mu[0][k])
                    d1 += (X[i][k] - mu[1][k]) * (X[i][k] - mu[1][k])
                lab = 1 if d1 < d0 else 0
                resp[i] = [1.0 if lab == 0 else 0.0, 1.0 if lab == 1 else 0.0]
                cnt[lab] += 1.0
                for k in range(r):
                    s[lab][k] += X[i][k]
            for cc in range(2):
                if cnt[cc] > 0.0:
                    mu[cc] = [s[cc][k] / cnt[cc] for k in range(r)]
    eps10, reg, LOG2PI = 10.0 * 2.220446049250313e-16, 1e-6, 1.8378770664093453
    st = {"w": [0.0, 0.0], "Lc": [None, None], "logdet": [0.0, 0.0], "ok": True}

    def mstep():
        nks = 0.0
        for cc in range(K):
            nk = eps10
            for i in range(m):
                nk += resp[i][cc]
            for k in range(r):
                sm = 0.0
                for i in range(m):
                    sm += resp[i][cc] * X[i][k]
                mu[cc][k] = sm / nk
            cov = [[0.0] * 4 for _ in range(4)]
            for a_ in range(r):
                for b_ in range(r):
                    sm = 0.0
                    for i in range(m):
                        sm += resp[i][cc] * (X[i][a_] - mu[cc][a_]) * (X[i][b_] - mu[cc][b_])
                    cov[a_][b_] = sm / nk + (reg if a_ == b_ else 0.0)
            st["w"][cc] = nk
            nks += nk
            Lc = _gmm_chol(cov, r)
            if Lc is None:
                st["ok"] = False
                Lc = np.eye(4)
            st["Lc"][cc] = Lc
            st["logdet"][cc] = 2.0 * sum(math.log(Lc[k][k]) for k in range(r))
        for cc in range(K):
            st["w"][cc] /= nks

    def wlogp(x, cc):
        return math.log(st["w"][cc]) - 0.5 * (r * LOG2PI + _gmm_md2(st["Lc"][cc], r, x, mu[cc]) + st["logdet"][cc])

    mstep()
    lb = -math.inf
    it = 0
    while it < 100 and st["ok"]:
        prev = lb
        tot = 0.0
        for i in range(m):
            lp = [wlogp(X[i], 0), wlogp(X[i], 1) if K == 2 else -math.inf]
            mx = max(lp)
            lse = mx + math.log(math.exp(lp[0] - mx) + math.exp(lp[1] - mx))
            tot += lse
            resp[i] = [math.exp(lp[0] - lse), math.exp(lp[1] - lse) if K == 2 else 0.0]
        mstep()
        lb = tot / m
        it += 1
        if abs(lb - prev) < 1e-3:
            break
    mds = [math.sqrt(_gmm_md2(st["Lc"][0], r, X[i], mu[0])) for i in range(nb)]
    if nb:
        mb = sum(mds) / nb
        thr = 3.0 * math.sqrt(sum((d - mb) ** 2 for d in mds) / nb)
    else:
        thr = math.inf
    keep = np.zeros(n, dtype=bool)
    for i in range(n):
        cc = 1 if (K == 2 and wlogp(Z[i], 1) > wlogp(Z[i], 0)) else 0
        keep[i] = st["ok"] and math.sqrt(_gmm_md2(st["Lc"][cc], r, Z[i], mu[cc])) <= thr
    return keep, thr, int(keep.sum()), st["ok"]


def gmm(U: torch.Tensor, sizes=None, attackers: Optional[torch.Tensor] = None, seed: int = 0,
        gmm_rank: Optional[int] = None, **_) -> AggResult:
    """GMM gradient filter (reference server.py:352-370; its full-covariance fit on raw P-dim updates crashes, A-8):
    a 2-component GMM on the updates' leading PCA scores, deterministic (agg.hip ``k_gmm_filter``, one fused
    launch on the device; ``gmm_filter_ref`` on the host).  The mean of the kept rows; the round fails when no
    row is kept (reference ``round_result = False``) — the only host read of the mode, one byte after the kernel.
    ``gmm_rank``: the PCA rank (engine ``gmm-rank``; None / 0 = max(1, min(4, n // 2 - 1)))."""
    n = U.shape[0]
    att = attackers.bool() if attackers is not None else torch.zeros(n, dtype=torch.bool)
    G = _centred_gram(U)
    if U.is_cuda and n <= 64:
        keep_d, inf_d = ops.native().gmm_filter(G.contiguous(), att.to(U.device, torch.uint8).contiguous(),
                                                int(gmm_rank or 0))
        keep = keep_d.bool()
        thr = inf_d[0]
        if not bool(inf_d[1] > 0):  # (the one synchronising read)
            return AggResult(None, False, {"kept": keep, "threshold": thr})
        return AggResult(_masked_mean(U, keep), True, {"kept": keep, "threshold": thr})
    keep, thr, kept, _ = gmm_filter_ref(G.cpu().numpy(), att.cpu().numpy(), rank=gmm_rank)
    if not kept:
        return AggResult(None, False, {"kept": []})
    return AggResult(mean_of(U[torch.from_numpy(np.nonzero(keep)[0]).to(U.device)]), True,
                     {"kept": np.nonzero(keep)[0].tolist(), "threshold": float(thr)})


def gmm_early(U: torch.Tensor, attackers: torch.Tensor, gmm_rank: Optional[int] = None):
    """``gmm`` without its host read, for the engine's early launch (device U, n <= 64): (mean of the kept
    rows, device bool "some row kept" = the rule's success, info).  ``attackers``: bool, host or device (a host
    tensor goes up pinned, never through a pageable copy that would wait for the stream)."""
    from ..ops.layers import upload

    att = attackers.to(torch.uint8)
    att = upload(att, U.device) if att.device.type == "cpu" else att
    G = _centred_gram(U)
    keep_d, inf_d = ops.native().gmm_filter(G.contiguous(), att.contiguous(), int(gmm_rank or 0))
    keep = keep_d.bool()
    return _masked_mean(U, keep), inf_d[1] > 0, {"kept": keep, "threshold": inf_d[0]}


def scionfl(U: torch.Tensor, sizes: torch.Tensor, seed: int = 0, **_) -> AggResult:
    """All on the device: quantisation, L2-from-counts, the 3x-mean clip, the cosine-distance threshold
    (the int(0.5 n)-th largest score) and the size-weighted FedAvg of the kept originals."""
    n = U.shape[0]
    sigma, smin, smax = ops.stochastic_quantize(U, seed)
    smin = smin.double()
    smax = smax.double()
    ones = sigma.double().sum(dim=1)
    zeros = U.shape[1] - ones
    l2 = torch.sqrt(zeros * smin ** 2 + ones * smax ** 2)
    MU, TOPK = 3.0, 0.5
    lim = MU * l2.mean()
    fac = torch.where(l2 > lim, lim / l2, torch.ones_like(l2))
    smin = smin * fac
    smax = smax * fac
    deq = smin.to(U.dtype)[:, None] + sigma * (smax - smin).to(U.dtype)[:, None]
    agg = mean_of(deq)
    cosd = 1.0 - ops.cosine_to(deq, agg, eps=1e-8).double()
    thr = torch.sort(cosd, descending=True).values[int(TOPK * n)] if n > 0 else torch.zeros((), device=U.device)
    keep = cosd > thr
    # (no client kept: the reference would crash; all clients are averaged instead)
    out = _masked_mean(U, keep, _device_weights(sizes, U.device))
    return AggResult(out, True, {"kept": keep, "scores": cosd, "threshold": thr})


def _median(x: torch.Tensor) -> torch.Tensor:
    """np.median: the mean of the two middle values for an even count."""
    s = torch.sort(x).values
    n = s.shape[0]
    return 0.5 * (s[(n - 1) // 2] + s[n // 2])


def _top_pc_scores(U: torch.Tensor, sweeps: int = 12) -> torch.Tensor:
    """First principal-component scores of the rows (sklearn ``PCA(1).fit_transform`` up to the sign) with no
    host synchronisation: the n x n Gram of the centred rows, its leading eigenpair by a fixed-sweep Jacobi
    eigen-decomposition on the device (``k_top_pc``, n <= 64; ``torch.linalg.eigh`` on the CPU / larger n),
    score = v sqrt(lambda).  Exact for any spectrum gap (repeated squaring, the round-4 form, let the second
    eigenvector leak in when the top two eigenvalues are close)."""
    G = _centred_gram(U)
    n = G.shape[0]
    if G.is_cuda and n <= 64:
        return ops.native().top_pc(G.contiguous(), int(sweeps))
    ev, V = torch.linalg.eigh(G)
    return V[:, -1] * torch.sqrt(ev[-1].clamp_min(0.0))


def fltracer(U: torch.Tensor, sizes: torch.Tensor, threshold: float = 2.5, **_) -> AggResult:
    """FLTracer anomaly filter (reference ``fltracer_detect_anomalies``, src/Utils.py:363-369): robust z-score
    |z - median| / (1.4826 MAD + 1e-6) of the first-PC scores, rows above ``threshold`` dropped, size-weighted
    FedAvg of the rest (every row when all are flagged).  All on the device."""
    z = _top_pc_scores(U)
    med = _median(z)
    mad = _median((z - med).abs())
    scores = (z - med).abs() / (1.4826 * mad + 1e-6)
    bad = scores > threshold
    out = _masked_mean(U, ~bad, _device_weights(sizes, U.device))
    return AggResult(out, True, {"anomalies": bad, "scores": scores})


def byzantine(U: torch.Tensor, sizes=None, threshold: float = 0.9, **_) -> AggResult:
    """Cosine >= 0.9 to model 0, mean of the kept rows (all rows when none passes), on the device."""
    keep = ops.cosine_to(U, U[0], eps=1e-8) >= threshold
    return AggResult(_masked_mean(U, keep), True, {"kept": keep})


# Contract of every aggregator: ``U`` is READ-ONLY and may be the live client-model rows (single rank: the
# engine hands ``local_params`` itself, FLEngine._plain_rows) — never write it in place; a returned tensor may
# alias one of its rows (Krum), which the engine clones before the next launch overwrites the rows.
AGGREGATORS = {
    "fedavg": fedavg,
    "trimmed_mean": trimmed_mean,
    "median": median,
    "krum": krum,
    "shieldfl": shieldfl,
    "gmm": gmm,
    "scionfl": scionfl,
    "fltracer": fltracer,
    "byzantine": byzantine,
}
