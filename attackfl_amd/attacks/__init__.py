"""Model-poisoning attacks on flat update matrices.

All attacks take the attacker's received genuine models as ONE matrix ``G [K, P]`` (rows in the
order the server sampled them) plus the attacker's own current model ``own [P]`` and return
``(ok, malicious [P])``.  Reference semantics (``src/Utils.py:30-214``,
dispatch ``src/RpcClient.py:119-145``) are kept, including the quirks that define the
effective attack:

* A-6  distances are ``sum_k ||Δ_k||_2`` per state_dict tensor with the *spectral* norm for 2-D
  tensors (``torch.linalg.norm(ord=2)``).  ``distance='flat'`` switches to the whole-vector L2
  (the Gram-matrix form).  For ≥3-D tensors (CNN convs, where the reference raises) the
  spectral mode uses the ``[out, in*k]`` matricisation — flagged in ``DEVIATIONS``.
* A-7  candidates are written into ``G[0]`` (alias), so the acceptance test sees a zero
  self-distance for row 0, and the bisection returns the *last tried* candidate.
* unbiased std (``torch.std`` default); ``K <= 1`` returns the attacker's own model for the
  bisection attacks, while LIE with ``K == 1`` yields NaN exactly like the reference.

The bisection only needs, per iteration, the K distances of one candidate.  In flat mode every
distance is ``sqrt(A_j - 2γB_j + γ²C)`` with coefficients from one pass over ``[K, P]``
(``ops.attack_coeffs``, a HIP kernel on GPU).  In spectral mode vector-shaped tensors use the same
closed form per tensor and matrix-shaped tensors use a batched σ_max (``ops.spectral_norm_sum``).

**Device-resident bisection (K-G5).**  The reference loop (``src/Utils.py:118-130,152-164,190-202``)
runs ``while |γ_succ - γ| > τ`` with the step halving every iteration; after iteration i that gap is
exactly γ0 / 2^(i+1) whatever was accepted (an accept sets γ_succ = γ and moves γ up by step/2, a
reject moves γ down by step/2 towards the last accepted value), so the iteration count is known up
front (6 for γ0 = 50, τ = 1) and only the path depends on the data.  ``_bisect_device`` therefore
unrolls the loop with γ, γ_succ and every accept decision as device scalars (``torch.where``
updates): no host synchronisation per γ — the whole attack is enqueued on the attacker's side stream
and its γ reaches the host only when the round's record is written.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from ..models import ParamLayout
from ..utils.log import print_with_color
from .. import ops

DEVIATIONS = {
    "spectral_3d": "reference torch.linalg.norm(ord=2) raises on 3-D conv weights (A-6); we matricise to [out, -1]",
}


@dataclass
class ColumnStats:
    mean: torch.Tensor
    std: torch.Tensor
    sign: torch.Tensor


def column_stats(G: torch.Tensor) -> ColumnStats:
    """Per-coordinate mean, unbiased std and sign(mean) over the K genuine rows."""
    mean, std = ops.column_mean_std(G)
    return ColumnStats(mean, std, torch.sign(mean))


# ----------------------------------------------------------------------------------------------
# distances
# ----------------------------------------------------------------------------------------------

class DistanceEngine:
    """Sum over tensors of per-tensor norms of (x - G_j), batched over rows j."""

    def __init__(self, layout: ParamLayout, mode: str = "spectral"):
        if mode not in ("spectral", "flat"):
            raise ValueError(mode)
        self.layout = layout
        self.mode = mode
        self.vec_slots = [s for s in layout.slots if len(s.shape) <= 1] if mode == "spectral" else []
        self.mat_slots = [s for s in layout.slots if len(s.shape) >= 2] if mode == "spectral" else []

    # pairwise among rows of G: returns [K, K] distance matrix
    def pairwise(self, G: torch.Tensor) -> torch.Tensor:
        K = G.shape[0]
        if self.mode == "flat":
            return ops.pairwise_l2(G)
        D = torch.zeros(K, K, dtype=torch.float64, device=G.device)
        if K < 2:
            return D
        iu = torch.triu_indices(K, K, offset=1, device=G.device)
        diffs = G[iu[0]] - G[iu[1]]                      # [M, P]
        d = self.rowwise_norm_sum(diffs)                  # [M]
        D[iu[0], iu[1]] = d
        D[iu[1], iu[0]] = d
        return D

    def rowwise_norm_sum(self, diffs: torch.Tensor) -> torch.Tensor:
        """sum_k ||diffs[m, slot_k]|| for every row m -> [M] float64."""
        if self.mode == "flat":
            return torch.linalg.vector_norm(diffs.double(), dim=1)
        out = torch.zeros(diffs.shape[0], dtype=torch.float64, device=diffs.device)
        if self.vec_slots:
            out += ops.segment_l2_sum(diffs, self.vec_slots)
        if self.mat_slots:
            out += ops.spectral_norm_sum(diffs, self.mat_slots)
        return out

    def to_rows(self, x: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
        return self.rowwise_norm_sum(x[None, :] - G)


def compute_distance(sd1: Dict[str, torch.Tensor], sd2: Dict[str, torch.Tensor], p: int = 2) -> float:
    """Reference ``compute_distance`` on two state_dicts (used by parity tests)."""
    total = 0.0
    for k in sd1.keys():
        if k in sd2:
            diff = sd1[k] - sd2[k]
            if diff.dim() >= 3:
                diff = diff.reshape(diff.shape[0], -1)
            total += torch.linalg.norm(diff, ord=p).item()
    return total


# ----------------------------------------------------------------------------------------------
# bisection (Min-Max / Min-Sum / Opt-Fang)
# ----------------------------------------------------------------------------------------------

class _CandidateDistances:
    """d(c(γ), G_j) for c(γ) = mean - γ·dev, j = 0..K-1 (row 0 aliased to the candidate)."""

    def __init__(self, engine: DistanceEngine, G: torch.Tensor, mean: torch.Tensor, dev: torch.Tensor):
        self.engine = engine
        self.G = G
        self.mean = mean
        self.dev = dev
        K = G.shape[0]
        if engine.mode == "flat":
            # ||m - g_j - γ d||^2 = A_j - 2γ B_j + γ^2 C  (all rows at once, one pass over [K, P])
            self.A, self.B, self.C = ops.attack_coeffs(G, mean, dev)
        else:
            self.vec = engine.vec_slots
            if self.vec:
                self.A, self.B, self.C = ops.attack_coeffs_segments(G, mean, dev, self.vec)  # [K,S],[K,S],[S]
            # device: the matrix slots' Grams of X_j = mean - G_j once; every γ is then one small launch
            self.fam = (ops.SpectralFamily(mean[None, :] - G[1:], engine.mat_slots, dev)
                        if engine.mat_slots and K > 1 and G.is_cuda else None)

    def __call__(self, gamma) -> torch.Tensor:
        """``gamma``: a float or a 0-d float64 tensor on the matrices' device."""
        K = self.G.shape[0]
        if self.engine.mode == "flat":
            q = (self.A - 2.0 * gamma * self.B + gamma * gamma * self.C).clamp_min(0.0)
            d = torch.sqrt(q)
        else:
            d = torch.zeros(K, dtype=torch.float64, device=self.G.device)
            if self.vec:
                q = (self.A - 2.0 * gamma * self.B + gamma * gamma * self.C[None, :]).clamp_min(0.0)
                d = d + torch.sqrt(q).sum(dim=1)
            if self.fam is not None:
                d = d + torch.cat([torch.zeros(1, dtype=torch.float64, device=d.device), self.fam(gamma)])
            elif self.engine.mat_slots and K > 1:
                cand = self.mean - gamma * self.dev
                diffs = cand[None, :] - self.G[1:]
                dm = torch.zeros(K, dtype=torch.float64, device=self.G.device)
                dm[1:] = ops.spectral_norm_sum(diffs, self.engine.mat_slots)
                d = d + dm
        d = d.clone()
        d[0] = 0.0  # A-7: row 0 *is* the candidate
        return d


def bisect_iterations(gamma: float = 50.0, tau: float = 1.0) -> int:
    """Iterations of the reference loop: the gap |γ_succ - γ| is γ0 / 2^i after i iterations."""
    n, gap = 0, float(gamma)
    while abs(gap) > tau:
        n += 1
        gap /= 2.0
    return n


def _bisect_device(accept: Callable[[torch.Tensor], torch.Tensor], gamma: float, tau: float, device):
    """The reference bisection with device-side state: ``accept(γ)`` returns a 0-d bool tensor.  Returns
    (last tried γ, iterations, last accepted γ, every tried γ [n], every decision [n]) with the γs as float64
    device tensors (the trace the reference prints as ``Gamma is {γ}``, ``src/Utils.py:119,153,191``)."""
    g = torch.full((), float(gamma), dtype=torch.float64, device=device)
    succ = torch.zeros((), dtype=torch.float64, device=device)
    last = g
    step = float(gamma)
    n = bisect_iterations(gamma, tau)
    tried, accs = [], []
    for _ in range(n):
        last = g
        acc = accept(g)
        tried.append(g)
        accs.append(acc)
        succ = torch.where(acc, g, succ)
        g = g + (acc.to(torch.float64) * step - step / 2.0)   # accept: +step/2, reject: -step/2
        step /= 2.0
    if n:
        return last, n, succ, torch.stack(tried), torch.stack(accs)
    return last, n, succ, torch.zeros(0, dtype=torch.float64), torch.zeros(0, dtype=torch.bool)


def _bisect_fused(cd: "_CandidateDistances", threshold: torch.Tensor, kind: str, gamma: float, tau: float):
    """The whole bisection as fused HIP launches (``linalg.hip`` ``bisect_decide``): ONE launch for every
    iteration when no distance needs a spectral norm (flat mode, or vector-shaped tensors only); otherwise
    one ``k_spec_eval<true>`` per γ whose last-arriving workgroup sums the K distances, makes the accept
    decision and moves γ on the device.  Returns the ``_bisect_device`` tuple, or None where a distance
    needs the generic path (matrix slots outside the Gram form, e.g. CNN fc1 / convs)."""
    from .. import ops

    n = bisect_iterations(gamma, tau)
    if n == 0 or n > 16:
        return None
    K = cd.G.shape[0]
    dev = cd.G.device
    if cd.engine.mode == "flat":
        vA, vB, vC = cd.A.reshape(K, 1), cd.B.reshape(K, 1), cd.C.reshape(1)
        fam = None
    else:
        if cd.engine.mat_slots and (cd.fam is None or cd.fam.rest or cd.fam.arena is None):
            return None
        fam = cd.fam if cd.engine.mat_slots else None
        vA, vB, vC = (cd.A, cd.B, cd.C) if cd.vec else (None, None, None)
    vA, vB, vC = [None if t is None else t.to(torch.float64).contiguous() for t in (vA, vB, vC)]
    st = torch.zeros(40, dtype=torch.float64, device=dev)
    st[:1].fill_(float(gamma))  # (st[0] = x is a pageable scalar copy: a host wait for the side stream)
    thr = threshold.to(device=dev, dtype=torch.float64).reshape(1)
    k = 1 if kind == "sum" else 0
    nat = ops.native()
    if fam is None:
        nat.bisect_vec(st, vA, vB, vC, thr, K, k, n, float(gamma))
    else:
        ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        step = float(gamma)
        for it in range(n):
            nat.spec_bisect(fam.arena, fam.tab, fam.sumq, K - 1, st, ctr, vA, vB, vC, thr, k, it, step)
            step /= 2.0
    return st[2], n, st[1], st[4:4 + n], st[20:20 + n] > 0.5


def host_info(info: Dict) -> Dict:
    """An attack's info dict with device values read back (call where the host synchronises anyway): 0-d
    tensors become floats, vectors (the per-γ trace) lists."""
    out = {}
    for k, v in info.items():
        if torch.is_tensor(v):
            v = float(v) if v.dim() == 0 else [float(x) if v.dtype != torch.bool else bool(x) for x in v.tolist()]
        out[k] = v
    return out


def _bisect(accept: Callable[[float], bool], gamma: float = 50.0, tau: float = 1.0) -> Tuple[float, int, float]:
    """Reference bisection with a host predicate: returns (last tried γ, iterations, last accepted γ)."""
    step = gamma
    gamma_succ = 0.0
    last = gamma
    it = 0
    while abs(gamma_succ - gamma) > tau:
        last = gamma
        it += 1
        if accept(gamma):
            gamma_succ = gamma
            gamma = gamma + step / 2
        else:
            gamma = gamma - step / 2
        step = step / 2
    return last, it, gamma_succ


@dataclass
class AttackResult:
    ok: bool
    params: Optional[torch.Tensor]
    info: Dict[str, float]


def _minmax_family(G: torch.Tensor, own: torch.Tensor, engine: DistanceEngine, kind: str, gamma: float = 50.0,
                   tau: float = 1.0) -> AttackResult:
    K = G.shape[0]
    if K <= 1:
        return AttackResult(True, own.clone(), {"gamma": 0.0, "iters": 0})
    st = column_stats(G)
    dev = st.sign if kind == "fang" else st.std
    D = engine.pairwise(G)
    threshold = (D ** 2).sum(dim=1).max() if kind == "sum" else D.max()   # device scalar
    cand_d = _CandidateDistances(engine, G, st.mean, dev)

    def accept(g: torch.Tensor) -> torch.Tensor:
        d = cand_d(g)
        return ((d ** 2).sum() < threshold) if kind == "sum" else (d.max() < threshold)

    fused = _bisect_fused(cand_d, threshold, kind, gamma, tau) if G.is_cuda else None
    last, iters, succ, tried, accs = fused if fused is not None else _bisect_device(accept, gamma, tau, G.device)
    mal = st.mean - last * dev
    return AttackResult(True, mal, {"gamma": last, "gamma_succ": succ, "iters": iters, "threshold": threshold,
                                    "gammas": tried, "accepted": accs})


def min_max(G, own, engine, **kw) -> AttackResult:
    return _minmax_family(G, own, engine, "max", **kw)


def min_sum(G, own, engine, **kw) -> AttackResult:
    return _minmax_family(G, own, engine, "sum", **kw)


def opt_fang(G, own, engine, **kw) -> AttackResult:
    return _minmax_family(G, own, engine, "fang", **kw)


def lie(G: torch.Tensor, own: torch.Tensor, engine: DistanceEngine = None, scaling_factor: float = 0.74) -> AttackResult:
    """Little-Is-Enough: mean + z·std (reference ``create_LIE_state_dict``)."""
    return AttackResult(True, ops.lie_candidate(G, float(scaling_factor)), {"z": float(scaling_factor)})


def random_noise(own: torch.Tensor, perturbation: float, seed: int = 0) -> AttackResult:
    """Random: own + N(0,1)·σ (reference ``create_random_base_model``): Philox4x32-10 normals keyed by
    ``seed`` (``k_noise_philox`` on GPU, the bit-identical uniform mirror on CPU)."""
    return AttackResult(True, ops.noise(own, float(perturbation), int(seed)), {"sigma": float(perturbation)})


def run_attack(mode: str, args: Sequence[float], own: torch.Tensor, G: Optional[torch.Tensor], engine: DistanceEngine,
               seed: int = 0, gamma: float = 50.0, tau: float = 1.0) -> AttackResult:
    """Dispatch by the reference's ``--attack_mode`` names.  ``seed`` keys the Random attack's noise;
    ``gamma`` / ``tau`` start and stop the bisection attacks (reference: fixed 50 / 1)."""
    if mode == "Random":
        sigma = args[0] if args else 1e6
        return random_noise(own, sigma, seed)
    if G is None or G.shape[0] == 0:
        raise ValueError("attack needs genuine models")
    if mode == "Min-Max":
        return min_max(G, own, engine, gamma=gamma, tau=tau)
    if mode == "Min-Sum":
        return min_sum(G, own, engine, gamma=gamma, tau=tau)
    if mode == "Opt-Fang":
        return opt_fang(G, own, engine, gamma=gamma, tau=tau)
    if mode == "LIE":
        z = args[0] if args else 0.74
        if G.shape[0] == 1:
            print_with_color("[Warning] LIE with a single genuine model: unbiased std is NaN (reference behaviour)",
                             "yellow")
        return lie(G, own, engine, z)
    raise ValueError(f"Attack client not contain '{mode}' algorithm.")


ATTACKS = ("Random", "Min-Max", "Min-Sum", "Opt-Fang", "LIE")
