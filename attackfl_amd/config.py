"""Typed ``config.yaml`` schema.

Same keys and defaults as the reference ``config.yaml:1-38`` (read at ``server.py:55-89``,
``client.py:42-48``).  Every reference key is accepted unchanged; the ``rabbit:`` section is
parsed and ignored (there is no broker: transport is RCCL / gloo, see ``parallel/comm.py``).

Extensions (all optional, defaults keep reference behaviour):

``comm:``
  backend: auto | nccl | gloo | loopback
  clients-per-rank: int (packed launcher; 0 = clients / world)
  one-shot-allgather: auto | true | false  (IPC xGMI all-gather of the update blocks on one node:
                            stream-ordered, no host staging; auto = on for GPU ranks of one host, verified
                            collectively at setup with a fallback to the process group's all-gather)
  fedavg-allreduce: auto | true | false  (fedavg without attackers/detection: one all_reduce of
                            [sum s_i w_i | sum s_i] instead of the update all-gather; auto = world > 1
                            without the IPC path)
  timeout-s: collective timeout (failure detection)
  attackers: {client_index: {mode, round, args}}  (launcher-side attack assignment)
``data:``
  synthetic: auto | true | false   (auto = use the reference pickles when present)
  train-size / test-size / seed / har-train-size / har-test-size
``engine:``
  trainer: auto | fused | graph | eager | oracle  (fused = HIP persistent TransformerModel / RNNModel
                                    kernels; graph = HIP-graph-replayed layer programs for CNN/RNN/HAR models;
                                    oracle = CPU fp32 twin of the fused TransformerModel trainer, same masks)
  distance: spectral | flat         (attack distance; spectral = reference ``torch.linalg.norm(ord=2)``)
  seed: int                         (torch / client RNG seed; the reference seeds only ``random``)
  metrics: path of the JSONL metrics file ('' disables)
  checkpoint-dir: where ``*.pth`` files go (reference: CWD)
  async-checkpoint: bool            (default True: the leader writes ``*.pth`` from a background thread)
  compat-hyper-resume: bool         (True = reproduce reference A-5: a loaded hyper checkpoint is discarded)
  compat-fltrust: bool              (True = reproduce reference A-10: FLTrust subtracts the global model twice)
  max-retries: int                  (consecutive failed rounds before the run aborts)
  trace: bool                       (roctx ranges around every round phase; also ATTACKFL_TRACE=1)
  phase-sync: bool                  (synchronise after the aggregate so per-phase times are device times)
  speculative: bool                 (default True: on GPU ranks, enqueue the next round's training
                                    before this round's validation / checkpoint, which overlap it)
  compat-har-train: bool            (True = reference train_HAR semantics: no size-1 batch skip, no NaN
                                    abort, client.py:114-131)
  compat-fedavg-alias: bool         (True = reproduce reference A-13: FedAvg writes the aggregate into the
                                    first client's stored update, which attackers may receive as "genuine")
  fault-inject: [{client, round}]   (NaN-poison a client's model before that training round)
  gmm-rank: int                     (gmm mode's PCA rank, default 1; 0 = max(1, min(4, n // 2 - 1)), the
                                    round-5 rule: profiles/gmm_rank_study_r6.md)
  save-state: bool                  (write {model}.state.pt + {model}.clients.r{rank}.pt every round)
  resume: bool                      (continue from those files: counters, RNGs, optimizer moments)
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

SERVER_MODES = ("fedavg", "hyper", "FLTrust", "trimmed_mean", "shieldfl", "gmm", "krum", "median", "scionfl",
                "fltracer", "byzantine")
ATTACK_MODES = ("Random", "Min-Max", "Min-Sum", "Opt-Fang", "LIE")
MODEL_NAMES = ("CNNModel", "RNNModel", "TransformerModel", "TransformerClassifier")
DATA_NAMES = ("ICU", "HAR", "CIFAR10")

REFERENCE_DEFAULTS: Dict[str, Any] = {
    "name": "Federated Learning poisoning attack testbed",
    "server": {
        "num-round": 30,
        "clients": 3,
        "mode": "hyper",
        "hyper-detection": {"enable": False, "cosine-search": 10, "n_components": 3, "eps": 0.007,
                            "min_samples": 3},
        "model": "TransformerModel",
        "data-name": "ICU",
        "parameters": {"load": False},
        "validation": True,
        "data-distribution": {"num-data-range": [12000, 15000]},
        "genuine-rate": 0.5,
        "random-seed": 1,
    },
    "rabbit": {"address": "192.0.0.1", "username": "admin", "password": "admin"},
    "log_path": ".",
    "learning": {"epoch": 5, "learning-rate": 0.004, "hyper-lr": 0.001, "momentum": 0.5, "batch-size": 128,
                 "clip-grad-norm": 1.0},
}

EXTENSION_DEFAULTS: Dict[str, Any] = {
    "comm": {"backend": "auto", "address": "", "port": 29517, "clients-per-rank": 0, "one-shot-allgather": "auto",
             "fedavg-allreduce": "auto", "timeout-s": 600, "attackers": {}},
    "data": {"synthetic": "auto", "train-size": 60000, "test-size": 10000, "seed": 1234,
             "har-train-size": 2048, "har-test-size": 512, "root": "."},
    "engine": {"trainer": "auto", "distance": "spectral", "seed": 0, "metrics": "", "checkpoint-dir": ".",
               "async-checkpoint": True, "compat-hyper-resume": False, "compat-fltrust": False, "max-retries": 50, "trace": False,
               "phase-sync": False, "fault-inject": [], "save-state": False, "resume": False,
               "speculative": True, "compat-har-train": False, "compat-fedavg-alias": False, "gmm-rank": 1},
}


def _deep_merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


@dataclass
class AttackSpec:
    """One attacker's schedule.  ``gamma`` / ``tau`` are the Min-Max / Min-Sum / Opt-Fang bisection's start
    value and stop gap; the reference hard-codes them to 50 and 1 (``src/Utils.py:101,134,167``), which
    stay the defaults.  With those the tried γs are 50, 25, ..., 1.5625 and a candidate can only be
    accepted at γ ≥ 1.5625 (profiles/attack_study/README.md shows why that rarely passes the distance check)."""
    mode: str
    round: int
    args: List[float] = field(default_factory=list)
    gamma: float = 50.0
    tau: float = 1.0

    def __post_init__(self):
        if self.mode not in ATTACK_MODES:
            raise ValueError(f"Attack mode '{self.mode}' is not valid (choose from {ATTACK_MODES}).")
        self.round = int(self.round)
        self.args = [float(a) for a in (self.args or [])]
        self.gamma, self.tau = float(self.gamma), float(self.tau)
        if not (self.gamma > 0 and self.tau > 0):
            raise ValueError(f"bisection gamma / tau must be positive (got {self.gamma}, {self.tau})")

    def to_dict(self) -> Dict[str, Any]:
        return {"mode": self.mode, "round": self.round, "args": self.args, "gamma": self.gamma, "tau": self.tau}

    @classmethod
    def from_dict(cls, v: Dict[str, Any]) -> "AttackSpec":
        return cls(v["mode"], v.get("round", 1), v.get("args", []), v.get("gamma", 50.0), v.get("tau", 1.0))


@dataclass
class Config:
    raw: Dict[str, Any]

    # ---- server ----
    @property
    def num_round(self) -> int:
        return int(self.raw["server"]["num-round"])

    @property
    def clients(self) -> int:
        return int(self.raw["server"]["clients"])

    @property
    def mode(self) -> str:
        return str(self.raw["server"]["mode"])

    @property
    def model(self) -> str:
        return str(self.raw["server"]["model"])

    @property
    def data_name(self) -> str:
        return str(self.raw["server"]["data-name"])

    @property
    def load_parameters(self) -> bool:
        return bool(self.raw["server"]["parameters"]["load"])

    @property
    def validation(self) -> bool:
        return bool(self.raw["server"]["validation"])

    @property
    def data_range(self) -> List[int]:
        r = self.raw["server"]["data-distribution"]["num-data-range"]
        return [int(r[0]), int(r[1])]

    @property
    def genuine_rate(self) -> float:
        return float(self.raw["server"]["genuine-rate"])

    @property
    def random_seed(self):
        return self.raw["server"]["random-seed"]

    @property
    def hyper_detection(self) -> Dict[str, Any]:
        return self.raw["server"]["hyper-detection"]

    # ---- learning ----
    @property
    def epoch(self) -> int:
        return int(self.raw["learning"]["epoch"])

    @property
    def batch_size(self) -> int:
        return int(self.raw["learning"]["batch-size"])

    @property
    def lr(self) -> float:
        return float(self.raw["learning"]["learning-rate"])

    @property
    def hyper_lr(self) -> float:
        return float(self.raw["learning"]["hyper-lr"])

    @property
    def momentum(self) -> float:
        return float(self.raw["learning"]["momentum"])

    @property
    def clip_grad_norm(self) -> float:
        return float(self.raw["learning"].get("clip-grad-norm", 0.0))

    @property
    def log_path(self) -> str:
        return str(self.raw["log_path"])

    # ---- extensions ----
    @property
    def comm(self) -> Dict[str, Any]:
        return self.raw["comm"]

    @property
    def data(self) -> Dict[str, Any]:
        return self.raw["data"]

    @property
    def engine(self) -> Dict[str, Any]:
        return self.raw["engine"]

    def attackers(self) -> Dict[int, AttackSpec]:
        out: Dict[int, AttackSpec] = {}
        for k, v in (self.raw["comm"].get("attackers") or {}).items():
            out[int(k)] = AttackSpec.from_dict(v)
        return out

    def validate(self) -> "Config":
        if self.mode not in SERVER_MODES:
            raise ValueError(f"Server mode '{self.mode}' is not valid.")
        if self.model not in MODEL_NAMES:
            raise ValueError(f"Model name '{self.model}' is not valid.")
        if self.data_name not in DATA_NAMES:
            raise ValueError(f"Data name '{self.data_name}' is not valid.")
        lo, hi = self.data_range
        if lo > hi or lo < 0:
            raise ValueError(f"num-data-range {self.data_range} is invalid")
        if self.clients < 1:
            raise ValueError("server.clients must be >= 1")
        if self.engine["distance"] not in ("spectral", "flat"):
            raise ValueError("engine.distance must be 'spectral' or 'flat'")
        return self

    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(self.raw)


def from_dict(d: Optional[Dict[str, Any]] = None) -> Config:
    raw = _deep_merge(REFERENCE_DEFAULTS, {})
    raw = _deep_merge(raw, EXTENSION_DEFAULTS)
    raw = _deep_merge(raw, d or {})
    return Config(raw).validate()


def load_config(path: str = "config.yaml", overrides: Optional[Dict[str, Any]] = None) -> Config:
    """Load ``config.yaml`` (reference schema + optional extensions)."""
    d: Dict[str, Any] = {}
    if path and os.path.exists(path):
        with open(path, "r") as fh:
            d = yaml.safe_load(fh) or {}
    elif path and path != "config.yaml":
        raise FileNotFoundError(path)
    if overrides:
        d = _deep_merge(d, overrides)
    return from_dict(d)
