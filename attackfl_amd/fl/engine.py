"""SPMD federated-learning round engine.

Replaces the reference's broker-driven state machines — server ``on_request`` /
``process_consumer`` / ``notify_clients`` (``server.py:205-624``) and client
``RpcClient.response_message`` (``src/RpcClient.py:64-172``) — with one synchronous loop that
every rank runs:

  START  (replicated decisions: per-client parameters, attackers' genuine-model sample)
  LOCAL  (this rank's clients: fused training kernel for all genuine clients at once, attacks)
  GATHER (one all-gather of fixed-layout ``[slots, W]`` blocks  == the UPDATE messages)
  SERVER (replicated aggregation/defense/hypernetwork update — deterministic kernels)
  CHECK  (replicated validation and hyper-detection decision; the leader logs and checkpoints)
  NEXT   (retry the same round on failure, exactly like the reference's ``round`` counter)

Server state is replicated on every rank instead of living in one process, and every decision that
ends a round (validation, detection) is computed by deterministic kernels on identical inputs on
every rank, so the only traffic per round is the update all-gather (or, for plain FedAvg over
RCCL, one all-reduce): no control broadcast, and the next round's training can be enqueued before
this round's validation at any world size (speculative launch, ``run_round``).
"""
from __future__ import annotations

import atexit
import contextlib
import os
import random
import time
import uuid
import weakref
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..agg import AGGREGATORS, AggResult, gmm_early
from ..agg import host_info as agg_host_info
from ..attacks import DistanceEngine, host_info, run_attack
from ..config import AttackSpec, Config
from ..data import DeviceTable, resolve_dataset
from ..detect import HyperDetector
from ..eval import Validation
from ..models import ParamLayout, build_model
from ..parallel.comm import Comm, LoopbackComm
from ..utils import trace
from ..utils.ckpt import CheckpointWriter
from ..utils.log import Logger, MetricsWriter, NullLogger, print_with_color
from .hyper_server import HyperServer
from .trainers import Plan, make_plan, make_trainer

# rules that run on the device without a host read: with one of them the aggregate and the next round's launch
# are enqueued before the host waits for the training, as for FedAvg (FLEngine._early_launch).  gmm (whose
# success the host reads after its wait, from a copy queued before the next launch) and FLTrust (server-model
# training + trust weights, device work too) take the early launch through branches of their own
EARLY_AGGREGATORS = ("trimmed_mean", "median", "krum", "shieldfl", "scionfl", "fltracer", "byzantine")

META = 5  # valid, result, size, is_attacker, decision word; then the client's per-epoch losses (E columns)
DECISION = 4  # column of the sender's decision word (``FLEngine._decision_word``)


class Staging:
    """Per-round host metadata -> device in ONE copy: the arrays are packed (8-byte aligned) into a
    reused pinned buffer, copied with one non-blocking H2D copy into a reused device buffer, and returned
    as typed device views — built once per layout (the same shapes every round), because the ~18 tensor
    view ops per round cost more host time than the copy.  Two buffers alternate, so the next round's
    metadata can be staged (``FLEngine._prepare_local``) while kernels of the current round that read the
    previous views are still queued; a buffer's copy is stream-ordered after the kernels of the round
    before that read it.  On a CPU device the arrays are simply wrapped."""

    SLOTS = 2

    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self._slots = [{"host": None, "dev": None, "done": None, "views": {}} for _ in range(self.SLOTS)]
        self._next = 0

    def upload(self, arrays: Sequence[np.ndarray]) -> List[torch.Tensor]:
        if self.device.type != "cuda":
            return [torch.from_numpy(np.ascontiguousarray(a)) for a in arrays]
        sl = self._slots[self._next]
        self._next = (self._next + 1) % self.SLOTS
        offs, n = [], 0
        for a in arrays:
            offs.append(n)
            n += (a.nbytes + 7) // 8 * 8
        n = max(n, 8)
        if sl["host"] is None or sl["host"].numel() < n:
            sl["host"] = torch.empty(max(n, 4096), dtype=torch.uint8, pin_memory=True)
            sl["dev"] = torch.empty(sl["host"].numel(), dtype=torch.uint8, device=self.device)
            sl["views"].clear()
        elif sl["done"] is not None:
            sl["done"].synchronize()  # this buffer's last copy finished long ago; never overwrite one in flight
        hb = sl["host"].numpy()
        for a, o in zip(arrays, offs):
            hb[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        sl["dev"][:n].copy_(sl["host"][:n], non_blocking=True)
        if sl["done"] is None:
            sl["done"] = torch.cuda.Event()
        sl["done"].record(torch.cuda.current_stream(self.device))
        key = tuple((a.shape, a.dtype.str) for a in arrays)
        out = sl["views"].get(key)
        if out is None:
            out = []
            for a, o in zip(arrays, offs):
                t = sl["dev"][o:o + a.nbytes].view(_TORCH_DT[a.dtype.str[1:]])
                out.append(t.reshape(a.shape))
            sl["views"][key] = out
        return out


def _no_dev_seed(s: int) -> int:
    return 0


_TORCH_DT = {"f4": torch.float32, "i4": torch.int32, "i8": torch.int64, "f8": torch.float64}


@dataclass
class ClientInfo:
    index: int
    uuid: str
    owner: int
    attack: Optional[AttackSpec] = None


@dataclass
class LocalClient:
    info: ClientInfo
    rng: random.Random
    seed: int
    training_round: int = 0
    has_model: bool = False
    genuine: Optional[torch.Tensor] = None     # last received genuine models [K, P]


def build_client_table(cfg: Config, world: int, attackers: Optional[Dict[int, AttackSpec]] = None,
                       clients_per_rank: int = 0) -> List[ClientInfo]:
    """Packed placement: client c lives on rank c // ceil(N / world) (contiguous blocks)."""
    n = cfg.clients
    cpr = clients_per_rank or -(-n // world)
    atk = attackers if attackers is not None else cfg.attackers()
    seed = int(cfg.engine.get("seed", 0))
    table = []
    for c in range(n):
        owner = min(c // cpr, world - 1)
        uid = str(uuid.UUID(int=(seed * 1000003 + c + 1) & ((1 << 128) - 1), version=4))
        table.append(ClientInfo(c, uid, owner, atk.get(c)))
    return table


_LIVE: "weakref.WeakSet[FLEngine]" = weakref.WeakSet()


@atexit.register
def _close_live_engines():
    """Interpreter exit: close every engine its script did not close (a pending speculative launch and the
    checkpoint writer thread would otherwise still run while the runtime tears down: abort at exit)."""
    for eng in list(_LIVE):
        try:
            eng.close()
        except Exception:  # noqa: BLE001 (best effort at exit)
            pass


class FLEngine:
    def __init__(self, cfg: Config, comm: Optional[Comm] = None, table: Optional[List[ClientInfo]] = None,
                 device=None, leader: Optional[bool] = None, verbose: bool = True, train_dataset=None,
                 test_dataset=None):
        _LIVE.add(self)
        self.cfg = cfg
        self.comm = comm or LoopbackComm(device or "cpu")
        self.device = torch.device(device) if device is not None else self.comm.device
        self.rank = self.comm.rank
        self.world = self.comm.world
        self.leader = (self.rank == 0) if leader is None else leader
        self.verbose = verbose and self.leader
        self.table = table if table is not None else build_client_table(cfg, self.world)
        self.n_clients = len(self.table)
        self.mode = cfg.mode
        self.model_name = cfg.model
        self.data_name = cfg.data_name
        self.seed = int(cfg.engine.get("seed", 0))
        self.ckpt_dir = cfg.engine.get("checkpoint-dir", ".")
        self.ckpt_writer = CheckpointWriter(bool(cfg.engine.get("async-checkpoint", True)))
        # synchronise after the aggregate so t_aggregate / t_validate are device times (diagnostics only)
        self.phase_sync = bool(cfg.engine.get("phase-sync", False))
        self._saved_params: Optional[torch.Tensor] = None
        self.max_retries = int(cfg.engine.get("max-retries", 50))
        self.layout = ParamLayout.for_model(self.model_name)
        self.P = self.layout.P
        self.E = cfg.epoch
        # update block row: [P update | META | E epoch losses], padded to 16 bytes (aligned IPC pushes)
        self.W = (self.P + META + self.E + 3) // 4 * 4
        self.dist = DistanceEngine(self.layout, cfg.engine.get("distance", "spectral"))

        # ---- logging (leader only, like the reference's single server process) ----
        if self.leader:
            os.makedirs(cfg.log_path, exist_ok=True)
            self.logger = Logger(os.path.join(cfg.log_path, "app.log"))
            self.metrics = MetricsWriter(cfg.engine.get("metrics") or None)
        else:
            self.logger = NullLogger()
            self.metrics = MetricsWriter(None)

        # ---- data (train set shared by all clients, resident on this rank's device) ----
        self.local = [LocalClient(ci, random.Random(self.seed * 7919 + ci.index), self.seed * 104729 + ci.index)
                      for ci in self.table if ci.owner == self.rank]
        need_train = len(self.local) > 0 or self.mode == "FLTrust"
        self.train_table = None
        if need_train:
            ds = train_dataset if train_dataset is not None else resolve_dataset(self.data_name, "train", cfg.data,
                                                                                 verbose=self.verbose)
            self.train_table = DeviceTable(ds, self.device)
        self.trainer = make_trainer(cfg.engine.get("trainer", "auto"), self.model_name, self.data_name,
                                    self.train_table, self.device) if self.train_table is not None else None
        if self.trainer is not None and hasattr(self.trainer, "compat_har"):
            self.trainer.compat_har = bool(cfg.engine.get("compat-har-train", False))
        # validation runs on EVERY rank: its kernels are deterministic and the global model is bit-identical
        # on all ranks, so each rank reaches the leader's decision without a control broadcast
        self.validation = None
        if cfg.validation:
            self.validation = Validation(self.model_name, self.data_name, self.logger, self.device, cfg.data,
                                         dataset=test_dataset, verbose=self.verbose)
        self.slots = max(sum(1 for ci in self.table if ci.owner == r) for r in range(self.world))
        # persistent per-client models (the reference's ``RpcClient.model``), own random init (A-16)
        self.local_params = torch.zeros(max(1, len(self.local)), self.P, dtype=torch.float32, device=self.device)
        for j, lc in enumerate(self.local):
            m = build_model(self.model_name, seed=lc.seed)
            self.local_params[j].copy_(self.layout.flatten(m.state_dict(), device=self.device))

        # ---- server state (replicated) ----
        self.server_rng = random.Random(cfg.random_seed) if cfg.random_seed else random.Random()
        self.global_params: Optional[torch.Tensor] = None
        self.selected: List[int] = []
        self._selection_done = False
        self.genuine_pool: Optional[torch.Tensor] = None
        self.hyper: Optional[HyperServer] = None
        self.fltrust_model: Optional[torch.Tensor] = None
        self.detector: Optional[HyperDetector] = None
        self.torch_gen = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        self.torch_gen.manual_seed(self.seed * 31337 + self.rank)
        self._init_server()
        self.round_no = 1
        self.rounds_left = cfg.num_round
        self.history: List[dict] = []
        if cfg.engine.get("trace", False):
            trace.enable(True)
        # fault injection: [{client: i, round: r}] -> client i's model is NaN-poisoned before
        # its local training of training-round r, which fails that client and retries the FL round
        self.faults = {(int(f["client"]), int(f["round"])) for f in (cfg.engine.get("fault-inject") or [])}
        self._phase_t: Dict[str, float] = {}
        # FedAvg fast path: with no attacker and no detection, the server needs only
        # sum_i s_i w_i and sum_i s_i -> ONE all_reduce of [P + 5] (+ #failed, #reported, the decision word and its
        # square) instead of the [N, P] all-gather
        # auto = world > 1 without the IPC one-shot gather (which moves whole blocks in one stream-ordered hop
        # and keeps FedAvg on the same deterministic kernel as a single rank)
        fa = str(cfg.comm.get("fedavg-allreduce", "auto")).lower()
        eligible = (self.mode == "fedavg" and all(ci.attack is None for ci in self.table)
                    and not cfg.hyper_detection.get("enable", False))
        self.fast_fedavg = eligible and (fa == "true" or (fa == "auto" and self.world > 1
                                                          and not getattr(self.comm, "one_shot", False)))
        # speculative next-round launch (run_round): replicated-state modes whose retry of a failed round
        # relaunches exactly the same client work (no detection, START from the in-memory global model /
        # hypernetwork; attackers draw from the pool set before the launch), no resume sidecars.  Any world
        # size: validation is replicated, so no rank waits for another's decision before the next launch.
        self._spec = None
        self._next_prep = None  # the next launch's host half, staged while the current training runs
        self._fedavg_w = None
        self._early_agg_info: dict = {}  # a robust rule's info of the last early launch (_early_info)
        self._early_agg_ok = None  # gmm: (pinned bool, event) of the early launch's filter success
        self._val_stream = None
        self._start_ready = None
        self._sel_cache = None
        self._meta_host = None
        self._plain_rows = False
        self._pending = None
        self._has_attackers = any(ci.attack is not None for ci in self.table)
        self._speculative = (bool(cfg.engine.get("speculative", True)) and self.device.type == "cuda"
                             and not cfg.hyper_detection.get("enable", False) and not cfg.load_parameters
                             and not cfg.engine.get("save-state", False) and not self.phase_sync
                             and self.trainer is not None)
        if cfg.engine.get("resume", False):
            self.load_state()
        self.logger.log_info("### Application start ###\n")

    # ------------------------------------------------------------------------------------------
    # server init / checkpoint
    # ------------------------------------------------------------------------------------------
    def _pth(self, hyper: bool = False) -> str:
        if hyper:
            return os.path.join(self.ckpt_dir, f"{self.model_name}_hyper_{self.cfg.clients}.pth")
        return os.path.join(self.ckpt_dir, f"{self.model_name}.pth")

    def _init_server(self):
        cfg = self.cfg
        if self.mode == "hyper":
            net = build_model(self.model_name, seed=self.seed + 99)
            target_sd = net.state_dict()
            hyper_ckpt = None
            if cfg.load_parameters:
                if os.path.exists(self._pth(True)):
                    hyper_ckpt = torch.load(self._pth(True), weights_only=True, map_location="cpu")
                elif os.path.exists(self._pth(False)):
                    net.load_state_dict(torch.load(self._pth(False), weights_only=True, map_location="cpu"))
                    target_sd = net.state_dict()
            self.hyper = HyperServer(target_sd, cfg.clients, cfg.hyper_lr, cfg.clip_grad_norm, self.device,
                                     seed=self.seed)
            if hyper_ckpt is not None:
                if cfg.engine.get("compat-hyper-resume", False):
                    print_with_color("[compat A-5] hyper checkpoint loaded then discarded", "yellow")
                else:
                    self.hyper.hnet.load_state_dict(hyper_ckpt)
                    print_with_color(f"Load state dict from hyper model: {self._pth(True)}", "yellow")
            hd = cfg.hyper_detection
            if hd.get("enable", False):
                # replicated like validation (the embeddings are bit-identical on every rank; PCA / DBSCAN are
                # deterministic host code); only the leader writes all_embeddings.npy and prints
                self.detector = HyperDetector(cfg.clients, int(hd.get("n_components", 3)), float(hd.get("eps", 0.007)),
                                              int(hd.get("min_samples", 3)),
                                              save_path=os.path.join(self.ckpt_dir, "all_embeddings.npy")
                                              if self.leader else "", verbose=self.leader)
        if self.mode == "FLTrust":
            m = build_model(self.model_name, seed=self.seed + 77)
            self.fltrust_model = self.layout.flatten(m.state_dict(), device=self.device)

    def save_checkpoint(self):
        """Reference ``server.py:551-553`` (same files and keys).  Every rank remembers the saved
        global model (what ``{model}.pth`` now holds) so ``load: True`` rounds need no file read;
        the leader writes the file in the background (``utils/ckpt.py``)."""
        if self.mode != "hyper" and self.global_params is not None:
            self._saved_params = self.global_params.detach().clone()
        if not self.leader:
            return
        os.makedirs(self.ckpt_dir, exist_ok=True)
        if self.mode == "hyper":
            hnet = self.hyper.hnet
            # deferred: the arena's copy is issued after the next training launch (utils/ckpt.py)
            if getattr(self, "_hyper_tail", None) is None:
                self._hyper_tail = hnet.target_tail()
            self.ckpt_writer.submit("hyper", hnet.arena, lambda a: hnet.state_dict_of(a, clone=False),
                                    self._pth(True), defer=True, tail=self._hyper_tail)
        elif self.global_params is not None:
            layout = self.layout
            # deferred too: an immediate copy let the writer thread's torch.save (GIL-bound, ~0.5 ms) run
            # in the gap between two rounds' training launches and stall the next round's preparation;
            # kicked after the next launch it runs while the GPU trains.  global_params is replaced, never
            # updated in place, so the submitted tensor stays valid until the copy.
            self.ckpt_writer.submit("global", self.global_params, lambda f: layout.unflatten(f, clone=False),
                                    self._pth(False), defer=True)

    # ---- resumable run state (new: the reference persists only the model) ----
    def _state_paths(self):
        base = os.path.join(self.ckpt_dir, self.model_name)
        return base + ".state.pt", f"{base}.clients.r{self.rank}.pt"

    def save_state(self) -> None:
        """Replicated server state (leader) + this rank's client state, loadable with
        ``torch.load(weights_only=True)``: round counters, RNG states, hypernetwork Adam moments,
        the genuine pool attackers sample from, and every local client's model and RNG."""
        os.makedirs(self.ckpt_dir, exist_ok=True)
        srv_path, cli_path = self._state_paths()
        if self.leader:
            v, st, gauss = self.server_rng.getstate()
            srv = {"round_no": self.round_no, "rounds_left": self.rounds_left, "rng_version": v,
                   "rng_state": list(st), "rng_gauss": gauss, "selected": list(self.selected),
                   "global": self.global_params.detach().cpu() if self.global_params is not None else None,
                   "genuine_pool": self.genuine_pool.detach().cpu() if self.genuine_pool is not None else None}
            if self.hyper is not None:
                srv.update(hyper_arena=self.hyper.hnet.arena.detach().cpu(), hyper_m=self.hyper.m.cpu(),
                           hyper_v=self.hyper.v.cpu(), hyper_step=self.hyper.step)
            torch.save(srv, srv_path + ".tmp")
            os.replace(srv_path + ".tmp", srv_path)
        cli = {"params": self.local_params.detach().cpu(), "index": [lc.info.index for lc in self.local],
               "training_round": [lc.training_round for lc in self.local],
               "rng": [[lc.rng.getstate()[0], list(lc.rng.getstate()[1]), lc.rng.getstate()[2]] for lc in self.local]}
        torch.save(cli, cli_path + ".tmp")
        os.replace(cli_path + ".tmp", cli_path)

    def load_state(self) -> bool:
        srv_path, cli_path = self._state_paths()
        if not os.path.exists(srv_path):
            return False
        srv = torch.load(srv_path, weights_only=True, map_location="cpu")
        self.round_no = int(srv["round_no"])
        self.rounds_left = int(srv["rounds_left"])
        self.server_rng.setstate((srv["rng_version"], tuple(srv["rng_state"]), srv["rng_gauss"]))
        if srv.get("selected"):
            self.selected = list(srv["selected"])
            self._selection_done = True
        if srv.get("global") is not None:
            self.global_params = srv["global"].to(self.device)
        if srv.get("genuine_pool") is not None:
            self.genuine_pool = srv["genuine_pool"].to(self.device)
        if self.hyper is not None and "hyper_m" in srv:
            self.hyper.load_arena(srv["hyper_arena"])
            self.hyper.m.copy_(srv["hyper_m"])
            self.hyper.v.copy_(srv["hyper_v"])
            self.hyper.step = int(srv["hyper_step"])
        if os.path.exists(cli_path):
            cli = torch.load(cli_path, weights_only=True, map_location="cpu")
            self.local_params.copy_(cli["params"].to(self.device))
            for lc, tr, rs in zip(self.local, cli["training_round"], cli["rng"]):
                lc.training_round = int(tr)
                lc.rng.setstate((rs[0], tuple(rs[1]), rs[2]))
        print_with_color(f"Resumed run state from {srv_path} at round {self.round_no}", "yellow")
        return True

    # ------------------------------------------------------------------------------------------
    # START
    # ------------------------------------------------------------------------------------------
    def client_selection(self):
        self._selection_done = True
        self.selected = list(range(self.n_clients))
        self.logger.log_info(f"Active with {len(self.selected)} client: {self.selected}")

    def _start_params(self, i: int) -> Optional[torch.Tensor]:
        if self.mode == "hyper":
            return self.hyper.generate(i)
        if self.cfg.load_parameters:
            if self._saved_params is not None:  # == the file this run last wrote
                return self._saved_params
            self.ckpt_writer.flush()
            p = self._pth(False)
            if os.path.exists(p):
                return self.layout.flatten(torch.load(p, weights_only=True, map_location="cpu"), device=self.device)
            return None
        return self.global_params

    def _genuine_for_attackers(self) -> Dict[int, Optional[torch.Tensor]]:
        """Replicated: every rank draws the same sample for every attacker (server RNG in sync)."""
        out: Dict[int, Optional[torch.Tensor]] = {}
        pool = self.genuine_pool
        for i in self.selected:
            ci = self.table[i]
            if ci.attack is None:
                continue
            if pool is not None and pool.shape[0] > 0:
                G = pool.shape[0]
                k = max(int(self.cfg.genuine_rate * G), 1)
                idx = self.server_rng.sample(range(G), k)
                out[i] = self._take_rows(pool, idx) if ci.owner == self.rank else None
            else:
                out[i] = None
        return out

    def _take_rows(self, pool: torch.Tensor, idx: List[int]) -> torch.Tensor:
        """``pool[idx]`` with the index list on the device through a small cache and a pinned, non-blocking
        upload: indexing a device tensor with a Python list (or a pageable ``.to``) makes a pageable host ->
        device copy, which synchronises the stream — the host would wait for the training launch already
        enqueued, the early launch's whole point (a random genuine sample misses the cache most rounds)."""
        if pool.device.type != "cuda":
            return pool[idx]
        from ..ops.layers import upload

        key = tuple(idx)
        cache = self.__dict__.setdefault("_rows_idx", {})
        ix = cache.get(key)
        if ix is None:
            if len(cache) > 1024:
                cache.clear()
            ix = cache[key] = upload(torch.tensor(idx, dtype=torch.long), pool.device)
        return pool.index_select(0, ix)

    # ------------------------------------------------------------------------------------------
    # LOCAL
    # ------------------------------------------------------------------------------------------
    @property
    def _dev_seed(self):
        ds = getattr(self.trainer, "device_seed", None)
        return ds if (ds is not None and self.device.type == "cuda") else _no_dev_seed

    @property
    def _staging(self) -> "Staging":
        st = getattr(self, "_staging_obj", None)
        if st is None:
            st = self._staging_obj = Staging(self.device)
        return st

    def _side_stream(self):
        if self.device.type != "cuda":
            return None
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def _local_work(self, genuine: Dict[int, Optional[torch.Tensor]]) -> torch.Tensor:
        return self._finish_local(self._launch_local(genuine))

    def _launch_local(self, genuine: Dict[int, Optional[torch.Tensor]]) -> dict:
        """Prepare this rank's clients for the round and enqueue the genuine clients' training (async).
        Uses the preparation staged ahead by ``run_round`` when there is one."""
        prep, self._next_prep = self._next_prep, None
        if prep is None or prep["selected"] != tuple(self.selected):
            prep = self._prepare_local()
        return self._enqueue_local(prep, genuine)

    def _prepare_local(self) -> dict:
        """Host half of a launch — client counters, the data draws, fault injection, the plan — none of which
        depends on the previous round's outcome, so ``run_round`` stages the NEXT launch's half before it
        waits for the current training (the draws are the same whenever they happen: one per launch, in
        launch order).  Uploads and the plan kernel are enqueued here; which clients attack is re-checked at
        enqueue time (an attacker's first attack round waits for its genuine sample)."""
        tq = time.perf_counter()
        cfg = self.cfg
        meta = np.zeros((self.slots, META + self.E), dtype=np.float32)  # host-built, uploaded once (+ losses)
        lo, hi = cfg.data_range
        clients, faults = [], []
        for j, lc in enumerate(self.local):
            i = lc.info.index
            if i not in self.selected:
                continue
            lc.training_round += 1
            if (i, lc.training_round) in self.faults:
                faults.append(j)
                print_with_color(f"[fault-inject] client {i} poisoned with NaN (training round {lc.training_round})",
                                 "red")
            num_data = lc.rng.randrange(lo, hi + 1)
            meta[j, 0] = 1.0
            meta[j, 2] = float(num_data)
            meta[j, 3] = 1.0 if lc.info.attack is not None else 0.0
            clients.append((j, i, lc, num_data))
        prep = {"tq": tq, "meta": meta, "clients": clients, "faults": faults, "selected": tuple(self.selected)}
        self._stage(prep, self._attack_decisions(prep))
        return prep

    def _prepare_staged(self) -> dict:
        """``_prepare_local`` with its device half (the upload and the plan kernel) on a staging stream: those
        depend on nothing the running training writes, and on the compute stream they sat behind it, in the gap
        between two training kernels.  The launch waits for the staging event (``_enqueue_local``)."""
        dev = self.device
        if dev.type != "cuda":
            return self._prepare_local()
        if getattr(self, "_stage_stream", None) is None:
            self._stage_stream = torch.cuda.Stream(device=dev)
        main = torch.cuda.current_stream(dev)
        with torch.cuda.stream(self._stage_stream):
            prep = self._prepare_local()
            ev = torch.cuda.Event()
            ev.record(self._stage_stream)
        plan = prep.get("plan")
        if plan is not None and plan.order.is_cuda:
            plan.order.record_stream(main)  # (allocated on the staging stream, read by the launch on main)
        prep["staged_ev"] = ev
        return prep

    @staticmethod
    def _attack_decisions(prep: dict) -> tuple:
        return tuple(lc.info.attack is not None and lc.training_round >= lc.info.attack.round
                     and lc.genuine is not None and lc.genuine.shape[0] > 0 for _, _, lc, _ in prep["clients"])

    def _stage(self, prep: dict, decisions: tuple) -> None:
        """Training rows / sizes / seeds for the given attack decisions, their ONE upload and the plan."""
        cfg, dev = self.cfg, self.device
        tq1 = time.perf_counter()
        train_rows, train_nd, train_seeds = [], [], []
        attack_rows = []
        for (j, i, lc, num_data), atk in zip(prep["clients"], decisions):
            if atk:
                attack_rows.append((j, lc))
            else:
                train_rows.append(j)
                train_nd.append(num_data)
                train_seeds.append(lc.seed * 7 + lc.training_round)
        if train_rows and attack_rows:
            # the attackers ride along with ZERO rows (nd = 0: the trainer leaves their models untouched), so the
            # launch covers every local client in place — no gather / scatter of the trained rows — and their
            # attack results are written into their local_params rows once the launch is done (_finish_local)
            for j, lc in attack_rows:
                train_rows.append(j)
                train_nd.append(0)
                train_seeds.append(lc.seed * 7 + lc.training_round)
            order = sorted(range(len(train_rows)), key=lambda k: train_rows[k])
            train_rows = [train_rows[k] for k in order]
            train_nd = [train_nd[k] for k in order]
            train_seeds = [train_seeds[k] for k in order]
        # FedAvg weights of the selected rows (single rank, every row stored): staged with the rest, so the
        # aggregate needs no host -> device copy after the training (== ops.fedavg's s / s.sum(), exact sums)
        sel_nd = np.asarray([prep["meta"][r, 2] for r in self._local_rows()], np.float64) if self.world == 1 else None
        fw = sel_nd / sel_nd.sum() if sel_nd is not None and sel_nd.size and sel_nd.sum() > 0 else np.zeros(1)
        # every per-round host value the device needs goes up in ONE asynchronous copy (a pageable
        # torch.tensor(..., device=) per item was a blocking copy each: ~1.5 ms of host time per round)
        js = [j for j, _, _, _ in prep["clients"]]
        plan_seeds = [sd * 1000003 + 17 for sd in train_seeds]
        meta_d, js_d, rows_d, pseed_d, nd_d, tseed_d, fw_d = self._staging.upload([
            prep["meta"][:, :META], np.asarray(js, np.int64), np.asarray(train_rows, np.int64),
            np.asarray([(s & 0xFFFFFFFFFFFFFFFF) - (1 << 64) if (s & 0xFFFFFFFFFFFFFFFF) >= (1 << 63)
                        else (s & 0xFFFFFFFFFFFFFFFF) for s in plan_seeds], np.int64),
            np.asarray(train_nd, np.int32),
            np.asarray([self._dev_seed(s) for s in train_seeds], np.int32), fw])
        tq2 = time.perf_counter()
        plan = None
        if train_rows:
            plan = make_plan(self.train_table.n, train_nd, cfg.epoch, plan_seeds, dev,
                             staged=(pseed_d, nd_d) if dev.type == "cuda" else None)
        prep.update({"dec": decisions, "train_rows": train_rows, "train_seeds": train_seeds,
                     "attack_rows": [j for j, _ in attack_rows], "js": js, "meta_d": meta_d, "js_d": js_d,
                     "rows_d": rows_d, "tseed_d": tseed_d, "plan": plan,
                     "fedavg_w": fw_d if sel_nd is not None and fw.size == len(self.selected) else None,
                     "sizes_h": torch.from_numpy(sel_nd) if sel_nd is not None else None,
                     "tq1": tq1, "tq2": tq2})

    def _enqueue_local(self, prep: dict, genuine: Dict[int, Optional[torch.Tensor]]) -> dict:
        """Device half of a launch: START parameters, the update block, the training launch."""
        cfg = self.cfg
        dev = self.device
        tq = time.perf_counter()
        if prep.get("staged_ev") is not None:  # uploads / plan staged on the staging stream (_prepare_staged)
            torch.cuda.current_stream(dev).wait_event(prep["staged_ev"])
        for j, i, lc, _ in prep["clients"]:
            g = genuine.get(i)
            if lc.info.attack is not None and g is not None and g.shape[0] > 0:
                lc.genuine = g
        dec = self._attack_decisions(prep)
        if dec != prep["dec"]:
            self._stage(prep, dec)  # (an attacker's first attack round)
        attack_jobs = [(j, i, lc, lc.info.attack) for (j, i, lc, _), a in zip(prep["clients"], dec) if a]
        train_rows, train_seeds, js, js_d = prep["train_rows"], prep["train_seeds"], prep["js"], prep["js_d"]
        rows_d = prep["rows_d"]
        n_local = len(self.local)
        # the common case (every local client trains) trains local_params in place: no gather / scatter
        in_place = train_rows == list(range(n_local))
        # single rank, every local client in the launch (attackers with zero rows), trained in place: the round
        # reads the update matrix straight from local_params and the meta columns from the host mirror, so
        # no update block is built at all
        plain = (bool(train_rows) and in_place and self.world == 1 and not self.fast_fedavg
                 and self._local_rows() == list(range(n_local)))
        block = None if plain else torch.zeros(self.slots, self.W, dtype=torch.float32, device=dev)
        tq2 = time.perf_counter()
        # START parameters of every started client (one batched generate / broadcast copy)
        if prep["clients"]:
            if self.mode == "hyper":
                start = self.hyper.generate_many([i for _, i, _, _ in prep["clients"]])
            else:
                p = self._start_params(prep["clients"][0][1])
                start = None if p is None else p[None, :].expand(len(js), -1)
            if start is not None:
                if js == list(range(len(js))):
                    self.local_params[:len(js)].copy_(start)
                else:
                    self.local_params.index_copy_(0, js_d, start.contiguous())
        if self._speculative and dev.type == "cuda":
            # START is generated (hyper: the memoised generate_many validation reuses): a speculative
            # round's validation stream waits for this point, not for the training launched below
            self._start_ready = torch.cuda.Event()
            self._start_ready.record(torch.cuda.current_stream(dev))
        for j in prep["faults"]:
            self.local_params[j, 0] = float("nan")
        if block is not None:
            block[:, self.P:self.P + META] = prep["meta_d"]
        tp0 = time.perf_counter()
        pending = None
        ready = None
        if attack_jobs and dev.type == "cuda":
            # the attackers' inputs are ready now; the side stream must not also wait for the training launch
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(dev))
        params = None
        if train_rows:
            params = self.local_params if in_place else self.local_params.index_select(0, rows_d).contiguous()
            pending = self.trainer.launch(params, prep["plan"], cfg.lr, cfg.batch_size, train_seeds,
                                          seeds_dev=prep["tseed_d"] if self._dev_seed is not _no_dev_seed else None)
        self.ckpt_writer.kick()  # last round's deferred checkpoint copy overlaps this round's training
        tp1 = time.perf_counter()
        return {"block": block, "attack_jobs": attack_jobs, "ready": ready, "pending": pending, "params": params,
                "in_place": in_place, "rows_d": rows_d, "n_local": n_local, "meta": prep["meta"],
                "train_rows": train_rows, "fedavg_w": prep["fedavg_w"], "sizes_h": prep.get("sizes_h"), "plain": plain,
                "t": (prep["tq"], prep["tq1"], prep["tq2"], tp0, tp1), "t_enqueue": tp0 - tq}

    def _finish_attacks(self, st: dict) -> None:
        """Attackers' math on a side stream; their results replace their local_params rows (stream-ordered
        after the training launch, which read / wrote back their untouched models: no host wait)."""
        attack_jobs, ready, pending, in_place = st["attack_jobs"], st["ready"], st["pending"], st["in_place"]
        dev = self.device
        tw = time.perf_counter()  # a speculative launch (run_round) may have been enqueued long before
        atk_out = []  # (row, ok, malicious update)
        if attack_jobs:
            # the attackers do not train: their math runs on a side stream while the genuine clients'
            # training launch occupies its own CUs (the reference runs every client concurrently too)
            side = self._side_stream()
            if side is not None:
                side.wait_event(ready)
            with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
                for j, i, lc, atk in attack_jobs:
                    res = run_attack(atk.mode, atk.args, self.local_params[j], lc.genuine, self.dist,
                                     seed=lc.seed * 1009 + lc.training_round, gamma=atk.gamma, tau=atk.tau)
                    atk_out.append((j, res.ok and res.params is not None, res.params))
                    self._attack_info = res.info
                    if self.verbose:  # (reads the attack's device scalars back: verbose runs only)
                        hi = host_info(res.info)
                        for g in hi.get("gammas", []):  # the reference's per-iteration print (src/Utils.py:119)
                            print(f"Gamma is {g}")
                        print_with_color(f"[===] Client {i} attacks with {atk.mode} "
                                         f"{ {k: v for k, v in hi.items() if not isinstance(v, list)} }", "red")
            if side is not None:
                torch.cuda.current_stream(dev).wait_stream(side)
        if pending is not None and in_place:
            for j, ok, mal in atk_out:
                if ok:
                    self.local_params[j].copy_(mal)
        st["atk_out"], st["tw"], st["tp2"] = atk_out, tw, time.perf_counter()

    def _finish_local(self, st: dict) -> Optional[torch.Tensor]:
        """Attackers' math (``_finish_attacks``, unless done already), then wait for the training launch and
        fill the update block (none at world 1 with plain rows)."""
        if "atk_out" not in st:
            self._finish_attacks(st)
        block, pending = st["block"], st["pending"]
        params, in_place, rows_d, n_local = st["params"], st["in_place"], st["rows_d"], st["n_local"]
        tq, tq1, tq2, tp0, tp1 = st["t"]
        atk_out, tw, tp2 = st["atk_out"], st["tw"], st["tp2"]
        dev = self.device
        hm = st["meta"]  # host mirror of the block's meta columns (ok filled in below): no device read needed
        self._plain_rows = pending is not None and st["plain"]  # (_enqueue_local: no update block)
        self._pending = pending
        P, E = self.P, self.E
        if pending is not None:
            ok_dev, loss_dev = pending.ok_device(), pending.losses_device()
            # world > 1: the ok flags and losses travel in the block and the host learns every rank's meta from
            # ONE read after the gather, so it does not wait for its own training here (one host round trip less)
            host_wait = self.world == 1 or ok_dev is None or loss_dev is None
            if host_wait:
                oks, losses = pending.result()
                for k, (j, o) in enumerate(zip(st["train_rows"], oks)):
                    hm[j, 1] = 1.0 if o else 0.0
                    hm[j, META:META + E] = np.asarray(losses[k], dtype=np.float32)[:E]
            tp3 = time.perf_counter()
            # A-15: an attacker still reports its num_data, ok = the attack's result (its row: _finish_attacks)
            for j, ok, mal in atk_out:
                hm[j, 1] = 1.0 if ok else 0.0
            if self._plain_rows:
                pass
            elif in_place:
                block[:n_local, :P] = self.local_params[:n_local]
                if ok_dev is not None:
                    block[:n_local, P + 1] = (ok_dev > 0).float()
                else:
                    block[:n_local, P + 1] = torch.tensor([1.0 if o else 0.0 for o in oks], device=dev)
                block[:n_local, P + META:P + META + E] = (loss_dev if loss_dev is not None
                                                         else losses.to(dev)).float()
                for j, ok, _ in atk_out:
                    block[j, P + 1] = 1.0 if ok else 0.0
            else:
                self.local_params.index_copy_(0, rows_d, params)
                block[rows_d, :P] = params
                okc = (ok_dev > 0).float() if ok_dev is not None else torch.tensor(
                    [1.0 if o else 0.0 for o in oks], device=dev)
                block[rows_d, P + 1] = okc
                block[rows_d, P + META:P + META + E] = (loss_dev if loss_dev is not None else losses.to(dev)).float()
                for j, ok, mal in atk_out:  # (only when no genuine client trains here: attackers are not launched)
                    if ok:
                        block[j, :P] = mal
                    block[j, P + 1] = 1.0 if ok else 0.0
        else:
            tp3 = time.perf_counter()
            for j, ok, mal in atk_out:  # every local client attacks: nothing was launched
                hm[j, 1] = 1.0 if ok else 0.0
                if ok:
                    block[j, :P] = mal
                block[j, P + 1] = 1.0 if ok else 0.0
        if block is not None:
            # every rank stamps its view of the replicated server state into its rows; the gather's reader checks
            # that all ranks agree (_check_decisions), so a rank whose validation / detection diverged fails loudly
            block[:, P + DECISION] = float(self._decision_word())
        self._fedavg_w = st.get("fedavg_w")
        self._lw_times = {"t_lw_prep": (tq2 - tq) + st.get("t_enqueue", 0.0), "t_lw_prep_host": tq1 - tq,
                          "t_lw_prep_upload": tq2 - tq1, "t_lw_launch": tp1 - tp0, "t_lw_attack": tp2 - tw,
                          "t_lw_wait": tp3 - tp2, "t_lw_post": time.perf_counter() - tp3}
        self._meta_host = hm
        return block

    def _local_rows(self) -> List[int]:
        """Block rows of the selected clients (cached per selection)."""
        key = tuple(self.selected)
        if self._sel_cache is None or self._sel_cache[0] != key:
            rows = [self.table[i].owner * self.slots + self._slot_of(i) for i in self.selected]
            idx = torch.tensor(rows, device=self.device, dtype=torch.long)
            self._sel_cache = (key, rows, idx)
        return self._sel_cache[1]

    # ------------------------------------------------------------------------------------------
    # SERVER
    # ------------------------------------------------------------------------------------------
    def _aggregate(self, U: torch.Tensor, sizes: torch.Tensor, attackers: torch.Tensor, round_ok: bool) -> dict:
        info: dict = {}
        if not round_ok:
            return info
        mode = self.mode
        if mode == "hyper":
            ups = {i: U[k] for k, i in enumerate(self.selected)}
            self.ckpt_writer.fence()  # the previous round's checkpoint copy of the arena, updated in place below
            self.hyper.train(self.selected, ups)
            info["_lazy"] = lambda: self.hyper.last_info  # read after validation: no sync between them
            return info
        if mode == "FLTrust":
            self.global_params = self._fltrust(U)
            return info
        if mode == "fedavg" and self._fedavg_w is not None and U.shape[0] == self._fedavg_w.shape[0] and U.is_cuda:
            # the weights were staged with the launch (sizes known then): no host -> device copy here
            self.global_params = ops.weighted_rows(U, self._fedavg_w)
            info["n"] = int(U.shape[0])
            return info
        fn = AGGREGATORS[mode]
        res: AggResult = fn(U, sizes, attackers=attackers, seed=self.seed * 13 + self.round_no,
                            gmm_rank=int(self.cfg.engine.get("gmm-rank", 1)))
        info.update({k: v for k, v in res.info.items() if k != "scores"})
        if not res.ok:
            info["agg_failed"] = True
        elif res.params is not None:
            g = res.params.to(torch.float32)
            if g.untyped_storage().data_ptr() == U.untyped_storage().data_ptr():
                g = g.clone()  # a selected row (e.g. Krum) of U, which may be the live client models
            self.global_params = g
        return info

    def _fltrust_setup(self):
        """Root set (first 200 test rows, ``server.py:290-293``), its device table and the server model's
        trainer: built once and reused every round."""
        if getattr(self, "_fl_root", None) is None:
            from ..data import ICUData

            root = resolve_dataset(self.data_name, "test", self.cfg.data, verbose=False)
            if isinstance(root, ICUData):
                root = ICUData(vitals=root.vitals[:200], labs=root.labs[:200], labels=root.labels[:200])
            table = DeviceTable(root, self.device)
            trainer = make_trainer(self.cfg.engine.get("trainer", "auto"), self.model_name, self.data_name, table,
                                   self.device)
            nd = min(200, table.n)
            # DataLoader(batch_size=100, shuffle=False): the same in-order visit every epoch
            order = torch.arange(nd, dtype=torch.int32, device=self.device)[None, None, :].expand(
                1, self.cfg.epoch, nd).contiguous()
            plan = Plan(order, torch.tensor([nd], dtype=torch.int32), self.cfg.epoch,
                        nd_dev=torch.tensor([nd], dtype=torch.int32, device=self.device))
            self._fl_root = (table, trainer, plan)
        return self._fl_root

    def _fltrust(self, U: torch.Tensor) -> torch.Tensor:
        """FLTrust with a server model trained on the first 200 test rows (``server.py:682-743``).
        Everything stays on the device: the server model's training is enqueued (its result is ignored,
        like the reference's ``train_on_device`` return value), and the trust scores, norms and the
        trust-weighted sum are device tensors; ``trust`` reaches the JSONL lazily after validation."""
        compat = bool(self.cfg.engine.get("compat-fltrust", False))
        g0 = self.global_params if self.global_params is not None else self.fltrust_model.clone()
        _, trainer, plan = self._fltrust_setup()
        params = g0.clone()[None]
        # kept and read at the round's host synchronisation (_finish_round): a NaN result is ignored like the
        # reference's train_on_device return value, a cross-workgroup timeout still raises
        seed = self.seed + self.round_no
        ds = getattr(trainer, "device_seed", None)
        seeds_dev = None
        if ds is not None and self.device.type == "cuda":
            # a pinned, non-blocking upload: the trainer's own upload of a host list is a pageable copy, which
            # waits for the clients' training (the early launch enqueues this before that ends)
            from ..ops.layers import upload
            seeds_dev = upload(torch.tensor([ds(seed)], dtype=torch.int32), self.device)
        self._fl_pending = trainer.launch(params, plan, self.cfg.lr, 100, [seed], seeds_dev=seeds_dev)
        server_new = params[0]
        g0_delta = server_new - g0
        if compat and self.global_params is None:
            g0_delta = torch.zeros_like(g0)  # round-1 alias: state_dict() views were trained in place
        deltas = U - g0[None, :]
        if compat:
            deltas = deltas - g0[None, :]   # A-10: the stored delta is reduced by g_0 a second time
        norm_g0 = torch.linalg.vector_norm(g0_delta.double())
        norms = ops.row_norms(deltas).double()
        cos = ops.cosine_to(deltas, g0_delta, eps=1e-8).double()
        trust = torch.clamp(cos, min=0.0)
        scale = (norm_g0 / (norms + 1e-6)) * trust
        w = scale / (trust.sum() + 1e-6)
        agg = ops.weighted_rows(deltas, w)
        self.fltrust_model = server_new
        self._trust = trust
        return g0 + agg

    # ------------------------------------------------------------------------------------------
    # one round
    # ------------------------------------------------------------------------------------------
    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def run_round(self, last: bool = False) -> dict:
        """One FL round.  ``last``: the caller will not run another round, so no speculative launch."""
        if not self._selection_done:
            self.client_selection()
        t0 = time.perf_counter()
        if self.verbose:
            print_with_color(f"Start training round {self.round_no}", "yellow")
        self._attack_info = None
        self._trust = None
        with trace.range("fl/local"):
            st, self._spec = self._spec, None
            if st is None:
                st = self._launch_local(self._genuine_for_attackers())
            if self._speculative and self.rounds_left > 1 and not last and self._next_prep is None:
                # the next launch's host half (draws, uploads, plan) while this round's training runs: after
                # it, only the aggregate, START and the launch itself separate two training kernels
                self._next_prep = self._prepare_staged()
            esl = self._early_launch(st, last)
            block = self._finish_local(st)
            if self.phase_sync:  # stream-ordered otherwise: the timing-only sync is skipped
                self._sync()
        t1 = time.perf_counter()
        P = self.P
        snapshot = None
        attackers = None
        stored = len(self.selected)
        if esl is not None:
            # FedAvg, one rank: the aggregate and the next launch went in before the wait (_early_launch)
            U = None
            meta = torch.from_numpy(self._meta_host[self._local_rows()])
            results = meta.numpy()[:, 1] > 0.5
            round_ok = bool(results.all())
            info = self._early_info(round_ok)
            if not self._early_agg_done() and round_ok:
                round_ok = False
                info = {**self._early_agg_info, "agg_failed": True}
            if not round_ok:
                self._early_launch_failed(esl, results)
            t2 = t3 = time.perf_counter()
        elif self.fast_fedavg:
            U = None
            round_ok, meta = self._fedavg_allreduce(block)
            info = {"path": "fedavg-allreduce"}
            t2 = t3 = time.perf_counter()
        else:
            trace.push("fl/gather")
            rows = self._local_rows()
            idx = self._sel_cache[2]
            if self.world == 1:  # every row is local: the host already knows the meta columns
                meta = torch.from_numpy(self._meta_host[rows])
                if self._plain_rows:
                    U = self.local_params[:len(rows)]  # the trained models ARE the update rows: no block at all
                else:
                    U = self.comm.all_gather_rows(block).index_select(0, idx)[:, :P].contiguous()
            else:
                allb = self.comm.all_gather_rows(block)                    # [world*slots, W]
                sel = allb.index_select(0, idx)
                U = sel[:, :P].contiguous()
                # the round's ONE host read: every client's [valid, result, size, attacker, decision | losses]; it
                # is queued BEFORE the early launch and waited for through its own event, so the host waits for
                # the gather (the slowest rank's clients), not for the next round's training queued behind it
                # (+ one row per rank — its first slot — so every rank's decision word is checked, also a rank
                # none of whose clients is selected or valid this round)
                nsel = sel.shape[0]
                per_rank = allb[0::block.shape[0], P:P + META + self.E] if block.shape[0] else allb[:0, P:P + META + self.E]
                mread = self._meta_read(torch.cat([sel[:, P:P + META + self.E], per_rank], 0))
                # FedAvg / hyper: the aggregate and the next launch go in on the device before the host read
                esl = self._early_launch(st, last, U=U, sel=sel)
                mall = mread()
                meta, rank_rows = mall[:nsel], mall[nsel:]
                self.comm.check()
                self._check_decisions(meta.numpy(), rank_rows.numpy()[:, DECISION])
                if self._pending is not None:
                    self._pending.result()  # the training has finished by now: surfaces hand-off timeouts
            if self.phase_sync:
                self._sync()
            trace.pop()
            t2 = time.perf_counter()
            mn = meta.numpy()  # (numpy: a handful of tiny host ops, cheaper than torch CPU tensors)
            results = mn[:, 1] > 0.5
            sizes = torch.from_numpy(mn[:, 2].copy())
            attackers = torch.from_numpy(mn[:, 3] > 0.5)
            round_ok = bool(results.all())
            # stored updates (arrival in client order; the reference stops storing after a failure)
            if not round_ok:
                stored = int(np.nonzero(~results)[0][0])
            snapshot = self.hyper.snapshot() if (self.mode == "hyper" and self.cfg.hyper_detection.get("enable")) \
                else None
            if esl is not None:  # (several ranks: the aggregate and the next launch are in already)
                info = self._early_info(round_ok)
                if not self._early_agg_done() and round_ok:
                    round_ok = False
                    info = {**self._early_agg_info, "agg_failed": True}
                if not round_ok:
                    self._early_launch_failed(esl, results)
            else:
                with trace.range("fl/aggregate"):
                    info = self._aggregate(U, sizes, attackers, round_ok)
                    if self.phase_sync:  # per-phase timings only; otherwise validation queues behind it
                        self._sync()
            if info.get("agg_failed"):
                round_ok = False
            t3 = time.perf_counter()
        self._round_meta = meta
        # ---- genuine pool for the next START (non-attacker rows stored this round; only attackers read it) ----
        if self._has_attackers and attackers is not None and esl is None:
            keep = [k for k in range(stored) if not bool(attackers[k])]
            self.genuine_pool = self._take_rows(U, keep) if keep else None  # (index_select: a new tensor)
            if (keep and keep[0] == 0 and round_ok and self.mode == "fedavg" and self.global_params is not None
                    and self.cfg.engine.get("compat-fedavg-alias", False)):
                # A-13: the reference averages INTO the first stored update's dict, which is also the first
                # genuine model in the pool (server.py:263-268,763): attackers may receive the aggregate
                self.genuine_pool[0] = self.global_params
        # Speculative next launch: the next round's local training is enqueued right behind the aggregate,
        # BEFORE this round's validation / checkpoint, which then run on a side stream next to it (the
        # trainer occupies a few CUs).  Valid whatever validation decides: a failed round is retried from the
        # same global model with the same client counters, i.e. exactly this launch.  Every rank decides
        # the same (replicated validation), so the ranks' launches and gathers stay in lockstep.
        vstream = None
        agg_done = None
        if esl is not None and self._spec is not None:
            agg_done = esl["agg_done"]
        elif self._speculative and round_ok and self.rounds_left > 1 and not last:
            if self.mode != "hyper":  # (test() falls back to the ordinary path if the model changes after this)
                self._prefetch_validation(self.global_params)
            agg_done = torch.cuda.Event()
            agg_done.record(torch.cuda.current_stream(self.device))
            self._spec = self._launch_local(self._genuine_for_attackers())
        if agg_done is not None:
            if self._val_stream is None:
                self._val_stream = torch.cuda.Stream(device=self.device)
            vstream = self._val_stream
            vstream.wait_event(agg_done)
            vstream.wait_event(self._start_ready)
        with (torch.cuda.stream(vstream) if vstream is not None else contextlib.nullcontext()):
            rec = self._finish_round(snapshot, info, round_ok, t0, t1, t2, t3)
        if vstream is not None:
            self.ckpt_writer.kick()  # the next launch is already in: copy + write while it trains
        return rec

    def _meta_read(self, cols: torch.Tensor):
        """Start the device -> host copy of the gathered meta columns; returns a callable that waits for THAT
        copy only (an event recorded right after it) and yields the fp64 host matrix."""
        if cols.device.type != "cuda":
            m = cols.double().cpu()
            return lambda: m
        buf = getattr(self, "_meta_pinned", None)
        if buf is None or buf.shape != cols.shape:
            buf = self._meta_pinned = torch.empty(cols.shape, dtype=torch.float32, pin_memory=True)
        buf.copy_(cols, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))

        def wait():
            ev.synchronize()
            return buf.double()  # (a copy: the pinned buffer is reused next round)
        return wait

    def _decision_word(self) -> int:
        """23-bit digest (exact in fp32) of the replicated server state every rank must agree on: the round
        counters (which encode every past round_ok) and the selected set (which encodes every removal)."""
        key = f"{self.round_no}|{self.rounds_left}|{','.join(map(str, self.selected))}".encode()
        return zlib.crc32(key) & 0x7FFFFF

    def _check_decisions(self, mn: np.ndarray, rank_words: np.ndarray = None) -> None:
        """Raise if the ranks' decision words differ: a rank's validation or detection decided otherwise (e.g.
        a mixed CPU / GPU gloo world whose kernels are not bit-identical), and continuing would desynchronise
        the collectives or silently diverge the replicated models.  ``rank_words``: one word per rank (its
        first slot row), so a rank without a selected, valid client is checked too (as the all-reduce path)."""
        valid = mn[:, 0] > 0.5
        words = mn[valid, DECISION]
        if rank_words is not None:
            words = np.concatenate([words, np.asarray(rank_words, dtype=words.dtype)])
        if words.size and not np.all(words == words[0]):
            raise RuntimeError(f"ranks disagree on the replicated server state (round {self.round_no}): decision "
                               f"words {sorted(set(int(w) for w in words))}; validation / detection must be "
                               "bit-identical on every rank (do not mix devices in one world)")

    def _fills_gpu(self) -> bool:
        """The training launch occupies every CU (the on-chip CNN trainer: 32 workgroups per client), so nothing
        queued beside it on another stream starts before it ends."""
        if self.device.type != "cuda" or getattr(self.trainer, "kind", "") != "graph" or self.model_name != "CNNModel":
            return False
        from .. import ops
        from ..parallel.launcher import gpu_sharers

        cus = torch.cuda.get_device_properties(self.device).multi_processor_count // gpu_sharers()
        return len(self.local) * int(ops.native().cnn2_wgs_per_client()) >= cus

    def _prefetch_validation(self, g: Optional[torch.Tensor]) -> None:
        """Ahead of a speculative launch that fills the GPU: this round's validation forward + AUC go in FIRST
        (stream order), so the host has its metric while the next training runs (Validation.prefetch)."""
        if g is not None and self.validation is not None and self._fills_gpu():
            self.validation.prefetch(g)

    def _early_ok(self, last: bool) -> bool:
        if self.mode == "hyper":
            mode_ok = self.device.type == "cuda" and self.hyper._native_ok()
        else:
            mode_ok = ((self.mode in ("fedavg", "FLTrust", "gmm") or self.mode in EARLY_AGGREGATORS)
                       and not (self.mode == "gmm" and len(self.selected) > 64) and not self.fast_fedavg
                       and self.global_params is not None
                       and not self.cfg.engine.get("compat-fedavg-alias", False))
        return self._speculative and mode_ok and self.rounds_left > 1 and not last

    def _early_launch(self, st: dict, last: bool, U: Optional[torch.Tensor] = None,
                      sel: Optional[torch.Tensor] = None) -> Optional[dict]:
        """FedAvg on one rank with plain rows: this round's aggregate and the NEXT round's launch are enqueued
        before the host waits for this round's training, so no host work separates two training kernels.
        The aggregate keeps the old global model on the device when a client failed (the host learns that
        after the wait), which makes the launch exactly this round's retry (same START, the next client
        draws); with attackers a failure discards it and restores the host state it consumed, because their
        genuine sample then comes from the stored prefix.  Returns None where the ordinary path runs."""
        if not self._early_ok(last):
            return None
        if sel is None:  # one rank, plain rows: called before _finish_local
            if not (self.world == 1 and st.get("plain") and st.get("fedavg_w") is not None):
                return None
            self._finish_attacks(st)
            if not all(ok for _, ok, _ in st["atk_out"]):
                return None
            n = len(self.selected)
            U = self.local_params[:n]
            ok_n = st["pending"].ok_device()[:n]
            ok_all = None if self.mode == "fedavg" else (ok_n > 0).all()  # (FedAvg: decided inside the aggregate)
            w = st["fedavg_w"]
            sizes = st["sizes_h"]
            attackers = torch.from_numpy(st["meta"][self._local_rows(), 3] > 0.5)
        else:  # several ranks: called on the gathered rows (device), before the host reads their meta
            P = self.P
            ok_n = None
            ok_all = ((sel[:, P] > 0.5) & (sel[:, P + 1] > 0.5)).all()
            s = sel[:, P + 2].double()
            w = s / s.sum()
            sizes = s
            attackers = sel[:, P + 3] > 0.5
        snap = ([(lc.rng.getstate(), lc.training_round, lc.genuine) for lc in self.local],
                self.server_rng.getstate(), self.genuine_pool)
        g_old, hyper_step, fl_old = self.global_params, None, None
        if self.mode == "hyper":  # the update runs, or leaves the hypernetwork untouched, as the device decides
            hyper_step = self.hyper.step
            self.ckpt_writer.fence()  # the previous round's checkpoint copy of the arena, updated in place below
            nxt = self._next_prep  # (staged ahead: its START models come out of the update's last launches)
            self.hyper.train(self.selected, {i: U[k] for k, i in enumerate(self.selected)},
                             enable=ok_all.to(torch.int32).reshape(1),
                             gen_key=[i for _, i, _, _ in nxt["clients"]] if nxt and nxt.get("clients") else None)
            g = g_old
        elif self.mode == "gmm":
            # the filter's success (some row kept) joins the clients' on the device; the host reads it after
            # its wait from a pinned copy queued BEFORE the next launch (run_round)
            params, ok_agg, self._early_agg_info = gmm_early(U, attackers, int(self.cfg.engine.get("gmm-rank", 1)))
            g = torch.where(ok_all & ok_agg, params, g_old)
            okh = torch.empty(1, dtype=torch.bool, pin_memory=True)
            okh.copy_(ok_agg.reshape(1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._early_agg_ok = (okh, ev)
        elif self.mode == "FLTrust":
            # the server model's training and the trust-weighted sum, all enqueued on the device (_fltrust); the
            # server model and the trust scores are rolled back if a client failed (_early_launch_failed)
            fl_old = self.fltrust_model
            g = torch.where(ok_all, self._fltrust(U), g_old)
        elif self.mode != "fedavg":
            # a robust rule, all on the device (no host read): its result kept only when every client succeeded
            res = AGGREGATORS[self.mode](U, sizes, attackers=None, seed=self.seed * 13 + self.round_no,
                                        gmm_rank=int(self.cfg.engine.get("gmm-rank", 1)))
            g = torch.where(ok_all, res.params.to(torch.float32), g_old)  # (a new tensor: never a row of U)
            self._early_agg_info = {k: v for k, v in res.info.items() if k != "scores"}
        else:
            if ok_n is not None and ok_n.dtype == torch.int32 and g_old is not None:
                g = ops.weighted_rows(U, w, ok_n, g_old)  # (the success check fused into the aggregate's pass)
            else:
                if ok_all is None:
                    ok_all = (ok_n > 0).all()
                g = torch.where(ok_all, ops.weighted_rows(U, w), g_old)
        keep = None
        if self._has_attackers:  # the pool of a fully stored round (before the next START overwrites U)
            keep = [k for k, i in enumerate(self.selected) if self.table[i].attack is None]
            self.genuine_pool = self._take_rows(U, keep) if keep else None  # (index_select: a new tensor)
        self.global_params = g
        if self.mode != "hyper":
            self._prefetch_validation(g)
        agg_done = torch.cuda.Event()
        agg_done.record(torch.cuda.current_stream(self.device))
        prep = self._next_prep  # (staged ahead: the snapshot above already includes its draws)
        self._spec = self._launch_local(self._genuine_for_attackers())
        return {"g_old": g_old, "snap": snap, "keep": keep, "pool": self.genuine_pool, "agg_done": agg_done,
                "prep": prep, "hyper_step": hyper_step, "fl_old": fl_old}

    def _early_info(self, round_ok: bool) -> dict:
        if not round_ok:
            return {}
        if self.mode == "hyper":
            return {"path": "early-launch", "_lazy": lambda: self.hyper.last_info}  # (as _aggregate)
        if self.mode == "FLTrust":
            return {"path": "early-launch"}  # (the trust scores join the record in _finish_round, as ever)
        if self.mode != "fedavg":
            return {**self._early_agg_info, "path": "early-launch"}
        return {"n": len(self.selected), "path": "early-launch"}

    def _early_agg_done(self) -> bool:
        """gmm's filter success of the early launch (True for every other rule): its pinned copy was queued before
        the next launch, so this waits for the filter only, not for the training queued behind it."""
        ok, self._early_agg_ok = self._early_agg_ok, None
        if ok is None:
            return True
        ok[1].synchronize()
        return bool(ok[0][0])

    def _early_launch_failed(self, esl: dict, results: np.ndarray) -> None:
        self.global_params = esl["g_old"]  # (the device selected the same values: the launch's START)
        if esl.get("fl_old") is not None:  # FLTrust: no server-model step and no trust scores for a failed round
            self.fltrust_model = esl["fl_old"]
            self._trust = None
            self._fl_pending = None
        if esl["hyper_step"] is not None:  # the device skipped the hypernetwork update: its step count too
            self.hyper.step = esl["hyper_step"]
            self.hyper._info_dev = None
        if esl["keep"] is None:
            return  # no attackers: the launch in flight is this round's retry
        # attackers sample the stored prefix's genuine rows: discard the launch, restore what it consumed
        # (every row is stored when only the aggregate failed: gmm kept no row)
        stored = int(np.nonzero(~results)[0][0]) if not results.all() else len(results)
        pos = [esl["keep"].index(k) for k in range(stored) if k in esl["keep"]]
        pool = esl["pool"][pos] if pos else None
        states, srng, _ = esl["snap"]
        for lc, (rs, tr, gen) in zip(self.local, states):
            lc.rng.setstate(rs)
            lc.training_round = tr
            lc.genuine = gen
        self.server_rng.setstate(srng)
        self._spec = None
        self._next_prep = esl["prep"]  # the launch's host half is reused as it was (same draws)
        self.genuine_pool = pool

    def _client_losses(self) -> Optional[List[Optional[List[float]]]]:
        """Per-epoch training loss of every selected client (None for attackers and failed clients), from
        the round's meta rows (host mirror on one rank, the gathered block's loss columns otherwise)."""
        meta = getattr(self, "_round_meta", None)
        if meta is None or meta.shape[1] < META + self.E:
            return None
        return [None if (meta[r, 3] > 0.5 or meta[r, 1] < 0.5)
                else [round(float(x), 6) for x in meta[r, META:META + self.E]] for r in range(len(self.selected))]

    def _finish_round(self, snapshot, info, round_ok, t0, t1, t2, t3) -> dict:
        trace.push("fl/validate")
        # ---- replicated detection + validation: every rank computes the same decision ----
        removed: List[int] = []
        metric = float("nan")
        # the reference validates len(all_model_parameters) generated models: the clients that reported this
        # round, counted before any removal (server.py:541)
        n_val = len(self.selected)
        if self.detector is not None:
            embs = {i: self.hyper.embedding(i).cpu().numpy()[None, :] for i in self.selected}
            removed = self.detector.step(self.round_no, self.selected, embs)
        if removed:
            # removal and rollback come BEFORE validation, so the logged metric and the round's success are
            # those of the rolled-back hypernetwork (server.py:532-543)
            for r in removed:
                if self.verbose:
                    print_with_color(f"Removing anomaly {r}, rolling back", "yellow")
                if r in self.selected:
                    self.selected.remove(r)
            self.hyper.restore(snapshot)
        if self.validation is not None and round_ok:
            if self.mode == "hyper":
                round_ok, metric = self.validation.test_hyper(self.hyper, n_val)
            else:
                if self.global_params is None:
                    round_ok = False
                else:
                    round_ok, metric = self.validation.test(self.global_params)
        trace.pop()
        fl_pending, self._fl_pending = getattr(self, "_fl_pending", None), None
        if fl_pending is not None:
            fl_pending.result()  # (FLTrust's root training: finished by now; raises on a hand-off timeout)
        t4 = time.perf_counter()
        if round_ok:
            with trace.range("fl/checkpoint"):
                self.save_checkpoint()
                self.rounds_left -= 1
                if self.cfg.engine.get("save-state", False):
                    self.round_no += 1
                    self.save_state()
                    self.round_no -= 1
        elif self.verbose:
            print_with_color("Training failed!", "yellow")
        t5 = time.perf_counter()
        rec = {"round": self.round_no, "ok": round_ok, "metric": metric, **getattr(self, "_lw_times", {}),
               "t_local": t1 - t0, "t_gather": t2 - t1,
               "t_aggregate": t3 - t2, "t_validate": t4 - t3, "t_checkpoint": t5 - t4, "t_round": t5 - t0,
               "n_selected": len(self.selected), "removed": removed}
        if self._attack_info:
            # every tried γ and its accept decision, not just the last one (the reference prints each γ)
            rec["attack"] = {k: v for k, v in host_info(self._attack_info).items() if isinstance(v, (int, float, list))}
        lazy = info.pop("_lazy", None)
        if lazy is not None:
            info.update(lazy())
        info = agg_host_info(info)  # (device-resident aggregator outputs: read now, after validation)
        if self._trust is not None:
            info["trust"] = [round(float(x), 6) for x in self._trust.tolist()]
        rec.update({k: v for k, v in info.items() if isinstance(v, (int, float, list, str))})
        losses = self._client_losses()
        if losses is not None:
            rec["client_loss"] = losses
            if self.verbose:
                self._print_losses(losses)
        self.metrics.write(rec)
        self.history.append(rec)
        if round_ok:
            self.round_no += 1
        return rec

    def _print_losses(self, losses) -> None:
        """Reference client prints (``client.py:109`` ICU: ``Loss {mean}`` per epoch; ``client.py:130`` HAR:
        ``Epoch {e}, Loss: {sum:.4f}``), one block per client, from the server's view of the round."""
        for i, ls in zip(self.selected, losses):
            if ls is None:
                continue
            if self.data_name == "HAR":
                nb = max(1, -(-int(self._round_meta[self.selected.index(i), 2]) // self.cfg.batch_size))
                for e, l in enumerate(ls):
                    print(f"[client {i}] Epoch {e + 1}, Loss: {l * nb:.4f}")
            else:
                for l in ls:
                    print_with_color(f"[client {i}] Loss {l} ", "yellow")

    def _fedavg_allreduce(self, block: torch.Tensor):
        """FedAvg over one all_reduce: [sum s_i w_i | sum s_i | #failed | #reported] (fp64).  Returns
        (round ok, host meta of this rank's rows); sets ``global_params`` on success."""
        P = self.P
        present = block[:, P] > 0.5
        size = torch.where(present, block[:, P + 2], torch.zeros_like(block[:, P + 2])).double()
        red = torch.zeros(P + 5, dtype=torch.float64, device=block.device)
        red[:P] = (size[:, None] * block[:, :P].double()).sum(0)
        red[P] = size.sum()
        red[P + 1] = (present & (block[:, P + 1] < 0.5)).double().sum()
        red[P + 2] = present.double().sum()
        # decision words: all equal iff n * sum(w^2) == (sum w)^2 (exact in fp64 for 23-bit words)
        word = float(self._decision_word())
        red[P + 3] = word
        red[P + 4] = word * word
        with trace.range("fl/allreduce"):
            if self.world > 1:
                self.comm.all_reduce_(red)
            if self.phase_sync:
                self._sync()
        fl = red[P + 1:P + 5].cpu()  # one device -> host read for the counters (waits for the reduce)
        if float(fl[2]) ** 2 != self.world * float(fl[3]):
            raise RuntimeError(f"ranks disagree on the replicated server state (round {self.round_no}); "
                               "validation / detection must be bit-identical on every rank")
        round_ok = int(fl[0]) == 0 and int(fl[1]) == len(self.selected)
        if round_ok:
            self.global_params = (red[:P] / red[P]).to(torch.float32)
        # per-client meta (losses for the JSONL): only a single rank knows every row without another read
        meta = torch.from_numpy(self._meta_host[self._local_rows()]) if self.world == 1 else None
        return round_ok, meta

    def _slot_of(self, i: int) -> int:
        owner = self.table[i].owner
        return sum(1 for c in self.table[:i] if c.owner == owner)

    def run(self, max_rounds: Optional[int] = None) -> List[dict]:
        if not self.selected:
            self.client_selection()
        fails = 0
        done = 0
        while self.rounds_left > 0:
            # the caller's last round launches nothing speculatively (no un-aggregated extra training)
            rec = self.run_round(last=max_rounds is not None and done + 1 >= max_rounds)
            done += 1
            fails = 0 if rec["ok"] else fails + 1
            if self.max_retries and fails > self.max_retries:
                raise RuntimeError(f"round {self.round_no} failed {fails} times in a row")
            if max_rounds is not None and done >= max_rounds:
                break
        if self.verbose and self.rounds_left <= 0:
            print_with_color("Training finished, stopping clients.", "green")
        self.ckpt_writer.flush()
        return self.history

    def close(self):
        if getattr(self, "_closed", False):
            return
        self._closed = True
        if self._spec is not None:
            # a speculative launch nobody consumed (bench.py drives run_round itself): wait for the GPU work,
            # skip the block / meta bookkeeping.  Client state (local_params, training_round, client RNGs) is
            # then one round ahead of history / round_no.
            st, self._spec = self._spec, None
            if st["pending"] is not None:
                st["pending"].result()
            self._sync()
        self.ckpt_writer.close()
        self.metrics.close()
        if hasattr(self.logger, "close"):
            self.logger.close()
