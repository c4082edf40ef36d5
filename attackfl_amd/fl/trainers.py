"""Client local training.

Semantics follow the reference trainers (``client.py:66-131``):
* fresh ``Adam(lr)`` (β=(0.9, 0.999), eps 1e-8) every round, ``momentum`` unused (A-19);
* ICU: ``BCELoss`` on sigmoid outputs, batches of size 1 skipped (A-21), a NaN loss aborts the
  client's round with ``result=False``; ``clip_grad_norm_`` is called before ``backward`` in the
  reference and therefore never clips (A-4) — we do not clip either;
* HAR: ``CrossEntropyLoss``;
* data: each round the client draws ``num_data`` rows without replacement from the shared
  train set (A-20) and visits them in a fresh random order each epoch (``DataLoader(shuffle=True)``).

Two implementations share one sampling plan (``make_plan``), so they see identical batches:
* ``EagerTrainer``  — PyTorch modules + ``torch.optim.Adam`` (the CPU path and the oracle);
* ``FusedTrainer``  — ONE persistent HIP kernel launch trains all of a rank's clients for all
  their local epochs (one workgroup per client, weights/activations in LDS, Adam state in
  registers) — ``ops/transformer.py``.  TransformerModel/ICU on gfx950.
* ``GraphTrainer``  — client-batched layer programs (``fl/programs.py``: CNNModel, RNNModel,
  TransformerClassifier/HAR) whose optimizer step is captured once into a HIP graph and replayed.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import time

import torch

from ..data import DeviceTable
from ..models import ParamLayout, build_model
from ..utils.log import print_with_color


@dataclass
class Plan:
    """Visit order of train rows for C clients: ``order [C, E, maxnd]`` int32 (+ ``nd [C]``)."""

    order: torch.Tensor
    nd: torch.Tensor
    epochs: int
    nd_dev: Optional[torch.Tensor] = None  # nd on the order's device, when the plan was built there

    def client(self, c: int) -> torch.Tensor:
        return self.order[c, :, : int(self.nd[c])]


class Pending:
    """A launched local-training job: ``result()`` synchronises and returns (ok per client, losses [C, E]).

    Trainers whose work is enqueued asynchronously (fused, graph) return before the GPU finishes, so the
    engine can run the attackers' math on a side stream while the genuine clients train."""

    def __init__(self, finish, ok_dev: Optional[torch.Tensor] = None, losses_dev: Optional[torch.Tensor] = None):
        self._finish = finish
        self._res = None
        self._ok_dev = ok_dev
        self._losses_dev = losses_dev

    def ok_device(self) -> Optional[torch.Tensor]:
        """Per-client success on the device (> 0 = ok) without a host round trip, when the trainer has it."""
        return self._ok_dev

    def losses_device(self) -> Optional[torch.Tensor]:
        """Per-client per-epoch mean losses ``[C, E]`` on the device, when the trainer has them."""
        return self._losses_dev

    def result(self) -> Tuple[List[bool], torch.Tensor]:
        if self._res is None:
            self._res = self._finish()
            self._finish = None
        return self._res


_M32 = 0xFFFFFFFF


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    """(x * c) mod 2^32 for int64 tensors holding uint32 values (no int64 overflow)."""
    return (x * (c & 0xFFFF) + (((x * (c >> 16)) & 0xFFFF) << 16)) & _M32


def _mix_t(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = _mul32(x, 0x85EBCA6B)
    x = x ^ (x >> 13)
    x = _mul32(x, 0xC2B2AE35)
    return x ^ (x >> 16)


def _mix_i(x: int) -> int:
    x &= _M32
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & _M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & _M32
    return x ^ (x >> 16)


def _half_bits(n: int) -> int:
    k = 2
    while (1 << k) < n:
        k += 2
    return k // 2


def _perm_t(x: torch.Tensor, n: int, k0: int, k1: int) -> torch.Tensor:
    """Keyed 6-round Feistel permutation of [0, n) with cycle walking (mirror of plan.hip:pl_perm)."""
    half = _half_bits(n)
    mask = (1 << half) - 1

    def feistel(v):
        L, R = v >> half, v & mask
        for r in range(6):
            F = _mix_t(R ^ k0 ^ ((k1 + 0x9E3779B9 * (r + 1)) & _M32)) & mask
            L, R = R, L ^ F
        return (L << half) | R

    x = feistel(x)
    while True:
        bad = x >= n
        if not bool(bad.any()):
            return x
        x = torch.where(bad, feistel(x), x)


def _plan_keys(seed: int, e: int):
    lo, hi = seed & _M32, (seed >> 32) & _M32
    ks0, ks1 = _mix_i(lo ^ 0x5BD1E995), _mix_i(hi ^ 0x27D4EB2F)
    ke0 = _mix_i(ks0 ^ ((0x165667B1 * (e + 1)) & _M32))
    ke1 = _mix_i((ks1 + 0xD3A2646C * (e + 1)) & _M32)
    return ks0, ks1, ke0, ke1


def _feistel_plan(n_train: int, num_data: List[int], epochs: int, seeds: List[int], device, staged=None) -> Plan:
    """Per-client subset + per-epoch shuffle from keyed Feistel permutations (``csrc/kernels/plan.hip``):
    one launch on GPU, a bit-identical vectorised mirror on CPU.  A client's plan depends only on its
    seed and num_data (placement-independent).  ``staged``: (seeds int64, num_data int32) already on the
    device (the engine uploads them with the rest of the round's metadata)."""
    dev = torch.device(device)
    C = len(num_data)
    maxnd = max(num_data)
    seeds = [s & 0xFFFFFFFFFFFFFFFF for s in seeds]
    nd = torch.tensor(num_data, dtype=torch.int32)
    if dev.type == "cuda":
        from .. import ops

        if staged is not None:
            st_d, nd_d = staged
        else:
            st_d = torch.tensor([s - (1 << 64) if s >= (1 << 63) else s for s in seeds], dtype=torch.int64).to(dev)
            nd_d = nd.to(dev)
        order = ops.native().make_plan(st_d, nd_d, int(n_train), int(epochs), int(maxnd))
        return Plan(order, nd, epochs, nd_d)
    order = torch.zeros(C, epochs, maxnd, dtype=torch.int64)
    for c in range(C):
        n = num_data[c]
        i = torch.arange(n, dtype=torch.int64)
        for e in range(epochs):
            ks0, ks1, ke0, ke1 = _plan_keys(seeds[c], e)
            order[c, e, :n] = _perm_t(_perm_t(i, n, ke0, ke1), n_train, ks0, ks1)
    return Plan(order.to(torch.int32).to(dev), nd, epochs)


def make_plan(n_train: int, num_data: Sequence[int], epochs: int, generator, device, staged=None) -> Plan:
    """Random subset (without replacement) per client + a fresh permutation per epoch.

    ``generator`` is one ``torch.Generator`` shared by all rows, or a list of per-client integer seeds
    (placement-independent: a client draws the same batches whichever rank hosts it).  The random keys
    are drawn on ``device`` and sorted with two batched argsorts (no per-client sort loops)."""
    C = len(num_data)
    if C == 0:
        return Plan(torch.zeros(0, epochs, 0, dtype=torch.int32, device=device), torch.zeros(0, dtype=torch.int32),
                    epochs)
    maxnd = max(num_data)
    if maxnd > n_train:
        raise ValueError(f"num_data {maxnd} exceeds the train set size {n_train}")
    if isinstance(generator, (list, tuple)):
        return _feistel_plan(n_train, list(num_data), epochs, [int(s) for s in generator], device, staged)
    gdev = generator.device if hasattr(generator, "device") else torch.device("cpu")
    keys = torch.rand(C, n_train, generator=generator, device=gdev)
    ek = None
    subset = torch.argsort(keys, dim=1)[:, :maxnd]                              # [C, maxnd]
    if ek is None:
        ek = torch.rand(C, epochs, maxnd, generator=generator, device=gdev)
    nd = torch.tensor(list(num_data), dtype=torch.long, device=gdev)
    pad = torch.arange(maxnd, device=gdev)[None, None, :] >= nd[:, None, None]
    ek = ek.masked_fill(pad, 2.0)                                               # padding sorts last
    perm = torch.argsort(ek, dim=2)                                             # [C, E, maxnd]
    order = torch.gather(subset[:, None, :].expand(C, epochs, maxnd), 2, perm)
    return Plan(order.to(device=device, dtype=torch.int32).contiguous(), nd.to(torch.int32).cpu(), epochs)


def batches(nd: int, batch: int, skip_single: bool = True):
    """(start, end) of each batch of one epoch; size-1 batches are skipped (A-21) unless ``skip_single``
    is False (the reference ``train_HAR`` loop)."""
    for a in range(0, nd, batch):
        b = min(nd, a + batch)
        if b - a == 1 and skip_single:
            continue
        yield a, b


def bce_loss(p: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``BCELoss`` (mean, log clamped at -100, torch's finite gradient at a saturated sigmoid) without the
    input-range check, so a NaN output reaches the NaN test (``client.py:100-102``) instead of raising
    inside the loss (``ops.composite.bce_loss``)."""
    from ..ops.composite import bce_loss as _bce

    return _bce(p, y)


class EagerTrainer:
    """Reference-semantics trainer on PyTorch modules (CPU oracle / fallback)."""

    kind = "eager"

    def __init__(self, model_name: str, data_name: str, table: DeviceTable, device, verbose: bool = False):
        self.model_name = model_name
        self.data_name = data_name
        self.table = table
        self.device = torch.device(device)
        self.model = build_model(model_name, seed=0).to(self.device)
        self.layout = ParamLayout.from_state_dict(self.model.state_dict())
        self.verbose = verbose
        self.compat_har = False  # engine.compat-har-train: reference train_HAR (no size-1 skip, no NaN abort)

    def train(self, params: torch.Tensor, plan: Plan, lr: float, batch: int, seeds: Sequence[int]
              ) -> Tuple[List[bool], torch.Tensor]:
        """Train every row of ``params`` [C, P] in place.  Returns (ok per client, losses [C, E])."""
        C = params.shape[0]
        losses = torch.zeros(C, plan.epochs, dtype=torch.float64)
        oks: List[bool] = []
        for c in range(C):
            torch.manual_seed(int(seeds[c]))  # dropout masks
            sd = self.layout.unflatten(params[c].to(self.device), clone=True)
            self.model.load_state_dict(sd)
            ok = self._train_one(plan.client(c), lr, batch, losses[c])
            with torch.no_grad():
                params[c].copy_(self.layout.flatten(self.model.state_dict(), device=params.device))
            oks.append(ok)
        return oks, losses

    def launch(self, params, plan, lr, batch, seeds, seeds_dev=None) -> Pending:
        res = self.train(params, plan, lr, batch, seeds)
        return Pending(lambda: res)

    def _train_one(self, order: torch.Tensor, lr: float, batch: int, loss_out: torch.Tensor) -> bool:
        model = self.model
        model.train()
        opt = torch.optim.Adam(model.parameters(), lr=lr)
        if self.data_name == "ICU":
            crit = bce_loss
        elif self.table.kind == "IMAGE":
            # the reference has no image trainer; its image validation scores log-probabilities with
            # nll_loss (src/Validation.py:80-82), so image models are trained on the same objective
            crit = torch.nn.NLLLoss()
        else:
            crit = torch.nn.CrossEntropyLoss()
        nd = order.shape[1]
        nbatches = max(1, (nd + batch - 1) // batch)
        har_compat = self.compat_har and self.data_name == "HAR"
        for e in range(order.shape[0]):
            total = torch.zeros((), dtype=torch.float64, device=self.device)
            for a, b in batches(nd, batch, skip_single=not har_compat):
                idx = order[e, a:b].long()
                opt.zero_grad()
                if self.data_name == "ICU":
                    v, l, y = self.table.icu_batch(idx)
                    out = model(v, l)
                    loss = crit(out, y[:, None])
                elif self.table.kind == "IMAGE":
                    x, y = self.table.image_batch(idx)
                    loss = crit(model(x), y)
                else:
                    x, y = self.table.har_batch(idx)
                    loss = crit(model(x), y)
                if not har_compat and bool(torch.isnan(loss).any()):
                    print_with_color("NaN detected in loss, stop training", "yellow")
                    return False
                total += loss.detach().double()
                loss.backward()
                opt.step()
            loss_out[e] = float(total.item()) / nbatches
            if self.verbose:
                print_with_color(f"Loss {float(loss_out[e]):.6f} ", "yellow")
        return True


_RB_STREAMS: dict = {}  # device -> the shared read-back stream (FusedTrainer._readback)


def _nd(plan: Plan):
    return plan.nd_dev if plan.nd_dev is not None else plan.nd


class FusedTrainer:
    """All local clients' local rounds in one persistent HIP launch: TransformerModel/ICU
    (``ops/transformer.py``) and RNNModel/ICU (``ops/rnn.py``, falls back to the graph trainer when
    its 3 workgroups per client do not all fit on the device)."""

    kind = "fused"
    MODELS = ("TransformerModel", "RNNModel")

    def __init__(self, model_name: str, data_name: str, table: DeviceTable, device, verbose: bool = False):
        if model_name not in self.MODELS or data_name != "ICU":
            raise ValueError("fused trainer supports TransformerModel/ICU and RNNModel/ICU")
        if torch.device(device).type != "cuda":
            raise ValueError("fused trainer needs a GPU")
        from ..ops import rnn as R
        from ..ops import transformer as T

        self.model_name = model_name
        self.T, self.R = T, R
        self.table = table
        self.device = torch.device(device)
        self.layout = ParamLayout.for_model(model_name)
        self.verbose = verbose
        self._fallback = None

    def train(self, params: torch.Tensor, plan: Plan, lr: float, batch: int, seeds: Sequence[int]
              ) -> Tuple[List[bool], torch.Tensor]:
        return self.launch(params, plan, lr, batch, seeds).result()

    def device_seed(self, s: int) -> int:
        """The kernel's int32 form of client seed ``s`` (the engine stages these on the device)."""
        return (self.R if self.model_name == "RNNModel" else self.T).device_seed(s)

    def launch(self, params: torch.Tensor, plan: Plan, lr: float, batch: int, seeds: Sequence[int],
               seeds_dev: Optional[torch.Tensor] = None) -> Pending:
        """``seeds_dev``: the same seeds already on the device in ``device_seed`` form (optional)."""
        if self.model_name == "RNNModel":
            if not self.R.fits(params.shape[0], self.device):
                if self._fallback is None:
                    self._fallback = GraphTrainer(self.model_name, "ICU", self.table, self.device, self.verbose)
                return self._fallback.launch(params, plan, lr, batch, seeds)
            ok, losses = self.R.train_clients_async(params, self.table.rows, plan.order, _nd(plan), plan.epochs, batch,
                                                    lr, seeds if seeds_dev is None else seeds_dev)
            what = "fused RNN trainer"
        else:
            ok, losses = self.T.train_clients_async(params, self.table.rows, plan.order, _nd(plan), plan.epochs, batch,
                                                    lr, seeds if seeds_dev is None else seeds_dev)
            what = "fused trainer"

        # ok + losses come back in ONE asynchronous copy into a pinned buffer, and result() waits on an event
        # (two blocking .cpu() reads cost two host round trips between the round's training and its aggregate)
        C, E = losses.shape
        buf = self._pinned(C, E)
        done = self._readback(ok, losses, buf)

        def fin():
            # poll instead of a blocking wait: the host then wakes within microseconds of the launch's end
            # (a blocking event wait sleeps on an interrupt); sleep(0) lets the checkpoint thread run
            while not done.query():
                time.sleep(0)
            okh = buf[:, 0].to(torch.int32)
            if bool((okh < 0).any()):
                raise RuntimeError(f"{what}: a cross-workgroup hand-off timed out (workgroups not co-resident?)")
            return [bool(x) for x in okh.tolist()], buf[:, 1:].clone()

        return Pending(fin, ok, losses)

    def _readback(self, ok: torch.Tensor, losses: torch.Tensor, buf: torch.Tensor) -> torch.cuda.Event:
        """Enqueue the result copy; returns its event.  When the launch leaves most CUs free (the on-chip trainers
        at a few clients per rank) the copy goes on a read-back stream that waits for the training: the compute
        stream then runs the round's aggregate and the next launch right away instead of three small kernels
        later.  A launch that fills the GPU keeps the copy on the compute stream (on another stream the copy
        could wait behind the NEXT launch's persistent workgroups)."""
        dev = self.device
        main = torch.cuda.current_stream(dev)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        side = 3 * ok.shape[0] * 2 <= cus
        if side:
            # ONE read-back stream per device for every trainer (FLTrust's server-model trainer too): a stream
            # waiting for a training blocks the hardware queue it is mapped to (GPU_MAX_HW_QUEUES = 4), and one
            # more stream moved the attack's side stream onto that queue, behind the wait (FLTrust + Min-Max: the
            # attack math started only after the clients' training, -10 %)
            rs = _RB_STREAMS.get(dev)
            if rs is None:
                rs = _RB_STREAMS[dev] = torch.cuda.Stream(device=dev)
            trained = torch.cuda.Event()
            trained.record(main)
            rs.wait_event(trained)
            ok.record_stream(rs)
            losses.record_stream(rs)
        else:
            rs = main
        with torch.cuda.stream(rs):
            buf.copy_(torch.cat([ok.to(torch.float32)[:, None], losses], 1), non_blocking=True)
            done = torch.cuda.Event()
            done.record(rs)
        return done

    def _pinned(self, C: int, E: int) -> torch.Tensor:
        """Pinned [C, 1 + E] result buffers, a ring of 3 (a launch's result is read before the launch after
        next is enqueued: at most two are in flight)."""
        ring = getattr(self, "_pin_ring", None)
        if ring is None or ring[0][0].shape != (C, 1 + E):
            ring = self._pin_ring = ([torch.empty(C, 1 + E, dtype=torch.float32, pin_memory=True) for _ in range(3)], [0])
        bufs, k = ring
        k[0] = (k[0] + 1) % len(bufs)
        return bufs[k[0]]


class OracleTrainer:
    """CPU twin of the fused TransformerModel trainer: ``ops.transformer.reference_train`` (fp32 autograd with
    the kernel's own hash dropout masks and Adam step sequence), so a CPU run follows the same client
    trajectories as the GPU run up to bf16-vs-fp32 rounding (the attack study compares the two)."""

    kind = "oracle"

    def __init__(self, model_name: str, data_name: str, table: DeviceTable, device, verbose: bool = False):
        if model_name != "TransformerModel" or data_name != "ICU":
            raise ValueError("oracle trainer: TransformerModel/ICU")
        from ..ops import transformer as T

        self.T = T
        self.table = table
        self.device = torch.device(device)
        self.verbose = verbose

    def train(self, params, plan, lr, batch, seeds):
        return self.launch(params, plan, lr, batch, seeds).result()

    def launch(self, params, plan, lr, batch, seeds, seeds_dev=None) -> Pending:
        p = params.detach().cpu().contiguous()
        ok, losses = self.T.reference_train(p, self.table.rows.cpu(), plan.order.cpu(), plan.nd, plan.epochs, batch,
                                            lr, [int(s) for s in seeds])
        params.copy_(p.to(params.device))
        res = ([bool(x) for x in ok.tolist()], losses.double())
        return Pending(lambda: res)


class GraphTrainer:
    """All local clients batched through a layer program; one HIP-graph replay per optimizer step."""

    kind = "graph"

    def __init__(self, model_name: str, data_name: str, table: DeviceTable, device, verbose: bool = False):
        from . import programs

        if model_name not in programs.PROGRAMS:
            raise ValueError(f"graph trainer supports {sorted(programs.PROGRAMS)}")
        if table.kind == "IMAGE":
            raise ValueError("graph trainer programs take ICU rows / HAR sequences; train image models eagerly")
        self.programs = programs
        self.model_name = model_name
        self.table = table
        self.device = torch.device(device)
        self.layout = ParamLayout.for_model(model_name)
        self.verbose = verbose
        self._runner = None
        self.compat_har = False  # engine.compat-har-train (HAR data only)

    def train(self, params: torch.Tensor, plan: Plan, lr: float, batch: int, seeds: Sequence[int]
              ) -> Tuple[List[bool], torch.Tensor]:
        return self.launch(params, plan, lr, batch, seeds).result()

    def launch(self, params: torch.Tensor, plan: Plan, lr: float, batch: int, seeds: Sequence[int],
               seeds_dev=None) -> Pending:
        C = params.shape[0]
        if self._runner is None or self._runner.prog.C != C or self._runner.prog.B != batch:
            self._runner = self.programs.ProgramRunner(
                self.programs.make_program(self.model_name, C, batch, self.device, train=True))
        ok, losses = self._runner.train(self.table, params, plan, lr, seeds, sync=False,
                                        compat_har=self.compat_har and self.table.kind == "HAR")
        if ok.is_cuda:
            # failed counts + losses come back in ONE asynchronous copy into a pinned buffer queued right behind
            # this launch, and fin() waits on its event: a .cpu() read in fin() went on the stream BEHIND the
            # speculative next launch enqueued meanwhile, so the host waited for that whole training too and
            # enqueued the round after it late (cnn2, which fills the GPU: ~1-2 ms idle per round)
            C, E = losses.shape
            buf = FusedTrainer._pinned(self, C, E)
            buf.copy_(torch.cat([ok.to(torch.float32)[:, None], losses], 1), non_blocking=True)
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.device))

            def host():
                while not done.query():
                    time.sleep(0)
                return buf[:, 0].to(torch.int32), buf[:, 1:].double()
        else:
            def host():
                return ok.cpu(), losses.double().cpu()

        def fin():
            fh, lh = host()
            if bool((fh == 2).any()):
                raise RuntimeError(self.programs.CNN2_TIMEOUT)
            okh = fh == 0
            if self.verbose:
                for c in range(C):
                    for e in range(plan.epochs):
                        print_with_color(f"Loss {float(lh[c, e]):.6f} ", "yellow")
            return [bool(x) for x in okh.tolist()], lh

        return Pending(fin, (ok == 0).to(torch.int32), losses)


def make_trainer(kind: str, model_name: str, data_name: str, table: DeviceTable, device, verbose=False):
    from .programs import PROGRAMS

    dev = torch.device(device)
    if kind == "auto":
        if dev.type != "cuda":
            kind = "eager"
        elif model_name in FusedTrainer.MODELS and data_name == "ICU":
            kind = "fused"
        elif model_name in PROGRAMS and data_name != "CIFAR10":
            kind = "graph"
        else:
            kind = "eager"
    if kind == "fused":
        return FusedTrainer(model_name, data_name, table, device, verbose)
    if kind == "oracle":
        return OracleTrainer(model_name, data_name, table, device, verbose)
    if kind == "graph":
        return GraphTrainer(model_name, data_name, table, device, verbose)
    return EagerTrainer(model_name, data_name, table, device, verbose)
