"""Process launch / rendezvous (replaces the RabbitMQ REGISTER handshake, ``server.py:205-235``,
``client.py:134-143``, and the broker queue janitor ``server.py:803-835``).

Two ways to start a run:

* **classic** — ``python server.py`` plus N x ``python client.py [--attack ...]``, exactly like the
  reference.  The server opens a TCPStore at ``comm.address`` (default: ``rabbit.address``) and waits
  for ``server.clients`` registrations; every client claims the next rank with an atomic counter and
  publishes its descriptor (uuid + attack flags + device).  Registration order defines the client index
  like the reference's ``list_clients``.  The N CLIENTS then form the ``torch.distributed`` group (client
  r = group rank r - 1, one client per rank: the packed layout with one client per process) and run the
  SPMD engine; server state is replicated on every client rank, and group rank 0 is the leader that writes
  ``app.log`` and the ``.pth`` checkpoints into the server's ``log_path`` / checkpoint directory.  The
  server process holds the store and the client table, echoes the leader's ``app.log`` to its console and
  exits when the leader reports the run done (``serve_until_done``) — it computes nothing, so it needs no
  GPU and is not in the device group: 8 clients on an 8-GPU node are 8 ranks on 8 distinct GPUs (RCCL).
  A fresh store per run plays the role of the queue janitor.
* **packed** — ``torchrun --nproc-per-node G launch.py`` (or ``bench.py``): one process per GPU, the
  ``server.clients`` clients packed N/G per rank, server state replicated on every rank.
"""
from __future__ import annotations

import datetime
import json
import time
import uuid
from typing import Dict, List, Optional, Tuple

import torch.distributed as dist

from ..config import AttackSpec, Config
from ..utils.log import print_with_color

PREFIX = "attackfl/"


def _host_port(cfg: Config) -> Tuple[str, int]:
    host = cfg.comm.get("address") or cfg.raw["rabbit"]["address"] or "127.0.0.1"
    return str(host), int(cfg.comm.get("port", 29517))


def gpu_key(index: int) -> str:
    """Physical identity of visible GPU ``index``, the same in every process whatever its device ordinals
    (HIP_VISIBLE_DEVICES narrowing renumbers them): the UUID, else the PCI location, else (last resort, per
    process) the ordinal."""
    import torch

    props = torch.cuda.get_device_properties(index)
    u = str(getattr(props, "uuid", "") or "")
    if u.strip("0-"):
        return "uuid:" + u
    bus = getattr(props, "pci_bus_id", None)
    if bus is not None:
        return f"pci:{getattr(props, 'pci_domain_id', 0)}:{bus}:{getattr(props, 'pci_device_id', 0)}"
    return f"ord:{index}"


def local_gpu_keys() -> Dict[str, int]:
    """gpu_key -> this process's ordinal, for every visible GPU."""
    import torch

    if not torch.cuda.is_available():
        return {}
    return {gpu_key(i): i for i in range(torch.cuda.device_count())}


def device_descriptor(device) -> Dict:
    """Where this process computes: host + physical GPU identity (``gpu_key``), so the server can tell whether
    every rank owns its own GPU (RCCL) or some share one (gloo + IPC)."""
    import socket

    import torch

    d = {"host": socket.gethostname(), "type": getattr(device, "type", "cpu"), "gpu": None}
    if d["type"] == "cuda" and torch.cuda.is_available():
        idx = device.index if device.index is not None else torch.cuda.current_device()
        d["gpu"] = gpu_key(idx)
    return d


def client_device(arg: Optional[str], rank: int, ndev: int) -> str:
    """Device of classic client ``rank`` (1..N, registration order).  An explicit ``--device cuda:i`` / ``cpu``
    wins; ``--device cuda`` or none puts client r on GPU ``(r - 1) % ndev`` — one FL client per MI355X (the
    server computes nothing and takes no GPU), round robin beyond ``ndev`` clients.  Reference: client.py:50-61
    (cuda if available)."""
    if arg and arg != "cuda":
        return arg
    if ndev <= 0:
        return arg or "cpu"
    return f"cuda:{(rank - 1) % ndev}"


def sync_gpu_sharers(device) -> int:
    """Collective (after ``init_process_group``): count the processes of the group on each physical GPU (by
    ``gpu_key``, so ranks whose visibility was narrowed to 'their' GPU are told apart) and record the count of
    THIS process's GPU as its co-residency budget (a rank that owns its GPU keeps the whole chip even when other
    ranks share one).  Returns it."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return gpu_sharers()
    descs: List[Dict] = [None] * dist.get_world_size()  # type: ignore[list-item]
    mine = device_descriptor(device)
    dist.all_gather_object(descs, mine)
    n = sharers_of(descs, mine)
    set_gpu_sharers(n)
    return n


_SHARERS: Optional[int] = None


def set_gpu_sharers(n: int) -> None:
    """Record how many processes of this run compute on this process's GPU (the classic launch learns it from
    the registered device descriptors, ``serve_rendezvous``)."""
    global _SHARERS
    _SHARERS = max(1, int(n))


def gpu_sharers() -> int:
    """Processes of this run sharing this process's GPU.  Kernels that need all their workgroups co-resident
    (the on-chip trainers spin on each other's counters) size themselves to ``CUs // gpu_sharers()``, because
    the other processes' persistent launches occupy CUs too.  Sources, in order: ``set_gpu_sharers``,
    ``AFL_GPU_SHARERS``, a packed launch with every rank pinned to one GPU (``AFL_BENCH_DEVICE`` or the
    ``AFL_SHARED_GPU`` flag launch.py sets: all local ranks), otherwise local ranks per visible GPU."""
    import os

    if _SHARERS is not None:
        return _SHARERS
    env = os.environ.get("AFL_GPU_SHARERS")
    if env:
        return max(1, int(env))
    local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")) or 1)
    if os.environ.get("AFL_BENCH_DEVICE") is not None or os.environ.get("AFL_SHARED_GPU") == "1":
        return max(1, local)
    # no explicit information: assume one process per GPU.  (Guessing local ranks / visible GPUs over-counts
    # when each rank sees only its own GPU; multi-process launches call sync_gpu_sharers, which counts the
    # processes per physical GPU.)
    return 1


def _gpu_counts(descs: List[Dict]) -> Dict[Tuple, int]:
    cnt: Dict[Tuple, int] = {}
    for d in descs:
        if d.get("type") == "cuda":
            k = (d.get("host"), d.get("gpu"))
            cnt[k] = cnt.get(k, 0) + 1
    return cnt


def max_sharers(descs: List[Dict]) -> int:
    """Largest number of registered processes on one physical GPU (1 when none shares)."""
    cnt = _gpu_counts(descs)
    return max(cnt.values()) if cnt else 1


def sharers_of(descs: List[Dict], mine: Dict) -> int:
    """Processes of ``descs`` on the physical GPU of descriptor ``mine`` (1 for a CPU process)."""
    if mine.get("type") != "cuda":
        return 1
    return max(1, _gpu_counts(descs).get((mine.get("host"), mine.get("gpu")), 1))


def choose_backend(descs: List[Dict]) -> Tuple[str, bool]:
    """(process-group backend, one-shot IPC) for the classic launch's client group: RCCL when every client owns
    a distinct GPU; gloo when some share one (RCCL refuses duplicate GPUs) or any is on the CPU.  The IPC
    all-gather is enabled when all GPU processes run on one host (it verifies itself and falls back
    collectively)."""
    if any(d.get("type") != "cuda" for d in descs):
        return "gloo", False
    one_host = len({d.get("host") for d in descs}) == 1
    gpus = [(d.get("host"), d.get("gpu")) for d in descs]
    return ("nccl" if len(set(gpus)) == len(gpus) else "gloo"), one_host


def serve_rendezvous(cfg: Config, timeout_s: float = 3600.0):
    """Server side: open the store, wait for ``clients`` registrations, publish the client table, the transport
    choice of the client group (``comm.backend: auto``) and where the leader writes (``leader_paths``).

    Returns (store, n_clients, table_json); the chosen (backend, one_shot) is in ``store`` under
    ``attackfl/transport`` (``read_transport``)."""
    import os
    import socket

    host, port = _host_port(cfg)
    n = cfg.clients
    store = dist.TCPStore(host, port, world_size=None, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=timeout_s), use_libuv=False)
    store.set(PREFIX + "n_clients", str(n))
    print_with_color(f"Server is waiting for {n} clients.", "green")
    t0 = time.time()
    while int(store.add(PREFIX + "next_rank", 0)) < n:
        if time.time() - t0 > timeout_s:
            raise TimeoutError("clients did not register in time")
        time.sleep(0.05)
    table, descs = [], []
    for r in range(1, n + 1):
        d = json.loads(store.get(PREFIX + f"client/{r}").decode())
        # client r is group rank r - 1 and owns exactly its own FL client (index r - 1)
        table.append({"index": r - 1, "uuid": d["uuid"], "owner": r - 1, "attack": d.get("attack")})
        descs.append(d.get("device") or {"type": "cpu"})
        print_with_color(f"[<<<] Received message from client: "
                         f"{ {k: v for k, v in d.items() if k != 'device'} }", "blue")
    backend, one_shot = choose_backend(descs)
    store.set(PREFIX + "transport", json.dumps({"backend": backend, "one_shot": one_shot,
                                                "sharers": [sharers_of(descs, d) for d in descs]}))
    # the leader (group rank 0) writes app.log and the checkpoints where the reference's server would: the
    # server's log_path and checkpoint directory, resolved against the server's working directory
    ckpt = cfg.engine.get("checkpoint-dir", ".")
    store.set(PREFIX + "leader_paths", json.dumps({"host": socket.gethostname(),
                                                   "log_path": os.path.abspath(cfg.log_path),
                                                   "checkpoint_dir": os.path.abspath(ckpt)}))
    store.set(PREFIX + "table", json.dumps(table))
    print_with_color("All clients are connected. Sending notifications.", "green")
    return store, n, table


def read_transport(store, rank: int = 0) -> Tuple[str, bool]:
    """(backend, one_shot) of the client group; records this client's co-residency budget (processes on its GPU)."""
    t = json.loads(store.get(PREFIX + "transport").decode())
    sh = t.get("sharers", 1)
    set_gpu_sharers(int(sh[rank] if isinstance(sh, list) else sh))
    return str(t["backend"]), bool(t["one_shot"])


def apply_leader_paths(store, cfg: Config) -> None:
    """Leader client: write ``app.log`` / ``.pth`` where the server would (its log_path / checkpoint directory)
    when both run on one host; elsewhere (a multi-host run) the leader's own configured paths are kept."""
    import socket

    p = json.loads(store.get(PREFIX + "leader_paths").decode())
    if p.get("host") == socket.gethostname():
        cfg.raw["log_path"] = p["log_path"]
        cfg.engine["checkpoint-dir"] = p["checkpoint_dir"]


DONE, FAILED, EXITED = PREFIX + "done", PREFIX + "failed", PREFIX + "exited"


def report_done(store, ok: bool, msg: str = "") -> None:
    """A client reports the run's end (leader: done; any client: failure, with its message)."""
    store.set(DONE if ok else FAILED, msg or ("ok" if ok else "failed"))


def report_exit(store) -> None:
    """A client is done with the store (the server keeps it open until every client has said so)."""
    store.add(EXITED, 1)


def serve_until_done(store, log_file: str, n_clients: int, timeout_s: float = 7 * 24 * 3600.0,
                     poll_s: float = 0.2) -> bool:
    """Server side after the rendezvous: echo the leader's ``app.log`` to the console as it grows (the reference
    server's console shows its own log) until a client reports the run done (True) or failed (False); then keep
    the store up until every client has left it (bounded)."""
    import os
    import sys

    pos = 0
    t0 = time.time()

    def echo():
        nonlocal pos
        if os.path.exists(log_file):
            with open(log_file, "rb") as fh:
                fh.seek(pos)
                chunk = fh.read()
            if chunk:
                pos += len(chunk)
                sys.stdout.write(chunk.decode(errors="replace"))
                sys.stdout.flush()

    while True:
        echo()
        if store.check([FAILED]):
            print_with_color(f"A client failed: {store.get(FAILED).decode()}", "red")
            return False
        if store.check([DONE]):
            echo()
            t1 = time.time()
            while int(store.add(EXITED, 0)) < n_clients and time.time() - t1 < 60.0:
                time.sleep(0.05)
            return True
        if time.time() - t0 > timeout_s:
            raise TimeoutError("the clients did not finish in time")
        time.sleep(poll_s)


def join_rendezvous(cfg: Config, attack: Optional[AttackSpec], timeout_s: float = 3600.0, device=None,
                    device_fn=None):
    """Client side: claim a client number (1..N), publish the descriptor, wait for the table.  ``device_fn(r)``
    (optional) picks the device once the number is known (``client_device``); it overrides ``device``.

    Returns (store, group rank = r - 1, group size = N, table_json, device)."""
    host, port = _host_port(cfg)
    store = dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s),
                          use_libuv=False)
    r = int(store.add(PREFIX + "next_rank", 1))
    n = int(store.get(PREFIX + "n_clients").decode())
    if r > n:
        raise RuntimeError(f"server expects {n} clients; this would be client #{r}")
    if device_fn is not None:
        device = device_fn(r)
    desc = {"uuid": str(uuid.uuid4()), "message": "Hello from Client!",
            "attack": None if attack is None else attack.to_dict(),
            "device": device_descriptor(device) if device is not None else {"type": "cpu"}}
    store.set(PREFIX + f"client/{r}", json.dumps(desc))
    print_with_color(f"[>>>] Client {desc['uuid']} registered as client {r}", "red")
    store.wait([PREFIX + "table"])
    table = json.loads(store.get(PREFIX + "table").decode())
    return store, r - 1, n, table, device


def table_from_json(table_json: List[Dict]):
    from ..fl.engine import ClientInfo

    out = []
    for d in table_json:
        a = d.get("attack")
        out.append(ClientInfo(int(d["index"]), str(d["uuid"]), int(d["owner"]),
                              AttackSpec.from_dict(a) if a else None))
    return out


def init_group(store, rank: int, world: int, backend: str, timeout_s: int = 600, device_index=None):
    import torch

    kw = dict(backend=backend, store=dist.PrefixStore(PREFIX + "pg", store), rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(device_index or 0)
        kw["device_id"] = torch.device("cuda", device_index or 0)
    elif torch.cuda.is_available() and device_index is not None:
        torch.cuda.set_device(device_index)
    dist.init_process_group(**kw)
