"""Process launch / rendezvous (replaces the RabbitMQ REGISTER handshake, ``server.py:205-235``,
``client.py:134-143``, and the broker queue janitor ``server.py:803-835``).

Two ways to start a run:

* **classic** — ``python server.py`` plus N x ``python client.py [--attack ...]``, exactly like the
  reference.  The server opens a TCPStore at ``comm.address`` (default: ``rabbit.address``) and waits
  for ``server.clients`` registrations; every client claims the next rank with an atomic counter and
  publishes its descriptor (uuid + attack flags).  Registration order defines the client index like
  the reference's ``list_clients``.  Then all processes join one ``torch.distributed`` group
  (rank 0 = server, ranks 1..N = clients) and run the SPMD engine.  A fresh store per run plays the
  role of the queue janitor.
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
    """Device of classic client ``rank`` (1..N; rank 0 is the server).  An explicit ``--device cuda:i`` / ``cpu``
    wins; ``--device cuda`` or none puts client r on GPU ``r % ndev`` — one FL client per MI355X, the server
    alone on GPU 0 whenever there are fewer clients than GPUs (with N = ndev clients the last one shares GPU 0
    with the server, the only way 9 processes fit 8 GPUs).  Reference: client.py:50-61 (cuda if available)."""
    if arg and arg != "cuda":
        return arg
    if ndev <= 0:
        return arg or "cpu"
    return f"cuda:{rank % ndev}"


def sync_gpu_sharers(device) -> int:
    """Collective (after ``init_process_group``): count the processes of the group on each physical GPU (by
    ``gpu_key``, so ranks whose visibility was narrowed to 'their' GPU are told apart) and record the largest
    count for this process's co-residency budget.  Returns it."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return gpu_sharers()
    descs: List[Dict] = [None] * dist.get_world_size()  # type: ignore[list-item]
    dist.all_gather_object(descs, device_descriptor(device))
    n = max_sharers(descs)
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


def max_sharers(descs: List[Dict]) -> int:
    """Largest number of registered processes on one physical GPU (1 when none shares)."""
    cnt: Dict[Tuple, int] = {}
    for d in descs:
        if d.get("type") == "cuda":
            k = (d.get("host"), d.get("gpu"))
            cnt[k] = cnt.get(k, 0) + 1
    return max(cnt.values()) if cnt else 1


def choose_backend(descs: List[Dict]) -> Tuple[str, bool]:
    """(process-group backend, one-shot IPC) for the classic launch: RCCL when every process owns a distinct
    GPU; gloo when some share one (RCCL refuses duplicate GPUs) or any is on the CPU.  The IPC all-gather is
    enabled when all GPU processes run on one host (it verifies itself and falls back collectively)."""
    if any(d.get("type") != "cuda" for d in descs):
        return "gloo", False
    one_host = len({d.get("host") for d in descs}) == 1
    gpus = [(d.get("host"), d.get("gpu")) for d in descs]
    return ("nccl" if len(set(gpus)) == len(gpus) else "gloo"), one_host


def serve_rendezvous(cfg: Config, timeout_s: float = 3600.0, device=None):
    """Server side: open the store, wait for ``clients`` registrations, publish the client table and the
    transport choice (``comm.backend: auto``).

    Returns (store, world_size, table_json); the chosen (backend, one_shot) is in ``store`` under
    ``attackfl/transport`` (``read_transport``)."""
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
    table = []
    descs = [device_descriptor(device) if device is not None else {"type": "cpu", "host": "", "gpu": None}]
    for r in range(1, n + 1):
        d = json.loads(store.get(PREFIX + f"client/{r}").decode())
        table.append({"index": r - 1, "uuid": d["uuid"], "owner": r, "attack": d.get("attack")})
        descs.append(d.get("device") or {"type": "cpu"})
        print_with_color(f"[<<<] Received message from client: "
                         f"{ {k: v for k, v in d.items() if k != 'device'} }", "blue")
    backend, one_shot = choose_backend(descs)
    store.set(PREFIX + "transport", json.dumps({"backend": backend, "one_shot": one_shot,
                                                "sharers": max_sharers(descs)}))
    store.set(PREFIX + "table", json.dumps(table))
    print_with_color("All clients are connected. Sending notifications.", "green")
    return store, n + 1, table


def read_transport(store) -> Tuple[str, bool]:
    t = json.loads(store.get(PREFIX + "transport").decode())
    set_gpu_sharers(int(t.get("sharers", 1)))
    return str(t["backend"]), bool(t["one_shot"])


def join_rendezvous(cfg: Config, attack: Optional[AttackSpec], timeout_s: float = 3600.0, device=None,
                    device_fn=None):
    """Client side: claim a rank, publish the descriptor, wait for the table.  ``device_fn(rank)`` (optional)
    picks the device once the rank is known (``client_device``); it overrides ``device``.

    Returns (store, rank, world_size, table_json, device)."""
    host, port = _host_port(cfg)
    store = dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s),
                          use_libuv=False)
    rank = int(store.add(PREFIX + "next_rank", 1))
    n = int(store.get(PREFIX + "n_clients").decode())
    if rank > n:
        raise RuntimeError(f"server expects {n} clients; this would be client #{rank}")
    if device_fn is not None:
        device = device_fn(rank)
    desc = {"uuid": str(uuid.uuid4()), "message": "Hello from Client!",
            "attack": None if attack is None else attack.to_dict(),
            "device": device_descriptor(device) if device is not None else {"type": "cpu"}}
    store.set(PREFIX + f"client/{rank}", json.dumps(desc))
    print_with_color(f"[>>>] Client {desc['uuid']} registered as rank {rank}", "red")
    store.wait([PREFIX + "table"])
    table = json.loads(store.get(PREFIX + "table").decode())
    return store, rank, n + 1, table, device


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
