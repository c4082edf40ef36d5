"""Classic-launch device placement and the co-residency budget (parallel/launcher.py): one FL client per GPU
(reference client.py:50-61 picks its own device; README.md:103-143 starts one client process per client)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from attackfl_amd.parallel import launcher as L


def _descs(devices, host="n0"):
    out = []
    for d in devices:
        if d.startswith("cuda"):
            out.append({"host": host, "type": "cuda", "gpu": f"uuid:{d.split(':')[1]}"})
        else:
            out.append({"host": host, "type": "cpu", "gpu": None})
    return out


def test_client_device_mapping():
    # explicit devices win
    assert L.client_device("cuda:5", 1, 8) == "cuda:5"
    assert L.client_device("cpu", 3, 8) == "cpu"
    # --device cuda / none: client r -> GPU (r - 1) % ndev (the server takes no GPU)
    assert [L.client_device(None, r, 8) for r in range(1, 9)] == [f"cuda:{i}" for i in range(8)]
    assert L.client_device("cuda", 3, 8) == "cuda:2"
    # more clients than GPUs: round robin, some GPUs shared
    assert [L.client_device(None, r, 2) for r in range(1, 5)] == ["cuda:0", "cuda:1", "cuda:0", "cuda:1"]
    # no GPU at all
    assert L.client_device(None, 1, 0) == "cpu"


def test_classic_backend_on_an_8_gpu_node():
    # the reference-style launch (server + 8 clients) on an 8-GPU node: the device group is the 8 clients
    # alone, each on its own GPU -> RCCL, IPC all-gather on the one host, every client with the whole chip
    devs8 = [L.client_device(None, r, 8) for r in range(1, 9)]
    assert L.choose_backend(_descs(devs8)) == ("nccl", True)
    assert L.max_sharers(_descs(devs8)) == 1
    # 16 clients on 8 GPUs: two per GPU -> gloo group, IPC data path, half the CUs each
    devs16 = [L.client_device(None, r, 8) for r in range(1, 17)]
    assert L.choose_backend(_descs(devs16)) == ("gloo", True)
    assert [L.sharers_of(_descs(devs16), d) for d in _descs(devs16)] == [2] * 16
    # one visible GPU (the GPU-box classic test): every client shares it
    devs1 = [L.client_device(None, r, 1) for r in range(1, 4)]
    assert devs1 == ["cuda:0"] * 3
    assert L.choose_backend(_descs(devs1)) == ("gloo", True)
    assert L.max_sharers(_descs(devs1)) == 3
    # CPU processes: gloo, no IPC
    assert L.choose_backend(_descs(["cpu", "cpu"])) == ("gloo", False)


def test_sharers_are_counted_per_gpu():
    """one shared GPU must not halve the budget of clients that own theirs."""
    devs = ["cuda:0", "cuda:0", "cuda:1", "cuda:2"]
    d = _descs(devs)
    assert [L.sharers_of(d, x) for x in d] == [2, 2, 1, 1]
    assert L.sharers_of(d, {"type": "cpu"}) == 1


def test_gpu_sharers_default_does_not_guess_from_local_world(monkeypatch):
    """with each rank's visibility narrowed to its own GPU (device_count() == 1) and 8 local ranks,
    the old fallback assumed all 8 share it and cut the CU budget 8x."""
    monkeypatch.setattr(L, "_SHARERS", None)
    monkeypatch.delenv("AFL_GPU_SHARERS", raising=False)
    monkeypatch.delenv("AFL_BENCH_DEVICE", raising=False)
    monkeypatch.delenv("AFL_SHARED_GPU", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert L.gpu_sharers() == 1
    monkeypatch.setenv("AFL_SHARED_GPU", "1")  # launch.py --device cuda:i: every local rank on one GPU
    assert L.gpu_sharers() == 8


def _sharers_worker(rank, world, port, same, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L._SHARERS = None
        gpu = "uuid:x" if same or rank < 2 else f"uuid:{rank}"
        L.device_descriptor = lambda dev: {"host": "n0", "type": "cuda", "gpu": gpu}
        q.put((rank, L.sync_gpu_sharers(None), L.gpu_sharers()))
    finally:
        dist.destroy_process_group()


def _run_sharers(world, same):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=_sharers_worker, args=(r, world, port, same, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_sync_gpu_sharers_counts_processes_per_physical_gpu():
    # 3 ranks, all on one GPU -> 3 each; ranks 0, 1 on one GPU and rank 2 on its own -> 2, 2 and 1 (each rank's
    # budget follows its own GPU)
    assert [(n, m) for _, n, m in _run_sharers(3, same=True)] == [(3, 3)] * 3
    assert [(n, m) for _, n, m in _run_sharers(3, same=False)] == [(2, 2), (2, 2), (1, 1)]
