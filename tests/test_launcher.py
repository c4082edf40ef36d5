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
    # --device cuda / none: client r -> GPU r % ndev (server = rank 0 on GPU 0)
    assert [L.client_device(None, r, 8) for r in range(1, 9)] == [f"cuda:{i}" for i in (1, 2, 3, 4, 5, 6, 7, 0)]
    assert L.client_device("cuda", 3, 8) == "cuda:3"
    # fewer GPUs than clients: round robin, some GPUs shared
    assert [L.client_device(None, r, 2) for r in range(1, 5)] == ["cuda:1", "cuda:0", "cuda:1", "cuda:0"]
    # no GPU at all
    assert L.client_device(None, 1, 0) == "cpu"


def test_classic_backend_on_an_8_gpu_node():
    server = "cuda:0"
    # 7 clients + server: every process owns a GPU -> RCCL, IPC all-gather on the one host
    devs7 = [server] + [L.client_device(None, r, 8) for r in range(1, 8)]
    assert L.choose_backend(_descs(devs7)) == ("nccl", True)
    assert L.max_sharers(_descs(devs7)) == 1
    # 8 clients + server on 8 GPUs: client 8 shares GPU 0 with the server -> gloo group, IPC data path
    devs8 = [server] + [L.client_device(None, r, 8) for r in range(1, 9)]
    assert L.choose_backend(_descs(devs8)) == ("gloo", True)
    assert L.max_sharers(_descs(devs8)) == 2
    # one visible GPU (the GPU-box classic test): everyone shares it
    devs1 = [server] + [L.client_device(None, r, 1) for r in range(1, 4)]
    assert devs1 == ["cuda:0"] * 4
    assert L.choose_backend(_descs(devs1)) == ("gloo", True)
    assert L.max_sharers(_descs(devs1)) == 4
    # CPU processes: gloo, no IPC
    assert L.choose_backend(_descs(["cpu", "cpu"])) == ("gloo", False)


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
    # 3 ranks, all on one GPU -> 3; ranks 0, 1 on one GPU and rank 2 on its own -> 2 (the largest group)
    assert [(n, m) for _, n, m in _run_sharers(3, same=True)] == [(3, 3)] * 3
    assert [(n, m) for _, n, m in _run_sharers(3, same=False)] == [(2, 2)] * 3
