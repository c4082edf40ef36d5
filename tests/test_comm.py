"""Transport logic on the CPU: the IPC path's collective verdict (every rank falls back together when any
rank cannot use it) and the process-group collectives over gloo at world 2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from attackfl_amd.parallel.ipc import IpcAllGather, IpcUnavailable, setup_verdict


def test_setup_verdict_rules():
    h = b"x" * 64
    ok = [("n0", 0, h), ("n0", 1, h), ("n0", 2, h)]
    assert setup_verdict("", ok, 0, lambda d: True) == ""
    assert "boom" in setup_verdict("boom", ok, 0, lambda d: True)
    assert "hosts" in setup_verdict("", [("n0", 0, h), ("n1", 0, h)], 0, lambda d: True)
    assert "export" in setup_verdict("", [("n0", 0, h), ("n0", 1, b"")], 0, lambda d: True)
    # no peer access from GPU 0 to GPU 2 (and 1 is fine)
    v = setup_verdict("", ok, 0, lambda d: d != 2)
    assert "GPU(s) ['2']" in v
    # ranks sharing one GPU need no peer access
    assert setup_verdict("", [("n0", 0, h), ("n0", 0, h)], 1, lambda d: False) == ""
    # physical identities: a peer GPU this process cannot see (visibility narrowed per rank) is unknown, not
    # refused — the open and the self-test decide
    ids = [("n0", "uuid:a", h), ("n0", "uuid:b", h), ("n0", "uuid:c", h)]
    seen = {"uuid:a": True, "uuid:c": False}
    assert setup_verdict("", ids, 0, lambda d: seen.get(d)) == "no peer access from GPU uuid:a to GPU(s) ['uuid:c']"
    seen["uuid:c"] = None
    assert setup_verdict("", ids, 0, lambda d: seen.get(d)) == ""


class _FakeCtx:
    fail_open_rank = -1

    def __init__(self, rank, world, n):
        self.rank = rank

    def handle(self):
        return b"h" * 64

    def open(self, handles):
        if self.rank == _FakeCtx.fail_open_rank:
            raise RuntimeError("hipIpcOpenMemHandle failed")

    def close(self):
        pass


class _FakeNative:
    IpcContext = _FakeCtx


def _worker(rank, world, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from attackfl_amd import ops

        ops.native = lambda: _FakeNative  # (the module-level accessor ipc.py calls)
        _FakeCtx.fail_open_rank = fail_rank
        ipc = IpcAllGather("cpu", rank, world)
        try:
            ipc.setup(16)
            q.put((rank, "ok"))
        except IpcUnavailable as e:
            q.put((rank, f"fallback: {e}"))
        # the process-group path every rank falls back to: gloo all-gather / all-reduce
        from attackfl_amd.parallel.comm import TorchComm

        comm = TorchComm("cpu", "gloo", one_shot=False)
        got = comm.all_gather_rows(torch.full((2, 3), float(rank)))
        red = comm.all_reduce_(torch.ones(4))
        q.put((rank, (got[:, 0].tolist(), red.tolist())))
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(4)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_ipc_open_failure_on_one_rank_falls_back_on_every_rank():
    out = _run(fail_rank=1)
    verdicts = {r: v for r, v in out if isinstance(v, str)}
    # rank 1 could not open rank 0's handle: BOTH ranks fall back, with rank 1's reason on rank 1
    assert verdicts[0].startswith("fallback") and verdicts[1].startswith("fallback")
    assert "open" in verdicts[1]
    colls = [v for _, v in out if not isinstance(v, str)]
    assert all(g == [0.0, 0.0, 1.0, 1.0] and red == [2.0] * 4 for g, red in colls)


@pytest.mark.parametrize("fail_rank", [-1])
def test_ipc_setup_agrees_when_every_rank_succeeds(fail_rank):
    out = _run(fail_rank)
    # (the fake context cannot run the self-test's device gather: the self-test's own failure is reported)
    verdicts = [v for _, v in out if isinstance(v, str)]
    assert len(verdicts) == 2 and len(set(v.startswith("fallback") for v in verdicts)) == 1
