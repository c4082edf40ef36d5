"""Checkpoint writer pieces that run on the CPU: the zip template (a ``torch.save`` archive re-emitted with
new storage bytes and a patched CRC-32) and zlib's CRC combination rule it relies on."""
import io
import os
import random
import zipfile
import zlib
from collections import OrderedDict

import pytest
import torch

from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.utils.ckpt import CheckpointWriter, ZipTemplate, crc32_combine


def test_crc32_combine_matches_zlib():
    rnd = random.Random(5)
    for _ in range(20):
        a = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 300)))
        b = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 300)))
        assert crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)


@pytest.mark.parametrize("model", ["TransformerModel", "CNNModel"])
def test_zip_template_rewrites_storage(tmp_path, model):
    lay = ParamLayout.for_model(model)
    host = lay.flatten(build_model(model, seed=0).state_dict()).contiguous()
    buf = io.BytesIO()
    torch.save(lay.unflatten(host, clone=False), buf)
    t = ZipTemplate(buf.getvalue(), host.numel() * 4)
    # a new state through the template: loadable, equal to torch.save of the same state, valid zip CRCs
    new = lay.flatten(build_model(model, seed=1).state_dict()).contiguous()
    path = str(tmp_path / "m.pth")
    t.write(path, memoryview(new.numpy()).cast("B"), zlib.crc32(new.numpy().tobytes()))
    got = torch.load(path, weights_only=True)
    ref = lay.unflatten(new, clone=True)
    assert list(got) == list(ref) and all(torch.equal(got[k], ref[k]) for k in ref)
    with zipfile.ZipFile(path) as z:
        assert z.testzip() is None
    buf2 = io.BytesIO()
    torch.save(lay.unflatten(new, clone=False), buf2)
    with zipfile.ZipFile(path) as a, zipfile.ZipFile(buf2) as b:   # record for record (but the per-save id)
        ra = {n.split("/", 1)[1]: a.read(n) for n in a.namelist()}
        rb = {n.split("/", 1)[1]: b.read(n) for n in b.namelist()}
        ra.pop(".data/serialization_id"), rb.pop(".data/serialization_id")
        assert ra == rb


def test_zip_template_rejects_several_storages():
    sd = OrderedDict(a=torch.zeros(4), b=torch.ones(3))
    buf = io.BytesIO()
    torch.save(sd, buf)
    with pytest.raises(ValueError):
        ZipTemplate(buf.getvalue(), 16)


def test_hyper_state_dict_views_one_storage():
    """With the target tail appended, every hypernetwork checkpoint tensor views one buffer (template path)
    and the dict equals the cloned reference layout."""
    from attackfl_amd.fl.hyper_server import HyperServer

    hs = HyperServer(build_model("TransformerModel", seed=0).state_dict(), 3, 0.01, 1.0, "cpu", seed=1)
    hnet = hs.hnet
    host = torch.cat([hnet.arena, hnet.target_tail()])
    sd = hnet.state_dict_of(host, clone=False)
    ref = hnet.state_dict()
    assert list(sd) == list(ref) and all(torch.equal(sd[k], ref[k]) for k in ref)
    assert {t.untyped_storage().data_ptr() for t in sd.values()} == {host.untyped_storage().data_ptr()}


def test_cpu_writer_writes_every_submit(tmp_path):
    w = CheckpointWriter()
    for v in range(3):
        w.submit("x", torch.full((10,), float(v)), lambda t: {"t": t}, str(tmp_path / "x.pth"))
    w.close()
    assert w.written == 3 and w.dropped == 0
    assert torch.equal(torch.load(tmp_path / "x.pth", weights_only=True)["t"], torch.full((10,), 2.0))
    assert not os.path.exists(tmp_path / "x.pth.tmp")
