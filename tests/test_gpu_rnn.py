"""Fused RNNModel trainers (split 4: csrc/kernels/rnn2.hip, on-chip; split 3: rnn.hip) against the
composite RNNProgram on CPU, which uses the same dropout-mask convention: raw SGD gradients with dropout on,
multi-step Adam trajectories, the partial / size-1 batches, the NaN abort, bit-reproducibility."""
import pytest
import torch

from attackfl_amd.data import DeviceTable, synthetic_icu
from attackfl_amd.fl.programs import ProgramRunner, make_program
from attackfl_amd.fl.trainers import Plan, make_plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import rnn as R

pytestmark = pytest.mark.gpu
SPLITS = pytest.mark.parametrize("split", [4, 3])


def _setup(C, nd, E=1, seed=0):
    ds = synthetic_icu(3000, seed=3)
    lay = ParamLayout.for_model("RNNModel")
    params = torch.stack([lay.flatten(build_model("RNNModel", seed=seed + i).state_dict()) for i in range(C)])
    plan = make_plan(len(ds), nd, E, [101 + i for i in range(C)], "cpu")
    return ds, params, plan


def _composite(ds, params, plan, lr, seeds, sgd=0.0):
    p = params.clone()
    prog = make_program("RNNModel", p.shape[0], 128, "cpu")
    ok, losses = ProgramRunner(prog).train(DeviceTable(ds, "cpu"), p, plan, lr=lr, seeds=seeds, sgd_lr=sgd)
    return p, ok, losses


@SPLITS
def test_sgd_gradients_match_program(gpu, split):
    """Raw SGD updates (dropout on): the fused kernel equals the GPU layer program (same bf16 operand
    rounding) to < 2 % per tensor, and both stay within the bf16 band of the fp32 composite."""
    ds, params, plan = _setup(2, [128, 100])
    ref, ok_r, _ = _composite(ds, params, plan, 0.0, [5, 6], sgd=1.0)
    dev = params.clone().to(gpu)
    ok, _ = R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, 1, 128, 1.0, [5, 6],
                            opt_mode=1, split=split)
    gp = params.clone().to(gpu)
    ProgramRunner(make_program("RNNModel", 2, 128, gpu), use_graph=False).train(
        DeviceTable(ds, gpu), gp, Plan(plan.order.to(gpu), plan.nd, 1), lr=0.0, seeds=[5, 6], sgd_lr=1.0)
    assert ok.tolist() == [1, 1] and ok_r.all()
    g_ref, g_dev, g_gp = params - ref, params - dev.cpu(), params - gp.cpu()
    bad = []
    for s in ParamLayout.for_model("RNNModel").slots:
        a = g_dev[:, s.offset:s.offset + s.numel]
        b = g_ref[:, s.offset:s.offset + s.numel]
        c = g_gp[:, s.offset:s.offset + s.numel]
        if b.abs().max().item() == 0.0:  # W_hh: exactly zero gradient (h0 = 0)
            if a.abs().max().item() != 0.0:
                bad.append((s.name, "nonzero"))
            continue
        vs_graph = float((a - c).norm() / c.norm())
        vs_fp32 = float((a - b).norm() / b.norm())
        if vs_graph > 0.02 or vs_fp32 > 0.12:
            bad.append((s.name, round(vs_graph, 4), round(vs_fp32, 4)))
    assert not bad, bad


@SPLITS
def test_adam_epochs_track_program(gpu, split):
    ds, params, plan = _setup(3, [700, 513, 300], E=2, seed=4)
    ref, ok_r, loss_r = _composite(ds, params, plan, 0.004, [7, 8, 9])
    dev = params.clone().to(gpu)
    ok, loss = R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, 2, 128, 0.004, [7, 8, 9],
                               split=split)
    assert ok.tolist() == [1, 1, 1] and ok_r.all()
    moved = (ref - params).abs().mean().item()
    assert (dev.cpu() - ref).abs().mean().item() < 0.1 * moved
    assert torch.allclose(loss.double(), loss_r, rtol=0.03, atol=0.01), (loss, loss_r)


@SPLITS
def test_nan_client_fails_others_train(gpu, split):
    ds, params, plan = _setup(2, [300, 300])
    params[1, 11] = float("nan")
    dev = params.clone().to(gpu)
    ok, _ = R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, 1, 128, 0.004, [1, 2],
                            split=split)
    assert ok.tolist() == [1, 0]
    assert torch.isfinite(dev[0]).all() and not torch.equal(dev[0].cpu(), params[0])


def test_onchip_bit_reproducible(gpu):
    """The on-chip trainer: a client's result may not depend on the launch that trains it (the multi-rank
    engine relies on it) — the same clients trained in one launch of 4 and in two launches of 2 are
    bit-identical, and so is a repeat."""
    ds, params, plan = _setup(4, [700, 650, 900, 301], E=2, seed=2)
    rows = DeviceTable(ds, gpu).rows
    order = plan.order.to(gpu)
    seeds = [11, 12, 13, 14]
    outs = []
    for _ in range(2):
        p = params.clone().to(gpu)
        ok, _ = R.train_clients(p, rows, order, plan.nd, 2, 128, 0.004, seeds)
        assert ok.tolist() == [1, 1, 1, 1]
        outs.append(p)
    assert torch.equal(outs[0], outs[1])
    sub = []
    for lo in (0, 2):
        p = params[lo:lo + 2].clone().to(gpu)
        R.train_clients(p, rows, order[lo:lo + 2].contiguous(), plan.nd[lo:lo + 2], 2, 128, 0.004, seeds[lo:lo + 2])
        sub.append(p)
    assert torch.equal(outs[0], torch.cat(sub))


def test_batch_sizes_and_tiny_clients(gpu):
    """Partial last batches, size-1 batches (skipped), batch sizes below 128 and clients with fewer rows
    than one batch: the on-chip trainer tracks the composite program."""
    ds, params, plan = _setup(3, [129, 65, 3], E=2, seed=6)
    for batch in (64, 32):
        prog = make_program("RNNModel", 3, batch, "cpu")
        ref = params.clone()
        ok_r, _ = ProgramRunner(prog).train(DeviceTable(ds, "cpu"), ref, plan, lr=0.003, seeds=[3, 4, 5])
        dev = params.clone().to(gpu)
        ok, _ = R.train_clients(dev, DeviceTable(ds, gpu).rows, plan.order.to(gpu), plan.nd, 2, batch, 0.003, [3, 4, 5])
        assert ok.tolist() == [1, 1, 1] and ok_r.all()
        moved = (ref - params).abs().mean().item()
        assert (dev.cpu() - ref).abs().mean().item() < 0.1 * moved, batch


def test_eval_many_matches_eager_model(gpu):
    """Fused forward-only eval of C models (k_rnn2_eval) against torch's fp32 RNNModel in eval mode (bf16
    MFMA operands: outputs within 2e-2, mean error far below)."""
    ds = synthetic_icu(1000, seed=5)
    n = 333  # not a multiple of the 128-row tile
    lay = ParamLayout.for_model("RNNModel")
    models = [build_model("RNNModel", seed=20 + i).eval() for i in range(3)]
    params = torch.stack([lay.flatten(m.state_dict()) for m in models]).to(gpu)
    rows = torch.cat([ds.vitals[:n], ds.labs[:n], ds.labels[:n, None]], 1)
    rows[::7, 2] = -2.0  # masked values
    out = R.eval_many(params, rows.to(gpu)).cpu()
    with torch.no_grad():
        ref = torch.stack([m(rows[:, :7], rows[:, 7:23]).reshape(-1) for m in models])
    assert out.shape == (3, n)
    err = (out - ref).abs()
    assert err.max().item() < 2e-2 and err.mean().item() < 3e-3, (err.max().item(), err.mean().item())
