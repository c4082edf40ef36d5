"""Fused TransformerModel training / eval kernels vs the fp32 PyTorch oracle of the same op."""
import pytest
import torch

from attackfl_amd.data import DeviceTable, synthetic_icu
from attackfl_amd.fl.trainers import make_plan
from attackfl_amd.models import ParamLayout, build_model
from attackfl_amd.ops import transformer as T

pytestmark = pytest.mark.gpu


def _setup(C, nd, seed=0):
    ds = synthetic_icu(2000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1)
    lay = ParamLayout.for_model("TransformerModel")
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=seed + i).state_dict()) for i in range(C)])
    g = torch.Generator().manual_seed(7)
    plan = make_plan(rows.shape[0], nd, 1, g, "cpu")
    return rows, params, plan


def test_eval_many_matches_single_model_eval(gpu):
    """Batched eval (grid.y = model, the hyper validation path) vs one launch per model: bit-identical."""
    from attackfl_amd.ops import native
    rows, params, _ = _setup(3, [10])
    pd, rd = params.to(gpu).contiguous(), rows[:1500].to(gpu).contiguous()
    many = native().tf_eval_many(pd, rd)
    assert many.shape == (3, 1500)
    for k in range(3):
        assert torch.equal(many[k], T.eval_forward(pd[k], rd))


def test_eval_forward_matches_reference(gpu):
    rows, params, _ = _setup(1, [10])
    out = T.eval_forward(params[0].to(gpu), rows.to(gpu)).cpu()
    sd = ParamLayout.for_model("TransformerModel").unflatten(params[0])
    ref = T.reference_forward(sd, rows[:, :7], rows[:, 7:23]).reshape(-1)
    assert torch.isfinite(out).all()
    assert (out - ref).abs().max().item() < 2e-2, (out - ref).abs().max()
    m = build_model("TransformerModel", seed=0).eval()
    with torch.no_grad():
        mod = m(rows[:, :7], rows[:, 7:23]).reshape(-1)
    assert (mod - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("split", [1, 2, 3, 4])
@pytest.mark.parametrize("batch", [128, 100])
def test_sgd_step_gradients_match(gpu, batch, split):
    """One SGD step (opt_mode 1) exposes the raw gradients: compare p1 - p0 with the oracle."""
    rows, params, plan = _setup(2, [batch, batch])
    lr = 1.0
    ref = params.clone()
    T.reference_train(ref, rows, plan.order, plan.nd, 1, batch, lr, [11, 12], opt_mode=1, max_steps=1)
    dev = params.clone().to(gpu)
    ok, _ = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 1, batch, lr, [11, 12], opt_mode=1,
                            split=split)
    assert ok.tolist() == [1, 1]
    g_ref = (params - ref)
    g_dev = (params - dev.cpu())
    lay = ParamLayout.for_model("TransformerModel")
    for s in lay.slots:
        a = g_dev[:, s.offset:s.offset + s.numel]
        b = g_ref[:, s.offset:s.offset + s.numel]
        scale = b.abs().max().item() + 1e-6
        err = (a - b).abs().max().item() / scale
        assert err < 0.08, (s.name, err, scale)


def test_adam_epoch_tracks_reference(gpu):
    """A full epoch of Adam steps: parameters stay close to the fp32 oracle and the loss falls."""
    nd = [1100, 900]
    rows, params, plan = _setup(2, nd, seed=5)
    ref = params.clone()
    ok_r, loss_r = T.reference_train(ref, rows, plan.order, plan.nd, 1, 128, 0.004, [3, 4])
    dev = params.clone().to(gpu)
    ok, loss = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 1, 128, 0.004, [3, 4])
    assert ok.tolist() == [1, 1]
    d = (dev.cpu() - ref).abs()
    moved = (ref - params).abs()
    # bf16 GEMM operands: the trajectories agree to a few % of the distance travelled
    assert d.mean().item() < 0.1 * moved.mean().item(), (d.mean(), moved.mean())
    assert torch.allclose(loss, loss_r, rtol=0.05, atol=0.02), (loss, loss_r)


@pytest.mark.parametrize("split", [1, 2, 3, 4])
def test_nan_params_fail_client(gpu, split):
    rows, params, plan = _setup(2, [300, 300])
    params[1, 5] = float("nan")
    dev = params.to(gpu)
    ok, _ = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 1, 128, 0.004, [1, 2], split=split)
    assert ok.tolist() == [1, 0]
    assert torch.isfinite(dev[0]).all()


def test_size_one_batch_skipped(gpu):
    rows, params, plan = _setup(1, [129])
    dev = params.clone().to(gpu)
    ok, _ = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 1, 128, 0.004, [9])
    ref = params.clone()
    T.reference_train(ref, rows, plan.order, plan.nd, 1, 128, 0.004, [9])
    assert ok.tolist() == [1]
    assert (dev.cpu() - ref).abs().max().item() < 0.02


def test_branch_parallel_matches_single_workgroup(gpu):  # noqa: D401
    """The two- and three-workgroup launches run the same arithmetic as the one-workgroup launch
    (hand-offs move exact bf16 values, and the one-workgroup launch rounds the branch gradient to bf16
    too; only the compiler's FMA contraction may differ per instantiation), so
    raw SGD updates agree to float rounding and Adam runs agree closely, including the partial and
    the skipped size-1 batch."""
    nd = [700, 513, 300]
    rows, params, plan = _setup(3, nd, seed=2)
    for opt_mode, lr in ((1, 1.0), (0, 0.004)):
        outs = []
        for split in (1, 2, 3):
            dev = params.clone().to(gpu)
            ok, loss = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 1, 128, lr, [5, 6, 7],
                                       opt_mode=opt_mode, split=split)
            assert ok.tolist() == [1, 1, 1]
            outs.append((dev.cpu(), loss))
        for o in outs[1:]:
            d = (outs[0][0] - o[0]).abs().max().item()
            if opt_mode == 1:
                assert d < 1e-5, d
            else:
                moved = (outs[0][0] - params).abs().max().item()
                assert d < 0.1 * moved, (d, moved)
            assert torch.allclose(outs[0][1], o[1], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("split", [3, 4])
def test_training_is_bit_reproducible(gpu, split):
    """A client's result may not depend on the launch that trains it: the multi-rank engine trains
    clients 0-1 on rank 0 and 2-3 on rank 1 and must equal the single-process run of all four (the
    on-chip trainer once summed LayerNorm gradients with fp32 LDS atomics in wave-arrival order)."""
    nd = [700, 650, 900, 801]
    ds = synthetic_icu(5000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(gpu)
    lay = ParamLayout.for_model("TransformerModel")
    params = torch.stack([lay.flatten(build_model("TransformerModel", seed=i).state_dict()) for i in range(4)]).to(gpu)
    plan = make_plan(rows.shape[0], nd, 2, torch.Generator().manual_seed(7), gpu)
    seeds = [101, 102, 103, 104]
    full = []
    for _ in range(2):
        p = params.clone()
        ok, _ = T.train_clients(p, rows, plan.order, plan.nd, 2, 128, 0.004, seeds, split=split)
        assert ok.tolist() == [1, 1, 1, 1]
        full.append(p)
    assert torch.equal(full[0], full[1])
    for lo in (0, 2):
        p = params[lo:lo + 2].clone()
        T.train_clients(p, rows, plan.order[lo:lo + 2].contiguous(), plan.nd[lo:lo + 2], 2, 128, 0.004,
                        seeds[lo:lo + 2], split=split)
        assert torch.equal(p, full[0][lo:lo + 2])


def test_saturated_sigmoid_start_matches_oracle(gpu):
    """The post-Opt-Fang start whose fp32 outputs saturate (tests/test_loss_parity.py): the fused trainer and
    the fp32 oracle both train it (no NaN abort) and end close — torch's BCELoss gradient on both sides."""
    from test_loss_parity import saturated_start

    ds = synthetic_icu(4000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1)
    start = saturated_start()
    plan = make_plan(rows.shape[0], [1000, 1000], 2, [5, 6], "cpu")
    params = torch.stack([start, start])
    ref = params.clone()
    ok_r, loss_r = T.reference_train(ref, rows, plan.order, plan.nd, 2, 128, 0.004, [11, 12])
    dev = params.clone().to(gpu)
    ok, loss = T.train_clients(dev, rows.to(gpu), plan.order.to(gpu), plan.nd, 2, 128, 0.004, [11, 12])
    assert ok.tolist() == ok_r.tolist() == [1, 1]
    assert torch.isfinite(dev).all()
    d = (dev.cpu() - ref).abs()
    moved = (ref - params).abs()
    assert d.mean().item() < 0.15 * moved.mean().item(), (d.mean(), moved.mean())
    assert torch.allclose(loss, loss_r, rtol=0.1, atol=0.05), (loss, loss_r)


def test_auto_split_choice(gpu):
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    assert T.auto_split(8, gpu) == 4
    assert T.auto_split(cus // 3, gpu) == 4
    assert T.auto_split(cus // 3 + 1, gpu) == 4  # more clients: back-to-back split-4 launches (chunked)
    assert T.onchip_capacity(gpu) == cus // 3


def test_cross_wave_column_sums_are_order_independent(gpu):
    """The on-chip trainers' cross-wave gradient column sums (onchip.h lds_addq: partials rounded to integer quanta
    of 2^-34, summed exactly in fp64 LDS atomics) give the same bits whatever order the 8 waves arrive in, with
    adversarial partials (|partial| < 2^16) whose exponents span more than 2^50 and cancel — the unquantised fp64
    atomics they replace were order-independent only within ~2^29 — and equal the exactly rounded sum."""
    from fractions import Fraction

    from attackfl_amd.ops import native

    g = torch.Generator().manual_seed(0)
    W = 8
    mant = 1.0 + torch.rand(W, 64, generator=g)
    expo = torch.tensor([15, -35, 15, -30, 10, -36, 14, -20], dtype=torch.float64)[:, None]
    sign = torch.where(torch.rand(W, 64, generator=g) < 0.5, -1.0, 1.0)
    vals = (sign * mant.double() * torch.pow(2.0, expo)).float()
    vals[2] = -vals[0]  # exact cancellation of the two largest partials: the result lives in the low bits
    outs = {native().fxsum_test(vals.to(gpu), seed, 0).cpu().numpy().tobytes() for seed in range(48)}
    assert len(outs) == 1
    got = torch.frombuffer(bytearray(outs.pop()), dtype=torch.float32)
    q = [[round(Fraction(float(v)) * 2 ** 34) for v in vals[:, j].tolist()] for j in range(64)]
    exp = torch.tensor([float(Fraction(sum(c), 2 ** 34)) for c in q], dtype=torch.float64).float()
    assert torch.equal(got, exp)
    # (the round-4 unquantised fp64 atomics on the same partials, for the log: distinct results over the orders)
    print("fp64 atomics:", len({native().fxsum_test(vals.to(gpu), seed, 1).cpu().numpy().tobytes() for seed in range(48)}),
          "distinct results over 48 launches")
    # a non-finite partial poisons its slot (decoded NaN, as an fp32 sum of a non-finite partial would give); the
    # other slots keep their exact sums
    for badv in (float("nan"), float("inf"), -float("inf")):
        bad = vals.clone()
        bad[3, 5] = badv
        res = native().fxsum_test(bad.to(gpu), 1, 0).cpu()
        assert torch.isnan(res[5]) and not torch.isnan(res[torch.arange(64) != 5]).any(), badv
        assert torch.equal(res[torch.arange(64) != 5], exp[torch.arange(64) != 5])
    # a FINITE partial at or beyond 2^16 saturates to +-(2^50 - 2^26) quanta: the slot stays finite (the fp32
    # reference keeps training such a client) and exact / order-independent; 65535.99 stays unsaturated
    sat = 2 ** 50 - 2 ** 26
    for badv, q_bad in ((65536.0, sat), (-70000.0, -sat), (3.0e38, sat), (65535.99, None)):
        bad = vals.clone()
        bad[3, 5] = badv
        outs = {native().fxsum_test(bad.to(gpu), seed, 0).cpu().numpy().tobytes() for seed in range(8)}
        assert len(outs) == 1, badv
        res = torch.frombuffer(bytearray(outs.pop()), dtype=torch.float32)
        col = [round(Fraction(float(v)) * 2 ** 34) for v in bad[:, 5].tolist()]
        if q_bad is not None:
            col[3] = q_bad
        want = torch.tensor(float(Fraction(sum(col), 2 ** 34)), dtype=torch.float64).float()  # (fp32 decode)
        assert torch.isfinite(res[5]) and torch.equal(res[5], want), (badv, res[5], want)
        assert torch.equal(res[torch.arange(64) != 5], exp[torch.arange(64) != 5])
    # eight poisoned partials in one slot decode as NaN
    bad = vals.clone()
    bad[:, 7] = float("inf")
    assert torch.isnan(native().fxsum_test(bad.to(gpu), 2, 0).cpu()[7])
