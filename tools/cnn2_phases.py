"""Per-phase timeline of the CNNModel on-chip trainer (csrc/kernels/cnn2.hip) from its s_memrealtime stamps.

  python tools/cnn2_phases.py [--clients 8] [--rows 13000]

Runs one local round (1 epoch) of C clients and prints, over active steps 8..63, the median per-step time of
each phase (microseconds): tower forward, forward -> head hand-off, head, head -> tower hand-off, tower
backward (+ partial publish), partial barrier, conv owner reduce + Adam + images, fc1 owner, image barrier.
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from attackfl_amd.data import DeviceTable, synthetic_icu
from attackfl_amd.fl.programs import ProgramRunner, make_program
from attackfl_amd.fl.trainers import make_plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rows", type=int, default=13000)
    ap.add_argument("--diag2", action="store_true", help="a -DCNN2_DIAG2 build: split b.dh1+dW into dh1 / dW3 / dW2")
    args = ap.parse_args()
    C, dev = args.clients, "cuda"
    ds = synthetic_icu(max(20000, args.rows + 1))
    table = DeviceTable(ds, dev)
    plan = make_plan(table.n, [args.rows] * C, 1, [11 + c for c in range(C)], dev)
    from attackfl_amd.models import ParamLayout, build_model

    lay = ParamLayout.for_model("CNNModel")
    params = lay.flatten(build_model("CNNModel", seed=0).state_dict())[None].repeat(C, 1).to(dev).contiguous()
    runner = ProgramRunner(make_program("CNNModel", C, 128, dev))
    runner.cnn2_stamps = torch.zeros(C * 32 * 64 * 16, dtype=torch.int64, device=dev)
    for _ in range(2):  # warm + measured
        runner.cnn2_stamps.zero_()
        p = params.clone()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        ok, _ = runner.train(table, p, plan, lr=1e-3, seeds=[5 + c for c in range(C)])
        t1.record()
        torch.cuda.synchronize()
    steps = (args.rows + 127) // 128
    print(f"round: {t0.elapsed_time(t1):.2f} ms for {steps} steps = {1e3 * t0.elapsed_time(t1) / steps:.1f} us/step")
    st = runner.cnn2_stamps.view(C, 32, 64, 16).cpu().double() * 0.01  # 100 MHz ticks -> us
    towers, headr, fc1 = st[:, :24], st[:, 24], st[:, 25:]
    rows = {k: [] for k in ("fwd", "to_head", "head", "to_tower", "bwd", "P_barrier", "conv_owner", "fc1_owner", "fc1_slack",
                            "W_barrier", "step")}
    for c in range(C):
        for k in range(8, 63):
            t = towers[c, :, k]
            tn = towers[c, :, k + 1]
            h = headr[c, k]
            rows["fwd"].append(float((t[:, 1] - t[:, 0]).max()))
            rows["to_head"].append(float(h[0] - t[:, 1].max()))
            rows["head"].append(float(h[1] - h[0]))
            rows["to_tower"].append(float(t[:, 2].min() - h[1]))
            rows["bwd"].append(float((t[:, 3] - t[:, 2]).max()))
            rows["P_barrier"].append(float(t[:, 4].min() - t[:, 3].max()))
            rows["conv_owner"].append(float((t[:, 6] - t[:, 4]).max()))
            rows["fc1_owner"].append(float((fc1[c, :, k, 1] - fc1[c, :, k, 0]).max()))
            rows["fc1_slack"].append(float(tn[:, 8].min() - fc1[c, :, k, 1].max()))
            rows["W_barrier"].append(float(tn[:, 0].min() - t[:, 6].max()))
            rows["step"].append(float(tn[:, 0].min() - t[:, 0].min()))
    fine = {"f.inputs+conv1": (0, 7), "f.conv2": (7, 14), "f.conv3": (14, 8), "o.wait+loads(diag)": (4, 15), "o.adam+publish(diag)": (15, 5), "o.arrive": (5, 6), "f.pool": (8, 9), "f.fc1+publish": (9, 1),
            "b.d1+dfeat": (2, 10), "b.dh3": (10, 11), "b.dh2": (11, 12), "b.dh1+dW": (12, 13), "b.partials": (13, 3)}
    if args.diag2 or not bool((towers[:, :, 8:63, 15] != 0).all()):  # stamp 15 only in -DCNN2_DIAG builds
        fine.pop("o.wait+loads(diag)")
        fine.pop("o.adam+publish(diag)")
    if args.diag2:  # slot 15 = dh1 done, slot 7 = dW3 done (f.inputs+conv1 / f.conv2 are not stamped then)
        for k in ("f.inputs+conv1", "f.conv2", "f.conv3", "o.wait+loads(diag)", "o.adam+publish(diag)"):
            fine.pop(k, None)
        fine.update({"b.dh1": (12, 15), "b.dW3": (15, 7), "b.dW2+sync": (7, 13)})
    for name, (a, b) in fine.items():
        rows[name] = [float((towers[c, :, k, b] - towers[c, :, k, a]).max()) for c in range(C) for k in range(8, 63)]
    # the head's own timeline (wave 0): z1 partial loads + ReLU, fc2 + fc3, output + BCE + d3, d2 + d1 (in
    # registers), the loss barrier, the d1 write-through stores + drain, the hand-off counters
    hfine = {"h.z1": (0, 3), "h.fc2+fc3": (3, 4), "h.out+d3": (4, 5), "h.d2+d1": (5, 6),
             "h.status+drain": (6, 8), "h.arrive": (8, 1)}  # (no loss barrier since the NaN check moved after it)
    if bool((headr[:, 8:63, 8] != 0).all()):
        for name, (a, b) in hfine.items():
            rows[name] = [float(headr[c, k, b] - headr[c, k, a]) for c in range(C) for k in range(8, 63)]
    for k, v in rows.items():
        print(f"{k:12s} median {statistics.median(v):7.2f} us   p90 {sorted(v)[int(0.9 * len(v))]:7.2f}")


if __name__ == "__main__":
    main()
