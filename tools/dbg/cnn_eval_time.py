"""Time the fused CNNModel validation kernel (cnn2.hip k_cnn2_eval) alone: one model over n ICU-shaped rows, the
round boundary's validation pass.  Loads attackfl_amd/_C.so or the build AFL_NATIVE_SO names (ablation builds:
AFL_DEV_DEFINES=-DCNN2_EVAL_ABL=1 no fc1 weight loads, =2 no conv towers)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from attackfl_amd.eval import cnn_eval_many  # noqa: E402
from attackfl_amd.models import ParamLayout, build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lay = ParamLayout.for_model("CNNModel")
    p = lay.flatten(build_model("CNNModel", seed=0).state_dict()).to(dev)[None].contiguous()
    rows = torch.randn(args.rows, 24, device=dev)
    for _ in range(5):
        cnn_eval_many(p, rows, lay)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(args.iters):
        cnn_eval_many(p, rows, lay)
    t1.record()
    torch.cuda.synchronize()
    print(json.dumps({"rows": args.rows, "us_per_eval": round(t0.elapsed_time(t1) * 1e3 / args.iters, 1)}))


if __name__ == "__main__":
    main()
