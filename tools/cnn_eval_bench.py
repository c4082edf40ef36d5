"""Times the fused CNNModel eval kernel (cnn2.hip k_cnn2_eval) on the ICU test-set shape: 10000 rows, C models.
Usage: python tools/cnn_eval_bench.py [C ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from attackfl_amd.data import synthetic_icu
from attackfl_amd.eval import cnn_eval_many
from attackfl_amd.models import ParamLayout, build_model


def main():
    dev = torch.device("cuda", 0)
    ds = synthetic_icu(10000, seed=1)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("CNNModel")
    for C in [int(c) for c in sys.argv[1:]] or [1, 8]:
        p = torch.stack([lay.flatten(build_model("CNNModel", seed=i).state_dict()) for i in range(C)]).to(dev)
        for _ in range(3):
            cnn_eval_many(p, rows, lay)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            cnn_eval_many(p, rows, lay)
        torch.cuda.synchronize()
        print(f"C={C}: {(time.perf_counter() - t0) / 10 * 1e6:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
