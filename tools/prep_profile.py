"""Host-side profile of the per-round engine path (bench config): cProfile of steady-state rounds only."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from attackfl_amd.config import from_dict  # noqa: E402
from attackfl_amd.fl.engine import FLEngine, build_client_table  # noqa: E402
from attackfl_amd.parallel.comm import LoopbackComm  # noqa: E402
from attackfl_amd.utils.log import set_quiet  # noqa: E402


def main():
    set_quiet(True)
    dev = torch.device("cuda", 0)
    cfg = from_dict({"server": {"num-round": 100, "clients": 8, "mode": sys.argv[1] if len(sys.argv) > 1 else "fedavg",
                                "model": "TransformerModel", "validation": True,
                                "data-distribution": {"num-data-range": [12000, 15000]}},
                     "learning": {"epoch": 5, "batch-size": 128, "learning-rate": 0.004},
                     "data": {"synthetic": True, "train-size": 60000, "test-size": 10000},
                     "engine": {"trainer": "auto", "checkpoint-dir": "/tmp/afl_prep", "seed": 1}, "log_path": "/tmp/afl_prep"})
    comm = LoopbackComm(dev)
    eng = FLEngine(cfg, comm=comm, table=build_client_table(cfg, 1), device=dev, verbose=False)
    eng.client_selection()
    for _ in range(3):
        eng.run_round()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        eng.run_round()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(60)
    print(s.getvalue())
    eng.close()


if __name__ == "__main__":
    main()
