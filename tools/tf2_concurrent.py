"""Two processes on one GPU, each training C clients with the on-chip trainer at the same time
(the multi-rank engine test shares one GPU this way): every client must finish ok with finite
parameters, identical to a single-process run of the same clients.  Diagnostics only."""
import multiprocessing as mp
import sys

sys.path.insert(0, ".")


def work(rank, C, q):
    import torch

    from attackfl_amd.data import synthetic_icu
    from attackfl_amd.fl.trainers import make_plan
    from attackfl_amd.models import ParamLayout, build_model
    from attackfl_amd.ops import transformer as T

    dev = torch.device("cuda", 0)
    ds = synthetic_icu(5000, seed=3)
    rows = torch.cat([ds.vitals, ds.labs, ds.labels[:, None]], 1).to(dev)
    lay = ParamLayout.for_model("TransformerModel")
    res = []
    for it in range(5):
        params = torch.stack([lay.flatten(build_model("TransformerModel", seed=10 * rank + i).state_dict())
                              for i in range(C)]).to(dev)
        plan = make_plan(rows.shape[0], [700 + 50 * i for i in range(C)], 2, [rank * 100 + i + it for i in range(C)], dev)
        ok, loss = T.train_clients(params, rows, plan.order, plan.nd, 2, 128, 0.004, [rank * 7 + i for i in range(C)])
        res.append((ok.tolist(), bool(torch.isfinite(params).all()), [round(float(x), 4) for x in loss[:, -1]]))
    q.put((rank, res))


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ps = [ctx.Process(target=work, args=(r, C, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in ps:
        print(q.get(), flush=True)
    for p in ps:
        p.join()
