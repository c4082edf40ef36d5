"""Host cost of small per-round uploads: pinned -> device .to(non_blocking) vs alternatives."""
import time

import torch

dev = torch.device("cuda", 0)
host = torch.empty(4096, dtype=torch.uint8, pin_memory=True)
dbuf = torch.empty(4096, dtype=torch.uint8, device=dev)
for name, fn in (("to_nonblocking", lambda: host[:512].to(dev, non_blocking=True)),
                 ("copy_nonblocking", lambda: dbuf[:512].copy_(host[:512], non_blocking=True)),
                 ("empty_like", lambda: torch.empty(512, dtype=torch.uint8, device=dev)),
                 ("fill", lambda: dbuf.zero_())):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        fn()
    dt = (time.perf_counter() - t) / 200
    torch.cuda.synchronize()
    print(f"{name}: {dt * 1e6:.1f} us host per call")
