"""Dump the HAR attention forward's keep words and the keep_rc reference for offline layout checks."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from attackfl_amd.ops import layers as Lx
from attackfl_amd.ops import masks, native


def main():
    gpu = torch.device("cuda:0")
    C, B, L, p = 1, 1, 200, 0.1
    Lp = (L + 63) // 64 * 64
    nat = native()
    ctl = Lx.StepCtl.create([3], gpu)
    cc = Lx.StepCtl.create([3], "cpu")
    hm = torch.zeros(C * B * 4, 3, Lp, 16, dtype=torch.bfloat16, device=gpu)
    hm[:, :, :L] = torch.randn(C * B * 4, 3, L, 16, generator=torch.Generator().manual_seed(1)).to(gpu, torch.bfloat16)
    o = torch.zeros(C, B * L, 64, dtype=torch.bfloat16, device=gpu)
    lse2 = torch.zeros(C * B * 4, Lp, device=gpu)
    mask = torch.zeros(C * B * 4, nat.har_mask_words(Lp), dtype=torch.int64, device=gpu)
    nat.har_attn_fwd(hm, o, lse2, B, L, ctl.seeds, ctl.stepctl, 12, p, mask)
    torch.cuda.synchronize()
    ref = masks.keep_rc(cc.key(0), 12, np.arange(L)[:, None], np.arange(L)[None, :], p).numpy()
    torch.save({"words": mask.cpu(), "ref": torch.from_numpy(ref), "L": L, "Lp": Lp}, "gpurun_out/har_mask_dump.pt")
    print("saved", mask.shape)


if __name__ == "__main__":
    main()
