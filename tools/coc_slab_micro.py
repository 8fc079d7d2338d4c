"""Time one GPU's co-cluster row slab at a BASELINE cfg4 shape (granular mode).

N = 250 000 cells, B = 60 000 columns (1000 bootstraps x 60 clusterings),
uint8 labels.  The 60 columns of one bootstrap share its sampling mask (10%
of cells unsampled) and have C rising from 2 to 60 with the resolution,
like getClustAssignments' granular cbind (R/consensusClust.R:688).  The
slab is rank 0's of an 8-GPU run (ccg_row_slabs), computed in the
library's column chunks of 16383; co + both outputs (uint16), 15.6 GB.
A is generated on the GPU (15 GB).  Reports ms, the algorithmic
2 * P * (sum C_b + B) rate and its fraction of the 5 POPS int8 peak.
Env: CS_N, CS_B, CS_G (GPUs in the plan), CS_RANK.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import Engine  # noqa: E402
from consensusclustr_amd.sharding import row_slabs, slab_pairs  # noqa: E402


def main():
    N = int(os.environ.get("CS_N", 250000))
    B = int(os.environ.get("CS_B", 60000))
    G = int(os.environ.get("CS_G", 8))
    rank = int(os.environ.get("CS_RANK", 0))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    per = 60
    nb = (B + per - 1) // per
    A = torch.empty((B, N), dtype=torch.uint8, device=dev)
    C = torch.empty(B, dtype=torch.int64)
    truth = torch.randint(0, 1 << 20, (N,), device=dev, generator=g)
    for b in range(nb):
        mask = torch.rand(N, device=dev, generator=g) < 0.1
        for t in range(per):
            col = b * per + t
            if col >= B:
                break
            c = 2 + (58 * t) // (per - 1)
            lab = (truth // (1 + t)) % c + 1
            flip = torch.rand(N, device=dev, generator=g) < 0.05
            lab = torch.where(flip, torch.randint(1, c + 1, (N,), device=dev, generator=g), lab)
            lab[mask] = 0
            A[col] = lab.to(torch.uint8)
            C[col] = c
    cuts = row_slabs(N, G)
    r0, r1 = cuts[rank], cuts[rank + 1]
    P = slab_pairs(N, r0, r1)
    co = torch.empty(P, dtype=torch.int16, device=dev)
    both = torch.empty(P, dtype=torch.int16, device=dev)
    eng = Engine(0)
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("cocluster")
    eng.cocluster_t(A, r0, r1, co=co, both=both)
    ms, cnt = eng.timing_read("cocluster")
    # spot check: one pair against a direct count on the device
    i, j = r0, r0 + 1
    ai, aj = A[:, i].long(), A[:, j].long()
    co_ref = int(((ai == aj) & (ai != 0)).sum())
    both_ref = int(((ai != 0) & (aj != 0)).sum())
    ok = int(co[0].item()) & 0xFFFF == co_ref and int(both[0].item()) & 0xFFFF == both_ref
    ops = 2.0 * P * (int(C.sum()) + B)
    print(json.dumps({"N": N, "B": B, "slab": [r0, r1], "of_gpus": G, "pairs": P, "sumC": int(C.sum()),
                      "coc_ms": ms, "tops": ops / (ms * 1e-3) / 1e12, "frac_of_5000": ops / (ms * 1e-3) / 5e15,
                      "spot_check_ok": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
