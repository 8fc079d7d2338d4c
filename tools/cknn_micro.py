"""Times the fused consensus kNN (ccg_consensus_knn_assign_dev, R/consensusClust.R
:421-425) against the co-clustering triangle at the same shape (cfg3: N =
100 000 cells, B = 1000 robust columns; 12 populations, relabelled per
column with 5% flips, 41% unsampled).  Both paths of the kNN are timed: the
triangle + candidate lists (default) and the full-row sub-slabs
(CCG_CKNN_PATH=slab).  Library hipEvent timers (CCG_KT_COCLUSTER covers the
whole kNN call).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import Engine  # noqa: E402


def robust_A(N, B, seed=31):
    g = torch.Generator(device="cuda").manual_seed(seed)
    pop = torch.randint(0, 12, (N,), generator=g, device="cuda")
    A = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    for b in range(B):
        Cb = int(torch.randint(2, 20, (1,), generator=g, device="cuda").item())
        col = (torch.randperm(12, generator=g, device="cuda") % Cb + 1)[pop]
        flip = torch.rand(N, generator=g, device="cuda") < 0.05
        col = torch.where(flip, torch.randint(1, Cb + 1, (N,), generator=g, device="cuda"), col)
        col[torch.rand(N, generator=g, device="cuda") < 0.41] = 0
        A[b] = col.to(torch.uint8)
    return A


def timed(eng, fn, reps=2):
    fn()
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("cocluster")
    for _ in range(reps):
        fn()
    ms, cnt = eng.timing_read("cocluster")
    eng.timing(False)
    return ms / max(cnt, 1)


def main():
    N, B, k = int(os.environ.get("CK_N", 100000)), int(os.environ.get("CK_B", 1000)), 20
    eng = Engine(0)
    A = robust_A(N, B)
    P = N * (N - 1) // 2
    co = torch.empty(P, dtype=torch.int16, device="cuda")
    both = torch.empty(P, dtype=torch.int16, device="cuda")
    t_tri = timed(eng, lambda: eng.cocluster_t(A, 0, N, co=co, both=both))
    del co, both
    out = torch.empty((N, k), dtype=torch.int32, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    t_cand = timed(eng, lambda: eng.consensus_knn_assign_t(A, k, 0, N, out, flag))
    ref = out.clone()
    t_slab, same = None, None
    if not os.environ.get("CK_NO_SLAB"):  # (CK_NO_SLAB=1: profiling runs skip the slow reference path)
        os.environ["CCG_CKNN_PATH"] = "slab"
        t_slab = timed(eng, lambda: eng.consensus_knn_assign_t(A, k, 0, N, out, flag))
        del os.environ["CCG_CKNN_PATH"]
        same = bool(torch.equal(ref, out))
    print(json.dumps({"N": N, "B": B, "k": k, "cocluster_triangle_ms": t_tri, "cknn_triangle_candidates_ms": t_cand,
                      "cknn_full_row_subslabs_ms": t_slab, "ratio_to_triangle": t_cand / t_tri,
                      "paths_identical": same, "nan_flag": int(flag.item())}))


if __name__ == "__main__":
    main()
