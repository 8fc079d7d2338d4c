"""Times ccg_pca_csc at BASELINE cfg3's producer shape (2000 genes x 100 000
cells, 50 PCs) from sparse counts.  Run under rocprofv3 --kernel-trace --stats
for per-kernel times; prints the whole call's wall time and the covariance
GEMM's algorithmic fp64 flops (ng (ng + 1) nc: the upper triangle of Z^T Z)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import Engine  # noqa: E402


def main():
    from scipy.sparse import random as sprandom
    G, N, npc = int(os.environ.get("PM_G", 2000)), int(os.environ.get("PM_N", 100000)), 50
    m = sprandom(G, N, density=0.08, format="csc", random_state=23, dtype=np.float64)
    m.data = np.ceil(m.data * 6.0)
    sf = np.random.default_rng(23).lognormal(0, 0.3, N)
    eng = Engine(0)
    eng.pca_csc(m.data, m.indices, m.indptr, G, sf, None, None, npc)  # warm-up (workspace)
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.pca_csc(m.data, m.indices, m.indptr, G, sf, None, None, npc)
        t.append(time.perf_counter() - t0)
    print(json.dumps({"genes": G, "cells": N, "npc": npc, "wall_s": min(t),
                      "cov_gemm_flop": float(G) * (G + 1) * N}))


if __name__ == "__main__":
    main()
