"""Micro-benchmark of ccg_knn_rows_dev at BASELINE cfg3 shapes (n=90000, d=30).

Times the screen kernel and the whole kNN with the library's hipEvent timers.
Variants come from environment variables read by libccg (CCG_KNN_F32,
CCG_KNN_EXP); run each in its own process.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import Engine  # noqa: E402


def main():
    n, d, reps = int(os.environ.get("KM_N", 90000)), int(os.environ.get("KM_D", 30)), 5
    rng = np.random.default_rng(0)
    centers = rng.normal(scale=3.0, size=(12, d))
    X = centers[rng.integers(0, 12, n)] + rng.normal(size=(n, d))
    eng = Engine(0)
    rows = torch.from_numpy(X).cuda()
    idx = torch.empty((n, 20), dtype=torch.int32, device="cuda")
    eng.knn_rows_t(rows, 20, idx)
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("knn_screen")
    eng.timing_read("knn_total")
    for _ in range(reps):
        eng.knn_rows_t(rows, 20, idx)
    scr = eng.timing_read("knn_screen")
    tot = eng.timing_read("knn_total")
    st = eng.knn_rows_t(rows, 20, idx, stats=True)
    out = {"variant": {k: os.environ.get(k) for k in ("CCG_KNN_F32", "CCG_KNN_EXP")},
           "screen_ms": scr[0] / scr[1], "knn_total_ms": tot[0] / tot[1], "fallback": st[1]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
