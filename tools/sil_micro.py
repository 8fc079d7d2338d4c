"""Micro-benchmark of the batched silhouette (ccg_silhouette_dev) at cfg3
shapes: one 90k-row bootstrap of bench.py's synthetic PCs (d = 30) and 60
synthetic clusterings (bench.synth_labels, drawn per cell).  Reports ms per
call (library hipEvent timer) of the row path (ccg_silhouette_dev) and of the
distinct-cell path (ccg_silhouette_cells_dev).  --lib selects a variant build (tools/build_variant.sh)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from consensusclustr_amd import _lib  # noqa: E402
if len(sys.argv) > 2 and sys.argv[1] == "--lib":
    _lib.LIB_PATH = os.path.abspath(sys.argv[2])
import bench  # noqa: E402
from consensusclustr_amd import Engine  # noqa: E402


def main():
    N, d, reps, L = 100000, 30, 10, 60
    n = int(0.9 * N)
    dev = torch.device("cuda", 0)
    pcs, pop = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, dev)
    boot = torch.from_numpy(np.random.default_rng(123).integers(0, N, n).astype(np.int32)).to(dev)
    eng = Engine(0)
    rows = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.gather_rows_t(pcs.t().contiguous(), N, d, boot, rows)
    labels = bench.synth_labels(torch, pop, boot, L, dev, 1000)
    cmax = int(labels.max().item())
    mean = torch.empty(L, dtype=torch.float64, device=dev)
    ncl = torch.empty(L, dtype=torch.int32, device=dev)
    mns = torch.empty(L, dtype=torch.int32, device=dev)
    eng.silhouette_t(rows, labels, cmax, mean, ncl, mns)
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("silhouette")
    for _ in range(reps):
        eng.silhouette_t(rows, labels, cmax, mean, ncl, mns)
    ms, cnt = eng.timing_read("silhouette")
    mean_rows = mean.clone()
    eng.silhouette_cells_t(rows, labels, cmax, boot, N, mean, ncl, mns)
    torch.cuda.synchronize()
    eng.timing_read("silhouette")
    for _ in range(reps):
        eng.silhouette_cells_t(rows, labels, cmax, boot, N, mean, ncl, mns)
    ms_c, cnt_c = eng.timing_read("silhouette")
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "sil_ms": ms / cnt, "sil_cells_ms": ms_c / cnt_c,
                      "cmax": cmax, "mean0": float(mean_rows[0].item()),
                      "max_abs_diff_cells": float((mean - mean_rows).abs().max().item())}))


if __name__ == "__main__":
    main()
