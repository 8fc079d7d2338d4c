"""Diagnostic: ccg_silhouette_segments_dev against per-segment
ccg_silhouette_cells_dev calls, one call at a time with a synchronise after
each (progress on stderr), for the ragged synthetic segments of
tests/test_gpu_sil_segments.py.  Prints per-segment max relative
differences: batch of all segments, and each segment as a batch of one."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    import torch
    from consensusclustr_amd import Engine
    import test_gpu_sil_segments as T
    eng = Engine(0)
    d = int(os.environ.get("DIAG_D", "15"))
    rng = np.random.default_rng(100 + d)
    sizes = [40, 130, 900, 2500, 61, 6000, 300]
    L = 12
    segs = T._segments(rng, sizes, d, L)
    cmax = max(int(s[2].max()) for s in segs)
    ncell = max(s[3] for s in segs)
    off = np.concatenate([[0], np.cumsum([s[0].shape[0] for s in segs])]).astype(np.int64)
    x = torch.from_numpy(np.concatenate([s[0] for s in segs])).cuda()
    cell = torch.from_numpy(np.concatenate([s[1] + q * ncell for q, s in enumerate(segs)]).astype(np.int32)).cuda()
    labels = [torch.from_numpy(s[2]).cuda() for s in segs]
    nseg = len(segs)
    torch.cuda.synchronize()
    log("inputs ok", d, cmax, ncell, off.tolist(), [float(np.abs(s[0]).max()) for s in segs])
    ref = []
    for q in range(nseg):
        mq = torch.empty(L, dtype=torch.float64, device="cuda")
        a, b = int(off[q]), int(off[q + 1])
        eng.silhouette_cells_t(x[a:b], labels[q], cmax, cell[a:b] - q * ncell, ncell, mq,
                               torch.empty(L, dtype=torch.int32, device="cuda"),
                               torch.empty(L, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        ref.append(mq.cpu().numpy())
        log("single", q, "ok")
    for q in range(nseg):  # each segment as a batch of one
        a, b = int(off[q]), int(off[q + 1])
        mq = torch.empty(L, dtype=torch.float64, device="cuda")
        eng.silhouette_segments_t(x[a:b].contiguous(), np.array([0, b - a], np.int64), [labels[q]], cmax,
                                  (cell[a:b] - q * ncell).contiguous(), ncell, [mq])
        torch.cuda.synchronize()
        r = np.abs(mq.cpu().numpy() - ref[q]) / np.abs(ref[q])
        log("batch-of-one", q, "max rel", float(r.max()))
    means = [torch.empty(L, dtype=torch.float64, device="cuda") for _ in range(nseg)]
    eng.silhouette_segments_t(x, off, labels, cmax, cell, nseg * ncell, means)
    torch.cuda.synchronize()
    log("batch ok")
    for q in range(nseg):
        r = np.abs(means[q].cpu().numpy() - ref[q]) / np.abs(ref[q])
        log("batch", q, "max rel", float(r.max()))
    eng.close()


if __name__ == "__main__":
    main()
