"""Micro-benchmark of the SNN pass (ccg_snn_multi_dev) on one bench-shaped bootstrap.

Same synthetic PCs as bench.py (100k cells x 30 PCs, 90k-row bootstrap),
exact kNN at k=20, then `reps` passes of the k = 10/15/20 NUMBER graphs,
timed with the library's hipEvent timers.  Variants are separate builds of libccg
(tools/build_variant.sh, --lib); run each in its own process.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from consensusclustr_amd import _lib  # noqa: E402
if len(sys.argv) > 2 and sys.argv[1] == "--lib":  # tools only: time a variant build of libccg
    _lib.LIB_PATH = os.path.abspath(sys.argv[2])
import bench  # noqa: E402
from consensusclustr_amd import Engine  # noqa: E402


def main():
    N, d, reps = 100000, 30, 5
    n = int(0.9 * N)
    dev = torch.device("cuda", 0)
    pcs, _ = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, dev)
    boot = torch.from_numpy(np.random.default_rng(123).integers(0, N, n).astype(np.int32)).to(dev)
    eng = Engine(0)
    rows = torch.empty((n, d), dtype=torch.float64, device=dev)
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    eng.gather_rows_t(pcs.t().contiguous(), N, d, boot, rows)
    eng.knn_rows_t(rows, 20, knn)
    caps = [120 * n, 240 * n, 400 * n]
    outs = [(torch.empty(c, dtype=torch.int32, device=dev), torch.empty(c, dtype=torch.int32, device=dev),
             torch.empty(c, dtype=torch.float64, device=dev)) for c in caps]
    ne = torch.zeros(3, dtype=torch.int64, device=dev)
    eng.snn_multi_t(knn, (10, 15, 20), "number", outs, ne)
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("snn")
    for _ in range(reps):
        eng.snn_multi_t(knn, (10, 15, 20), "number", outs, ne)
    ms, cnt = eng.timing_read("snn")
    # the bench's form: union-graph rows only (ccg_snn_rows_dev, no per-graph emit)
    rcap = 700 * n
    ro = (torch.zeros(n + 1, dtype=torch.int64, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),
          torch.empty(rcap, dtype=torch.int32, device=dev), torch.empty(rcap, dtype=torch.int32, device=dev))
    ne2 = torch.zeros(3, dtype=torch.int64, device=dev)
    eng.snn_rows_t(knn, (10, 15, 20), "number", *ro, ne2)
    torch.cuda.synchronize()
    eng.timing_read("snn")
    for _ in range(reps):
        eng.snn_rows_t(knn, (10, 15, 20), "number", *ro, ne2)
    ms2, cnt2 = eng.timing_read("snn")
    assert ne2.tolist() == ne.tolist()
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "snn_multi_ms": ms / cnt, "snn_rows_ms": ms2 / cnt2,
                      "edges": [int(x) for x in ne.tolist()]}))


if __name__ == "__main__":
    main()
