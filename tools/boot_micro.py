"""Per-bootstrap chain at BASELINE cfg3 shapes on ONE stream, timed per stage.

The bench step's bootstrap part (bench.py: gather, kNN from the cell table,
SNN rows for kNum 10/15/20, silhouette of the 60 clusterings over distinct
cells) for BM_BOOTS bootstraps one after another, with the library's hipEvent
timers per stage, plus the cell-table build once.  No overlap between
bootstraps, so stage times are the kernels' isolated cost.  --lib selects a
variant build of libccg (tools/build_variant.sh); run each in its own
process.  Prints one JSON line (ms per bootstrap per stage)."""
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
    N, d, KT, B = 100000, 30, 48, int(os.environ.get("BM_BOOTS", 8))
    n = int(0.9 * N)
    dev = torch.device("cuda", 0)
    pcs, pop = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, dev)
    pcs_cm = pcs.t().contiguous()
    eng = Engine(0)
    boots_np = [np.random.default_rng(123 + b).integers(0, N, n).astype(np.int32) for b in range(B)]
    boots = [torch.from_numpy(b).to(dev) for b in boots_np]
    uniq = [int(np.count_nonzero(np.bincount(b, minlength=N))) for b in boots_np]
    labels = [bench.synth_labels(torch, pop, boots[b], 60, dev, 1000 + b) for b in range(B)]
    cmax = max(int(lb.max().item()) for lb in labels)
    tab_idx = torch.empty((N, KT), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, KT), dtype=torch.float64, device=dev)
    rows = torch.empty((n, d), dtype=torch.float64, device=dev)
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    rcap = 700 * n
    snn = (torch.zeros(n + 1, dtype=torch.int64, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),
           torch.empty(rcap, dtype=torch.int32, device=dev), torch.empty(rcap, dtype=torch.int32, device=dev))
    ned = torch.zeros(3, dtype=torch.int64, device=dev)
    sb = bench.SnnBufs(torch, n, 300 * n, dev)  # the class-level pass (bench.py's)
    info = torch.zeros(6, dtype=torch.int64, device=dev)
    mean = torch.empty(60, dtype=torch.float64, device=dev)
    ncl = torch.empty(60, dtype=torch.int32, device=dev)
    mns = torch.empty(60, dtype=torch.int32, device=dev)

    mode = os.environ.get("BM_SNN", "classes")

    def one(b):
        eng.gather_rows_rm_t(pcs, N, d, boots[b], rows)
        eng.knn_boot_table_t(pcs_cm, N, d, boots[b], uniq[b], rows, 20, tab_idx, tab_d2, knn)
        if mode == "rows":
            eng.snn_rows_t(knn, bench.K_NUM, "number", *snn, ned)
        else:
            sb.run(eng, knn, boots[b], info)
        eng.silhouette_cells_t(rows, labels[b], cmax, boots[b], N, mean, ncl, mns)

    eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
    one(0)
    torch.cuda.synchronize()
    stages = ("knn_screen", "knn_total", "snn", "silhouette")
    eng.timing(True)
    for w in stages:
        eng.timing_read(w)
    eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
    torch.cuda.synchronize()
    table = eng.timing_read("knn_total")
    eng.timing_read("knn_screen")
    for b in range(B):
        one(b)
    torch.cuda.synchronize()
    out = {"lib": os.path.basename(_lib.LIB_PATH), "boots": B, "table_ms": table[0] / max(table[1], 1)}
    for w in stages[1:]:
        ms, cnt = eng.timing_read(w)
        out[w + "_ms_per_boot"] = ms / max(cnt, 1)
    eng.timing(False)
    out["means0"] = float(mean[0].item())
    out["snn_mode"] = mode
    out["edges"] = [int(e) for e in ned.tolist()] if mode == "rows" else [int(e) for e in info.tolist()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
