"""Micro-benchmark of one launch set of the batched bench step (cfg3 shapes):
nb bootstraps (default 8) of bench.py's synthetic PCs through
ccg_knn_boots_table_dev, one class-level SNN pass over the batch and one
ccg_silhouette_segments_dev, each stage timed in isolation by the library's
hipEvent timers (ms per bootstrap), plus digests of the outputs so variant
builds (--lib, tools/build_variant.sh) can be checked for equal results."""
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
    N, d, L, KT = 100000, 30, 60, 48
    nb = int(os.environ.get("SM_NB", 8))
    reps = int(os.environ.get("SM_REPS", 4))
    n = int(0.9 * N)
    dev = torch.device("cuda", 0)
    pcs, pop = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, dev)
    pcs_cm = pcs.t().contiguous()
    boots_np = np.stack([np.random.default_rng(123 + b).integers(0, N, n) for b in range(nb)]).astype(np.int32)
    boots = torch.from_numpy(boots_np).to(dev)
    uniq = np.array([np.unique(b).size for b in boots_np], np.int32)
    labels = torch.stack([bench.synth_labels(torch, pop, boots[j], L, dev, 1000 + j) for j in range(nb)])
    cmax = int(labels.max().item())
    keys = (boots + (torch.arange(nb, dtype=torch.int32, device=dev) * N)[:, None]).reshape(-1).contiguous()
    eng = Engine(0)
    tab_idx = torch.empty((N, KT), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, KT), dtype=torch.float64, device=dev)
    eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
    m = nb * n
    rows = torch.empty((m, d), dtype=torch.float64, device=dev)
    knn = torch.empty((m, 20), dtype=torch.int32, device=dev)
    sb = bench.SnnBufs(torch, m, 300 * m, dev)
    info = torch.zeros(3 + len(bench.K_NUM), dtype=torch.int64, device=dev)
    means = torch.empty((nb, L), dtype=torch.float64, device=dev)
    nclust = torch.empty((nb, L), dtype=torch.int32, device=dev)
    minsize = torch.empty((nb, L), dtype=torch.int32, device=dev)
    off = np.arange(nb + 1, dtype=np.int64) * n

    def run():
        eng.gather_rows_rm_t(pcs, N, d, boots.reshape(-1), rows)
        eng.knn_boots_table_t(N, d, boots, uniq, rows, 20, tab_idx, tab_d2, knn)
        sb.run(eng, knn, keys, info, n=m)
        eng.silhouette_segments_t(rows, off, [labels[j] for j in range(nb)], cmax, keys, nb * N,
                                  [means[j] for j in range(nb)], [nclust[j] for j in range(nb)],
                                  [minsize[j] for j in range(nb)])
    run()
    torch.cuda.synchronize()
    eng.timing(True)
    for w in ("knn_total", "snn", "silhouette"):
        eng.timing_read(w)
    for _ in range(reps):
        run()
    out = {"lib": os.path.basename(_lib.LIB_PATH), "nb": nb}
    for w in ("knn_total", "snn", "silhouette"):
        ms, c = eng.timing_read(w)
        out[w + "_ms_per_boot"] = round(ms / c / nb, 4)
    torch.cuda.synchronize()
    used = int(sb.off[m].item())
    out["digest_knn"] = int(knn.to(torch.int64).sum().item())
    out["digest_snn"] = [int(x) for x in info.tolist()] + [int(sb.nbr[:used].to(torch.int64).sum().item()),
                                                            int(sb.wpk[:used].to(torch.int64).sum().item())]
    out["digest_sil"] = float(means.sum().item())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
