"""End-to-end consensus_cluster at BASELINE cfg2 shapes with the host
clusterer, split into engine time and host time ("end-to-end
time with host Leiden, reported separately").

20k cells x 20 PCs (bench.py's synthetic PCs), robust mode, kNum 10/15/20 x
the 20 default resolutions, E2E_BOOTS bootstraps (default 100; cfg2 names
500), then the co-clustering, the consensus kNN, the consensus SNN-rank
graphs, their clusterings and the consensus silhouettes
(consensus.consensus_cluster, R/consensusClust.R:388-456).  The host
clusterer is the drop-in's default, libccg's host Louvain (ccg_host_louvain)
on 16 host threads -- igraph's Leiden is not in this image, so the host
figure is the stand-in's, not igraph's.

Prints one JSON line: wall seconds, and per bootstrap the engine calls
(device work with their host<->device copies, by call), the host clustering
(wall time of the clustering batches) and the rest of the host work.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from consensusclustr_amd import Engine, consensus  # noqa: E402


def main():
    N, d = 20000, 20
    nboots = int(os.environ.get("E2E_BOOTS", 100))
    dev = torch.device("cuda", 0)
    pcs, _ = bench.synth_pcs(torch, N, d, 2000, 20241024 + 2, dev)
    pca = pcs.double().cpu().numpy()
    eng = Engine(0)
    spent = {}

    def timed(name, f):
        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                spent[name] = spent.get(name, 0.0) + time.perf_counter() - t0
        return g

    for name in ("knn_boot", "snn_multi", "silhouette_cells", "cocluster", "consensus_knn_assign", "snn",
                 "silhouette"):
        setattr(eng, name, timed(name, getattr(eng, name)))
    consensus._cluster_all = timed("host_clustering", consensus._cluster_all)
    # warm-up (library load, workspaces, thread pool) on one bootstrap (a
    # consensus over a few bootstraps would leave never-co-sampled pairs: NA
    # distances, which the consensus kNN refuses as dbscan::kNN does)
    consensus.getClustAssignments(pca, consensus.bootstrap_indices(N, 1, 0.9, 99)[0], engine=eng)
    spent.clear()
    t0 = time.perf_counter()
    out = consensus.consensus_cluster(pca, nboots=nboots, engine=eng, return_matrix=False)
    wall = time.perf_counter() - t0
    torch.cuda.synchronize()
    eng_s = sum(v for k, v in spent.items() if k != "host_clustering")
    host_c = spent.get("host_clustering", 0.0)
    res = {
        "workload": f"BASELINE cfg2 end to end: {N} cells x {d} PCs, robust, {nboots} bootstraps (bootSize 0.9), "
                    "kNum 10/15/20 x 20 resolutions, consensus co-clustering + kNN + SNN-rank + clusterings + "
                    "silhouettes (consensus.consensus_cluster)",
        "data": "synthetic: bench.py's NB counts -> PCA",
        "host_clusterer": "ccg_host_louvain (libccg's host Louvain, the Python drop-in's stand-in for "
                          "igraph::cluster_leiden, which is not in this image)",
        "host_threads": min(16, os.cpu_count() or 1),
        "nboots": nboots,
        "wall_s": round(wall, 3),
        "per_boot_ms": {
            "total": round(1e3 * wall / nboots, 2),
            "engine_calls": round(1e3 * eng_s / nboots, 2),
            "host_clustering": round(1e3 * host_c / nboots, 2),
            "other_host": round(1e3 * (wall - eng_s - host_c) / nboots, 2),
        },
        "engine_calls_s": {k: round(v, 3) for k, v in sorted(spent.items()) if k != "host_clustering"},
        "note": "per_boot_ms divides the whole job (bootstraps + consensus stage) by the bootstraps; engine calls "
                "are the host-flavour entry points (copies to and from the device included); the device-resident "
                "bootstrap path bench.py times runs cfg2 at ~7800 bootstraps/s",
        "clusters_chosen": int(np.unique(out["assignments"]).size),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
