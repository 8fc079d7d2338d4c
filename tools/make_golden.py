"""Generate tests/golden/*.npz parity fixtures with the CPU restatement.

Usage: python tools/make_golden.py
The reference (R) cannot run in this image (no R / Bioconductor), so the
fixtures come from the oracle (oracle/ccg_oracle.c), itself pinned by the
hand-derived known-answer tests in tests/golden/kat.json.  Inputs are
seeded and stored with the outputs; re-running reproduces the files.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def mixture(rng, N, d, C=6, spread=4.0):
    centers = rng.normal(scale=spread, size=(C, d))
    lab = rng.integers(0, C, N)
    return centers[lab] + rng.normal(size=(N, d)), lab


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20241024)

    # --- kNN + SNN on a bootstrap of a Gaussian mixture (duplicates included)
    N, d = 400, 7
    pcs, truth = mixture(rng, N, d)
    boot = rng.integers(0, N, int(0.9 * N)).astype(np.int32)
    X = O.gather_rows(pcs, boot)
    idx, dist = O.knn(X, 20)
    snn = {}
    for k in (10, 15, 20):
        for t in ("number", "rank"):
            ei, ej, w = O.snn(idx, k, t)
            snn[f"snn_{t}_{k}_i"] = ei
            snn[f"snn_{t}_{k}_j"] = ej
            snn[f"snn_{t}_{k}_w"] = w
    np.savez_compressed(os.path.join(OUT, "knn_snn_boot.npz"), pcs=pcs, boot=boot, knn_idx=idx, knn_dist=dist,
                        **snn)

    # --- kNN with exact distance ties (integer lattice, duplicated rows)
    lat = rng.integers(-3, 4, size=(150, 4)).astype(np.float64)
    lat = np.concatenate([lat, lat[:30]])  # explicit duplicates
    tidx, tdist = O.knn(lat, 20)
    np.savez_compressed(os.path.join(OUT, "knn_ties.npz"), rows=lat, knn_idx=tidx, knn_dist=tdist)

    # --- silhouette: several labelings incl. singleton, 1 cluster, identical points
    Xs, lab = mixture(rng, 300, 5, C=4)
    Xs[:10] = Xs[0]  # identical points
    labs = [lab + 1,
            (rng.integers(0, 7, 300) + 1),
            np.ones(300, np.int64),
            np.where(np.arange(300) == 5, 9, lab + 1),  # singleton cluster code 9
            (np.arange(300) % 2) + 1]
    labs = np.stack(labs).astype(np.int32)
    widths, means, ncl = [], [], []
    for l_ in labs:
        w, m, C = O.silhouette(Xs, l_)
        widths.append(w)
        means.append(m)
        ncl.append(C)
    np.savez_compressed(os.path.join(OUT, "silhouette.npz"), x=Xs, labels=labs, widths=np.stack(widths),
                        means=np.array(means), nclust=np.array(ncl))

    # --- co-clustering, robust-sized B with NAs
    B, Nc = 40, 150
    A = rng.integers(1, 9, size=(B, Nc))
    A[rng.random((B, Nc)) < 0.1] = -1
    cc = O.cocluster(A)
    cknn = {f"cknn_{k}": O.consensus_knn(cc["dist"], Nc, k) for k in (10, 15, 20)}
    np.savez_compressed(os.path.join(OUT, "cocluster.npz"), A=A, co=cc["co"], both=cc["both"], dist=cc["dist"],
                        **cknn)

    # --- co-clustering at a granular-sized B (many columns, many clusters)
    Bg, Ng = 6000, 48
    Ag = rng.integers(1, 40, size=(Bg, Ng))
    Ag[rng.random((Bg, Ng)) < 0.3] = -1
    cg = O.cocluster(Ag)
    np.savez_compressed(os.path.join(OUT, "cocluster_granular.npz"), A=Ag.astype(np.int16), co=cg["co"],
                        both=cg["both"], dist=cg["dist"])
    # --- adversarial fp32 collision: two distinct rationals with equal float
    #     ratio (co/both = a/b vs c/d), realisable only at granular-sized B
    b, d = 60001, 60013
    for a in range(30000, 30500):
        c = int(round(a * d / b))
        if a * d != b * c and np.float32(a) / np.float32(b) == np.float32(c) / np.float32(d):
            break
    Bc = max(b, d)
    Acol = np.full((Bc, 4), -1, np.int64)
    Acol[:, 0] = 1
    Acol[:b, 1] = 2
    Acol[:a, 1] = 1
    Acol[:d, 2] = 3
    Acol[:c, 2] = 1
    Acol[:, 3] = rng.integers(1, 3, Bc)
    cc2 = O.cocluster(Acol)
    np.savez_compressed(os.path.join(OUT, "cocluster_collide.npz"), A=Acol.astype(np.int8), co=cc2["co"],
                        both=cc2["both"], dist=cc2["dist"], frac=np.array([a, b, c, d]))
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
