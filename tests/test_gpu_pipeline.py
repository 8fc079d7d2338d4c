"""End-to-end parity of the host mirror (consensusclustr_amd.consensus) with
the same pipeline assembled from oracle calls, at BASELINE cfg1's shape
(N = 2700 cells, 5 PCs, 100 bootstraps; PBMC3k itself is not on disk, so the
PCs are synthetic).  Covers R/consensusClust.R:388-456 (bootstrap loop,
assignment matrix, co-clustering, consensus kNN + SNN rank, consensus
resolution choice) and :650-692 (getClustAssignments: kNN, SNN number, the
(k, res) loop order, robust scoring and selection, first-copy map-back,
granular cbind).

The clustering function is host code in the reference (Leiden) and is not
part of the engine; here it is a deterministic stand-in (connected
components of the SNN graph above a resolution-dependent weight quantile),
applied identically to the engine's and the oracle's graphs, so any wiring
difference between kNN, SNN, clustering, silhouette and selection shows up.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

N_CELLS, D, NBOOTS = 2700, 5, 100
RES = np.concatenate([np.linspace(0.01, 0.3, 10), np.linspace(0.25, 1.5, 10)])
KNUM = (10, 15, 20)


def components(n, ei, ej, w, res, seed):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    w = np.asarray(w)
    thr = np.quantile(w, min(0.97, 0.35 + 0.4 * res)) if w.size else 0.0
    keep = w >= thr
    g = coo_matrix((np.ones(int(keep.sum())), (np.asarray(ei)[keep], np.asarray(ej)[keep])), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    _, first, inv = np.unique(lab, return_index=True, return_inverse=True)
    rank = np.empty(first.size, np.int64)
    rank[np.argsort(first)] = np.arange(first.size)
    return (rank[inv] + 1).astype(np.int32)  # codes 1..C by first appearance


def _pcs():
    rng = np.random.default_rng(2700)
    centers = rng.normal(scale=3.0, size=(9, D))
    return centers[rng.integers(0, 9, N_CELLS)] + rng.normal(size=(N_CELLS, D))


def _boots():
    return np.stack([np.random.default_rng(123 + b).integers(0, N_CELLS, int(0.9 * N_CELLS))
                     for b in range(NBOOTS)]).astype(np.int32)


def oracle_get_clust_assignments(pca, boot, mode):
    """getClustAssignments (:650-692) from oracle calls."""
    X = O.gather_rows(pca, boot)
    idx, _ = O.knn(X, max(KNUM))
    labs, scores = [], []
    for k in KNUM:
        ei, ej, w = O.snn(idx, k, "number")
        for res in RES:
            lab = components(X.shape[0], ei, ej, w, float(res), 123)
            labs.append(lab)
            if mode == "robust":
                _, m, C = O.silhouette(X, lab)
                scores.append(O.robust_score(C, m, True))  # minSize = 0: min(table) > 0 always
    if mode == "robust":
        choice = O.robust_choice(scores)
        return O.mapback(boot, labs[choice], pca.shape[0]), np.array(scores), choice
    return np.stack([O.mapback(boot, l_, pca.shape[0]) for l_ in labs], axis=1), None, None


@pytest.fixture(scope="module")
def pca():
    return _pcs()


@pytest.mark.parametrize("mode", ["robust", "granular"])
def test_getClustAssignments_matches_oracle_pipeline(engine, pca, mode):
    from consensusclustr_amd.consensus import getClustAssignments
    boots = _boots()
    for b in range(0, NBOOTS, 9 if mode == "robust" else 33):
        got = getClustAssignments(pca, boots[b], clusterFun=components, resRange=RES, kNum=KNUM, mode=mode,
                                  engine=engine, return_details=True)
        want, scores, choice = oracle_get_clust_assignments(pca, boots[b], mode)
        out, det = got
        assert np.array_equal(out, want)
        if mode == "robust":
            np.testing.assert_allclose(det["scores"], scores, rtol=1e-5)
            assert det["choice"] == choice


@pytest.mark.parametrize("via", ["ctx", "group"])
def test_consensus_cluster_matches_oracle_pipeline(engine, pca, via):
    """The R drop-in's loop (R/ccg.R ccgConsensusCore): every bootstrap drawn
    first, batched kNN over bootstraps (through a device group: split over
    its GPUs, ccg_group_knn_boot), then SNN + host clustering + one batched
    silhouette per bootstrap."""
    from consensusclustr_amd.consensus import assignment_matrix, consensus_cluster
    from consensusclustr_amd.sharding import DeviceGroup
    boots = _boots()
    grp = DeviceGroup.open([0]) if via == "group" else None
    try:
        got = consensus_cluster(pca, clusterFun=components, resRange=RES, kNum=KNUM, engine=engine,
                                boot_indices=boots, return_matrix=True, group=grp)
    finally:
        if grp is not None:
            grp.close()
    # oracle: the bootstrap columns, co-clustering, consensus kNN + SNN rank, scoring
    cols = [oracle_get_clust_assignments(pca, boots[b], "robust")[0] for b in range(NBOOTS)]
    A = assignment_matrix(cols)
    assert np.array_equal(got["clustAssignments"], A)
    Ao = A.astype(np.int32)
    Ao[Ao == 0] = -1
    cc = O.cocluster(Ao)
    assert np.array_equal(got["co"], cc["co"].astype(np.uint16))
    assert np.array_equal(got["both"], cc["both"].astype(np.uint16))
    assert np.array_equal(got["jaccardDist"], cc["dist"], equal_nan=True)
    finals = []
    for k in KNUM:
        knn = O.consensus_knn(cc["dist"], N_CELLS, k)
        assert np.array_equal(got["consensus_knn"][:, :k], knn)
        ei, ej, w = O.snn(knn, k, "rank")
        for res in RES:
            finals.append(components(N_CELLS, ei, ej, w, float(res), 123))
    scores = []
    for lab in finals:
        C = np.unique(lab).size
        m = O.silhouette(pca, lab)[1] if 1 < C < N_CELLS / 10 else 0.0
        scores.append(O.consensus_score(C, N_CELLS, m))
    np.testing.assert_allclose(got["scores"], scores, rtol=1e-5)
    choice = O.consensus_choice(scores)
    assert got["choice"] == choice
    assert np.array_equal(got["assignments"], finals[choice])


def test_null_statistics_match_oracle_pipeline(engine):
    """generateNullStatistic's clustering + silhouette (:796-813) for a batch of
    null PC matrices (one batched kNN) vs the oracle run per simulation."""
    from consensusclustr_amd.consensus import NULL_RES_RANGE, null_statistics, null_test_pvalue
    rng = np.random.default_rng(77)
    nulls = [rng.normal(size=(int(n), d)) for n, d in [(600, 5), (750, 5), (420, 8), (900, 3)]]
    nulls.insert(2, None)  # a failed prcomp_irlba -> score 0
    got = null_statistics(nulls, kNum=KNUM, clusterFun=components, engine=engine)
    want = []
    for X in nulls:
        if X is None:
            want.append(0.0)
            continue
        idx, _ = O.knn(X, max(KNUM))
        labs, scores, means, ncl = [], [], [], []
        for k in KNUM:
            ei, ej, w = O.snn(idx, k, "number")
            for res in NULL_RES_RANGE:
                lab = components(X.shape[0], ei, ej, w, float(res), 123)
                _, m, C = O.silhouette(X, lab)
                ok = np.bincount(lab)[1:].min() > 5
                scores.append(O.robust_score(C, m, ok))
                means.append(m)
                ncl.append(C)
        c = O.robust_choice(scores)
        want.append(0.0 if ncl[c] < 2 else means[c])
    assert np.allclose(got, want, rtol=1e-5, atol=0)
    p = null_test_pvalue(0.5, got)
    assert 0.0 <= p <= 1.0
