"""The consensusClust mirror end to end on the GPU (R/consensusClust.R:122-632):
counts -> PCs (ccg_pca) -> bootstrap consensus -> merging -> null test ->
iterate.  Community detection is the deterministic components stand-in of
test_gpu_pipeline (Leiden is host code the engine does not replace); the
checks are on wiring and on recovering well separated populations.  nboots is
60: with fewer bootstraps some cell pairs are never co-sampled and the
consensus kNN stops on NA distances, as dbscan::kNN does in the reference."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _counts(rng, groups, G=200, boost=4.0):
    """Poisson counts for nested populations: groups = list of (top, sub, n)."""
    base = rng.lognormal(0.0, 1.0, G)
    prof = {}
    cols, truth_top, truth_sub = [], [], []
    for top, sub, n in groups:
        key_t = ("t", top)
        if key_t not in prof:
            prof[key_t] = np.exp(boost * (rng.random(G) < 0.2) * rng.choice([-1, 1], G))
        key_s = ("s", top, sub)
        if key_s not in prof:
            prof[key_s] = np.exp(0.7 * boost * (rng.random(G) < 0.15) * rng.choice([-1, 1], G))
        mu = base * prof[key_t] * prof[key_s]
        sf = rng.lognormal(0, 0.2, n)
        cols.append(rng.poisson(mu[:, None] * sf[None, :]))
        truth_top += [top] * n
        truth_sub += [f"{top}_{sub}"] * n
    counts = np.concatenate(cols, axis=1).astype(np.float64)
    sf = counts.sum(0) / counts.sum(0).mean()
    return counts, sf, np.array(truth_top), np.array(truth_sub)


def _components(n, ei, ej, w, res, seed):
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
    return (rank[inv] + 1).astype(np.int32)


def _ari(a, b):
    from sklearn.metrics import adjusted_rand_score
    return adjusted_rand_score(a, b)


def test_consensus_clust_recovers_populations(engine):
    from consensusclustr_amd.pipeline import consensusClust
    rng = np.random.default_rng(1)
    counts, sf, top, _ = _counts(rng, [(1, 1, 400), (2, 1, 350), (3, 1, 300)])
    genes = np.flatnonzero(counts.std(1) > 0).astype(np.int32)
    out = consensusClust(counts, sf, genes, pcNum=10, nboots=60, clusterFun=_components, engine=engine,
                         silhouetteThresh=0.0)
    lab = np.array(out["assignments"])
    assert lab.size == counts.shape[1]
    assert _ari(lab, top) > 0.9, (np.unique(lab, return_counts=True), out)


def test_consensus_clust_null_test_rejects_noise_clusters(engine):
    """A null distribution at least as well clustered as the data -> pval >= alpha -> one cluster (:967-970)."""
    from consensusclustr_amd.pipeline import consensusClust
    rng = np.random.default_rng(2)
    counts, sf, top, _ = _counts(rng, [(1, 1, 300), (2, 1, 300)])
    genes = np.flatnonzero(counts.std(1) > 0).astype(np.int32)

    def null_pcs(depth, cells, k):  # far better separated "null" data
        r = np.random.default_rng(depth)
        return [np.concatenate([r.normal(0, 0.1, (cells.size // 2, 10)),
                                r.normal(50, 0.1, (cells.size - cells.size // 2, 10))]) for _ in range(k)]

    out = consensusClust(counts, sf, genes, pcNum=10, nboots=60, clusterFun=_components, engine=engine,
                         silhouetteThresh=1.0, null_pcs=null_pcs)
    assert out["pval"] is not None and out["pval"] >= 0.05
    assert set(out["assignments"]) == {"1"}


def test_consensus_clust_iterates_into_subclusters(engine):
    from consensusclustr_amd.pipeline import consensusClust
    rng = np.random.default_rng(3)
    counts, sf, top, sub = _counts(rng, [(1, 1, 250), (1, 2, 250), (2, 1, 250), (2, 2, 250)], boost=5.0)
    genes = np.flatnonzero(counts.std(1) > 0).astype(np.int32)
    out = consensusClust(counts, sf, genes, pcNum=10, nboots=60, clusterFun=_components, engine=engine,
                         silhouetteThresh=0.0, iterate=True, minSize=50)
    lab = np.array(out["assignments"])
    # the four groups come out either at the top level or as "c_sub" labels
    # of an iteration (:576); homogeneous subsets must not split further
    assert _ari(lab, sub) > 0.9, np.unique(lab, return_counts=True)
    top_of = np.array([x.split("_")[0] for x in lab])
    for t in np.unique(top_of):  # a subclustered cluster's members all carry its prefix
        parts = {x for x in lab if x.split("_")[0] == t}
        assert len(parts) == 1 or all("_" in x for x in parts)


def test_level_batched_iterate_equals_depth_first_recursion(engine):
    """BASELINE config 5: iterate=TRUE walked level by level with ONE batched
    bootstrap kNN per level (ccg_knn_boot_segments) returns exactly what the
    depth-first recursion of :546-567 returns, on a 4-subcluster case."""
    from consensusclustr_amd.pipeline import consensusClust
    rng = np.random.default_rng(4)
    groups = [(t, s, 180) for t in (1, 2, 3, 4) for s in (1, 2)]
    counts, sf, top, sub = _counts(rng, groups, boost=5.0)
    genes = np.flatnonzero(counts.std(1) > 0).astype(np.int32)
    kw = dict(pcNum=10, nboots=60, clusterFun=_components, engine=engine, silhouetteThresh=0.0, iterate=True,
              minSize=50, seed=7)
    a = consensusClust(counts, sf, genes, batch_levels=True, **kw)
    b = consensusClust(counts, sf, genes, batch_levels=False, **kw)
    assert a["assignments"] == b["assignments"]
    assert a["silhouette"] == b["silhouette"] and a["pcNum"] == b["pcNum"]
    lab = np.array(a["assignments"])
    assert len({x.split("_")[0] for x in lab}) >= 2
