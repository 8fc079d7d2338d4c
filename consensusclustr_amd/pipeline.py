"""Host mirror of consensusClust's clustering core over the engine
(R/consensusClust.R:122-632): PCs of the cells, bootstrap consensus, cluster
merging, the null-simulation test and iterative subclustering.

What the reference computes with third-party R packages and what stays on
the host here:
  * size factors (scran deconvolution) and variable features (scry deviance)
    are inputs (``sizeFactors``, ``variableFeatures``); subclusters reuse them
    (the reference recomputes both per subset, :274-299 -- pass
    ``subset_inputs`` to do the same);
  * null count matrices come from scDesign3 in the reference (:909-936); here
    ``null_pcs(depth, cells, n_sims)`` returns the null PC matrices (None = no
    null test);
  * community detection is the host clusterFun (Leiden in R).
Everything of size cells x cells or bootstraps x cells runs in libccg.so.
"""
import numpy as np

from ._lib import CCG_ENAN, CcgError
from .consensus import (K_NUM, RES_RANGE, consensus_cluster, default_engine, null_statistics, null_test_pvalue,
                        subset_pcs)


def live_genes(counts, sf, genes, cells, chunk=256):
    """The genes of `genes` (None = all) whose log1p(counts / sf) varies
    across `cells`.  The reference re-selects deviance features for every
    subset (R/consensusClust.R:290-298, variableFeatures=NULL in the
    recursive call :562-566), which never picks a gene that is constant over
    the subset; prcomp_irlba would fail on one (:368-379)."""
    g = np.arange(counts.shape[0]) if genes is None else np.asarray(genes)
    c = np.asarray(cells)
    s = np.asarray(sf, np.float64)[c]
    keep = np.zeros(g.size, bool)
    for a in range(0, g.size, chunk):
        y = np.log1p(counts[g[a:a + chunk]][:, c] / s[None, :])
        keep[a:a + chunk] = (y.max(1) > y.min(1))
    return g[keep].astype(np.int32)


def _silhouette_mean(eng, pca, labels):
    codes = np.unique(np.asarray(labels), return_inverse=True)[1].astype(np.int32) + 1
    return float(eng.silhouette(np.asarray(pca, np.float64), codes[None, :])[0][0])


def consensusClust(counts, sizeFactors, variableFeatures=None, pcNum="find", pcVar=0.2, nboots=100, bootSize=0.9,
                   minStability=0.175, clusterFun="leiden", resRange=RES_RANGE, kNum=K_NUM, silhouetteThresh=0.45,
                   alpha=0.05, minSize=50, mode="robust", seed=123, iterate=False, null_pcs=None, depth=1,
                   engine=None, subset_inputs=None, cells=None):
    """consensusClust (R/consensusClust.R:122-632) from counts.

    counts: genes x cells; sizeFactors: per cell; variableFeatures: gene
    indices (None = every gene that varies over the cells; subclusters always
    drop genes constant over their cells).  sizeFactors: one per column of
    counts (subset_inputs must return a full-length array too).  Returns dict(assignments = list of str
    labels, nested "c_sub" under iterate=True as :576, pcNum, silhouette,
    pval)."""
    counts = np.asarray(counts, np.float64)
    all_cells = np.arange(counts.shape[1]) if cells is None else np.asarray(cells)
    N = all_cells.size
    sf = np.asarray(sizeFactors, np.float64)
    if sf.size != counts.shape[1]:
        raise ValueError(f"sizeFactors has {sf.size} entries for {counts.shape[1]} cells (one per column of counts)")
    # explicit top-level features are used as given (a constant one fails the
    # PCA, as in the reference); the reference's own selection (None, and every
    # subcluster) never picks a gene that is constant over the cells
    if variableFeatures is None or depth > 1:
        genes = live_genes(counts, sf, variableFeatures, all_cells)
    else:
        genes = np.asarray(variableFeatures, np.int32)
    eng = engine or default_engine()
    if nboots <= 1:
        raise NotImplementedError("nboots <= 1 (the un-bootstrapped path, :498-511) is not mirrored")
    # :337-382 -- PCs of these cells on the variable genes (a failed PCA -> one cluster;
    # prcomp_irlba cannot return more components than genes or cells)
    npc = 50 if (pcNum == "find" or int(pcNum) > 30) else int(pcNum)
    if genes.size <= npc or N <= npc:
        return {"assignments": ["1"] * N, "pcNum": None, "silhouette": None, "pval": None}
    try:
        pca, _sdev = subset_pcs(counts, sf, genes, all_cells.astype(np.int32), pcNum, pcVar, eng)
    except CcgError as e:
        if e.code != CCG_ENAN:
            raise
        return {"assignments": ["1"] * N, "pcNum": None, "silhouette": None, "pval": None}
    # :388-497 -- bootstraps, consensus graph, resolution choice, merging
    res = consensus_cluster(pca, nboots=nboots, bootSize=bootSize, clusterFun=clusterFun, resRange=resRange,
                            kNum=kNum, mode=mode, seed=seed + depth - 1, engine=eng, return_matrix=False,
                            merge=True, minStability=minStability)
    final = np.asarray(res["final_assignments"]).astype(np.int64)
    out = {"pcNum": pca.shape[1], "silhouette": None, "pval": None}
    if np.unique(final).size <= 1:  # :628-630
        out["assignments"] = [str(v) for v in final]
        return out
    # :515-539 -- the null test runs when the silhouette is at or below the
    # threshold (testSplits, :907; the `min(table(...) < 50)` term of :521
    # only opens the branch, testSplits then checks the silhouette itself)
    sil = _silhouette_mean(eng, pca, final)
    out["silhouette"] = sil
    if sil <= silhouetteThresh and null_pcs is not None:
        scores = list(null_statistics(null_pcs(depth, all_cells, 20), kNum, clusterFun, engine=eng, seed=seed))
        p = null_test_pvalue(sil, scores)
        if 0.05 <= p < 0.1:  # :943-952: 20 more simulations
            scores += list(null_statistics(null_pcs(depth, all_cells, 20), kNum, clusterFun, engine=eng, seed=seed))
            p = null_test_pvalue(sil, scores)
        if 0.05 <= p < 0.075:  # :955-964
            scores += list(null_statistics(null_pcs(depth, all_cells, 20), kNum, clusterFun, engine=eng, seed=seed))
            p = null_test_pvalue(sil, scores)
        out["pval"] = p
        if p >= alpha:  # :967-970 (test_splits_seperately = FALSE): reject every split
            final = np.ones_like(final)
    labels = [str(v) for v in final]
    # :542-578 -- iterate into clusters above minSize
    uniq = list(dict.fromkeys(final.tolist()))
    sizes = {c: int((final == c).sum()) for c in uniq}
    if len(uniq) > 1 and iterate and any(s > minSize for s in sizes.values()):
        for c in [c for c in uniq if sizes[c] > minSize]:
            idx = np.flatnonzero(final == c)
            sub_sf, sub_genes = sf, genes
            if subset_inputs is not None:
                sub_sf, sub_genes = subset_inputs(all_cells[idx])
            # the reference's recursive call (:562-566) does not forward
            # silhouetteThresh, alpha, minSize or seed: subclusters use the defaults
            sub = consensusClust(counts, sub_sf, sub_genes, "find", pcVar, nboots, bootSize, minStability,
                                 clusterFun, resRange, kNum, 0.45, 0.05, 50, mode, 123, True,
                                 null_pcs, depth + 1, eng, subset_inputs, all_cells[idx])["assignments"]
            if len(set(sub)) > 1:  # :575-577
                for t, i in enumerate(idx):
                    labels[i] = f"{labels[i]}_{sub[t]}"
    out["assignments"] = labels
    return out
