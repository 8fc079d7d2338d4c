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
from .consensus import (K_NUM, RES_RANGE, bootstrap_indices, consensus_cluster, default_engine, null_statistics,
                        null_test_pvalue, subset_pcs)


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


def _node_pcs(counts, sf, variableFeatures, all_cells, depth, pcNum, pcVar, nboots, eng):
    """:273-382 for one (sub)cluster: the genes, the PC matrix, or the early
    one-cluster result (returned as ("done", result))."""
    N = all_cells.size
    # explicit top-level features are used as given (a constant one fails the
    # PCA, as in the reference); the reference's own selection (None, and every
    # subcluster) never picks a gene that is constant over the cells
    if variableFeatures is None or depth > 1:
        genes = live_genes(counts, sf, variableFeatures, all_cells)
    else:
        genes = np.asarray(variableFeatures, np.int32)
    if nboots <= 1:
        raise NotImplementedError("nboots <= 1 (the un-bootstrapped path, :498-511) is not mirrored")
    one = {"assignments": ["1"] * N, "pcNum": None, "silhouette": None, "pval": None}
    # :337-382 -- PCs of these cells on the variable genes (a failed PCA -> one cluster;
    # prcomp_irlba cannot return more components than genes or cells)
    npc = 50 if (pcNum == "find" or int(pcNum) > 30) else int(pcNum)
    if genes.size <= npc or N <= npc:
        return "done", one
    try:
        pca, _sdev = subset_pcs(counts, sf, genes, all_cells.astype(np.int32), pcNum, pcVar, eng)
    except CcgError as e:
        if e.code != CCG_ENAN:
            raise
        return "done", one
    return "pca", (pca, genes)


def _node_consensus(pca, all_cells, depth, nboots, bootSize, minStability, clusterFun, resRange, kNum,
                    silhouetteThresh, alpha, mode, seed, boot_seed, null_pcs, eng, boot_knn=None):
    """:388-539 for one (sub)cluster with its PC matrix: bootstraps,
    consensus graph, resolution choice, merging and the null test.  Returns
    (out, final labels)."""
    res = consensus_cluster(pca, nboots=nboots, bootSize=bootSize, clusterFun=clusterFun, resRange=resRange,
                            kNum=kNum, mode=mode, seed=seed, engine=eng, return_matrix=False,
                            merge=True, minStability=minStability, boot_seed=boot_seed, boot_knn=boot_knn)
    final = np.asarray(res["final_assignments"]).astype(np.int64)
    out = {"pcNum": pca.shape[1], "silhouette": None, "pval": None}
    if np.unique(final).size <= 1:  # :628-630
        return out, final, False
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
    return out, final, True


def _children(final, minSize):
    """:542-546: the clusters to subcluster, in unique() order."""
    uniq = list(dict.fromkeys(final.tolist()))
    sizes = {c: int((final == c).sum()) for c in uniq}
    if len(uniq) > 1 and any(s > minSize for s in sizes.values()):
        return [c for c in uniq if sizes[c] > minSize]
    return []


def _attach(labels, idx, sub):
    """:575-577: a subcluster's own labels become c_sub when it split."""
    if len(set(sub)) > 1:
        for t, i in enumerate(idx):
            labels[i] = f"{labels[i]}_{sub[t]}"


def consensusClust(counts, sizeFactors, variableFeatures=None, pcNum="find", pcVar=0.2, nboots=100, bootSize=0.9,
                   minStability=0.175, clusterFun="leiden", resRange=RES_RANGE, kNum=K_NUM, silhouetteThresh=0.45,
                   alpha=0.05, minSize=50, mode="robust", seed=123, iterate=False, null_pcs=None, depth=1,
                   engine=None, subset_inputs=None, cells=None, boot_seed=None, batch_levels=True):
    """consensusClust (R/consensusClust.R:122-632) from counts.

    counts: genes x cells; sizeFactors: per cell; variableFeatures: gene
    indices (None = every gene that varies over the cells; subclusters always
    drop genes constant over their cells).  sizeFactors: one per column of
    counts (subset_inputs must return a full-length array too).  seed: the
    clustering seed; boot_seed (default seed) seeds the bootstrap draws, like
    BPPARAM = SerialParam(RNGseed = seed): the recursive call of :562-566
    forwards BPPARAM but not seed, so subclusters draw their bootstraps from
    the caller's stream seed and cluster with seed 123.
    iterate=True with batch_levels (default): the subcluster tree is walked
    level by level, and the bootstrap kNN of every subcluster of a level is
    one batched engine call (ccg_knn_boot_segments, BASELINE config 5); the
    result equals the depth-first recursion (batch_levels=False) exactly.
    Returns dict(assignments = list of str labels, nested "c_sub" under
    iterate=True as :576, pcNum, silhouette, pval)."""
    counts = np.asarray(counts, np.float64)
    all_cells = np.arange(counts.shape[1]) if cells is None else np.asarray(cells)
    sf = np.asarray(sizeFactors, np.float64)
    if sf.size != counts.shape[1]:
        raise ValueError(f"sizeFactors has {sf.size} entries for {counts.shape[1]} cells (one per column of counts)")
    eng = engine or default_engine()
    if boot_seed is None:
        boot_seed = seed
    common = dict(nboots=nboots, bootSize=bootSize, minStability=minStability, clusterFun=clusterFun,
                  resRange=resRange, kNum=kNum, mode=mode, boot_seed=boot_seed, null_pcs=null_pcs)
    if iterate and batch_levels and depth == 1:
        return _consensus_levels(counts, sf, variableFeatures, all_cells, pcNum, pcVar, silhouetteThresh, alpha,
                                 minSize, seed, subset_inputs, eng, common)
    kind, v = _node_pcs(counts, sf, variableFeatures, all_cells, depth, pcNum, pcVar, nboots, eng)
    if kind == "done":
        return v
    pca, genes = v
    out, final, split = _node_consensus(pca, all_cells, depth, silhouetteThresh=silhouetteThresh, alpha=alpha,
                                        seed=seed, eng=eng, **common)
    labels = [str(v) for v in final]
    if split and iterate:  # :542-578 -- iterate into clusters above minSize
        for c in _children(final, minSize):
            idx = np.flatnonzero(final == c)
            sub_sf, sub_genes = sf, genes
            if subset_inputs is not None:
                sub_sf, sub_genes = subset_inputs(all_cells[idx])
            # the reference's recursive call (:562-566) forwards BPPARAM (the
            # bootstrap streams) but not silhouetteThresh, alpha, minSize or seed
            sub = consensusClust(counts, sub_sf, sub_genes, "find", pcVar, nboots, bootSize, minStability,
                                 clusterFun, resRange, kNum, 0.45, 0.05, 50, mode, 123, True,
                                 null_pcs, depth + 1, eng, subset_inputs, all_cells[idx], boot_seed, False)
            _attach(labels, idx, sub["assignments"])
    out["assignments"] = labels
    return out


def level_bootstrap_knn(pcas, nboots, bootSize, boot_seed, kmax, engine, batch=32):
    """The bootstrap kNN of every subcluster of one iterate=TRUE level in
    batched engine calls (ccg_knn_boot_segments: one segment per (subcluster,
    bootstrap), `batch` bootstraps of every subcluster per call).  Returns
    per PC matrix an (nboots, n, kmax) array, or None for a matrix whose
    bootstraps are too small for a segment (its own consensus_cluster call
    then searches them)."""
    boots = [bootstrap_indices(p.shape[0], nboots, bootSize, boot_seed) for p in pcas]
    ok = [s for s, b in enumerate(boots) if min(np.unique(r).size for r in b) >= kmax + 1]
    out = [None] * len(pcas)
    for s in ok:
        out[s] = np.empty((nboots, boots[s].shape[1], kmax), np.int32)
    # the library's (segment, cell) keys are 31-bit: a call's segments x its
    # stacked cells must stay below 2^31.  Subclusters go into groups that fit
    # with one bootstrap each; each group's batch is cut to fit.
    groups, cur = [], []
    for s in ok:
        trial = cur + [s]
        if len(trial) * sum(pcas[t].shape[0] for t in trial) < 2 ** 31:
            cur = trial
            continue
        if cur:
            groups.append(cur)
        cur = [s] if pcas[s].shape[0] < 2 ** 31 else []
        if not cur:  # too large for any segment call: its own consensus_cluster searches it
            out[s] = None
    if cur:
        groups.append(cur)
    for grp in groups:
        Ntot = sum(pcas[s].shape[0] for s in grp)
        bg = max(1, min(batch, (2 ** 31 - 1) // (Ntot * len(grp))))
        for b0 in range(0, nboots, bg):
            b1 = min(nboots, b0 + bg)
            res = engine.knn_boot_segments([pcas[s] for s in grp], [boots[s][b0:b1] for s in grp], kmax=kmax,
                                           want_dist=False)
            for s, (idx, _) in zip(grp, res):
                out[s][b0:b1] = idx
    return out


def _consensus_levels(counts, sf, variableFeatures, all_cells, pcNum, pcVar, silhouetteThresh, alpha, minSize, seed,
                      subset_inputs, eng, common):
    """iterate=TRUE walked level by level (BASELINE config 5).  Every node of
    a level gets its PCs, then ONE batched bootstrap kNN serves all of them,
    then each node runs its consensus, merging and null test and lists its
    children.  Labels are assembled bottom-up exactly as the recursion does
    (:575-577)."""
    kmax = max(common["kNum"])
    # node: cells, depth, sf, genes(for subset_inputs default), parent link
    root = {"cells": all_cells, "depth": 1, "sf": sf, "vf": variableFeatures, "pcNum": pcNum,
            "thr": silhouetteThresh, "alpha": alpha, "minSize": minSize, "seed": seed}
    order = []
    level = [root]
    while level:
        for nd in level:
            kind, v = _node_pcs(counts, nd["sf"], nd["vf"], nd["cells"], nd["depth"], nd["pcNum"], pcVar,
                                common["nboots"], eng)
            nd["done"] = v if kind == "done" else None
            nd["pca"], nd["genes"] = (None, None) if kind == "done" else v
        live = [nd for nd in level if nd["done"] is None]
        knns = level_bootstrap_knn([nd["pca"] for nd in live], common["nboots"], common["bootSize"],
                                   common["boot_seed"], kmax, eng) if live else []
        nxt = []
        for nd, kn in zip(live, knns):
            out, final, split = _node_consensus(nd["pca"], nd["cells"], nd["depth"], silhouetteThresh=nd["thr"],
                                                alpha=nd["alpha"], seed=nd["seed"], eng=eng, boot_knn=kn, **common)
            nd["out"], nd["final"], nd["kids"] = out, final, []
            nd["pca"] = None
            if not split:
                continue
            for c in _children(final, nd["minSize"]):
                idx = np.flatnonzero(final == c)
                sub_sf, sub_genes = nd["sf"], nd["genes"]
                if subset_inputs is not None:
                    sub_sf, sub_genes = subset_inputs(nd["cells"][idx])
                kid = {"cells": nd["cells"][idx], "depth": nd["depth"] + 1, "sf": sub_sf, "vf": sub_genes,
                       "pcNum": "find", "thr": 0.45, "alpha": 0.05, "minSize": 50, "seed": 123}
                nd["kids"].append((idx, kid))
                nxt.append(kid)
        order += level
        level = nxt
    for nd in reversed(order):  # children before parents
        if nd["done"] is not None:
            nd["result"] = nd["done"]
            continue
        labels = [str(v) for v in nd["final"]]
        for idx, kid in nd["kids"]:
            _attach(labels, idx, kid["result"]["assignments"])
        nd["out"]["assignments"] = labels
        nd["result"] = nd["out"]
    return root["result"]
