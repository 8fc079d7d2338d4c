"""Host-side mirror of consensusClust's bootstrap path over the HIP engine.

Function names, argument meaning and return shapes follow the reference
(R/consensusClust.R); all kNN / SNN / silhouette / co-clustering arithmetic
runs in libccg.so.  The host keeps what the reference keeps on the host:
the RNG draw of bootstrap indices, community detection (Leiden), and the
small per-bootstrap decision logic.

Indices are 0-based; "NA" cluster assignments are -1 as after :408.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .cluster_host import louvain
from .engine import Engine

# consensusClust defaults (R/consensusClust.R:126-127)
RES_RANGE = np.concatenate([np.linspace(0.01, 0.3, 10), np.linspace(0.25, 1.5, 10)])
K_NUM = (10, 15, 20)

_DEFAULT_ENGINE = None


def default_engine():
    global _DEFAULT_ENGINE
    if _DEFAULT_ENGINE is None:
        _DEFAULT_ENGINE = Engine(0)
    return _DEFAULT_ENGINE


def _native_louvain(n, ei, ej, w, res, seed):
    return louvain(n, ei, ej, w, resolution=res, seed=seed)


def _cluster_fn(clusterFun):
    if callable(clusterFun):
        return clusterFun
    if clusterFun in ("leiden", "louvain"):
        return _native_louvain
    raise ValueError(f"clusterFun must be 'leiden', 'louvain' or a callable, got {clusterFun!r}")


_POOL = None


def _cluster_all(fn, jobs):
    """fn(*job) for every job, in order.  The built-in clusterer
    (ccg_host_louvain: no shared state, the GIL released) runs the jobs on
    host threads -- the reference runs one bootstrap per BiocParallel worker
    (:391-400); here the clusterings of one bootstrap share the workers.  A
    caller's callable runs serially (its thread safety is unknown)."""
    global _POOL
    if fn is not _native_louvain or len(jobs) < 2:
        return [fn(*j) for j in jobs]
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)))
    return list(_POOL.map(lambda j: fn(*j), jobs))


# ------------------------------------------------------------ decisions --
def _rank_max_position(scores, ties):
    """which(rank(scores, ties.method=ties) == max(...)), na.last=TRUE.

    NaN scores are ranked last (highest) in order of appearance, so the last
    NaN wins; among finite scores ties="first" picks the last maximum and
    ties="last" the first maximum.
    """
    s = np.asarray(scores, dtype=np.float64)
    nan = np.flatnonzero(np.isnan(s))
    if nan.size:
        return int(nan[-1])
    hits = np.flatnonzero(s == s.max())
    return int(hits[-1] if ties == "first" else hits[0])


def robust_choice(scores):
    """R/consensusClust.R:685-686 -- rank(ties.method="first"), which max."""
    return _rank_max_position(scores, "first")


def consensus_choice(scores):
    """R/consensusClust.R:445-456 -- rank(ties.method="last"), which max."""
    return _rank_max_position(scores, "last")


def robust_scores(means, nclust, minsize, minSize=0):
    """Per-clustering scores, R/consensusClust.R:662-670."""
    out = np.empty(len(means))
    for t, (m, c, s) in enumerate(zip(means, nclust, minsize)):
        if c > 1 and s > minSize:
            out[t] = m
        elif s > minSize:
            out[t] = 0.0
        else:
            out[t] = 0.15
    return out


def bootstrap_indices(N, nboots, bootSize=0.9, seed=123):
    """Host RNG draw of bootstrap cell indices (R: sample(..., replace=TRUE), :394).

    n = trunc(bootSize * N) as R's sample() truncates the size.  The stream is
    numpy's (default_rng(seed + b)), not R's L'Ecuyer-CMRG streams; an R
    front-end passes R's own draws through the C ABI instead.
    """
    n = int(bootSize * N)
    return np.stack([np.random.default_rng(seed + b).integers(0, N, n) for b in range(nboots)]).astype(np.int32)


def mapback(boot_idx, labels_boot, N):
    """assignments[match(cellOrder, names(assignments))] (:673), NA -> -1 (:408)."""
    out = np.full(N, -1, np.int32)
    cells, first = np.unique(np.asarray(boot_idx), return_index=True)  # first copy in sample order
    out[cells] = np.asarray(labels_boot)[first]
    return out


# ------------------------------------------------------- bootstrap path --
def getClustAssignments(pca, boot_idx=None, clusterFun="leiden", resRange=RES_RANGE, kNum=K_NUM,
                        mode="robust", cellOrder=None, seed=123, minSize=0, engine=None,
                        return_details=False, knn=None):
    """Mirror of getClustAssignments (R/consensusClust.R:650-692).

    pca: N x d PC matrix of all cells; the clustered matrix is pca[boot_idx]
    (the reference receives pca[sample(...), ] with duplicated row names,
    :394).  boot_idx=None clusters pca itself (the nboots == 1 path, :500).
    cellOrder: only the identity order of pca's rows is supported (the
    reference always passes rownames(pca)).  knn: this bootstrap's n x kmax
    neighbour rows when the caller already searched them in a batch
    (consensus_cluster); None searches here.
    Returns length-N int32 labels (robust) or N x (|kNum|*|resRange|) (granular),
    -1 for cells not in the bootstrap.
    """
    if cellOrder is not None and not np.array_equal(np.asarray(cellOrder), np.arange(pca.shape[0])):
        raise ValueError("cellOrder must be the identity order of pca's rows")
    eng = engine or default_engine()
    pca = np.asarray(pca, dtype=np.float64)
    N = pca.shape[0]
    boot_idx = np.arange(N, dtype=np.int32) if boot_idx is None else np.asarray(boot_idx, np.int32)
    n = boot_idx.size
    kmax = max(kNum)
    if knn is None:
        knn, _ = eng.knn_boot(pca, boot_idx, kmax=kmax, want_dist=False)
        knn = knn[0]
    elif knn.shape != (n, kmax):
        raise ValueError(f"knn must be {n} x {kmax}, got {knn.shape}")
    fn = _cluster_fn(clusterFun)
    # every k in one pass (:656-658); copies of a cell share a row class
    graphs = eng.snn_multi(knn, [int(k) for k in kNum], "number", cell=boot_idx)
    jobs = [(n, *graphs[g], float(res), seed) for g in range(len(kNum)) for res in resRange]  # :653-654, k outer
    lab = np.stack([np.asarray(x, np.int32) for x in _cluster_all(fn, jobs)])
    if mode == "robust":
        X = pca[boot_idx]
        # :664 on the bootstrap rows: widths once per (cell, label), copies weighted
        means, nclust, minsize = eng.silhouette_cells(X, lab, boot_idx, N)
        scores = robust_scores(means, nclust, minsize, minSize)
        choice = robust_choice(scores)
        out = mapback(boot_idx, lab[choice], N)
        if return_details:
            return out, {"scores": scores, "choice": choice, "labels": lab, "knn": knn}
        return out
    if mode == "granular":
        out = np.stack([mapback(boot_idx, l_, N) for l_ in lab], axis=1)  # :688
        return (out, {"labels": lab, "knn": knn}) if return_details else out
    raise ValueError("mode must be 'robust' or 'granular'")


def subcluster_bootstrap_knn(pcas, boot_idx, kmax=20, engine=None):
    """The kNN step of every subcluster's bootstrap in ONE batched call.

    iterate=TRUE (R/consensusClust.R:541-566) re-runs consensusClust on each
    cluster with > minSize cells; each run starts with its own bootstrap loop
    (CS1 -> getClustAssignments, :391-400 / :650-658) on a small N_c x d_c PC
    matrix.  The engine searches all of them together (BASELINE config 5):
    pcas: list of N_c x d_c PC matrices (d_c may differ; smaller ones are
    zero-padded); boot_idx: list of index arrays into each pca (R's sample()
    - 1).  Returns a list of n_c x kmax int32 bootstrap-row indices, each
    identical to eng.knn_boot(pcas[c], boot_idx[c], kmax).
    """
    eng = engine or default_engine()
    mats = [np.asarray(p_, dtype=np.float64)[np.asarray(b_, dtype=np.int64)] for p_, b_ in zip(pcas, boot_idx)]
    return [idx for idx, _ in eng.knn_segments(mats, kmax=kmax, want_dist=False)]


def assignment_matrix(columns):
    """do.call(cbind, ...) (:404) with NA -> -1 (:408), as the B x N
    column-major matrix of the C ABI (0 = not sampled): uint8 when every code
    fits in 1..255, else uint16 (codes up to 65535)."""
    cols = []
    for c in columns:
        c = np.asarray(c)
        cols.extend([c] if c.ndim == 1 else list(c.T))
    A = np.stack(cols).astype(np.int64)
    if A.max() > 65535:
        raise ValueError("cluster codes above 65535 are not supported by the assignment matrix")
    A[A < 0] = 0
    return A.astype(np.uint8 if A.max() <= 255 else np.uint16)


def bootstrap_knn_batches(pca, boots, kmax, engine=None, group=None, batch=32):
    """The kNN of every bootstrap, searched in batches of `batch` bootstraps
    per call (ccg_knn_boot, or ccg_group_knn_boot splitting each batch over
    the group's GPUs).  Yields (b0, knn[b0:b1]) with knn (b1-b0, n, kmax)."""
    eng = engine or default_engine()
    search = group.knn_boot if group is not None else eng.knn_boot
    for b0 in range(0, boots.shape[0], batch):
        b1 = min(boots.shape[0], b0 + batch)
        try:
            knn, _ = search(pca, boots[b0:b1], kmax=kmax, want_dist=False)
        except Exception:  # one bootstrap at a time, so a failure hits only its own column (:397-399)
            knn = None
        yield b0, b1, knn


def consensus_cluster(pca, nboots=100, bootSize=0.9, clusterFun="leiden", resRange=RES_RANGE, kNum=K_NUM,
                      mode="robust", seed=123, engine=None, boot_indices=None, return_matrix=None,
                      merge=False, minStability=0.175, group=None, boot_seed=None, boot_knn=None):
    """The bootstrap + consensus core of consensusClust (R/consensusClust.R:388-456).

    The bootstrap loop runs as the R drop-in does (R/ccg.R ccgConsensusCore):
    every bootstrap's indices are drawn first, the kNN of a batch of
    bootstraps is one engine call (a DeviceGroup `group` splits each batch
    over its GPUs), then per bootstrap the SNN graphs, host clustering and
    one batched silhouette.  seed is the clustering seed (getClustAssignments'
    and cluster_leiden's `seed`); boot_seed (default: seed) seeds the
    bootstrap draws, as BPPARAM = SerialParam(RNGseed = seed) does in the
    reference -- iterate=TRUE forwards BPPARAM but not seed (:562-566).
    boot_knn: (nboots, n, max(kNum)) neighbour rows of every bootstrap when a
    caller already searched them (the level-batched iterate driver).
    Returns dict(assignments=<chosen consensus labels>, clustAssignments=<B x N
    uint8/uint16>, scores=<consensus scores>, choice=<index>, candidates,
    consensus_knn=<N x max(kNum)>) and, when return_matrix (default: N <=
    20000), the packed R-dist-order jaccardDist, co and both.  The consensus
    kNN (:425) comes straight from the assignment matrix through the fused
    co-clustering top-k (ccg_consensus_knn_assign), so the N x N distance is
    only materialised on request.  merge=True adds the cluster merging of
    :458-497 (merge_unstable_clusters) as final_assignments / stability.
    """
    eng = engine or default_engine()
    pca = np.asarray(pca, dtype=np.float64)
    N = pca.shape[0]
    if boot_seed is None:
        boot_seed = seed
    boots = bootstrap_indices(N, nboots, bootSize, boot_seed) if boot_indices is None else np.asarray(boot_indices)
    fn = _cluster_fn(clusterFun)
    columns = []
    if boot_knn is not None:
        batches = [(0, boots.shape[0], boot_knn)]
    else:
        batches = bootstrap_knn_batches(pca, boots, max(kNum), eng, group)
    for b0, b1, knn in batches:  # bplapply(1:nboots), :391-400
        for b in range(b0, b1):
            try:
                columns.append(getClustAssignments(pca, boots[b], clusterFun=fn, resRange=resRange, kNum=kNum,
                                                   mode=mode, seed=seed, engine=eng,
                                                   knn=None if knn is None else knn[b - b0]))
            except Exception:  # tryCatch(..., error = rep(1, N)), :397-399
                columns.append(np.ones(N, np.int32))
    A = assignment_matrix(columns)
    out = {"clustAssignments": A}
    if return_matrix is None:
        return_matrix = N <= 20000
    if return_matrix:
        cc = eng.cocluster(A)  # 1 - parDist(customDist), :411-421
        out.update(jaccardDist=cc["dist"], co=cc["co"], both=cc["both"])
    kmax = max(kNum)
    cknn = eng.consensus_knn_assign(A, kmax)  # dbscan::kNN(jaccardDist, k), :425 (k < kmax: prefixes)
    jobs = []
    for k in kNum:  # :423-441
        ei, ej, w = eng.snn(np.ascontiguousarray(cknn[:, :k]), k, "rank")  # neighborsToSNNGraph(knn, "rank"), :426
        jobs += [(N, ei, ej, w, float(res), seed) for res in resRange]
    finals = [np.asarray(x, np.int32) for x in _cluster_all(fn, jobs)]
    lab = np.stack(finals)
    nuniq = np.array([np.unique(l_).size for l_ in finals])
    # approxSilhouette on the full pca only where it is used, 1 < C < N/10 (:446-452)
    scored = np.flatnonzero((nuniq > 1) & (nuniq < N / 10))
    means = np.zeros(len(finals))
    if scored.size:
        codes = np.stack([np.unique(finals[t], return_inverse=True)[1] + 1 for t in scored]).astype(np.int32)
        means[scored] = eng.silhouette(pca, codes)[0]
    scores = np.where((nuniq > 1) & (nuniq < N / 10), means, np.where(nuniq == N, -1.0, 0.15))
    choice = consensus_choice(scores)
    out.update(assignments=lab[choice], scores=scores, choice=choice, candidates=lab, consensus_knn=cknn)
    if merge:
        m = merge_unstable_clusters(lab[choice], A, kNum, minStability, eng)
        out.update(final_assignments=m["assignments"], stability=m["stability"])
    return out


# ------------------------------------------- after the consensus choice --
# R/consensusClust.R:458-497.  finalAssignments starts as cluster_leiden's
# integer membership; the first small-cluster merge assigns a character
# (colnames(clustDist)[...]), which turns the whole vector into character, so
# from then on table()/factor level order is the lexicographic order of the
# decimal labels.  Labels stay integers here; `is_char` tracks that order.
def _level_order(values, is_char):
    vals = sorted(set(int(v) for v in values))
    return sorted(vals, key=str) if is_char else vals


def _unique_order(values):
    _, first = np.unique(values, return_index=True)
    return [int(values[i]) for i in np.sort(first)]


def _exact_block_sums(simsum, npairs):
    """(K, K, 2) uint64 words -> exact Python-int sums (object array)."""
    K = npairs.shape[0]
    S = np.empty((K, K), dtype=object)
    for p in range(K):
        for q in range(K):
            S[p, q] = (int(simsum[p, q, 1]) << 64) + int(simsum[p, q, 0])
    return S, npairs.astype(object)


def merge_small_clusters(final, A, kNum=K_NUM, engine=None, max_iter=100000):
    """while (min(table(f)) < max(kNum[1], 20)) merge the smallest cluster into
    its nearest by determineHierachy(as.matrix(jaccardDist), f) (:462-467).

    The block sums come from the assignment matrix in one GPU pass
    (ccg_cluster_block_sums); merges add exact sums, so every iteration's
    distance row is the exact block mean, correctly rounded (R: long-double
    two-pass mean).  Returns (labels, is_char)."""
    from fractions import Fraction
    eng = engine or default_engine()
    f = np.asarray(final).astype(np.int64).copy()
    thr = max(int(kNum[0]), 20)
    base = sorted(set(f.tolist()))
    pos = {v: t for t, v in enumerate(base)}
    S, Np = _exact_block_sums(*eng.cluster_block_sums(A, np.array([pos[v] for v in f], np.int32), len(base)))
    members = {v: [pos[v]] for v in base}  # current label -> original clusters
    is_char = False
    for _ in range(max_iter):
        levels = _level_order(f, is_char)
        counts = {v: int((f == v).sum()) for v in levels}
        small = min(levels, key=lambda v: (counts[v], levels.index(v)))  # which.min(table(f))
        if counts[small] >= thr:
            return f, is_char
        best, bestd = None, None
        for v in _unique_order(f):  # which.min over clustDist[small, ] in unique() order
            if v == small:
                d = Fraction(1)  # diag(clustDist) = 1
            else:
                s = sum(S[p, q] + S[q, p] for p in members[small] for q in members[v])
                n = sum(Np[p, q] + Np[q, p] for p in members[small] for q in members[v])
                if n == 0:
                    continue  # NaN: which.min skips NA
                d = 1 - Fraction(s, n << 39)
            if bestd is None or d < bestd:
                best, bestd = v, d
        if best == small:
            raise RuntimeError("merge target is the cluster itself (the reference loops forever here)")
        f[f == small] = best
        members[best] = members[best] + members.pop(small)
        is_char = True
    raise RuntimeError("small-cluster merging did not converge")


def stability_matrix(final, A, is_char=False, engine=None):
    """apply(simplify2array(lapply(boots, pairwiseRand(f[mask], A[, b][mask],
    mode="ratio", adjusted=TRUE))), 2, rowMeans2, na.rm=TRUE) (:470-481).

    Contingency tables of every bootstrap column come from one GPU pass
    (ccg_contingency); the ratio is host arithmetic (ccg_pairwise_rand_ratio).
    Returns None where the reference's tryCatch returns NULL (per-bootstrap
    matrices of different sizes), else the K x K matrix in level order with
    diag 1 and NA -> 1 (:485-487).  pairwiseRand(mode="ratio") fills only the
    lower triangle, so the upper one averages to NA and becomes 1: the merge's
    which(stab == min) then sees each pair once (parity unpinned: bluster is
    not installed; restated from its documented output)."""
    import math
    from .engine import pairwise_rand_ratio
    eng = engine or default_engine()
    f = np.asarray(final).astype(np.int64)
    levels = _level_order(f, is_char)
    pos = {v: t for t, v in enumerate(levels)}
    K = len(levels)
    tab = eng.contingency(A, np.array([pos[v] for v in f], np.int32), K)
    mats = []
    for b in range(tab.shape[0]):
        t = tab[b]
        present = np.flatnonzero(t[:, 1:].sum(1) > 0)  # ref levels in f[mask]
        r = pairwise_rand_ratio(t[present])
        r[np.triu_indices_from(r, 1)] = np.nan  # bluster fills the lower triangle only (upper NA)
        mats.append(r)
    if len({m.shape for m in mats}) != 1:
        return None  # simplify2array cannot stack -> apply() errors -> NULL
    arr = np.stack(mats)
    Kb = arr.shape[1]
    out = np.empty((Kb, Kb))
    for i in range(Kb):
        for j in range(Kb):
            v = arr[:, i, j]
            v = v[~np.isnan(v)]
            out[i, j] = math.fsum(v) / v.size if v.size else np.nan
    np.fill_diagonal(out, 1.0)
    out[np.isnan(out)] = 1.0
    return out


def stability_merge(final, A, stab, minStability=0.175, max_iter=100000):
    """while (min(stabilityMat) < minStability) (:489-495): clustersToMerge =
    as.numeric(which(stab == min, arr.ind=TRUE)) -- 1-based positions, whose
    first two entries are the rows of the first two matches in column-major
    order -- and labels EQUAL to those positions are relabelled (the
    reference compares labels with matrix indices)."""
    f = np.asarray(final).astype(np.int64).copy()
    A = np.array(A, copy=True)
    stab = np.array(stab, dtype=np.float64, copy=True)
    for _ in range(max_iter):
        m = stab.min()
        if not m < minStability:
            return f, A, stab
        rows, cols = np.nonzero((stab == m).T)  # column-major scan: (col, row) pairs
        hits = list(zip(cols, rows))  # (row, col) in column-major order
        flat = [r + 1 for r, _ in hits] + [c + 1 for _, c in hits]
        c1, c2 = flat[0], flat[1]
        f[f == c2] = c1
        A[A == c2] = c1
        stab[c1 - 1, c2 - 1] = 1.0
        stab[c2 - 1, c1 - 1] = 1.0
    raise RuntimeError("stability merging did not converge (the reference loops forever here)")


def merge_unstable_clusters(final, A, kNum=K_NUM, minStability=0.175, engine=None):
    """R/consensusClust.R:458-497 as one step: small-cluster merging by the
    co-clustering block distances, then bootstrap-stability merging.
    Returns dict(assignments, stability (or None), clustAssignments)."""
    f = np.asarray(final).astype(np.int64)
    if np.unique(f).size <= 1:
        return {"assignments": f, "stability": None, "clustAssignments": A}
    f, is_char = merge_small_clusters(f, A, kNum, engine)
    stab = stability_matrix(f, A, is_char, engine)
    if stab is None:
        return {"assignments": np.ones_like(f), "stability": None, "clustAssignments": A}
    f, A2, stab = stability_merge(f, A, stab, minStability)
    return {"assignments": f, "stability": stab, "clustAssignments": A2}


# ------------------------------------------------ null-simulation test --
# testSplits / generateNullStatistic (R/consensusClust.R:759-814, :891-964).
# The null count matrices come from scDesign3 (R, host) and their PCA from
# prcomp_irlba; the engine clusters all null PC matrices of one test together:
# ONE batched kNN over the simulations (ccg_knn_segments), then per
# simulation the SNN graphs, host clustering and one batched silhouette over
# the 3 x 19 candidate clusterings.
NULL_RES_RANGE = np.concatenate([np.arange(0.01, 0.3 + 1e-12, 0.03), np.arange(0.3, 2 + 1e-12, 0.2)])  # :803


def null_statistics(pca_nulls, kNum=K_NUM, clusterFun="leiden", resRange=NULL_RES_RANGE, minSize=5, seed=123,
                    engine=None):
    """generateNullStatistic (:796-813) for every null PC matrix: the mean
    approxSilhouette of getClustAssignments(pcaNull, robust, minSize=5), 0 if
    the PCA failed (None / all NaN) or one cluster was chosen."""
    eng = engine or default_engine()
    fn = _cluster_fn(clusterFun)
    kmax = max(kNum)
    ok = [t for t, p in enumerate(pca_nulls) if p is not None and not np.all(np.isnan(np.asarray(p, np.float64)))]
    out = np.zeros(len(pca_nulls))
    if not ok:
        return out
    mats = [np.asarray(pca_nulls[t], np.float64) for t in ok]
    knns = eng.knn_segments(mats, kmax=kmax, want_dist=False)  # every simulation in one set of launches
    for t, X, (knn, _) in zip(ok, mats, knns):
        n = X.shape[0]
        labels = []
        graphs = eng.snn_multi(np.ascontiguousarray(knn), [int(k) for k in kNum], "number")
        for g, k in enumerate(kNum):  # getClustAssignments' k-outer / resolution-inner loop (:653-654)
            ei, ej, w = graphs[g]
            for res in resRange:
                labels.append(np.asarray(fn(n, ei, ej, w, float(res), seed), np.int32))
        lab = np.stack(labels)
        means, nclust, minsize, _ = eng.silhouette(X, lab)
        choice = robust_choice(robust_scores(means, nclust, minsize, minSize))
        out[t] = 0.0 if nclust[choice] < 2 else means[choice]  # :806-811 (same labels, same mean)
    return out


def null_test_pvalue(silhouette, null_scores):
    """fitdistr(nullDist, 'normal') (MLE: mean, sd with divisor n) and
    1 - pnorm(silhouette, mean, sd) (:939-940)."""
    import math
    x = np.asarray(null_scores, np.float64)
    mu = math.fsum(x) / x.size
    sd = math.sqrt(math.fsum((x - mu) ** 2) / x.size)
    if sd == 0.0:  # pnorm(q, mu, 0) is a point mass at mu: 1 for q >= mu
        return 0.0 if silhouette >= mu else 1.0
    return 1.0 - 0.5 * math.erfc(-((silhouette - mu) / sd) / math.sqrt(2.0))


# ------------------------------------------------------- PCs of a subset --
def choose_pc_num(sdev, pcVar=0.2):
    """pcNum = max(which(cumsum(sdev[1:50]) / sum(sdev) > pcVar)[1], 5) (:356):
    the first (1-based) component count whose share of the summed sdev of
    the top 50 exceeds pcVar, at least 5."""
    s = np.asarray(sdev, np.float64)[:50]
    frac = np.cumsum(s) / s.sum()
    hit = np.flatnonzero(frac > pcVar)
    return max(int(hit[0]) + 1 if hit.size else 5, 5)


def subset_pcs(counts, sf, genes=None, cells=None, pcNum="find", pcVar=0.2, engine=None):
    """The PC matrix of a (sub)cluster (:287, :337-382, iterate=TRUE at :562):
    log1p(counts / sf) on the variable genes, prcomp_irlba with per-gene
    centring and scaling (ccg_pca on the GPU); pcNum "find" (or > 30) takes
    50 components and keeps the first choose_pc_num(sdev, pcVar).
    Returns (pca: n_cells x pcNum, sdev)."""
    eng = engine or default_engine()
    if pcNum == "find" or int(pcNum) > 30:
        x, sdev = eng.pca(counts, sf, genes, cells, npc=50)
        k = choose_pc_num(sdev, pcVar)
        return x[:, :k], sdev
    x, sdev = eng.pca(counts, sf, genes, cells, npc=int(pcNum))
    return x, sdev
