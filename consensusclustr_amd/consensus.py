"""Host-side mirror of consensusClust's bootstrap path over the HIP engine.

Function names, argument meaning and return shapes follow the reference
(R/consensusClust.R); all kNN / SNN / silhouette / co-clustering arithmetic
runs in libccg.so.  The host keeps what the reference keeps on the host:
the RNG draw of bootstrap indices, community detection (Leiden), and the
small per-bootstrap decision logic.

Indices are 0-based; "NA" cluster assignments are -1 as after :408.
"""
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


def _cluster_fn(clusterFun):
    if callable(clusterFun):
        return clusterFun
    if clusterFun in ("leiden", "louvain"):
        return lambda n, ei, ej, w, res, seed: louvain(n, ei, ej, w, resolution=res, seed=seed)
    raise ValueError(f"clusterFun must be 'leiden', 'louvain' or a callable, got {clusterFun!r}")


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
                        return_details=False):
    """Mirror of getClustAssignments (R/consensusClust.R:650-692).

    pca: N x d PC matrix of all cells; the clustered matrix is pca[boot_idx]
    (the reference receives pca[sample(...), ] with duplicated row names,
    :394).  boot_idx=None clusters pca itself (the nboots == 1 path, :500).
    cellOrder: only the identity order of pca's rows is supported (the
    reference always passes rownames(pca)).
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
    knn, _ = eng.knn_boot(pca, boot_idx, kmax=kmax, want_dist=False)
    knn = knn[0]
    fn = _cluster_fn(clusterFun)
    labels = []
    for k in kNum:  # :653-654, k outer, resolution inner
        ei, ej, w = eng.snn(knn, k, "number")  # SNNGraphParam(type="number"), :656-658
        for res in resRange:
            labels.append(np.asarray(fn(n, ei, ej, w, float(res), seed), np.int32))
    lab = np.stack(labels)
    if mode == "robust":
        X = pca[boot_idx]
        means, nclust, minsize, _ = eng.silhouette(X, lab)  # :664 on the bootstrap rows
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


def consensus_cluster(pca, nboots=100, bootSize=0.9, clusterFun="leiden", resRange=RES_RANGE, kNum=K_NUM,
                      mode="robust", seed=123, engine=None, boot_indices=None, return_matrix=None):
    """The bootstrap + consensus core of consensusClust (R/consensusClust.R:388-456).

    Returns dict(assignments=<chosen consensus labels>, clustAssignments=<B x N
    uint8/uint16>, scores=<consensus scores>, choice=<index>, candidates,
    consensus_knn=<N x max(kNum)>) and, when return_matrix (default: N <=
    20000), the packed R-dist-order jaccardDist, co and both.  The consensus
    kNN (:425) comes straight from the assignment matrix through the fused
    co-clustering top-k (ccg_consensus_knn_assign), so the N x N distance is
    only materialised on request.  The later host stages (cluster merging
    :459-497, null test, dendrogram) are out of scope.
    """
    eng = engine or default_engine()
    pca = np.asarray(pca, dtype=np.float64)
    N = pca.shape[0]
    boots = bootstrap_indices(N, nboots, bootSize, seed) if boot_indices is None else np.asarray(boot_indices)
    fn = _cluster_fn(clusterFun)
    columns = []
    for b in range(boots.shape[0]):  # bplapply(1:nboots, ...), :391-400
        try:
            columns.append(getClustAssignments(pca, boots[b], clusterFun=fn, resRange=resRange, kNum=kNum,
                                               mode=mode, seed=seed, engine=eng))
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
    finals = []
    for k in kNum:  # :423-441
        ei, ej, w = eng.snn(np.ascontiguousarray(cknn[:, :k]), k, "rank")  # neighborsToSNNGraph(knn, "rank"), :426
        for res in resRange:
            finals.append(np.asarray(fn(N, ei, ej, w, float(res), seed), np.int32))
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
    return out
