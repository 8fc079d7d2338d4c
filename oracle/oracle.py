"""ctypes binding of liboracle.so plus small pure-numpy restatements.

TEST INFRASTRUCTURE ONLY (see package docstring).  Each function cites the
reference line it restates (paths relative to /root/reference).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

__all__ = [
    "build", "lib", "gather_rows", "knn", "snn", "silhouette", "mapback",
    "cocluster", "consensus_knn", "robust_choice", "consensus_choice",
    "py_knn", "py_snn", "py_cocluster", "packed_index", "RES_RANGE", "K_NUM",
    "robust_score", "consensus_score", "knn_queries", "cocluster_rows",
    "block_means", "contingency", "pairwise_rand_ratio", "consensus_knn_rows",
]

# consensusClust defaults, R/consensusClust.R:126-127
RES_RANGE = np.concatenate([np.linspace(0.01, 0.3, 10), np.linspace(0.25, 1.5, 10)])
K_NUM = (10, 15, 20)


def build():
    """Compile liboracle.so with the committed Makefile (gcc, OpenMP)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        i64, i32, p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        L.orc_gather_rows.argtypes = [p, i64, i32, p, i64, p]
        L.orc_knn.argtypes = [p, i64, i32, i32, p, p, i32]
        L.orc_snn.argtypes = [p, i64, i32, i32, i32, p, p, p, p, i64]
        L.orc_silhouette.argtypes = [p, i64, i32, p, p, p]
        L.orc_mapback.argtypes = [p, i64, p, i64, p]
        L.orc_cocluster.argtypes = [p, i64, i64, p, p, p, i32]
        L.orc_consensus_knn.argtypes = [p, i64, i32, p, i32]
        L.orc_knn_queries.argtypes = [p, i64, i32, i32, p, i64, p, p, i32]
        L.orc_cocluster_rows.argtypes = [p, i32, i64, i64, p, i64, p, p, i32]
        L.orc_block_means.argtypes = [p, i64, p, i32, p, i32]
        L.orc_contingency.argtypes = [p, i32, i64, i64, p, i32, i32, p]
        L.orc_consensus_knn_rows.argtypes = [p, i32, i64, i64, p, i64, i32, p, p, i32]
        for f in (L.orc_gather_rows, L.orc_knn, L.orc_snn, L.orc_silhouette,
                  L.orc_mapback, L.orc_cocluster, L.orc_consensus_knn,
                  L.orc_knn_queries, L.orc_cocluster_rows, L.orc_block_means, L.orc_contingency,
                  L.orc_consensus_knn_rows):
            f.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"oracle {what} failed with code {rc}")
    return rc


def gather_rows(pcs, idx):
    """pca[idx, ] (R/consensusClust.R:394) -> n x d row-major float64."""
    pcs_f = np.asfortranarray(pcs, dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    N, d = pcs_f.shape
    X = np.empty((idx.size, d), dtype=np.float64)
    _check(lib().orc_gather_rows(_ptr(pcs_f), N, d, _ptr(idx), idx.size, _ptr(X)), "gather")
    return X


def knn(X, k, nthreads=0):
    """Exact kNN, self excluded, order (fp64 sq-distance, row); see header."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    idx = np.empty((n, k), dtype=np.int32)
    dist = np.empty((n, k), dtype=np.float64)
    _check(lib().orc_knn(_ptr(X), n, d, k, _ptr(idx), _ptr(dist), nthreads), "knn")
    return idx, dist


def knn_queries(X, k, qidx, nthreads=0):
    """orc_knn for the rows qidx only: (idx, dist) of shape (len(qidx), k)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    q = np.ascontiguousarray(qidx, dtype=np.int32)
    n, d = X.shape
    idx = np.empty((q.size, k), dtype=np.int32)
    dist = np.empty((q.size, k), dtype=np.float64)
    _check(lib().orc_knn_queries(_ptr(X), n, d, k, _ptr(q), q.size, _ptr(idx), _ptr(dist), nthreads), "knn_queries")
    return idx, dist


def cocluster_rows(A, rows, nthreads=0):
    """customDist counts of selected rows against every column j.

    A: B x N uint8/uint16 codes (0 = NA).  Returns (co, both) uint32 arrays of
    shape (len(rows), N); entry j = i is included.
    """
    A = np.ascontiguousarray(A)
    assert A.dtype in (np.uint8, np.uint16)
    r = np.ascontiguousarray(rows, dtype=np.int32)
    B, N = A.shape
    co = np.empty((r.size, N), np.uint32)
    both = np.empty((r.size, N), np.uint32)
    _check(lib().orc_cocluster_rows(_ptr(A), 8 * A.dtype.itemsize, N, B, _ptr(r), r.size, _ptr(co), _ptr(both),
                                    nthreads), "cocluster_rows")
    return co, both


def consensus_knn_rows(A, rows, k, nthreads=0):
    """dbscan::kNN(jaccardDist, k)$id rows (R/consensusClust.R:421-425) for
    the selected rows only, from the assignment matrix (orc_consensus_knn_rows).

    A: B x N uint8/uint16 codes (0 = NA).  Returns (idx (len(rows), k) int32
    0-based, nan_row (len(rows),) bool: the row has a never co-sampled pair)."""
    A = np.ascontiguousarray(A)
    assert A.dtype in (np.uint8, np.uint16)
    r = np.ascontiguousarray(rows, dtype=np.int32)
    B, N = A.shape
    out = np.empty((r.size, k), np.int32)
    nan = np.empty(r.size, np.int32)
    _check(lib().orc_consensus_knn_rows(_ptr(A), 8 * A.dtype.itemsize, N, B, _ptr(r), r.size, k, _ptr(out),
                                        _ptr(nan), nthreads), "consensus_knn_rows")
    return out, nan.astype(bool)


def snn(knn_idx, k, type="number"):
    """bluster neighborsToSNNGraph edges (i<j sorted) and weights."""
    knn_idx = np.ascontiguousarray(knn_idx, dtype=np.int32)
    n, ks = knn_idx.shape
    t = {"number": 0, "rank": 1}[type]
    ne = ctypes.c_int64(0)
    L = lib()
    rc = L.orc_snn(_ptr(knn_idx), n, ks, k, t, ctypes.byref(ne), None, None, None, 0)
    if rc not in (0, -4):
        _check(rc, "snn")
    m = ne.value
    ei = np.empty(m, np.int32)
    ej = np.empty(m, np.int32)
    w = np.empty(m, np.float64)
    _check(L.orc_snn(_ptr(knn_idx), n, ks, k, t, ctypes.byref(ne), _ptr(ei), _ptr(ej), _ptr(w), m), "snn")
    return ei, ej, w


def silhouette(X, labels):
    """approxSilhouette(x, labels)[,3] and mean(na.rm=TRUE); returns (width, mean, C)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    m, d = X.shape
    w = np.empty(m, np.float64)
    mean = ctypes.c_double(0)
    C = _check(lib().orc_silhouette(_ptr(X), m, d, _ptr(labels), _ptr(w), ctypes.byref(mean)), "silhouette")
    return w, mean.value, C


def mapback(idx, labels_n, N):
    """assignments[match(cellOrder, names(assignments))] (:673); NA -> -1 (:408)."""
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    labels_n = np.ascontiguousarray(labels_n, dtype=np.int32)
    out = np.empty(N, np.int32)
    _check(lib().orc_mapback(_ptr(idx), idx.size, _ptr(labels_n), N, _ptr(out)), "mapback")
    return out


def cocluster(A, nthreads=0, want=("co", "both", "dist")):
    """customDist + 1 - parDist (:411-421).  A: B x N int labels, -1 = NA.

    Returns dict of packed (R "dist" order) arrays: co, both (uint32), dist (f64).
    """
    A = np.ascontiguousarray(A, dtype=np.int32)
    B, N = A.shape
    P = N * (N - 1) // 2
    co = np.empty(P, np.uint32) if "co" in want else None
    both = np.empty(P, np.uint32) if "both" in want else None
    dist = np.empty(P, np.float64) if "dist" in want else None
    _check(lib().orc_cocluster(_ptr(A), N, B, _ptr(co), _ptr(both), _ptr(dist), nthreads), "cocluster")
    return {"co": co, "both": both, "dist": dist}


def consensus_knn(dist, N, k, nthreads=0):
    """dbscan::kNN(jaccardDist, k)$id (:425), 0-based."""
    dist = np.ascontiguousarray(dist, dtype=np.float64)
    out = np.empty((N, k), np.int32)
    rc = lib().orc_consensus_knn(_ptr(dist), N, k, _ptr(out), nthreads)
    if rc == -3:
        raise ValueError("distances cannot contain NAs for kNN")
    _check(rc, "consensus_knn")
    return out


def packed_index(i, j, N):
    """0-based (i<j) -> offset in the packed upper triangle (== R dist order)."""
    i = np.asarray(i, np.int64)
    j = np.asarray(j, np.int64)
    return i * N - i * (i + 1) // 2 + (j - i - 1)


# ---- host selection rules ---------------------------------------------
def _rank_max_position(scores, ties):
    """which(rank(scores, ties.method=ties) == max(...)) with na.last=TRUE.

    R's rank() ranks NaN/NA last in order of appearance, so any NaN wins
    and the LAST NaN gets the top rank.  Among finite values:
    ties="first" -> the last-occurring maximum gets the top rank;
    ties="last"  -> the first-occurring maximum does.
    """
    s = np.asarray(scores, dtype=np.float64)
    nan = np.flatnonzero(np.isnan(s))
    if nan.size:
        return int(nan[-1])
    mx = s.max()
    hits = np.flatnonzero(s == mx)
    return int(hits[-1] if ties == "first" else hits[0])


def robust_choice(scores):
    """getClustAssignments (:685-686): rank(ties.method="first"), which max."""
    return _rank_max_position(scores, "first")


def consensus_choice(scores):
    """consensusClust (:445-456): rank(ties.method="last"), which max."""
    return _rank_max_position(scores, "last")


def robust_score(n_clusters, sil_mean, min_size_ok=True):
    """Per-bootstrap score rules (:663-670) with minSize=0 (always > minSize)."""
    if n_clusters > 1 and min_size_ok:
        return sil_mean
    if min_size_ok:
        return 0.0
    return 0.15


def consensus_score(n_clusters, N, sil_mean):
    """Consensus scoring rules (:446-452)."""
    if n_clusters > 1 and n_clusters < N / 10:
        return sil_mean
    if n_clusters == N:
        return -1.0
    return 0.15


# ---- independent pure-numpy restatements (small inputs only) ----------
def py_knn(X, k):
    X = np.asarray(X, np.float64)
    n, d = X.shape
    out = np.empty((n, k), np.int64)
    for i in range(n):
        s = np.zeros(n)
        for kk in range(d):  # dimension order, unfused
            t = X[i, kk] - X[:, kk]
            s = s + t * t
        s[i] = np.inf
        order = np.lexsort((np.arange(n), s))
        out[i] = order[:k]
    return out


def py_snn(knn_idx, k, type="number"):
    knn_idx = np.asarray(knn_idx)[:, :k]
    n = knn_idx.shape[0]
    plus = [dict([(i, 0)] + [(int(x), r + 1) for r, x in enumerate(knn_idx[i])]) for i in range(n)]
    edges = {}
    for i in range(n):
        for j in range(i + 1, n):
            shared = set(plus[i]) & set(plus[j])
            if not shared:
                continue
            if type == "number":
                edges[(i, j)] = float(len(shared))
            else:
                r = min(plus[i][s] + plus[j][s] for s in shared)
                edges[(i, j)] = max(k - 0.5 * r, 1e-6)
    keys = sorted(edges)
    ei = np.array([a for a, _ in keys], np.int32)
    ej = np.array([b for _, b in keys], np.int32)
    w = np.array([edges[t] for t in keys], np.float64)
    return ei, ej, w


def py_cocluster(A):
    A = np.asarray(A, np.int64)
    B, N = A.shape
    P = N * (N - 1) // 2
    co = np.empty(P, np.uint32)
    both = np.empty(P, np.uint32)
    dist = np.empty(P, np.float64)
    o = 0
    for i in range(N):
        for j in range(i + 1, N):
            a, c = A[:, i], A[:, j]
            ov = int(np.sum((a == c) & (a != -1)))
            un = int(np.sum((a != -1) & (c != -1)))
            co[o], both[o] = ov, un
            with np.errstate(invalid="ignore", divide="ignore"):
                q = np.float32(ov) / np.float32(un)
            dist[o] = 1.0 - float(q)
            o += 1
    return {"co": co, "both": both, "dist": dist}


def block_means(dist, N, f, K, nthreads=0):
    """determineHierachy(as.matrix(jaccardDist), assignments, return="distance")
    (:699-721) with f = positions 0..K-1 in unique(assignments) order."""
    dist = np.ascontiguousarray(dist, dtype=np.float64)
    f = np.ascontiguousarray(f, dtype=np.int32)
    out = np.empty((K, K), np.float64)
    _check(lib().orc_block_means(_ptr(dist), N, _ptr(f), K, _ptr(out), nthreads), "block_means")
    return out


def contingency(A, f, K, C=None):
    """table(f, A[b, ]) for every bootstrap column b: (B, K, C+1) int32."""
    A = np.ascontiguousarray(A)
    B, N = A.shape
    C = int(A.max()) if C is None else C
    f = np.ascontiguousarray(f, dtype=np.int32)
    tab = np.empty((B, K, C + 1), np.int32)
    _check(lib().orc_contingency(_ptr(A), 8 * A.dtype.itemsize, N, B, _ptr(f), K, C, _ptr(tab)), "contingency")
    return tab


def pairwise_rand_ratio(tab, adjusted=True):
    """bluster::pairwiseRand(ref, alt, mode="ratio", adjusted) from the
    contingency table(ref, alt) (K ref levels x alt levels), :470-474.

    PARITY UNPINNED: bluster is absent; restated from its documented
    definition -- diagonal: fraction of the C(n_p, 2) pairs inside ref cluster
    p that share an alt cluster; off-diagonal: fraction of the n_p n_q pairs
    across p and q that are split in alt; adjusted: (obs - E)/(total - E)
    with E the expectation under random alt labels (p_same = sum_a C(n_a, 2) /
    C(n, 2)).  0/0 -> NaN."""
    t = np.asarray(tab, dtype=np.float64)
    c2 = lambda x: x * (x - 1.0) / 2.0
    n_p = t.sum(1)
    n_a = t.sum(0)
    n = t.sum()
    p_same = c2(n_a).sum() / c2(n) if n > 1 else np.nan
    K = t.shape[0]
    out = np.empty((K, K))
    with np.errstate(invalid="ignore", divide="ignore"):
        for p in range(K):
            for q in range(K):
                if p == q:
                    obs, tot = c2(t[p]).sum(), c2(n_p[p])
                    exp = tot * p_same
                else:
                    tot = n_p[p] * n_p[q]
                    obs = tot - (t[p] * t[q]).sum()
                    exp = tot * (1.0 - p_same)
                out[p, q] = (obs - exp) / (tot - exp) if adjusted else obs / tot
    return out
