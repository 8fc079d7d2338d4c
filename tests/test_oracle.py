"""The CPU restatement (oracle) against the hand-derived KATs, its own
independent numpy restatement, and the committed golden fixtures."""
import numpy as np
import pytest

import oracle as O


def test_kat_cocluster(kat):
    c = kat["cocluster_4x3"]
    r = O.cocluster(np.array(c["A"]))
    assert r["co"].tolist() == c["co"]
    assert r["both"].tolist() == c["both"]
    assert r["dist"].tolist() == c["dist"]  # bit-exact, incl. the float division


def test_kat_knn_and_snn(kat):
    c = kat["knn_dups_1d"]
    idx, _ = O.knn(np.array(c["rows"]), c["k"])
    assert idx.tolist() == c["idx"]
    for t in ("number", "rank"):
        e = kat[f"snn_{t}_k2"]
        ei, ej, w = O.snn(idx, 2, t)
        assert ei.tolist() == e["i"] and ej.tolist() == e["j"]
        assert np.array_equal(w, np.array(e["w"], float))


def test_kat_silhouette(kat):
    c = kat["silhouette_1d"]
    w, m, C = O.silhouette(np.array(c["x"]), np.array(c["labels"]))
    assert C == 2
    np.testing.assert_allclose(w, c["widths"], rtol=1e-10)
    np.testing.assert_allclose(m, c["mean"], rtol=1e-10)


def test_kat_selection_rules(kat):
    for scores, want in kat["robust_choice"]["cases"]:
        assert O.robust_choice(scores) == want
    for scores, want in kat["consensus_choice"]["cases"]:
        assert O.consensus_choice(scores) == want


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_knn_matches_numpy_restatement(seed):
    rng = np.random.default_rng(seed)
    pcs = rng.normal(size=(120, 6))
    idx = rng.integers(0, 120, 108)
    X = O.gather_rows(pcs, idx)
    a, _ = O.knn(X, 20)
    assert np.array_equal(a, O.py_knn(X, 20))


def test_knn_ties_lattice():
    rng = np.random.default_rng(5)
    X = rng.integers(-2, 3, size=(80, 3)).astype(float)
    a, _ = O.knn(X, 15)
    assert np.array_equal(a, O.py_knn(X, 15))


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_matches_set_restatement(t):
    rng = np.random.default_rng(3)
    X = rng.normal(size=(90, 4))
    idx, _ = O.knn(X, 12)
    for k in (5, 12):
        a = O.snn(idx, k, t)
        b = O.py_snn(idx, k, t)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def test_cocluster_matches_numpy_restatement():
    rng = np.random.default_rng(4)
    A = rng.integers(-1, 5, size=(25, 40))
    A[A == 0] = 3
    a = O.cocluster(A)
    b = O.py_cocluster(A)
    for key in ("co", "both", "dist"):
        assert np.array_equal(a[key], b[key], equal_nan=True)


def test_golden_reproduces(golden):
    g = golden("knn_snn_boot.npz")
    X = O.gather_rows(g["pcs"], g["boot"])
    idx, dist = O.knn(X, 20)
    assert np.array_equal(idx, g["knn_idx"])
    assert np.array_equal(dist, g["knn_dist"])
    for k in (10, 15, 20):
        for t in ("number", "rank"):
            ei, ej, w = O.snn(g["knn_idx"], k, t)
            assert np.array_equal(ei, g[f"snn_{t}_{k}_i"])
            assert np.array_equal(w, g[f"snn_{t}_{k}_w"])
    c = golden("cocluster.npz")
    r = O.cocluster(c["A"])
    assert np.array_equal(r["co"], c["co"]) and np.array_equal(r["dist"], c["dist"])
    for k in (10, 15, 20):
        assert np.array_equal(O.consensus_knn(c["dist"], c["A"].shape[1], k), c[f"cknn_{k}"])


def test_collision_fixture_has_fp32_collisions(golden):
    """customDist holds overlap/U in float (:412-416): distinct rationals can
    share one fp32 ratio at granular B.  The fixture must contain such a pair
    so the GPU epilogue is held to the float division, not the exact ratio."""
    g = golden("cocluster_collide.npz")
    a, b, c, d = (int(v) for v in g["frac"])
    assert a * d != b * c
    assert g["co"][0] == a and g["both"][0] == b and g["co"][1] == c and g["both"][1] == d
    assert g["dist"][0] == g["dist"][1]
    r = O.cocluster(g["A"].astype(np.int32))
    assert np.array_equal(r["dist"], g["dist"])


def test_knn_queries_equals_full_search_rows():
    rng = np.random.default_rng(31)
    X = rng.normal(size=(700, 6))
    X[100:140] = X[0:40]  # duplicates
    full_i, full_d = O.knn(X, 15)
    q = np.array([0, 5, 100, 139, 699], np.int32)
    qi, qd = O.knn_queries(X, 15, q)
    assert np.array_equal(qi, full_i[q])
    assert np.array_equal(qd, full_d[q])
    assert np.array_equal(qi[:, :10], O.py_knn(X, 10)[q])


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
def test_cocluster_rows_equals_packed_triangle(dtype):
    rng = np.random.default_rng(32)
    B, N = 40, 150
    A = rng.integers(0, 300 if dtype == np.uint16 else 6, (B, N)).astype(dtype)
    Ao = A.astype(np.int32)
    Ao[Ao == 0] = -1
    ref = O.py_cocluster(Ao)
    rows = np.array([0, 7, 149], np.int32)
    co, both = O.cocluster_rows(A, rows)
    for t, i in enumerate(rows):
        for j in range(N):
            if j == i:
                continue
            o = O.packed_index(min(i, j), max(i, j), N)
            assert co[t, j] == ref["co"][o] and both[t, j] == ref["both"][o]
        assert both[t, i] == B - (A[:, i] == 0).sum()  # the diagonal: sampled count


def test_block_means_vs_literal_restatement():
    """orc_block_means == determineHierachy(as.matrix(D), f, "distance") restated
    with numpy on the square matrix (within an ulp: R's two-pass long-double mean)."""
    from fractions import Fraction
    rng = np.random.default_rng(11)
    B, N = 30, 160
    A = rng.integers(-1, 5, (B, N)).astype(np.int32)
    D = O.cocluster(A, want=("dist",))["dist"]
    sq = np.zeros((N, N))
    iu = np.triu_indices(N, 1)
    sq[iu] = D
    sq = sq + sq.T
    f = rng.integers(0, 6, N).astype(np.int32)
    got = O.block_means(D, N, f, 6)
    for p in range(6):
        assert got[p, p] == 0
        for q in range(6):
            if p == q:
                continue
            blk = sq[np.ix_(f == p, f == q)].ravel()
            blk = blk[~np.isnan(blk)]
            want = float(sum(Fraction(x) for x in blk) / len(blk))
            assert abs(got[p, q] - want) <= np.spacing(want)


def test_contingency_vs_numpy():
    rng = np.random.default_rng(12)
    A = rng.integers(0, 7, (9, 300)).astype(np.uint8)
    f = rng.integers(0, 4, 300).astype(np.int32)
    tab = O.contingency(A, f, 4, 6)
    for b in range(9):
        for p in range(4):
            for a in range(7):
                assert tab[b, p, a] == np.sum((f == p) & (A[b] == a))


def test_consensus_knn_rows_matches_the_full_distance_path():
    """orc_consensus_knn_rows (from A, rows only) equals orc_cocluster ->
    orc_consensus_knn (the N x N dist) on the same rows, ties included."""
    rng = np.random.default_rng(12)
    for B, N, C in ((30, 257, 3), (400, 600, 9)):
        A = rng.integers(1, C + 1, (B, N)).astype(np.uint8)
        A[rng.random((B, N)) < 0.3] = 0
        Ai = A.astype(np.int32)
        Ai[Ai == 0] = -1
        full = O.consensus_knn(O.cocluster(Ai)["dist"], N, 20)
        rows = np.array([0, 1, N // 2, N - 1], np.int32)
        got, nan = O.consensus_knn_rows(A, rows, 20)
        assert not nan.any()
        assert np.array_equal(got, full[rows])
    A = np.zeros((3, 10), np.uint8)
    A[:, :5] = 1
    _, nan = O.consensus_knn_rows(A, np.array([0, 7], np.int32), 3)
    assert nan.tolist() == [True, True]
