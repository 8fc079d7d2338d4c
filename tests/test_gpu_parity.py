"""HIP engine vs the oracle and the golden fixtures, through the C ABI.

Bar: bit-exact kNN indices, SNN edges/weights, co/both counts and co-cluster
distances (the distance is a pure function of the integer counts); kNN
distances and silhouette scores within 1e-5 relative (north_star tolerance).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north_star: distances and silhouette scores within 1e-5 relative


def _mixture(rng, N, d, C=8, spread=3.0):
    centers = rng.normal(scale=spread, size=(C, d))
    return centers[rng.integers(0, C, N)] + rng.normal(size=(N, d))


# ----------------------------------------------------------------- kNN --
def test_knn_kat(engine, kat):
    c = kat["knn_dups_1d"]
    rows = np.array(c["rows"])
    idx, _ = engine.knn_boot(rows, np.arange(rows.shape[0]), kmax=c["k"])
    assert idx[0].tolist() == c["idx"]


def test_knn_golden_bootstrap(engine, golden):
    g = golden("knn_snn_boot.npz")
    idx, dist = engine.knn_boot(g["pcs"], g["boot"], kmax=20)
    assert np.array_equal(idx[0], g["knn_idx"])
    np.testing.assert_allclose(dist[0], g["knn_dist"], rtol=RTOL, atol=1e-12)


def test_knn_golden_ties(engine, golden):
    g = golden("knn_ties.npz")
    rows = g["rows"]
    idx, dist = engine.knn_boot(rows, np.arange(rows.shape[0]), kmax=20)
    assert np.array_equal(idx[0], g["knn_idx"])
    np.testing.assert_allclose(dist[0], g["knn_dist"], rtol=RTOL, atol=1e-12)
    # a lattice is full of exact ties at the k-th distance: certification must
    # have refused some rows and sent them to the exact fallback
    q, fb = engine.last_knn_stats
    assert q == rows.shape[0] and fb > 0


@pytest.mark.parametrize("N,d,k", [(3000, 30, 20), (2500, 20, 20), (1800, 5, 15), (700, 50, 10), (1200, 63, 20)])
def test_knn_random_vs_oracle(engine, N, d, k):
    rng = np.random.default_rng(N + d)
    pcs = _mixture(rng, N, d)
    boot = rng.integers(0, N, int(0.9 * N)).astype(np.int32)
    idx, dist = engine.knn_boot(pcs, boot, kmax=k)
    X = O.gather_rows(pcs, boot)
    oi, od = O.knn(X, k)
    assert np.array_equal(idx[0], oi)
    np.testing.assert_allclose(dist[0], od, rtol=RTOL, atol=1e-12)


def test_knn_multi_bootstrap_batch(engine):
    rng = np.random.default_rng(7)
    N, d = 1500, 12
    pcs = _mixture(rng, N, d)
    boots = rng.integers(0, N, (3, 1350)).astype(np.int32)
    idx, _ = engine.knn_boot(pcs, boots, kmax=20)
    for b in range(3):
        oi, _ = O.knn(O.gather_rows(pcs, boots[b]), 20)
        assert np.array_equal(idx[b], oi)


def test_knn_tiny_and_degenerate(engine):
    # n = kmax + 1 (every other row is a neighbour), all-identical rows
    rows = np.zeros((21, 3))
    idx, dist = engine.knn_boot(rows, np.arange(21), kmax=20)
    oi, od = O.knn(rows, 20)
    assert np.array_equal(idx[0], oi)
    assert np.all(dist[0] == 0)
    rng = np.random.default_rng(1)
    rows = rng.normal(size=(33, 2))
    idx, _ = engine.knn_boot(rows, np.arange(33), kmax=20)
    assert np.array_equal(idx[0], O.knn(rows, 20)[0])


def test_knn_heavy_duplication_forces_fallback(engine):
    # 60 distinct cells, 900 draws: every cell has ~15 copies at distance 0.
    # Searched as rows (ccg_knn_rows_dev) the k-th and (k+1)-th neighbours tie
    # and certification must fail; the bootstrap path (ccg_knn_boot ->
    # ccg_knn_boot_dev) searches the 60 distinct cells and expands the copies.
    import torch
    rng = np.random.default_rng(11)
    pcs = rng.normal(size=(60, 8))
    boot = rng.integers(0, 60, 900).astype(np.int32)
    rows = O.gather_rows(pcs, boot)
    oi, _ = O.knn(rows, 20)
    idx, _ = engine.knn_boot(pcs, boot, kmax=20)
    assert np.array_equal(idx[0], oi)
    tr = torch.from_numpy(rows).cuda()
    out = torch.empty((900, 20), dtype=torch.int32, device="cuda")
    _, fb = engine.knn_rows_t(tr, 20, out, stats=True)
    assert np.array_equal(out.cpu().numpy(), oi)
    assert fb > 0


def test_knn_segments_vs_oracle(engine):
    """iterate=TRUE (BASELINE cfg 5): many subclusters' bootstrap matrices in
    one batched call; each segment must equal its own independent kNN."""
    rng = np.random.default_rng(41)
    sizes = [21, 64, 127, 128, 129, 900, 2000, 333, 4100]
    dims = [5, 7, 12, 15, 5, 10, 15, 8, 14]
    mats = []
    for n_s, d_s in zip(sizes, dims):
        X = _mixture(rng, n_s, d_s, C=4)
        if n_s > 300:
            X[: n_s // 10] = X[n_s // 10: 2 * (n_s // 10)]  # bootstrap-like duplicates
        mats.append(X)
    res = engine.knn_segments(mats, kmax=20)
    for X, (idx, dist) in zip(mats, res):
        oi, od = O.knn(X, 20)
        assert np.array_equal(idx, oi)
        np.testing.assert_allclose(dist, od, rtol=RTOL, atol=1e-12)


def test_knn_segments_single_equals_rows(engine):
    rng = np.random.default_rng(42)
    X = _mixture(rng, 3000, 30)
    (idx, _), = engine.knn_segments([X], kmax=15)
    ref, _ = engine.knn_boot(X, np.arange(3000), kmax=15)
    assert np.array_equal(idx, ref[0])


def test_subcluster_bootstrap_knn_matches_per_cluster(engine):
    from consensusclustr_amd.consensus import subcluster_bootstrap_knn
    rng = np.random.default_rng(43)
    pcas = [_mixture(rng, n_c, d_c, C=3) for n_c, d_c in ((400, 5), (1500, 9), (90, 6), (3000, 13))]
    boots = [rng.integers(0, p_.shape[0], int(0.9 * p_.shape[0])) for p_ in pcas]
    got = subcluster_bootstrap_knn(pcas, boots, kmax=20, engine=engine)
    for p_, b_, g in zip(pcas, boots, got):
        ref, _ = engine.knn_boot(p_, b_, kmax=20)
        assert np.array_equal(g, ref[0])


def test_knn_rejects_bad_args(engine):
    from consensusclustr_amd import CcgError
    with pytest.raises(CcgError):
        engine.knn_boot(np.zeros((10, 3)), np.arange(10), kmax=10)  # kmax > n-1
    with pytest.raises(CcgError):
        engine.knn_boot(np.zeros((10, 3)), np.array([0, 1, 50]), kmax=1)  # index out of range


# ----------------------------------------------------------------- SNN --
def test_snn_kat(engine, kat):
    idx = np.array(kat["knn_dups_1d"]["idx"], np.int32)
    for t in ("number", "rank"):
        e = kat[f"snn_{t}_k2"]
        ei, ej, w = engine.snn(idx, 2, t)
        assert ei.tolist() == e["i"] and ej.tolist() == e["j"]
        assert np.array_equal(w, np.array(e["w"], float))


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_golden(engine, golden, t):
    g = golden("knn_snn_boot.npz")
    for k in (10, 15, 20):
        ei, ej, w = engine.snn(g["knn_idx"], k, t)
        assert np.array_equal(ei, g[f"snn_{t}_{k}_i"])
        assert np.array_equal(ej, g[f"snn_{t}_{k}_j"])
        assert np.array_equal(w, g[f"snn_{t}_{k}_w"])


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_large_vs_oracle(engine, t):
    rng = np.random.default_rng(21)
    X = _mixture(rng, 20000, 10)
    idx, _ = engine.knn_boot(X, np.arange(20000), kmax=20)
    for k in (10, 20):
        a = engine.snn(idx[0], k, t)
        b = O.snn(idx[0], k, t)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_hub_overflow_dense_path(engine, t):
    # every node lists nodes 0..k-1 (a hub set) -> gathered lists overflow
    # the LDS capacity and take the dense path
    n, k = 3000, 20
    rng = np.random.default_rng(2)
    idx = np.empty((n, k), np.int32)
    for i in range(n):
        cand = [x for x in range(k + 1) if x != i][:k]
        if i < k + 1:
            idx[i] = cand
        else:
            idx[i, :10] = cand[:10]
            idx[i, 10:] = rng.choice(np.setdiff1d(np.arange(n), [i] + cand[:10]), k - 10, replace=False)
    a = engine.snn(idx, k, t)
    b = O.snn(idx, k, t)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_table_tiers_vs_oracle(engine, t):
    # two groups whose members all list the group's 5 hub nodes: node j's
    # partners p > j are the later group members, so the partner count runs
    # from 0 to ~4000 and crosses the 1024-slot tier, the 2048-slot tier and
    # the block-table path
    n, k = 6000, 20
    rng = np.random.default_rng(5)
    idx = np.empty((n, k), np.int32)
    for i in range(n):
        base = 0 if i < 2000 else 2000
        hubs = [base + h for h in range(6) if base + h != i][:5]
        rest = rng.choice(n, 3 * k, replace=False)
        rest = [int(x) for x in rest if x != i and x not in hubs][:k - 5]
        idx[i] = hubs + rest
    a = engine.snn(idx, k, t)
    b = O.snn(idx, k, t)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_multi_pass_matches_single_graphs(engine, t):
    """One pass over kmax=20 builds the k=10/15/20 graphs (kNum, :653)."""
    import torch
    rng = np.random.default_rng(31)
    X = _mixture(rng, 12000, 16)
    idx, _ = engine.knn_boot(X, np.arange(12000), kmax=20)
    knn_t = torch.from_numpy(idx[0]).cuda()
    ks = (10, 15, 20)
    cap = 12000 * 400
    outs = [(torch.empty(cap, dtype=torch.int32, device="cuda"), torch.empty(cap, dtype=torch.int32, device="cuda"),
             torch.empty(cap, dtype=torch.float64, device="cuda")) for _ in ks]
    ne = torch.zeros(len(ks), dtype=torch.int64, device="cuda")
    engine.snn_multi_t(knn_t, ks, t, outs, ne)
    torch.cuda.synchronize()
    for g, k in enumerate(ks):
        m = int(ne[g].item())
        ei, ej, w = O.snn(idx[0], k, t)
        assert m == ei.size
        assert np.array_equal(outs[g][0][:m].cpu().numpy(), ei)
        assert np.array_equal(outs[g][1][:m].cpu().numpy(), ej)
        assert np.array_equal(outs[g][2][:m].cpu().numpy(), w)


# ---------------------------------------------------------- silhouette --
def test_silhouette_kat(engine, kat):
    c = kat["silhouette_1d"]
    mean, nc, ms, w = engine.silhouette(np.array(c["x"]), np.array(c["labels"]), want_width=True)
    np.testing.assert_allclose(w[0], c["widths"], rtol=RTOL)
    np.testing.assert_allclose(mean[0], c["mean"], rtol=RTOL)
    assert nc[0] == 2 and ms[0] == 2


def test_silhouette_golden(engine, golden):
    g = golden("silhouette.npz")
    lab = g["labels"]
    mean, nc, ms, w = engine.silhouette(g["x"], lab, want_width=True)
    np.testing.assert_allclose(mean, g["means"], rtol=RTOL)
    assert np.array_equal(nc, g["nclust"])
    ok = ~np.isnan(g["widths"])
    assert np.array_equal(np.isnan(w), ~ok)
    np.testing.assert_allclose(w[ok], g["widths"][ok], rtol=RTOL, atol=1e-9)
    for l_ in range(lab.shape[0]):
        assert ms[l_] == np.bincount(lab[l_])[np.bincount(lab[l_]) > 0].min()


def test_silhouette_batch_vs_oracle(engine):
    rng = np.random.default_rng(9)
    X = _mixture(rng, 20000, 30, C=12)
    L = 12
    labs = np.stack([rng.integers(1, 2 + 3 * l_, 20000) for l_ in range(L)]).astype(np.int32)
    mean, nc, _, _ = engine.silhouette(X, labs)
    for l_ in range(L):
        _, m, C = O.silhouette(X, labs[l_])
        np.testing.assert_allclose(mean[l_], m, rtol=RTOL)
        assert nc[l_] == C


def test_silhouette_deterministic(engine):
    rng = np.random.default_rng(10)
    X = _mixture(rng, 5000, 20)
    labs = rng.integers(1, 9, (6, 5000)).astype(np.int32)
    a = engine.silhouette(X, labs)[0]
    b = engine.silhouette(X, labs)[0]
    assert np.array_equal(a, b)  # fixed-point reductions: bitwise reproducible


# -------------------------------------------------------- co-clustering --
def _to_u8(A):
    A = np.array(A, np.int64)
    A[A < 0] = 0
    return A.astype(np.uint8)


def test_cocluster_kat(engine, kat):
    c = kat["cocluster_4x3"]
    r = engine.cocluster(_to_u8(c["A"]))
    assert r["co"].tolist() == c["co"]
    assert r["both"].tolist() == c["both"]
    assert r["dist"].tolist() == c["dist"]


@pytest.mark.parametrize("name", ["cocluster.npz", "cocluster_granular.npz", "cocluster_collide.npz"])
def test_cocluster_golden(engine, golden, name):
    g = golden(name)
    r = engine.cocluster(_to_u8(g["A"]))
    assert np.array_equal(r["co"], g["co"].astype(np.uint16))
    assert np.array_equal(r["both"], g["both"].astype(np.uint16))
    assert np.array_equal(r["dist"], g["dist"], equal_nan=True)  # bitwise, NaN where both == 0


@pytest.mark.parametrize("B,N,C", [(100, 700, 12), (7, 300, 255), (257, 513, 3), (1000, 1024, 40),
                                   (16383, 64, 3), (300, 2048, 17), (33, 1028, 31)])
def test_cocluster_vs_oracle(engine, B, N, C):
    """N % 4 == 0 and B <= 16383 take the fused one-hot kernel (co + 16384*both in
    one accumulator); the others the two-GEMM kernel.  Edge cases: an all-unsampled
    column (no K slots), a column using label 255 (16 slots), B at the fused limit."""
    rng = np.random.default_rng(B * N)
    A = rng.integers(1, C + 1, (B, N))
    A[rng.random((B, N)) < 0.1] = -1
    A[0, :] = -1
    if B > 2:
        A[1, ::7] = 255
    r = engine.cocluster(_to_u8(A))
    o = O.cocluster(A)
    assert np.array_equal(r["co"], o["co"].astype(np.uint16))
    assert np.array_equal(r["both"], o["both"].astype(np.uint16))
    assert np.array_equal(r["dist"], o["dist"], equal_nan=True)


def test_cocluster_row_slabs_concatenate(engine):
    """Row-slab outputs (the multi-GPU split) concatenate to the full triangle."""
    import torch
    from consensusclustr_amd.sharding import row_slabs, slab_pairs
    rng = np.random.default_rng(3)
    B, N = 60, 1000
    A = rng.integers(0, 9, (B, N)).astype(np.uint8)
    full = engine.cocluster(A)
    At = torch.from_numpy(A).cuda()
    parts = []
    for G in (2, 4, 8):
        cuts = row_slabs(N, G)
        parts = []
        for g in range(G):
            P = slab_pairs(N, cuts[g], cuts[g + 1])
            co = torch.empty(max(P, 1), dtype=torch.int16, device="cuda")
            both = torch.empty(max(P, 1), dtype=torch.int16, device="cuda")
            engine.cocluster_t(At, cuts[g], cuts[g + 1], co=co, both=both)
            torch.cuda.synchronize()
            parts.append((co[:P].cpu().numpy().view(np.uint16), both[:P].cpu().numpy().view(np.uint16)))
        assert np.array_equal(np.concatenate([p[0] for p in parts]), full["co"])
        assert np.array_equal(np.concatenate([p[1] for p in parts]), full["both"])


# ------------------------------------------------------ consensus kNN --
def test_consensus_knn_golden(engine, golden):
    g = golden("cocluster.npz")
    N = g["A"].shape[1]
    for k in (10, 15, 20):
        out = engine.consensus_knn(g["co"].astype(np.uint16), g["both"].astype(np.uint16), N, k)
        assert np.array_equal(out, g[f"cknn_{k}"])


def test_consensus_knn_nan_raises(engine):
    A = np.zeros((3, 5), np.uint8)
    A[:, :3] = 1  # cells 3, 4 never sampled
    r = engine.cocluster(A)
    with pytest.raises(ValueError):
        engine.consensus_knn(r["co"], r["both"], 5, 2)


# ---------------------------------------------------- selection + map-back --
def test_select_mapback_robust_and_granular(engine):
    import torch
    from consensusclustr_amd.consensus import mapback, robust_choice, robust_scores
    rng = np.random.default_rng(4)
    N, n, nb, L = 500, 450, 3, 6
    boots = rng.integers(0, N, (nb, n)).astype(np.int32)
    labels = rng.integers(1, 7, (nb, L, n)).astype(np.int32)
    means = rng.random((nb, L))
    means[1, 2] = np.nan
    means[2, 1] = means[2, 4] = means[2].max() + 1  # tie at the max -> last wins
    nclust = np.full((nb, L), 5, np.int32)
    nclust[0, 3] = 1
    minsize = np.full((nb, L), 10, np.int32)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    A = torch.zeros((nb, N), dtype=torch.uint8, device="cuda")
    choice = torch.zeros(nb, dtype=torch.int32, device="cuda")
    engine.select_mapback_t("robust", dev(labels), dev(boots), N, A, 0, means=dev(means), nclust=dev(nclust),
                            minsize=dev(minsize), out_choice=choice)
    Ag = torch.zeros((nb * L, N), dtype=torch.uint8, device="cuda")
    engine.select_mapback_t("granular", dev(labels), dev(boots), N, Ag, 0)
    torch.cuda.synchronize()
    for b in range(nb):
        want = robust_choice(robust_scores(means[b], nclust[b], minsize[b]))
        assert choice[b].item() == want
        col = mapback(boots[b], labels[b, want], N)
        col[col < 0] = 0
        assert np.array_equal(A[b].cpu().numpy(), col.astype(np.uint8))
        for l_ in range(L):
            col = mapback(boots[b], labels[b, l_], N)
            col[col < 0] = 0
            assert np.array_equal(Ag[b * L + l_].cpu().numpy(), col.astype(np.uint8))
