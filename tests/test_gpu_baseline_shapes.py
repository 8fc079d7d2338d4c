"""Parity at the BASELINE.json configurations' sizes.

cfg2 (20k cells, 20 PCs, n = 18 000): the whole bootstrap kNN against the
oracle's full scan, SNN k = 10/15/20 and silhouettes.  cfg3 (100k cells, 30
PCs, n = 90 000): every row's kNN from the engine, 4096 sampled rows checked
against the oracle's exact scan (orc_knn_queries); SNN at n = 90 000 against
orc_snn on the same neighbour lists.  cfg4 (250k cells, granular, B = 60 000
columns): co-clustering counts through the column-chunked kernel, sampled
rows checked against orc_cocluster_rows, at N = 4096 over the whole
triangle and on row slabs of the full N = 250 000 matrix.  cfg5
(iterate=TRUE): batched subcluster segments at realistic sizes.

Synthetic PC matrices: a Gaussian mixture with bootstrap-like duplication
(the kNN contract is exercised by the sampling with replacement itself).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _pcs(seed, N, d, C=12):
    rng = np.random.default_rng(seed)
    centers = rng.normal(scale=4.0, size=(C, d)) / np.sqrt(np.arange(1, d + 1))  # PC-like decaying spread
    sd = 1.0 / np.sqrt(np.arange(1, d + 1))
    return centers[rng.integers(0, C, N)] + rng.normal(size=(N, d)) * sd


def _edges_equal(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


def test_cfg2_full_bootstrap_knn_snn_silhouette(engine):
    N, d = 20000, 20
    pcs = _pcs(20241026, N, d)
    boot = np.random.default_rng(123).integers(0, N, int(0.9 * N)).astype(np.int32)
    idx, dist = engine.knn_boot(pcs, boot, kmax=20)
    X = O.gather_rows(pcs, boot)
    oi, od = O.knn(X, 20)
    assert np.array_equal(idx[0], oi)
    np.testing.assert_allclose(dist[0], od, rtol=RTOL, atol=1e-12)
    for k in (10, 15, 20):
        assert _edges_equal(engine.snn(idx[0], k, "number"), O.snn(oi, k, "number"))
    rng = np.random.default_rng(5)
    labs = np.stack([rng.integers(1, c + 1, X.shape[0]) for c in (2, 7, 19, 40)]).astype(np.int32)
    mean, nc, _, _ = engine.silhouette(X, labs)
    for l_ in range(labs.shape[0]):
        _, m, C = O.silhouette(X, labs[l_])
        np.testing.assert_allclose(mean[l_], m, rtol=RTOL)
        assert nc[l_] == C


@pytest.fixture(scope="module")
def cfg3(engine):
    N, d = 100000, 30
    pcs = _pcs(20241027, N, d)
    boot = np.random.default_rng(124).integers(0, N, int(0.9 * N)).astype(np.int32)
    idx, dist = engine.knn_boot(pcs, boot, kmax=20)
    return pcs, boot, idx[0], dist[0], engine.last_knn_stats


def test_cfg3_knn_sampled_rows_vs_oracle(cfg3):
    pcs, boot, idx, dist, stats = cfg3
    X = O.gather_rows(pcs, boot)
    q = np.random.default_rng(7).choice(X.shape[0], 4096, replace=False).astype(np.int32)
    q[:64] = np.sort(np.unique(boot, return_index=True)[1])[:64]  # first copies of duplicated cells too
    oi, od = O.knn_queries(X, 20, q)
    assert np.array_equal(idx[q], oi)
    np.testing.assert_allclose(dist[q], od, rtol=RTOL, atol=1e-12)
    assert stats[0] == X.shape[0] and stats[1] < X.shape[0] // 50  # the screen certifies >98% of rows


def test_cfg3_knn_size_independent_properties(cfg3):
    """Every row: ascending distances, no self, indices distinct and in range."""
    pcs, boot, idx, dist, _ = cfg3
    n = boot.size
    assert np.all(np.diff(dist, axis=1) >= 0)
    assert np.all((idx >= 0) & (idx < n))
    assert not np.any(idx == np.arange(n)[:, None])
    s = np.sort(idx, axis=1)
    assert not np.any(s[:, 1:] == s[:, :-1])
    # duplicated cells are at distance 0 from each other
    cells = boot[idx[:, 0]]
    zero = dist[:, 0] == 0
    assert np.all(cells[zero] == boot[zero])


@pytest.mark.parametrize("t", ["number", "rank"])
def test_cfg3_snn_n90k_vs_oracle(engine, cfg3, t):
    _, _, idx, _, _ = cfg3
    for k in ((10, 15, 20) if t == "number" else (20,)):
        assert _edges_equal(engine.snn(idx, k, t), O.snn(idx, k, t))


def _granular_A(rng, B, N, dtype=np.uint8):
    """60 clusterings per bootstrap sharing its sampling mask, C rising 2..60."""
    nb = (B + 59) // 60
    A = np.empty((B, N), dtype)
    for b in range(nb):
        mask = rng.random(N) < 0.6  # ~ a bootstrap's sampled cells
        base = rng.integers(0, 1 << 30, N)
        for r in range(60):
            c = b * 60 + r
            if c >= B:
                break
            C = 2 + (58 * r) // 59
            col = (base % C + 1).astype(dtype)
            col[~mask] = 0
            A[c] = col
            base = base // 3 + rng.integers(0, 7, N) * (rng.random(N) < 0.05)
    return A


def test_cfg4_granular_B60000_triangle_rows_vs_oracle(engine):
    rng = np.random.default_rng(4)
    B, N = 60000, 4096
    A = _granular_A(rng, B, N)
    r = engine.cocluster(A)
    rows = np.concatenate([[0, 1, 4095], rng.choice(N, 61, replace=False)]).astype(np.int32)
    co, both = O.cocluster_rows(A, rows)
    j = np.arange(N)
    for t, i in enumerate(rows):
        m = j != i
        o = O.packed_index(np.minimum(i, j[m]), np.maximum(i, j[m]), N)
        assert np.array_equal(r["co"][o], co[t, m].astype(np.uint16))
        assert np.array_equal(r["both"][o], both[t, m].astype(np.uint16))
        with np.errstate(invalid="ignore", divide="ignore"):
            q = (co[t, m].astype(np.float32) / both[t, m].astype(np.float32)).astype(np.float64)
        assert np.array_equal(r["dist"][o], 1.0 - q, equal_nan=True)


def test_cfg4_full_N250k_row_slabs_vs_oracle(engine):
    """Row slabs of the N = 250 000, B = 60 000 matrix (15 GB of uint8 labels
    in HBM): the first and the last slab, 64-bit offsets included."""
    import torch
    from consensusclustr_amd.sharding import slab_offset
    B, N = 60000, 250000
    g = torch.Generator(device="cuda").manual_seed(11)
    Cb = torch.randint(2, 61, (B, 1), device="cuda", generator=g, dtype=torch.int32)
    At = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    for c0 in range(0, B, 4000):  # bounded temporaries
        c1 = min(B, c0 + 4000)
        v = (torch.rand((c1 - c0, N), device="cuda", generator=g) * Cb[c0:c1]).to(torch.int32) + 1
        v[torch.rand((c1 - c0, N), device="cuda", generator=g) < 0.35] = 0
        At[c0:c1] = v.to(torch.uint8)
        del v
    A = At.cpu().numpy()
    rng = np.random.default_rng(3)
    for r0, r1 in ((0, 128), (249856, N)):
        P = (r1 - r0) * N - (r1 * (r1 + 1) - r0 * (r0 + 1)) // 2
        co = torch.empty(P, dtype=torch.int16, device="cuda")
        both = torch.empty(P, dtype=torch.int16, device="cuda")
        engine.cocluster_t(At, r0, r1, co=co, both=both)
        torch.cuda.synchronize()
        co_h = co.cpu().numpy().view(np.uint16)
        both_h = both.cpu().numpy().view(np.uint16)
        rows = np.unique(np.concatenate([[r0, r1 - 2], rng.integers(r0, r1 - 1, 4)])).astype(np.int32)
        oco, oboth = O.cocluster_rows(A, rows)
        for t, i in enumerate(rows.tolist()):  # Python ints: the offsets exceed 2^31
            j = np.arange(i + 1, N, dtype=np.int64)
            o = (i * N - i * (i + 1) // 2 + (j - i - 1)) - slab_offset(N, r0)
            assert np.array_equal(co_h[o], oco[t, i + 1:].astype(np.uint16))
            assert np.array_equal(both_h[o], oboth[t, i + 1:].astype(np.uint16))
    del At


def test_cfg5_subcluster_segments_realistic_sizes(engine):
    """iterate=TRUE: a 100k-cell run's subclusters (5k-20k cells, d_c 5-15),
    each bootstrapped, searched in one batched call; sampled rows per segment
    against the oracle."""
    rng = np.random.default_rng(55)
    sizes = [20000, 12000, 9000, 5000, 7000]
    dims = [15, 9, 12, 5, 7]
    mats, boots = [], []
    for s_, d_ in zip(sizes, dims):
        p_ = _pcs(int(rng.integers(1 << 30)), s_, d_, C=4)
        b_ = rng.integers(0, s_, int(0.9 * s_)).astype(np.int32)
        mats.append(O.gather_rows(p_, b_))
    res = engine.knn_segments(mats, kmax=20)
    for X, (idx, dist) in zip(mats, res):
        q = rng.choice(X.shape[0], 512, replace=False).astype(np.int32)
        oi, od = O.knn_queries(X, 20, q)
        assert np.array_equal(idx[q], oi)
        np.testing.assert_allclose(dist[q], od, rtol=RTOL, atol=1e-12)
