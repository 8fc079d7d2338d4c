"""Bootstrap kNN over distinct cells (ccg_knn_boot_dev) against the oracle's
full-row scan of the gathered bootstrap (R/consensusClust.R:394, :656-658).

The device path searches the bootstrap's distinct cells and expands their
lists back to rows; these cases pin the expansion's tie rules: copies of a
cell at distance 0 (more copies than kmax), distinct cells at equal distance
(integer lattices, where the kmax-th entry is often a tie the distinct-cell
list cuts and the exact fallback takes over), bootstraps with fewer distinct
cells than kmax + 1, kmax = 32, and a wrong distinct-cell count.  Every case
runs through both the per-bootstrap screen and the cell-table path
(ccg_knn_table_dev once over the N cells, then ccg_knn_boot_table_dev: the
first kq present entries of each distinct cell's table row).
"""
import numpy as np
import pytest
import torch

import oracle as O
from consensusclustr_amd import CcgError

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["screen", "table"])
def path(request):
    return request.param


def _table(engine, pcs_cm, N, d, K):
    dev = pcs_cm.device
    ti = torch.empty((N, K), dtype=torch.int32, device=dev)
    td = torch.empty((N, K), dtype=torch.float64, device=dev)
    engine.knn_table_t(pcs_cm, N, d, K, ti, td)
    return ti, td


def _boot_knn(engine, pcs, idx, kmax, want_dist=True, n_unique=None, path="screen", K=48):
    N, d = pcs.shape
    dev = torch.device("cuda", engine.device)
    pcs_cm = torch.from_numpy(np.ascontiguousarray(np.asarray(pcs, np.float64).T)).to(dev)
    ti = torch.from_numpy(np.ascontiguousarray(idx, np.int32)).to(dev)
    n = idx.size
    rows = torch.empty((n, d), dtype=torch.float64, device=dev)
    engine.gather_rows_t(pcs_cm, N, d, ti, rows)
    out = torch.empty((n, kmax), dtype=torch.int32, device=dev)
    dist = torch.empty((n, kmax), dtype=torch.float64, device=dev) if want_dist else None
    u = len(np.unique(idx)) if n_unique is None else n_unique
    if path == "table":
        tab = _table(engine, pcs_cm, N, d, min(K, N - 1))
        q, fb = engine.knn_boot_table_t(pcs_cm, N, d, ti, u, rows, kmax, *tab, out, dist, stats=True)
    else:
        q, fb = engine.knn_boot_t(pcs_cm, N, d, ti, u, rows, kmax, out, dist, stats=True)
    torch.cuda.synchronize()
    return out.cpu().numpy(), (dist.cpu().numpy() if want_dist else None), fb


def _check(engine, pcs, idx, kmax, path="screen", K=48):
    oi, od = O.knn(O.gather_rows(pcs, idx), kmax)
    gi, gd, fb = _boot_knn(engine, pcs, idx, kmax, path=path, K=K)
    assert np.array_equal(gi, oi)
    # distances: sqrt of the same fp64 sums; the device sqrt may differ in the last ulp
    np.testing.assert_allclose(gd, od, rtol=1e-12, atol=1e-12)
    return fb


@pytest.mark.parametrize("N,n,d,kmax", [(4000, 3600, 30, 20), (3000, 6000, 12, 32), (2500, 2250, 50, 15)])
def test_knn_boot_dev_random_bootstraps(engine, path, N, n, d, kmax):
    rng = np.random.default_rng(N + n)
    centers = rng.normal(scale=3.0, size=(10, d))
    pcs = centers[rng.integers(0, 10, N)] + rng.normal(size=(N, d))
    idx = rng.integers(0, N, n).astype(np.int32)
    _check(engine, pcs, idx, kmax, path)


def test_knn_boot_dev_cell_copies_beyond_kmax(engine, path):
    """One cell drawn 45 times (> kmax + 1): its rows' lists are its other
    copies only, in row order; a second cell drawn 12 times sits among them."""
    rng = np.random.default_rng(3)
    N, d = 800, 8
    pcs = rng.normal(size=(N, d))
    idx = rng.integers(0, N, 1000).astype(np.int32)
    idx[rng.choice(1000, 45, replace=False)] = 17
    idx[rng.choice(np.flatnonzero(idx != 17), 12, replace=False)] = 99
    _check(engine, pcs, idx, 20, path)


def test_knn_boot_dev_cells_drawn_over_64_times(engine, path):
    """Cells drawn 150 and 70 times (the grouping's big-cell path: ranks by
    counting beyond 64 rows, a wave sort up to 64) among ordinary cells."""
    rng = np.random.default_rng(4)
    N, d = 200, 5
    pcs = rng.normal(size=(N, d))
    idx = rng.integers(0, N, 1200).astype(np.int32)
    idx[rng.choice(1200, 150, replace=False)] = 5
    idx[rng.choice(np.flatnonzero(idx != 5), 70, replace=False)] = 7
    _check(engine, pcs, idx, 20, path)


@pytest.mark.parametrize("kmax", [20, 32])
def test_knn_boot_dev_lattice_ties(engine, path, kmax):
    """Integer lattice cells (many distinct cells at exactly equal distance)
    with heavy duplication: equal-d2 groups are merged by row index, and a
    group cut by the distinct-cell list goes to the exact search."""
    g = np.arange(6, dtype=np.float64)
    pcs = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)  # 216 cells
    rng = np.random.default_rng(kmax)
    idx = rng.integers(0, pcs.shape[0], 600).astype(np.int32)
    fb = _check(engine, pcs, idx, kmax, path)
    if path == "screen":
        assert fb > 0  # the screen cannot certify the lattice's cut ties: the exact path took them


def test_knn_boot_dev_few_distinct_cells(engine, path):
    """9 distinct cells, 60 rows, kmax 20: every distinct cell is listed
    (kq = u - 1 < kmax) and the rows come from the copies."""
    rng = np.random.default_rng(5)
    pcs = rng.normal(size=(9, 4))
    idx = np.concatenate([np.arange(9), rng.integers(0, 9, 51)]).astype(np.int32)
    rng.shuffle(idx)
    _check(engine, pcs, idx, 20, path)


def test_knn_boot_dev_single_cell(engine, path):
    """Every row is the same cell: each list is the other rows in order."""
    pcs = np.ones((5, 3))
    idx = np.full(30, 2, np.int32)
    _check(engine, pcs, idx, 20, path)


def test_knn_boot_dev_counts_distinct_cells(engine, path):
    """n_unique = -1: the device counts the distinct cells itself."""
    rng = np.random.default_rng(13)
    pcs = rng.normal(size=(700, 9))
    idx = rng.integers(0, 700, 630).astype(np.int32)
    oi, od = O.knn(O.gather_rows(pcs, idx), 20)
    gi, gd, _ = _boot_knn(engine, pcs, idx, 20, n_unique=-1, path=path)
    assert np.array_equal(gi, oi)
    np.testing.assert_allclose(gd, od, rtol=1e-12, atol=1e-12)


def test_knn_boot_dev_wrong_unique_count(engine, path):
    rng = np.random.default_rng(7)
    pcs = rng.normal(size=(500, 6))
    idx = rng.integers(0, 500, 400).astype(np.int32)
    u = len(np.unique(idx))
    _boot_knn(engine, pcs, idx, 10, want_dist=False, n_unique=u - 3, path=path)
    with pytest.raises(CcgError, match="n_unique"):
        engine.check_errors()
    # the context is usable again afterwards
    _check(engine, pcs, idx, 10, path)


def test_knn_boot_hint_warm_start_is_exact(engine):
    """ccg_knn_boot_hint_dev: each bootstrap's certified k-th distances seed
    the next bootstrap's screen; outputs equal the un-hinted search bit for
    bit, with good hints (few fallbacks), absurdly tight hints (every row to
    the exact fallback) and loose ones."""
    import torch
    rng = np.random.default_rng(91)
    N, d = 30000, 20
    centers = rng.normal(scale=3.0, size=(9, d))
    pcs = centers[rng.integers(0, 9, N)] + rng.normal(size=(N, d))
    pcs_cm = torch.from_numpy(np.ascontiguousarray(pcs.T)).cuda()
    hint = torch.zeros(N, dtype=torch.float32, device="cuda")
    n = int(0.9 * N)
    rows = torch.empty((n, d), dtype=torch.float64, device="cuda")
    a = torch.empty((n, 20), dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    da = torch.empty((n, 20), dtype=torch.float64, device="cuda")
    db = torch.empty_like(da)
    fb = []
    for t in range(5):
        boot_np = rng.integers(0, N, n).astype(np.int32)
        boot = torch.from_numpy(boot_np).cuda()
        u = len(np.unique(boot_np))
        engine.gather_rows_t(pcs_cm, N, d, boot, rows)
        engine.knn_boot_t(pcs_cm, N, d, boot, u, rows, 20, a, out_dist=da)
        if t == 3:
            hint.fill_(1e-6)       # far too tight: every hinted row falls back
        elif t == 4:
            hint.fill_(1e6)        # far too loose: a plain screen
        fb.append(engine.knn_boot_hint_t(pcs_cm, N, d, boot, u, rows, 20, b, hint, out_dist=db, stats=True)[1])
        torch.cuda.synchronize()
        assert torch.equal(a, b) and torch.equal(da, db), t
        assert float(hint.min()) >= 0.0
    assert max(fb[1:3]) < n // 100  # warm-started bootstraps certify almost every row


def test_knn_table_matches_oracle(engine):
    """ccg_knn_table_dev: each cell's K = 48 nearest other cells among all N
    (ids and certified squared distances) equal the oracle's exact kNN of the
    N cells, clustered data with exact duplicate cells included."""
    rng = np.random.default_rng(401)
    N, d = 6000, 30
    centers = rng.normal(scale=3.0, size=(12, d))
    pcs = centers[rng.integers(0, 12, N)] + rng.normal(size=(N, d))
    pcs[100:140] = pcs[7]  # 41 cells at one point
    K = 48
    oi, od = O.knn(pcs, K)
    pcs_cm = torch.from_numpy(np.ascontiguousarray(pcs.T)).cuda()
    ti, td = _table(engine, pcs_cm, N, d, K)
    torch.cuda.synchronize()
    assert np.array_equal(ti.cpu().numpy(), oi)
    np.testing.assert_allclose(np.sqrt(td.cpu().numpy()), od, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("frac,K", [(0.9, 48), (0.2, 48), (0.9, 8), (2.0, 48)])
def test_knn_boot_table_presence_rates(engine, frac, K):
    """Table path at presence rates from ~18% (most cells short of kq present
    table entries: the exact search among distinct cells) to ~86%, and a
    table shorter than kq (K = 8 < 20: every cell searched exactly)."""
    rng = np.random.default_rng(int(frac * 100) + K)
    N, d = 5000, 16
    centers = rng.normal(scale=3.0, size=(8, d))
    pcs = centers[rng.integers(0, 8, N)] + rng.normal(size=(N, d))
    idx = rng.integers(0, N, int(frac * N)).astype(np.int32)
    fb = _check(engine, pcs, idx, 20, "table", K=K)
    if K < 20:
        assert fb >= len(np.unique(idx))
