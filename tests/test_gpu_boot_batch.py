"""Bootstrap batches (ccg_knn_boots_table_dev): nb bootstraps of the same
PCs through one set of launches must give every bootstrap exactly
ccg_knn_boot_table_dev's result (ids and distances bit for bit), and so the
oracle's (R/consensusClust.R:394 + :656-658: findKNN on each
pca[sample(...), ]).

* cfg3 shapes (100 000 cells x 30 PCs, n = 90 000, the bench's first
  bootstraps): the batch against the per-bootstrap calls, in both id modes,
  and the cut-tie rows the batch reports against the per-bootstrap ones;
* small integer-valued PCs (exact distance ties everywhere: the tie merge and
  the cut-tie radius search), a short table (K = 21 of kmax = 20: most cells
  take the segmented radius search), nb = 1 and nb = 64, every row against
  the oracle;
* the sticky error for a wrong n_unique and the host checks.
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _table(engine, torch, pcs_cm, N, d, K):
    dev = pcs_cm.device
    tab_idx = torch.empty((N, K), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, K), dtype=torch.float64, device=dev)
    engine.knn_table_t(pcs_cm, N, d, K, tab_idx, tab_d2)
    return tab_idx, tab_d2


def _batch_vs_single(engine, torch, pcs, boots_np, K, kmax=20, local_ids=True):
    """(batch idx, batch dist, per-bootstrap idx, per-bootstrap dist, cut rows
    of the batch, union of the per-bootstrap cut rows, both shifted to the
    concatenation)."""
    dev = pcs.device
    N, d = pcs.shape
    nb, n = boots_np.shape
    pcs_cm = pcs.t().contiguous()
    tab_idx, tab_d2 = _table(engine, torch, pcs_cm, N, d, K)
    boots = torch.from_numpy(np.ascontiguousarray(boots_np, dtype=np.int32)).to(dev)
    uniq = [int(np.unique(b).size) for b in boots_np]
    rows = torch.empty((nb * n, d), dtype=torch.float64, device=dev)
    engine.gather_rows_rm_t(pcs, N, d, boots.reshape(-1), rows)
    bi = torch.empty((nb * n, kmax), dtype=torch.int32, device=dev)
    bd = torch.empty((nb * n, kmax), dtype=torch.float64, device=dev)
    engine.knn_boots_table_t(N, d, boots, uniq, rows, kmax, tab_idx, tab_d2, bi, out_dist=bd, local_ids=local_ids)
    cut_b = engine.knn_last_fallback()
    engine.synchronize()
    si = torch.empty((n, kmax), dtype=torch.int32, device=dev)
    sd = torch.empty((n, kmax), dtype=torch.float64, device=dev)
    ref_i, ref_d, cut_s = [], [], []
    for s in range(nb):
        engine.knn_boot_table_t(pcs_cm, N, d, boots[s], uniq[s], rows[s * n:(s + 1) * n], kmax, tab_idx, tab_d2,
                                si, out_dist=sd)
        cut_s.append(engine.knn_last_fallback() + s * n)
        ref_i.append(si.cpu().numpy() + (0 if local_ids else s * n))
        ref_d.append(sd.cpu().numpy())
    return (bi.cpu().numpy(), bd.cpu().numpy(), np.concatenate(ref_i), np.concatenate(ref_d), np.sort(cut_b),
            np.sort(np.concatenate(cut_s)), rows)


@pytest.fixture(scope="module")
def cfg3_pcs():
    import torch
    import bench
    pcs, _ = bench.synth_pcs(torch, 100000, 30, 2000, 20241024 + 3, torch.device("cuda", 0))
    return pcs


@pytest.mark.parametrize("local_ids", [True, False])
def test_cfg3_batch_equals_per_bootstrap_calls(engine, cfg3_pcs, local_ids):
    import torch
    N, n, nb = 100000, 90000, 6
    boots = np.stack([np.random.default_rng(123 + b).integers(0, N, n) for b in range(nb)]).astype(np.int32)
    bi, bd, ri, rd, cut_b, cut_s, _ = _batch_vs_single(engine, torch, cfg3_pcs, boots, 48, local_ids=local_ids)
    assert np.array_equal(bi, ri)
    assert np.array_equal(bd, rd)
    assert np.array_equal(cut_b, cut_s)


def test_cfg3_batch_vs_oracle_sampled_rows(engine, cfg3_pcs):
    import torch
    N, n, nb = 100000, 90000, 3
    boots = np.stack([np.random.default_rng(500 + b).integers(0, N, n) for b in range(nb)]).astype(np.int32)
    bi, bd, _, _, cut_b, _, rows = _batch_vs_single(engine, torch, cfg3_pcs, boots, 48, local_ids=True)
    X_all = rows.cpu().numpy()
    pcs_np = cfg3_pcs.cpu().numpy()
    tab = None
    rng = np.random.default_rng(9)
    for s in range(nb):
        X = X_all[s * n:(s + 1) * n]
        assert np.array_equal(X, O.gather_rows(pcs_np, boots[s]))
        cut = cut_b[(cut_b >= s * n) & (cut_b < (s + 1) * n)] - s * n
        q = np.unique(np.concatenate([cut[:2048], rng.choice(n, 1024, replace=False), [0, n - 1]])).astype(np.int32)
        oi, od = O.knn_queries(X, 20, q, nthreads=THREADS)
        assert np.array_equal(bi[s * n + q], oi), s
        np.testing.assert_allclose(bd[s * n + q], od, rtol=1e-12, atol=1e-12)
    del tab


@pytest.mark.parametrize("N,d,K,nb,seed", [(3000, 7, 48, 5, 1), (3000, 7, 21, 4, 2), (2500, 12, 30, 1, 3),
                                           (400, 5, 24, 64, 4)])
def test_small_tied_batches_vs_per_bootstrap_and_oracle(engine, N, d, K, nb, seed):
    """Integer-valued PCs: exact ties between distinct cells everywhere (the
    expansion's per-row merge and the cut-tie radius search); K = 21 leaves
    most cells short of 20 present table entries (the segmented radius search
    over each bootstrap's distinct cells); nb = 64 is the batch maximum."""
    import torch
    rng = np.random.default_rng(seed)
    pcs = torch.from_numpy(rng.integers(-3, 4, (N, d)).astype(np.float64)).to("cuda:0")
    n = int(0.9 * N)
    boots = rng.integers(0, N, (nb, n)).astype(np.int32)
    for local_ids in (True, False):
        bi, bd, ri, rd, cut_b, cut_s, rows = _batch_vs_single(engine, torch, pcs, boots, K, local_ids=local_ids)
        assert np.array_equal(bi, ri)
        assert np.array_equal(bd, rd)
        assert np.array_equal(cut_b, cut_s)
    X_all = rows.cpu().numpy()
    for s in sorted({0, nb - 1}):
        X = X_all[s * n:(s + 1) * n]
        oi, od = O.knn(X, 20)
        assert np.array_equal(bi[s * n:(s + 1) * n] - s * n, oi), s
        np.testing.assert_allclose(bd[s * n:(s + 1) * n], od, rtol=1e-12, atol=1e-12)


def test_wrong_n_unique_sets_the_sticky_error_and_host_checks(engine):
    import torch
    from consensusclustr_amd import CcgError
    rng = np.random.default_rng(5)
    N, d, n, nb = 2000, 6, 1800, 3
    pcs = torch.from_numpy(rng.normal(size=(N, d))).to("cuda:0")
    boots_np = rng.integers(0, N, (nb, n)).astype(np.int32)
    pcs_cm = pcs.t().contiguous()
    tab_idx, tab_d2 = _table(engine, torch, pcs_cm, N, d, 48)
    boots = torch.from_numpy(boots_np).to("cuda:0")
    rows = torch.empty((nb * n, d), dtype=torch.float64, device="cuda:0")
    engine.gather_rows_rm_t(pcs, N, d, boots.reshape(-1), rows)
    out = torch.empty((nb * n, 20), dtype=torch.int32, device="cuda:0")
    uniq = [int(np.unique(b).size) for b in boots_np]
    # the same total, moved between bootstraps: caught per bootstrap only by the count
    bad = [uniq[0] + 1, uniq[1] - 1, uniq[2]]
    engine.knn_boots_table_t(N, d, boots, bad, rows, 20, tab_idx, tab_d2, out)
    engine.synchronize()  # (the total still matches: the per-bootstrap distinct ids come from the device)
    bad = [uniq[0] + 1, uniq[1], uniq[2]]
    engine.knn_boots_table_t(N, d, boots, bad, rows, 20, tab_idx, tab_d2, out)
    with pytest.raises(CcgError):
        engine.synchronize()
    with pytest.raises(CcgError):  # fewer than kmax + 1 distinct cells
        engine.knn_boots_table_t(N, d, boots, [20, uniq[1], uniq[2]], rows, 20, tab_idx, tab_d2, out)
    with pytest.raises(ValueError):
        engine.knn_boots_table_t(N, d, boots, uniq[:2], rows, 20, tab_idx, tab_d2, out)
