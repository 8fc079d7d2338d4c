"""Parity at the BASELINE sizes for the paths the smaller tests cannot reach.

* Fused consensus kNN (R/consensusClust.R:421-425: 1 - parDist(customDist),
  then dbscan::kNN(dist, k)) at cfg3's N = 100 000 x B = 1000, which runs
  ten 4 GB row sub-slabs, and on a cfg4-shaped N = 250 000 granular matrix
  (B = 6000: 100 bootstraps x 60 clusterings), first and last sub-slabs;
  sampled rows bit-exact against orc_consensus_knn_rows, sub-slab edges
  included.
* Silhouette at cfg3 (:664): 90 000 bootstrap rows x 30 PCs with 60
  labelings, C from 2 to 40, means within 1e-5 of the oracle.
* Bootstrap kNN at cfg4's size (:656-658): n = 225 000 rows of 250 000
  cells, 512 sampled rows against the oracle's exact scan.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5
THREADS = min(16, os.cpu_count() or 1)


def _pcs(seed, N, d, C=12):
    rng = np.random.default_rng(seed)
    centers = rng.normal(scale=4.0, size=(C, d)) / np.sqrt(np.arange(1, d + 1))
    sd = 1.0 / np.sqrt(np.arange(1, d + 1))
    pop = rng.integers(0, C, N)
    return centers[pop] + rng.normal(size=(N, d)) * sd, pop


def _robust_A(seed, B, N, pop, C=12):
    """B bootstrap columns like the robust path's (generated on the GPU): a
    relabelled population with 5% flips, cells not drawn -> 0 (about 41%)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    popt = torch.from_numpy(pop).cuda()
    A = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    for b in range(B):
        Cb = int(torch.randint(2, 20, (1,), generator=g, device="cuda").item())
        perm = torch.randperm(C, generator=g, device="cuda") % Cb + 1
        col = perm[popt]
        flip = torch.rand(N, generator=g, device="cuda") < 0.05
        col = torch.where(flip, torch.randint(1, Cb + 1, (N,), generator=g, device="cuda"), col)
        col[torch.rand(N, generator=g, device="cuda") < 0.41] = 0
        A[b] = col.to(torch.uint8)
    return A


def _subslab_rows(N):
    """Rows per fused sub-slab (cocluster.hip: 4 GB of co|both rows, a
    multiple of the 128-row tile)."""
    return (4 << 30) // (4 * N) // 128 * 128


def test_consensus_knn_fused_n100k_b1000_vs_oracle(engine):
    N, B = 100000, 1000
    rng = np.random.default_rng(31)
    _, pop = _pcs(31, N, 2)
    A = _robust_A(31, B, N, pop).cpu().numpy()
    got = engine.consensus_knn_assign(A, 20)
    R = _subslab_rows(N)
    edges = [r for a in range(0, N, R) for r in (a, a + 1, min(N, a + R) - 1)]
    rows = np.unique(np.concatenate([edges, [N - 1], rng.choice(N, 256, replace=False)])).astype(np.int32)
    ref, nan = O.consensus_knn_rows(A, rows, 20, nthreads=THREADS)
    assert not nan.any()
    assert np.array_equal(got[rows], ref)
    # k = 10 and 15 (kNum): prefixes of the same stable order
    got10 = engine.consensus_knn_assign(A, 10)
    assert np.array_equal(got10[rows], ref[:, :10])
    assert np.array_equal(got10, got[:, :10])


def test_consensus_knn_fused_n250k_granular_first_last_subslabs(engine):
    import torch
    N, nb = 250000, 100
    rng = np.random.default_rng(41)
    _, pop = _pcs(41, N, 2)
    B = 60 * nb
    g = torch.Generator(device="cuda").manual_seed(41)
    popt = torch.from_numpy(pop).cuda()
    At = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    for b in range(nb):  # a bootstrap's 60 clusterings share its sampling mask
        mask = torch.rand(N, generator=g, device="cuda") < 0.41
        base = popt * 7919 + torch.randint(0, 3, (N,), generator=g, device="cuda")
        for r in range(60):
            C = 2 + (58 * r) // 59
            col = base % C + 1
            flip = torch.rand(N, generator=g, device="cuda") < 0.05
            col = torch.where(flip, torch.randint(1, C + 1, (N,), generator=g, device="cuda"), col)
            col[mask] = 0
            At[b * 60 + r] = col.to(torch.uint8)
    A = At.cpu().numpy()
    R = _subslab_rows(N)
    k = 20
    out = torch.full((N, k), -1, dtype=torch.int32, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    spans = [(0, 2 * R + 128), (N // 128 * 128 - R - 128, N)]
    rows = []
    for r0, r1 in spans:
        engine.consensus_knn_assign_t(At, k, r0, r1, out, flag)
        torch.cuda.synchronize()
        assert flag.item() == 0
        edges = [r for a in range(r0, r1, R) for r in (a, a + 1, min(r1, a + R) - 1)]
        rows += edges + rng.integers(r0, r1, 24).tolist()
    rows = np.unique(np.asarray(rows)).astype(np.int32)
    got = out.cpu().numpy()
    ref, nan = O.consensus_knn_rows(A, rows, k, nthreads=THREADS)
    assert not nan.any()
    assert np.array_equal(got[rows], ref)
    del At


def test_silhouette_cfg3_60_labelings_vs_oracle(engine):
    N, d = 100000, 30
    pcs, pop = _pcs(51, N, d)
    rng = np.random.default_rng(52)
    boot = rng.integers(0, N, int(0.9 * N)).astype(np.int32)
    X = O.gather_rows(pcs, boot)
    L, n = 60, boot.size
    Cl = 2 + (38 * (np.arange(L) % 20)) // 19  # C from 2 to 40 rising with resolution, 3 kNum blocks
    labs = np.empty((L, n), np.int32)
    for l_ in range(L):
        lab = (pop[boot] * 7 + l_ // 20) % Cl[l_] + 1
        flip = rng.random(n) < 0.05
        lab[flip] = rng.integers(1, Cl[l_] + 1, int(flip.sum()))
        labs[l_] = lab
    mean, nc, ms, _ = engine.silhouette(X, labs)
    with cf.ThreadPoolExecutor(THREADS) as ex:  # ctypes releases the GIL
        ref = list(ex.map(lambda l_: O.silhouette(X, labs[l_]), range(L)))
    for l_, (_, m, C) in enumerate(ref):
        np.testing.assert_allclose(mean[l_], m, rtol=RTOL)
        assert nc[l_] == C == np.unique(labs[l_]).size
        assert ms[l_] == np.bincount(labs[l_])[1:].min()


def test_knn_boot_cfg4_n225k_sampled_rows_vs_oracle(engine):
    N, d = 250000, 30
    pcs, _ = _pcs(61, N, d)
    boot = np.random.default_rng(62).integers(0, N, int(0.9 * N)).astype(np.int32)
    idx, dist = engine.knn_boot(pcs, boot, kmax=20)
    X = O.gather_rows(pcs, boot)
    rng = np.random.default_rng(63)
    q = rng.choice(X.shape[0], 512, replace=False).astype(np.int32)
    q[:32] = np.sort(np.unique(boot, return_index=True)[1])[:32]
    q[32:34] = [0, X.shape[0] - 1]
    oi, od = O.knn_queries(X, 20, q, nthreads=THREADS)
    assert np.array_equal(idx[0][q], oi)
    np.testing.assert_allclose(dist[0][q], od, rtol=RTOL, atol=1e-12)


def test_consensus_knn_candidate_path_equals_subslab_path_with_fallback(engine, monkeypatch):
    """The triangle + candidate-list path and the full-row sub-slab path give
    identical neighbour matrices (N = 40 000 > the candidate path's minimum),
    and a matrix whose similarities all tie (every row overflows its
    candidate list) falls back to the sub-slab path and still matches the
    oracle's stable order."""
    import torch
    N, B = 40000, 300
    _, pop = _pcs(71, N, 2)
    At = _robust_A(71, B, N, pop)
    k = 20
    outs = []
    for path in ("", "slab"):
        monkeypatch.setenv("CCG_CKNN_PATH", path)
        out = torch.full((N, k), -1, dtype=torch.int32, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        engine.consensus_knn_assign_t(At, k, 0, N, out, flag)
        torch.cuda.synchronize()
        assert flag.item() == 0
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    A = At.cpu().numpy()
    rows = np.array([0, 1, 777, N - 1], np.int32)
    ref, nan = O.consensus_knn_rows(A, rows, k, nthreads=THREADS)
    assert np.array_equal(outs[0][rows], ref)
    # all similarities tie: one label per column, 10% unsampled
    monkeypatch.setenv("CCG_CKNN_PATH", "")
    g = torch.Generator(device="cuda").manual_seed(72)
    Ae = torch.ones((60, N), dtype=torch.uint8, device="cuda")
    Ae[torch.rand((60, N), generator=g, device="cuda") < 0.1] = 0
    out = torch.full((N, k), -1, dtype=torch.int32, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.consensus_knn_assign_t(Ae, k, 0, N, out, flag)
    torch.cuda.synchronize()
    ref, nan = O.consensus_knn_rows(Ae.cpu().numpy(), rows, k, nthreads=THREADS)
    assert flag.item() == int(nan.any())
    if not nan.any():
        assert np.array_equal(out.cpu().numpy()[rows], ref)
