"""Host-side logic of the drop-in (no GPU): selection rules, map-back,
assignment matrix, sharding arithmetic and the host clustering stand-in."""
import numpy as np
import pytest

import oracle as O
from consensusclustr_amd import consensus as C
from consensusclustr_amd import _lib
from consensusclustr_amd.cluster_host import louvain, louvain_py
from consensusclustr_amd.sharding import boot_shard, row_slabs, slab_offset, slab_pairs


def test_selection_rules_match_kat_and_oracle(kat):
    for scores, want in kat["robust_choice"]["cases"]:
        assert C.robust_choice(scores) == want == O.robust_choice(scores)
    for scores, want in kat["consensus_choice"]["cases"]:
        assert C.consensus_choice(scores) == want == O.consensus_choice(scores)
    rng = np.random.default_rng(0)
    for _ in range(200):
        s = rng.integers(0, 4, 12).astype(float) / 4
        if rng.random() < 0.2:
            s[rng.integers(0, 12)] = np.nan
        assert C.robust_choice(s) == O.robust_choice(s)
        assert C.consensus_choice(s) == O.consensus_choice(s)


def test_robust_score_rules():
    # :663-670 with minSize: >1 cluster & min size > minSize -> silhouette; 1 cluster -> 0; small -> 0.15
    s = C.robust_scores([0.3, 0.4, 0.5], [3, 1, 4], [10, 100, 2], minSize=5)
    assert s.tolist() == [0.3, 0.0, 0.15]
    assert C.robust_scores([0.7], [1], [50])[0] == 0.0


def test_mapback_first_copy_and_na():
    rng = np.random.default_rng(1)
    N, n = 200, 180
    idx = rng.integers(0, N, n).astype(np.int32)
    lab = rng.integers(1, 9, n).astype(np.int32)
    got = C.mapback(idx, lab, N)
    assert np.array_equal(got, O.mapback(idx, lab, N))
    assert (got[np.setdiff1d(np.arange(N), idx)] == -1).all()


def test_assignment_matrix():
    cols = [np.array([1, -1, 3]), np.array([[2, 1], [-1, 5], [4, 4]])]
    A = C.assignment_matrix(cols)
    assert A.dtype == np.uint8 and A.shape == (3, 3)
    assert A.tolist() == [[1, 0, 3], [2, 0, 4], [1, 5, 4]]
    wide = C.assignment_matrix([np.array([1, 300]), np.array([-1, 2])])  # codes > 255: uint16 matrix
    assert wide.dtype == np.uint16 and wide.tolist() == [[1, 300], [0, 2]]
    with pytest.raises(ValueError):
        C.assignment_matrix([np.array([1, 70000])])


@pytest.mark.parametrize("N,G", [(100000, 8), (100000, 2), (250000, 8), (1000, 4), (130, 8)])
def test_row_slabs_partition_and_balance(N, G):
    cuts = row_slabs(N, G)
    assert cuts[0] == 0 and cuts[-1] == N and all(a <= b for a, b in zip(cuts, cuts[1:]))
    assert all(c % 128 == 0 for c in cuts[1:-1])
    P = N * (N - 1) // 2
    pairs = [slab_pairs(N, cuts[g], cuts[g + 1]) for g in range(G)]
    assert sum(pairs) == P
    assert slab_offset(N, cuts[-1]) == P
    if N >= 100000:
        assert max(pairs) / (P / G) < 1.02


def test_boot_shard_covers():
    for nb, G in [(1000, 8), (10, 3), (5, 8)]:
        spans = [boot_shard(nb, G, r) for r in range(G)]
        assert spans[0][0] == 0 and spans[-1][1] == nb
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_bootstrap_indices():
    b = C.bootstrap_indices(1000, 3, 0.9, seed=123)
    assert b.shape == (3, 900) and b.dtype == np.int32
    assert np.array_equal(b, C.bootstrap_indices(1000, 3, 0.9, seed=123))
    assert b.min() >= 0 and b.max() < 1000


def test_louvain_recovers_two_cliques():
    ei, ej = [], []
    for base in (0, 10):
        for a in range(10):
            for b in range(a + 1, 10):
                ei.append(base + a)
                ej.append(base + b)
    ei.append(0)
    ej.append(10)
    for f in (louvain, louvain_py):
        lab = f(20, np.array(ei), np.array(ej), np.ones(len(ei)), resolution=1.0, seed=0)
        assert len(set(lab[:10])) == 1 and len(set(lab[10:])) == 1 and lab[0] != lab[10]
        assert lab.min() == 1 and lab[0] == 1


def _planted(n, blocks, m, p_out, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n, m)
    size = n // blocks
    b = np.where(rng.random(m) < p_out, rng.integers(0, n, m), (a // size) * size + rng.integers(0, size, m))
    keep = a != b
    a, b = a[keep], b[keep]
    key = np.unique(np.minimum(a, b) * n + np.maximum(a, b))
    return key // n, key % n, rng.random(key.size) + 0.5


def test_native_louvain_recovers_planted_blocks_like_the_python_restatement():
    """ccg_host_louvain (the drop-in's default clusterer) and louvain_py (the
    same algorithm in Python) both recover a planted 4-block partition."""
    n = 2000
    ei, ej, w = _planted(n, 4, 40000, 0.1, 3)
    truth = np.arange(n) // 500
    for f in (louvain, louvain_py):
        lab = f(n, ei, ej, w, resolution=1.0, seed=7)
        assert lab.dtype == np.int32 and lab.min() == 1
        # same partition as the truth (labels in order of first appearance)
        assert np.array_equal(lab, np.unique(truth, return_inverse=True)[1] + 1)


def test_native_louvain_is_deterministic_and_thread_safe():
    from concurrent.futures import ThreadPoolExecutor
    n = 3000
    ei, ej, w = _planted(n, 12, 30000, 0.4, 5)
    jobs = [(float(r), s) for r in (0.3, 0.8, 1.5) for s in (1, 2)]
    serial = [louvain(n, ei, ej, w, resolution=r, seed=s) for r, s in jobs]
    with ThreadPoolExecutor(6) as ex:
        par = list(ex.map(lambda j: louvain(n, ei, ej, w, resolution=j[0], seed=j[1]), jobs * 3))
    for t, lab in enumerate(par):
        assert np.array_equal(lab, serial[t % len(jobs)])
    # more resolution, more clusters
    assert np.unique(serial[0]).size <= np.unique(serial[4]).size


def test_native_louvain_rejects_bad_edges():
    with pytest.raises(_lib.CcgError):
        louvain(4, np.array([0, 1]), np.array([1, 1]), np.ones(2))  # self loop
    with pytest.raises(_lib.CcgError):
        louvain(4, np.array([0]), np.array([4]), np.ones(1))  # out of range
    with pytest.raises(_lib.CcgError):
        louvain(4, np.array([0]), np.array([1]), -np.ones(1))  # negative weight
    assert np.array_equal(louvain(3, np.array([], np.int32), np.array([], np.int32), np.array([])), [1, 2, 3])


@pytest.mark.parametrize("N,G", [(300, 8), (1000, 3), (129, 2), (257, 4)])
def test_row_slabs_small_n_cuts_stay_aligned(N, G):
    """A cut must never equal an unaligned N (it would be the next rank's r0)."""
    cuts = row_slabs(N, G)
    assert all(c % 128 == 0 for c in cuts[:-1])
    assert cuts[-1] == N


@pytest.mark.parametrize("N,G", [(1000, 3), (250000, 8), (300, 8), (100, 2)])
def test_rect_slabs_cover_evenly(N, G):
    from consensusclustr_amd.sharding import rect_slabs
    cuts = rect_slabs(N, G)
    assert cuts[0] == 0 and cuts[-1] == N and all(a <= b for a, b in zip(cuts, cuts[1:]))
    assert all(c % 128 == 0 for c in cuts[1:-1])
    if N >= 128 * G * 4:
        sizes = np.diff(cuts)
        assert sizes.max() - sizes.min() <= 2 * 128


def test_row_slabs_formula():
    """ccg_row_slabs (libccg, host-only) = the closed form r_g = N(1 - sqrt(1 - g/G)) rounded to 128."""
    import math
    N, G = 100000, 8
    want = [0] + [int(round(N * (1 - math.sqrt(1 - g / G)) / 128)) * 128 for g in range(1, G)] + [N]
    assert row_slabs(N, G) == want


def test_pairwise_rand_ratio_matches_oracle_restatement():
    """libccg's host ratio (ccg_pairwise_rand_ratio) == the oracle's numpy restatement, bitwise."""
    import oracle as O
    from consensusclustr_amd.engine import pairwise_rand_ratio
    rng = np.random.default_rng(5)
    for K, C in [(2, 3), (5, 9), (7, 1), (3, 12)]:
        tab = rng.integers(0, 40, (K, C + 1)).astype(np.int32)
        tab[rng.integers(0, K), 1:] = 0  # a ref cluster with no sampled cells -> NaN entries
        for adj in (True, False):
            got = pairwise_rand_ratio(tab, adj)
            want = O.pairwise_rand_ratio(tab[:, 1:], adj)
            assert np.array_equal(got, want, equal_nan=True)


def test_pairwise_rand_ratio_known_values():
    """Hand-computed: ref {0: 4 cells, 1: 2 cells}; alt puts 3 of cluster 0 together."""
    from consensusclustr_amd.engine import pairwise_rand_ratio
    tab = np.array([[0, 3, 1], [0, 0, 2]], np.int32)  # column 0 = unsampled
    r = pairwise_rand_ratio(tab, adjusted=False)
    assert r[0, 0] == 3 / 6          # C(3,2) of C(4,2) pairs stay together
    assert r[1, 1] == 1.0            # the 2 cells of cluster 1 stay together
    assert r[0, 1] == (8 - 2) / 8    # 8 cross pairs, 2 share alt cluster 2
    assert r[0, 1] == r[1, 0]


def test_cluster_block_means_exact():
    """ccg_cluster_block_means from 128-bit sums: symmetrised, diag 0, NaN when empty,
    equal to the correctly rounded rational mean."""
    from fractions import Fraction
    from consensusclustr_amd.engine import cluster_block_means
    rng = np.random.default_rng(9)
    K = 4
    sims = {}
    simsum = np.zeros((K, K, 2), np.uint64)
    npairs = np.zeros((K, K), np.int64)
    for p in range(K):
        for q in range(K):
            if p == 3 or q == 3:
                continue  # cluster 3 has no co-sampled pairs
            co = rng.integers(0, 50, 200)
            both = rng.integers(50, 60000, 200)
            s = [int(np.float32(np.float32(c) / np.float32(b)) * np.float32(2.0 ** 39)) for c, b in zip(co, both)]
            tot = sum(s) * 3000  # large totals exercise the high word
            simsum[p, q, 0] = tot & ((1 << 64) - 1)
            simsum[p, q, 1] = tot >> 64
            npairs[p, q] = 200 * 3000
            sims[p, q] = (tot, 200 * 3000)
    out = cluster_block_means(simsum, npairs)
    assert np.all(np.diag(out) == 0)
    assert np.isnan(out[0, 3]) and np.isnan(out[3, 1])
    for p in range(3):
        for q in range(3):
            if p == q:
                continue
            s = sims[p, q][0] + sims[q, p][0]
            n = sims[p, q][1] + sims[q, p][1]
            want = float(1 - Fraction(s, n << 39))
            assert abs(out[p, q] - want) <= np.spacing(want)
            assert out[p, q] == out[q, p]


def test_stability_merge_follows_the_reference_index_rule():
    """which(stab == min, arr.ind=TRUE) -> rows of the first two column-major matches;
    labels EQUAL to those 1-based positions are merged (R/consensusClust.R:489-495)."""
    from consensusclustr_amd.consensus import stability_merge
    stab = np.ones((3, 3))
    stab[0, 2] = stab[2, 0] = 0.1
    f = np.array([1, 1, 2, 3, 3, 2])
    A = np.array([[1, 3, 3, 2, 0, 1]], np.uint8)
    f2, A2, s2 = stability_merge(f, A, stab, 0.175)
    # matches in column-major order: (3,1) then (1,3) -> merge label 1 into label 3
    assert f2.tolist() == [3, 3, 2, 3, 3, 2]
    assert A2.tolist() == [[3, 3, 3, 2, 0, 3]]
    assert s2.min() == 1.0


def test_null_test_pvalue_is_normal_mle_tail():
    """fitdistr(x, 'normal') (MLE sd, divisor n) + 1 - pnorm (:939-940)."""
    from scipy.stats import norm
    from consensusclustr_amd.consensus import null_test_pvalue
    x = np.array([0.21, 0.25, 0.19, 0.3, 0.22, 0.27, 0.24, 0.2, 0.26, 0.23])
    mu, sd = x.mean(), x.std()  # numpy std: divisor n
    for s in (0.1, 0.24, 0.31, 0.5):
        assert abs(null_test_pvalue(s, x) - norm.sf(s, mu, sd)) < 1e-12


def test_choose_pc_num_rule():
    """pcNum = max(which(cumsum(sdev)/sum(sdev) > pcVar)[1], 5) (:356)."""
    from consensusclustr_amd.consensus import choose_pc_num
    sdev = np.array([10.0, 5, 3] + [1.0] * 47)
    # cumulative shares: 10/65 = 0.154, 15/65 = 0.23 -> first above 0.2 is component 2 -> max(2, 5) = 5
    assert choose_pc_num(sdev, 0.2) == 5
    assert choose_pc_num(sdev, 0.5) == 1 + int(np.flatnonzero(np.cumsum(sdev) / sdev.sum() > 0.5)[0])
    assert choose_pc_num(sdev, 0.5) == 18  # 33/65 = 0.508 at component 18


def test_live_genes_drops_genes_constant_over_the_subset():
    """Subclusters re-select features (R/consensusClust.R:290-298, :562-566):
    genes constant over the subset's cells never reach the PCA."""
    from consensusclustr_amd.pipeline import live_genes
    rng = np.random.default_rng(0)
    counts = rng.poisson(3.0, (6, 40)).astype(np.float64)
    counts[1] = 0.0                 # all-zero gene
    counts[4, :20] = 0.0            # zero only over the first 20 cells
    sf = np.ones(40)
    assert live_genes(counts, sf, None, np.arange(40)).tolist() == [0, 2, 3, 4, 5]
    assert live_genes(counts, sf, None, np.arange(20)).tolist() == [0, 2, 3, 5]
    assert live_genes(counts, sf, np.array([1, 4, 5]), np.arange(20)).tolist() == [5]


def test_consensus_clust_rejects_subset_length_size_factors():
    from consensusclustr_amd.pipeline import consensusClust
    import pytest
    with pytest.raises(ValueError, match="one per column"):
        consensusClust(np.ones((5, 30)), np.ones(10), engine=object())


def test_null_test_pvalue_sd_zero_is_point_mass():
    """1 - pnorm(q, mu, 0): pnorm is 1 for q >= mu (R's point mass)."""
    from consensusclustr_amd.consensus import null_test_pvalue
    assert null_test_pvalue(0.3, [0.3, 0.3, 0.3]) == 0.0
    assert null_test_pvalue(0.31, [0.3, 0.3]) == 0.0
    assert null_test_pvalue(0.29, [0.3, 0.3]) == 1.0


@pytest.mark.parametrize("G", [1, 3, 8])
def test_allgather_plan_unequal_and_equal_counts(G):
    """ccg_allgather_plan: the collective group_allgather_rows issues (one
    ncclAllGather for equal blocks, one ncclBroadcast per non-empty root
    otherwise), checked on CPU for every rank count the node can have."""
    from consensusclustr_amd.sharding import allgather_plan
    rng = np.random.default_rng(G)
    for nboots in (0, G, 3 * G, 1000, 1000 + G - 1, G - 1 if G > 1 else 0):
        counts = [boot_shard(nboots, G, r)[1] - boot_shard(nboots, G, r)[0] for r in range(G)]
        off, equal, roots = allgather_plan(counts)
        assert off == [0] + np.cumsum(counts).tolist()
        assert equal == (len(set(counts)) == 1)
        assert roots == ([] if equal else [r for r in range(G) if counts[r] > 0])
    counts = rng.integers(0, 5, G).tolist()
    counts[0] = 0
    off, equal, roots = allgather_plan(counts)
    assert off[-1] == sum(counts) and 0 not in roots
    # simulate the broadcasts: every rank ends with every block at its offset
    full = rng.integers(0, 9, (sum(counts), 4))
    for me in range(G):
        buf = np.zeros_like(full)
        buf[off[me]:off[me + 1]] = full[off[me]:off[me + 1]]
        for root in (roots if not equal else range(G)):
            buf[off[root]:off[root + 1]] = full[off[root]:off[root + 1]]
        assert np.array_equal(buf, full)
    with pytest.raises(Exception):
        allgather_plan([1, -1])


@pytest.mark.parametrize("batch_levels", [True, False])
def test_iterate_forwards_bootstrap_seed_and_resets_clustering_seed(monkeypatch, batch_levels):
    """R/consensusClust.R:562-566 forwards BPPARAM (SerialParam(RNGseed =
    seed): the bootstrap streams) to the recursive call but not `seed`, which
    falls back to 123 there.  Subclusters therefore draw their bootstraps
    from the caller's seed and cluster with seed 123."""
    import consensusclustr_amd.pipeline as P
    calls = []

    def fake_pcs(counts, sf, vf, cells, depth, pcNum, pcVar, nboots, eng):
        return "pca", (np.zeros((cells.size, 5)), np.arange(3, dtype=np.int32))

    def fake_consensus(pca, **kw):
        calls.append((pca.shape[0], kw["seed"], kw["boot_seed"], kw.get("boot_knn") is None))
        n = pca.shape[0]
        fin = np.where(np.arange(n) < n // 2, 1, 2) if n >= 400 else np.ones(n, np.int64)
        return {"final_assignments": fin}

    monkeypatch.setattr(P, "_node_pcs", fake_pcs)
    monkeypatch.setattr(P, "consensus_cluster", fake_consensus)
    monkeypatch.setattr(P, "_silhouette_mean", lambda eng, pca, f: 0.9)
    monkeypatch.setattr(P, "level_bootstrap_knn", lambda pcas, *a, **k: [None] * len(pcas))
    for top_seed in (7, 11):
        calls.clear()
        out = P.consensusClust(np.ones((3, 800)), np.ones(800), np.arange(3), nboots=5, seed=top_seed,
                               iterate=True, engine=object(), batch_levels=batch_levels)
        assert len(out["assignments"]) == 800
        top = [c for c in calls if c[0] == 800]
        subs = [c for c in calls if c[0] == 400]
        assert top == [(800, top_seed, top_seed, True)]
        assert len(subs) == 2 and all(c[1] == 123 and c[2] == top_seed for c in subs)
