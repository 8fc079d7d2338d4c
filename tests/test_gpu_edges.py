"""Adversarial and boundary cases of the HIP engine (round-2 review items).

kNN certification: a lane-half owning a query's whole top-k with a tie at
rank k (the evicted-ref bound), near-origin points beside a huge outlier (the
fp16 representation floor), kmax = 32 (the KP_BIG screen).  Co-clustering:
all-zero columns inside a slot stage, uint16 labels, B > 16383 (column
chunks), odd N.  Boundary: labels wider than the assignment matrix, invalid
SNN input through the device ABI, the fused consensus kNN.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _mixture(rng, N, d, C=8, spread=3.0):
    centers = rng.normal(scale=spread, size=(C, d))
    return centers[rng.integers(0, C, N)] + rng.normal(size=(N, d))


def _unit(rng, d):
    v = rng.normal(size=d)
    return v / np.linalg.norm(v)


# ----------------------------------------------------------------- kNN --
def _half_owner_rows(seed=0):
    """Segment positions are rows (identity order), 64-row chunks, 32-row
    tiles; a ref at tile offset r % 8 < 4 lands in lane-half 0.  Query 130
    (block 1, scanned chunk order 2, 3, 1, 4, 0) gets its 19 nearest refs and
    a duplicated pair (rows 136 and 0, identical) at rank 20, all in half 0.
    Row 136 is seen in the first chunk, row 0 in the last: the screen keeps
    136 and drops 0, so only a correct bound sends the query to the exact
    path, which returns row 0 (the lower index) at rank 20."""
    rng = np.random.default_rng(seed)
    n, d = 320, 4
    X = np.empty((n, d))
    for i in range(n):
        X[i] = (10.0 + 0.37 * i) * _unit(rng, d)  # far, distinct radii
    X[130] = 0.0
    near = [128, 129, 131, 137, 138, 139, 144, 145, 146, 147, 152, 153, 154, 155, 160, 161, 162, 163, 168]
    for t, r in enumerate(near):
        X[r] = 0.1 * (t + 1) * _unit(rng, d)
    X[136] = 2.0 * _unit(rng, d)
    X[0] = X[136]
    return X


@pytest.mark.parametrize("kmax", [20, 10])
def test_knn_certify_half_owns_topk_with_tie(engine, kmax):
    X = _half_owner_rows()
    if kmax == 10:  # move the duplicated pair to rank 10
        X = X.copy()
        rng = np.random.default_rng(9)
        near = [128, 129, 131, 137, 138, 139, 144, 145, 146]
        for t, r in enumerate(near):
            X[r] = 0.1 * (t + 1) * _unit(rng, 4)
        for r in [147, 152, 153, 154, 155, 160, 161, 162, 163, 168]:
            X[r] = (3.0 + 0.05 * r) * _unit(rng, 4)
        X[136] = 0.95 * _unit(rng, 4)
        X[0] = X[136]
    oi, od = O.knn(X, kmax)
    assert oi[130, kmax - 1] == 0  # the tie resolves to the lower row index
    (idx, dist), = engine.knn_segments([X], kmax=kmax)
    assert np.array_equal(idx, oi)
    np.testing.assert_allclose(dist, od, rtol=RTOL, atol=1e-12)
    idx2, _ = engine.knn_boot(X, np.arange(X.shape[0]), kmax=kmax)  # Morton-ordered path
    assert np.array_equal(idx2[0], oi)


def test_knn_near_origin_cluster_beside_huge_outlier(engine):
    """Scaled coordinates of the near-origin points fall below the fp16 normal
    range (2^-14): the screen cannot rank them, so the certification's
    absolute term must refuse them and the exact path must answer."""
    rng = np.random.default_rng(12)
    X = rng.normal(scale=1e-6, size=(2000, 10))
    X[0, 0] = 1e4
    X[1:40] += rng.normal(scale=3.0, size=(39, 10))  # a few ordinary-scale rows
    idx, dist = engine.knn_boot(X, np.arange(2000), kmax=20)
    oi, od = O.knn(X, 20)
    assert np.array_equal(idx[0], oi)
    np.testing.assert_allclose(dist[0], od, rtol=RTOL, atol=0)
    assert engine.last_knn_stats[1] >= 1900  # the tiny rows went to the exact fallback


@pytest.mark.parametrize("kmax,d", [(32, 20), (25, 30), (32, 7), (21, 40)])
def test_knn_kp_big_vs_oracle(engine, kmax, d):
    rng = np.random.default_rng(kmax * 100 + d)
    N = 3000
    pcs = _mixture(rng, N, d)
    boot = rng.integers(0, N, int(0.9 * N)).astype(np.int32)
    idx, dist = engine.knn_boot(pcs, boot, kmax=kmax)
    oi, od = O.knn(O.gather_rows(pcs, boot), kmax)
    assert np.array_equal(idx[0], oi)
    np.testing.assert_allclose(dist[0], od, rtol=RTOL, atol=1e-12)


# -------------------------------------------------------- co-clustering --
def _to_oracle(A):
    A = np.array(A, np.int64)
    A[A == 0] = -1
    return A.astype(np.int32)


def _check_cocluster(engine, A):
    r = engine.cocluster(A)
    o = O.cocluster(_to_oracle(A))
    assert np.array_equal(r["co"], o["co"].astype(np.uint16))
    assert np.array_equal(r["both"], o["both"].astype(np.uint16))
    assert np.array_equal(r["dist"], o["dist"], equal_nan=True)


def test_cocluster_zero_columns_inside_a_stage(engine):
    """Never-sampled columns own no K slot; 20 one-slot columns interleaved
    with all-zero ones span 39 columns in one 32-slot stage."""
    rng = np.random.default_rng(20)
    B, N = 40, 512
    A = rng.integers(1, 4, (B, N)).astype(np.uint8)
    A[1::2] = 0
    A[rng.random((B, N)) < 0.1] = 0
    _check_cocluster(engine, A)


@pytest.mark.parametrize("B,N,C", [(50, 600, 1000), (33, 257, 300), (7, 130, 65535)])
def test_cocluster_uint16_labels(engine, B, N, C):
    rng = np.random.default_rng(B + N)
    A = rng.integers(1, C + 1, (B, N)).astype(np.uint16)
    A[:, ::5] = rng.integers(1, 4, (B, (N + 4) // 5))  # frequent co-assignment too
    A[rng.random((B, N)) < 0.1] = 0
    _check_cocluster(engine, A)


@pytest.mark.parametrize("B,N,dtype", [(20000, 260, np.uint8), (16500, 257, np.uint16), (16384, 128, np.uint8)])
def test_cocluster_column_chunks(engine, B, N, dtype):
    """B > 16383 (granular mode): counts of 16383-column chunks are added."""
    rng = np.random.default_rng(B)
    Cb = rng.integers(2, 8, B)
    A = (rng.random((B, N)) * Cb[:, None]).astype(dtype) + 1
    A[rng.random((B, N)) < 0.1] = 0
    _check_cocluster(engine, A)


def test_cocluster_chunks_dist_only_matches(engine):
    import torch
    rng = np.random.default_rng(77)
    B, N = 17000, 384
    A = rng.integers(0, 5, (B, N)).astype(np.uint8)
    full = engine.cocluster(A)
    At = torch.from_numpy(A).cuda()
    P = N * (N - 1) // 2
    dist = torch.empty(P, dtype=torch.float64, device="cuda")
    engine.cocluster_t(At, 0, N, dist=dist)  # co/both NULL: chunk partials in scratch
    torch.cuda.synchronize()
    assert np.array_equal(dist.cpu().numpy(), full["dist"], equal_nan=True)


# ---------------------------------------------------- selection + map-back --
def test_mapback_label_range_raises_and_uint16_holds(engine):
    import torch
    from consensusclustr_amd import CcgError
    from consensusclustr_amd.consensus import mapback
    rng = np.random.default_rng(5)
    N, n, nb, L = 400, 360, 2, 3
    boots = torch.from_numpy(rng.integers(0, N, (nb, n)).astype(np.int32)).cuda()
    lab_np = rng.integers(1, 700, (nb, L, n)).astype(np.int32)
    labels = torch.from_numpy(lab_np).cuda()
    A8 = torch.zeros((nb * L, N), dtype=torch.uint8, device="cuda")
    engine.select_mapback_t("granular", labels, boots, N, A8, 0)
    with pytest.raises(CcgError) as e:
        engine.synchronize()
    assert e.value.code == -6  # CCG_ERANGE, never a silent clamp
    engine.check_errors()  # the sticky error was cleared
    A16 = torch.zeros((nb * L, N), dtype=torch.int16, device="cuda")  # uint16 storage (non-uint8 = 16-bit labels)
    engine.select_mapback_t("granular", labels, boots, N, A16, 0)
    engine.synchronize()
    got = A16.cpu().numpy().view(np.uint16)
    bn = boots.cpu().numpy()
    for b in range(nb):
        for l_ in range(L):
            col = mapback(bn[b], lab_np[b, l_], N)
            col[col < 0] = 0
            assert np.array_equal(got[b * L + l_], col.astype(np.uint16))


# ----------------------------------------------------------------- SNN --
def test_snn_dev_invalid_index_is_reported(engine):
    import torch
    from consensusclustr_amd import CcgError
    n, k = 500, 10
    rng = np.random.default_rng(3)
    idx = np.stack([rng.choice(np.setdiff1d(np.arange(n), [i]), k, replace=False) for i in range(n)]).astype(np.int32)
    idx[7, 3] = n + 5  # out of range
    knn_t = torch.from_numpy(idx).cuda()
    cap = n * 200
    out = (torch.empty(cap, dtype=torch.int32, device="cuda"), torch.empty(cap, dtype=torch.int32, device="cuda"),
           torch.empty(cap, dtype=torch.float64, device="cuda"))
    ne = torch.zeros(1, dtype=torch.int64, device="cuda")
    engine.snn_multi_t(knn_t, (k,), "number", [out], ne)
    with pytest.raises(CcgError):
        engine.synchronize()
    engine.check_errors()


# ------------------------------------------------------ consensus kNN --
@pytest.mark.parametrize("B,N,dtype", [(100, 1100, np.uint8), (60, 700, np.uint16), (300, 1025, np.uint8)])
def test_consensus_knn_fused_vs_oracle(engine, B, N, dtype):
    """dbscan::kNN(jaccardDist) from the assignment matrix without the N x N
    matrix, vs the oracle's stable order() over the full distance."""
    rng = np.random.default_rng(B * 7 + N)
    C = rng.integers(2, 12, B)
    A = ((rng.random((B, N)) * C[:, None]).astype(np.int64) + 1)
    A[rng.random((B, N)) < 0.1] = 0
    A = A.astype(dtype)
    o = O.cocluster(_to_oracle(A), want=("dist",))
    got = engine.consensus_knn_assign(A, 20)
    for k in (10, 15, 20):  # kNum: k < 20 are prefixes of the stable order
        assert np.array_equal(got[:, :k], O.consensus_knn(o["dist"], N, k))


def test_consensus_knn_fused_row_ranges(engine):
    import torch
    rng = np.random.default_rng(8)
    B, N, k = 80, 900, 15
    A = rng.integers(1, 6, (B, N)).astype(np.uint8)
    ref = engine.consensus_knn_assign(A, k)
    At = torch.from_numpy(A).cuda()
    out = torch.full((N, k), -1, dtype=torch.int32, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    for r0, r1 in ((0, 128), (128, 512), (512, 900)):
        engine.consensus_knn_assign_t(At, k, r0, r1, out, flag)
    torch.cuda.synchronize()
    assert flag.item() == 0
    assert np.array_equal(out.cpu().numpy(), ref)


def test_consensus_knn_fused_nan_raises(engine):
    A = np.zeros((3, 5), np.uint8)
    A[:, :3] = 1  # cells 3, 4 never sampled
    with pytest.raises(ValueError):
        engine.consensus_knn_assign(A, 2)


# ---------------------------------------------------------- silhouette --
@pytest.mark.parametrize("m,d,C", [(6000, 30, 1000), (4000, 50, 200), (3000, 12, 2900), (5000, 64, 300),
                                   (3000, 64, 40), (3000, 9, 100), (2000, 32, 90)])
def test_silhouette_many_clusters_vs_oracle(engine, m, d, C):
    """More than 256 clusters (high-resolution clusterings are scored too,
    R/consensusClust.R:663-664): global accumulation and chunked centroid
    staging instead of the LDS fast path.  The last three cases keep the
    sorted-segment sums (LDS) at each padded width, up to its cmax limit."""
    rng = np.random.default_rng(m + C)
    X = _mixture(rng, m, d, C=16)
    labs = np.stack([rng.integers(1, C + 1, m), rng.integers(1, 9, m)]).astype(np.int32)
    labs[0, :5] = C  # make sure the top code is present
    mean, nc, ms, w = engine.silhouette(X, labs, want_width=True)
    for l_ in range(2):
        ow, om, oC = O.silhouette(X, labs[l_])
        np.testing.assert_allclose(mean[l_], om, rtol=RTOL)
        assert nc[l_] == oC
        ok = ~np.isnan(ow)
        assert np.array_equal(np.isnan(w[l_]), ~ok)
        np.testing.assert_allclose(w[l_][ok], ow[ok], rtol=RTOL, atol=1e-9)


# ------------------------------------------------------------ SNN rows --
def _rows_to_graphs(off, ln, nbr, wpk, ks, t):
    out = []
    for g, k in enumerate(ks):
        ei, ej, w = [], [], []
        for j in range(ln.size):
            for c in range(off[j], off[j] + ln[j]):
                b = (int(wpk[c]) >> (8 * g)) & 0xFF
                if (b != 0) if t == "number" else (b != 0xFF):
                    ei.append(j)
                    ej.append(nbr[c])
                    w.append(float(b) if t == "number" else max(k - 0.5 * b, 1e-6))
        out.append((np.array(ei, np.int32), np.array(ej, np.int32), np.array(w)))
    return out


@pytest.mark.parametrize("t", ["number", "rank"])
def test_snn_rows_match_per_graph_edges(engine, t):
    """The compact union-graph rows (ccg_snn_rows_dev) carry every graph of
    kNum with the same edges and weights as the per-graph lists."""
    import torch
    rng = np.random.default_rng(33)
    X = _mixture(rng, 6000, 12)
    X[:600] = X[600:1200]  # duplicates
    idx, _ = engine.knn_boot(X, np.arange(6000), kmax=20)
    n = idx.shape[1]
    knn_t = torch.from_numpy(idx[0]).cuda()
    ks = (10, 15, 20)
    off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = torch.zeros(n, dtype=torch.int32, device="cuda")
    cap = n * 400
    nbr = torch.empty(cap, dtype=torch.int32, device="cuda")
    wpk = torch.empty(cap, dtype=torch.int32, device="cuda")
    ne = torch.zeros(3, dtype=torch.int64, device="cuda")
    engine.snn_rows_t(knn_t, ks, t, off, ln, nbr, wpk, ne)
    torch.cuda.synchronize()
    got = _rows_to_graphs(off.cpu().numpy(), ln.cpu().numpy(), nbr.cpu().numpy(),
                          wpk.cpu().numpy().view(np.uint32), ks, t)
    for g, k in enumerate(ks):
        ref = O.snn(idx[0], k, t)
        assert ne[g].item() == ref[0].size
        for a, b in zip(got[g], ref):
            assert np.array_equal(a, b)
    # too small a capacity: rows are not written, the totals report -(required)
    ne2 = torch.zeros(3, dtype=torch.int64, device="cuda")
    engine.snn_rows_t(knn_t, ks, t, off, ln, nbr[:100], wpk[:100], ne2)
    torch.cuda.synchronize()
    assert ne2[0].item() < 0 and -ne2[0].item() == off[-1].item()


def test_snn_rows_copy_nodes_from_bootstrap_copies(engine):
    """Bootstrap rows repeat cells, and the rows of a cell's copies are
    copied from its first copy's row (identical N+ sets for every k).  Cases:
    copies in twos and threes, a cell copied 14 times (more than the smallest
    k + 1, so its copies' sets differ and they are built), and distinct cells
    at one point (zero-distance groups mixing cells).  Every graph equals the
    oracle's."""
    import torch
    rng = np.random.default_rng(35)
    N = 5000
    X = _mixture(rng, N, 10)
    X[100:108] = X[7]  # 9 distinct cells at one point
    boot = rng.integers(0, N, 4500).astype(np.int32)
    boot[rng.choice(4500, 14, replace=False)] = 3  # one cell drawn 14 times
    boot[rng.choice(4500, 5, replace=False)] = 104
    idx, _ = engine.knn_boot(X, boot, kmax=20)
    n = idx.shape[1]
    knn_t = torch.from_numpy(idx[0]).cuda()
    ks = (10, 15, 20)
    off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = torch.zeros(n, dtype=torch.int32, device="cuda")
    cap = n * 400
    nbr = torch.empty(cap, dtype=torch.int32, device="cuda")
    wpk = torch.empty(cap, dtype=torch.int32, device="cuda")
    ne = torch.zeros(3, dtype=torch.int64, device="cuda")
    engine.snn_rows_t(knn_t, ks, "number", off, ln, nbr, wpk, ne)
    torch.cuda.synchronize()
    got = _rows_to_graphs(off.cpu().numpy(), ln.cpu().numpy(), nbr.cpu().numpy(),
                          wpk.cpu().numpy().view(np.uint32), ks, "number")
    for g, k in enumerate(ks):
        ref = O.snn(idx[0], k, "number")
        assert ne[g].item() == ref[0].size
        for a, b in zip(got[g], ref):
            assert np.array_equal(a, b)


def test_snn_host_flavour_grows_row_reservation(engine):
    rng = np.random.default_rng(34)
    X = _mixture(rng, 3000, 8)
    idx, _ = engine.knn_boot(X, np.arange(3000), kmax=20)
    engine.snn_reserve(1000)  # far too small for the default-sized per-graph path...
    try:
        a = engine.snn(idx[0], 20, "number")  # ...the host flavour grows it and reruns
    finally:
        engine.snn_reserve(0)
    for x, y in zip(a, O.snn(idx[0], 20, "number")):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("n,bits", [(1, 5), (4095, 17), (4097, 3), (90000, 17), (1_800_000, 17), (70001, 30),
                                    (5000, 0)])
def test_sort_pairs_is_a_stable_radix_sort(engine, n, bits):
    """ccg_sort_pairs_dev (the hand-written LSD radix sort behind the
    distinct-cell grouping and the SNN host lists) equals numpy's stable
    argsort on the low key_bits bits, duplicates kept in input order."""
    import torch
    rng = np.random.default_rng(n + bits)
    hi = 1 << bits if bits else 1
    keys = rng.integers(0, min(hi, max(2, n // 3)), n).astype(np.int32)  # many equal keys
    vals = rng.permutation(n).astype(np.int32)
    kt, vt = torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda()
    ko, vo = torch.empty_like(kt), torch.empty_like(vt)
    engine.sort_pairs_t(kt, vt, ko, vo, bits)
    torch.cuda.synchronize()
    o = np.argsort(keys & (hi - 1), kind="stable")
    assert np.array_equal(ko.cpu().numpy(), keys[o])
    assert np.array_equal(vo.cpu().numpy(), vals[o])


@pytest.mark.parametrize("labels_per", ["cell", "row"])
def test_silhouette_cells_matches_row_path_and_oracle(engine, labels_per):
    """ccg_silhouette_cells_dev: widths once per (cell, label), weighted by
    the copies sharing it (R/consensusClust.R:664 on pca[sample(...), ]).
    Labels per cell (as Leiden gives copies of a cell): bit-identical to the
    per-row path.  Labels per row (copies may disagree: the exception path):
    within 1e-12 of it, and within 1e-5 of the oracle."""
    import torch
    rng = np.random.default_rng(81)
    N, d, L = 6000, 20, 9
    centers = rng.normal(scale=3.0, size=(7, d))
    pop = rng.integers(0, 7, N)
    pcs = centers[pop] + rng.normal(size=(N, d))
    boot = rng.integers(0, N, int(0.9 * N)).astype(np.int32)
    X = pcs[boot]
    n = boot.size
    labs = np.empty((L, n), np.int32)
    for l_ in range(L):
        C = 2 + 4 * l_
        if labels_per == "cell":
            lc = (pop * 3 + l_) % C + 1
            flip = rng.random(N) < 0.1
            lc[flip] = rng.integers(1, C + 1, int(flip.sum()))
            labs[l_] = lc[boot]
        else:
            labs[l_] = rng.integers(1, C + 1, n)
    cmax = int(labs.max())
    xt = torch.from_numpy(X).cuda()
    lt = torch.from_numpy(labs).cuda()
    ct = torch.from_numpy(boot).cuda()
    outs = []
    for cells in (False, True):
        mean = torch.empty(L, dtype=torch.float64, device="cuda")
        nc = torch.empty(L, dtype=torch.int32, device="cuda")
        ms = torch.empty(L, dtype=torch.int32, device="cuda")
        if cells:
            engine.silhouette_cells_t(xt, lt, cmax, ct, N, mean, nc, ms)
        else:
            engine.silhouette_t(xt, lt, cmax, mean, nc, ms)
        torch.cuda.synchronize()
        outs.append((mean.cpu().numpy(), nc.cpu().numpy(), ms.cpu().numpy()))
    (m0, c0, s0), (m1, c1, s1) = outs
    assert np.array_equal(c0, c1) and np.array_equal(s0, s1)
    if labels_per == "cell":
        assert np.array_equal(m0, m1)
    else:
        np.testing.assert_allclose(m1, m0, rtol=1e-12)
    for l_ in range(L):
        _, m, C = O.silhouette(X, labs[l_])
        np.testing.assert_allclose(m1[l_], m, rtol=1e-5)
        assert c1[l_] == C


@pytest.mark.parametrize("knum", [(10, 10, 15), (5, 8, 10, 15, 20), (20, 10, 15)])
def test_snn_graphs_any_knum_vs_oracle(engine, knum):
    """Engine.snn_multi over ccg_snn_graphs + ccg_snn_graph_fetch: kNum in
    any order, with repeats and with more than 4 distinct values (one device
    pass per 4 distinct k); every graph equals the oracle's, aligned with
    kNum (getClustAssignments loops k in kNum order, :653)."""
    rng = np.random.default_rng(41)
    X = _mixture(rng, 4000, 10)
    idx, _ = engine.knn_boot(X, rng.integers(0, 4000, 3600), kmax=20)
    graphs = engine.snn_multi(idx[0], list(knum), "number")
    assert len(graphs) == len(knum)
    for k, got in zip(knum, graphs):
        for a, b in zip(got, O.snn(idx[0], k, "number")):
            assert np.array_equal(a, b)


def test_snn_multi_ecap_keeps_graphs_staged(engine):
    """ccg_snn_multi with too-small capacities returns CCG_ECAP with every
    count set; the graphs stay staged, so ccg_snn_graph_fetch serves them
    without a second device pass."""
    import ctypes
    from consensusclustr_amd import _lib
    rng = np.random.default_rng(42)
    X = _mixture(rng, 3000, 8)
    idx, _ = engine.knn_boot(X, np.arange(3000), kmax=20)
    knn = np.ascontiguousarray(idx[0])
    ks = (10, 20)
    ne = (ctypes.c_int64 * 2)()
    P = ctypes.c_void_p * 2
    rc = engine.lib.ccg_snn_multi(engine.ctx, knn.ctypes.data_as(ctypes.c_void_p), knn.shape[0], knn.shape[1],
                                  (ctypes.c_int * 2)(*ks), 2, _lib.CCG_SNN_NUMBER, P(), P(), P(),
                                  (ctypes.c_int64 * 2)(0, 0), ne)
    assert rc == _lib.CCG_ECAP
    for t, k in enumerate(ks):
        got = engine._snn_fetch(t, ne[t])
        for a, b in zip(got, O.snn(knn, k, "number")):
            assert np.array_equal(a, b)
    small = np.empty(1, np.int32)
    rc = engine.lib.ccg_snn_graph_fetch(engine.ctx, 0, small.ctypes.data_as(ctypes.c_void_p), None, None, 1)
    assert rc == _lib.CCG_ECAP


def test_snn_copy_node_chains_of_distinct_points(engine):
    """Copy nodes are found from each node's first neighbour; distinct points
    with identical N+ sets for every k (a tight ball of 11 cells far from
    the rest) chain first neighbours (src of a src), and their rows come from
    the built end of the chain.  Graphs equal the oracle's, through the
    device rows and through the host flavour."""
    import torch
    rng = np.random.default_rng(43)
    N, d = 3000, 8
    X = _mixture(rng, N, d)
    X[200:211] = X[50] + 1e-7 * rng.normal(size=(11, d)) + 500.0  # an isolated tight ball of 11 cells
    boot = np.concatenate([np.arange(N), rng.integers(0, N, 600)]).astype(np.int32)
    idx, _ = engine.knn_boot(X, boot, kmax=20)
    ks = (10, 15, 20)
    for k, got in zip(ks, engine.snn_multi(idx[0], list(ks), "number")):
        for a, b in zip(got, O.snn(idx[0], k, "number")):
            assert np.array_equal(a, b)
    n = idx.shape[1]
    knn_t = torch.from_numpy(idx[0]).cuda()
    off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = torch.zeros(n, dtype=torch.int32, device="cuda")
    nbr = torch.empty(n * 400, dtype=torch.int32, device="cuda")
    wpk = torch.empty(n * 400, dtype=torch.int32, device="cuda")
    ne = torch.zeros(3, dtype=torch.int64, device="cuda")
    engine.snn_rows_t(knn_t, ks, "number", off, ln, nbr, wpk, ne)
    torch.cuda.synchronize()
    got = _rows_to_graphs(off.cpu().numpy(), ln.cpu().numpy(), nbr.cpu().numpy(),
                          wpk.cpu().numpy().view(np.uint32), ks, "number")
    for g, k in enumerate(ks):
        for a, b in zip(got[g], O.snn(idx[0], k, "number")):
            assert np.array_equal(a, b)


def _classes(engine, knn_np, cell, ks=(10, 15, 20), cap=None):
    import torch
    import bench
    n = knn_np.shape[0]
    knn_t = torch.from_numpy(np.ascontiguousarray(knn_np)).cuda()
    sb = bench.SnnBufs(torch, n, cap if cap is not None else 300 * n, "cuda")
    info = torch.zeros(3 + len(ks), dtype=torch.int64, device="cuda")
    cl = None if cell is None else torch.from_numpy(np.ascontiguousarray(cell, dtype=np.int32)).cuda()
    engine.snn_classes_t(knn_t, ks, sb.row_class, sb.class_root, sb.off, sb.ln, sb.nbr, sb.wpk, info, cell=cl)
    torch.cuda.synchronize()
    return sb, info.cpu().numpy()


@pytest.mark.parametrize("with_cell", [True, False])
def test_snn_classes_bootstrap_copies_vs_oracle(engine, with_cell):
    """ccg_snn_classes_dev on a bootstrap with copies in twos and threes, a
    cell drawn 14 times (more than kmin + 1: its rows are singletons) and 9
    distinct cells at one point: the class rows expand to the oracle's
    graphs, with and without the cell ids; the roots are each class's lowest
    row; too small a capacity reports -(required) and writes nothing."""
    rng = np.random.default_rng(35)
    N = 5000
    X = _mixture(rng, N, 10)
    X[100:108] = X[7]
    boot = rng.integers(0, N, 4500).astype(np.int32)
    boot[rng.choice(4500, 14, replace=False)] = 3
    boot[rng.choice(4500, 5, replace=False)] = 104
    idx, _ = engine.knn_boot(X, boot, kmax=20)
    sb, inf = _classes(engine, idx[0], boot if with_cell else None)
    n = idx.shape[1]
    u = int(inf[0])
    assert inf[1] == 0 and u < n
    rc = sb.row_class.cpu().numpy()
    roots = sb.class_root[:u].cpu().numpy()
    assert np.array_equal(roots, np.array([np.flatnonzero(rc == c)[0] for c in range(u)]))
    if with_cell:  # a class never mixes cells
        assert all(np.unique(boot[rc == c]).size == 1 for c in range(u))
    got = sb.decode(n, u)
    for g, k in enumerate((10, 15, 20)):
        ref = O.snn(idx[0], k, "number")
        assert int(inf[3 + g]) > 0
        for a, b in zip(got[g], ref):
            assert np.array_equal(a, b)
    _, inf2 = _classes(engine, idx[0], boot if with_cell else None, cap=100)
    assert inf2[3:].max() < 0 and -inf2[3] == inf2[2] == inf[2]


def test_snn_classes_contract_check_and_host_fallback(engine):
    """Distinct points with identical N+ sets (a tight ball of 11 cells far
    from the rest) may share a class only if every list holds them in row
    order; the check reports a violation in d_info[1], and the host flavour
    then takes the row-level pass -- both flavours stay exact."""
    rng = np.random.default_rng(43)
    N, d = 3000, 8
    X = _mixture(rng, N, d)
    X[200:211] = X[50] + 1e-7 * rng.normal(size=(11, d)) + 500.0
    boot = np.concatenate([np.arange(N), rng.integers(0, N, 600)]).astype(np.int32)
    idx, _ = engine.knn_boot(X, boot, kmax=20)
    n = idx.shape[1]
    for cell in (None, boot):
        sb, inf = _classes(engine, idx[0], cell)
        if cell is not None:
            assert inf[1] == 0  # the cells keep the ball's points in classes of their own
        if inf[1] == 0:
            got = sb.decode(n, int(inf[0]))
            for g, k in enumerate((10, 15, 20)):
                for a, b in zip(got[g], O.snn(idx[0], k, "number")):
                    assert np.array_equal(a, b)
        for k, got in zip((10, 15, 20), engine.snn_multi(idx[0], [10, 15, 20], "number", cell=cell)):
            for a, b in zip(got, O.snn(idx[0], k, "number")):
                assert np.array_equal(a, b)
