"""Parity of the cfg4 and cfg5 paths bench.py times, at the sizes it times them.

cfg4 (BASELINE config 4: 250 000 cells x 30 PCs, n = 225 000 rows per
bootstrap; bench.py --workload cfg4): the cell table ccg_knn_table_dev at
K = 48 over the 250k cells, then one bootstrap's kNN from it
(ccg_knn_boot_table_dev), against orc_knn_queries:
* the table: a sample of the cells the table build sent to the exact search
  (ccg_knn_last_fallback) plus 2048 sampled cells;
* the bootstrap: every row of a cell short of kq present table entries, a
  sample of the cut-tie rows and 2048 sampled rows.

cfg5 (BASELINE config 5: one iterate=TRUE level, 10 subclusters of 5k-20k
cells with 5-15 PCs; bench.py --workload cfg5): the bench's first launch set
-- 16 bootstraps of every subcluster = 160 segments through ONE
ccg_knn_boot_segments_dev (global row ids) and ONE ccg_snn_rows_dev over the
disjoint union -- against per-segment oracle rows (R/consensusClust.R:
541-567 runs each subcluster's bootstrap loop, :394, :656-658):
* every segment: 128 sampled kNN rows plus every exact-search row, segment-
  local ids; all three SNN graphs of the segment against orc_snn of its rows;
* the smallest subcluster's first segment: every kNN row;
* the first bootstrap of every subcluster: the 60 cell silhouettes within 1e-5.
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
K_NUM = (10, 15, 20)


@pytest.fixture(scope="module")
def cfg4(engine):
    import torch
    import bench
    dev = torch.device("cuda", 0)
    N, D, KT = 250000, 30, 48
    pcs, _ = bench.synth_pcs(torch, N, D, 2000, 20241024 + 3, dev)  # bench.py's PCs for every non-cfg5 workload
    pcs_cm = pcs.t().contiguous()
    tab_idx = torch.empty((N, KT), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, KT), dtype=torch.float64, device=dev)
    st = engine.knn_table_t(pcs_cm, N, D, KT, tab_idx, tab_d2, stats=True)
    tab_fb = engine.knn_last_fallback()
    assert st[1] == tab_fb.size
    n = int(0.9 * N)
    boot_np = np.random.default_rng(123).integers(0, N, n).astype(np.int32)  # the bench's bootstrap 0
    boot = torch.from_numpy(boot_np).to(dev)
    u = int(np.count_nonzero(np.bincount(boot_np, minlength=N)))
    rows = torch.empty((n, D), dtype=torch.float64, device=dev)
    engine.gather_rows_rm_t(pcs, N, D, boot, rows)
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    kd = torch.empty((n, 20), dtype=torch.float64, device=dev)
    bst = engine.knn_boot_table_t(pcs_cm, N, D, boot, u, rows, 20, tab_idx, tab_d2, knn, out_dist=kd, stats=True)
    cut = engine.knn_last_fallback()
    torch.cuda.synchronize()
    out = dict(N=N, D=D, KT=KT, n=n, u=u, pcs_np=pcs.cpu().numpy(), tab_idx=tab_idx.cpu().numpy(),
               tab_d2=tab_d2.cpu().numpy(), tab_fb=tab_fb, boot_np=boot_np, knn=knn.cpu().numpy(),
               kd=kd.cpu().numpy(), boot_stats=bst, cut=cut)
    del rows, tab_idx, tab_d2, pcs, pcs_cm
    torch.cuda.empty_cache()
    return out


def test_knn_table_cfg4_fallback_and_sampled_cells_vs_oracle(cfg4):
    c = cfg4
    rng = np.random.default_rng(17)
    fb = c["tab_fb"]
    if fb.size > 4096:
        fb = rng.choice(fb, 4096, replace=False)
    q = np.unique(np.concatenate([fb, rng.choice(c["N"], 2048, replace=False), [0, c["N"] - 1]])).astype(np.int32)
    oi, od = O.knn_queries(c["pcs_np"], c["KT"], q, nthreads=THREADS)
    assert np.array_equal(c["tab_idx"][q], oi)
    np.testing.assert_allclose(np.sqrt(c["tab_d2"][q]), od, rtol=1e-12, atol=1e-12)


def test_knn_boot_table_cfg4_short_cells_cut_ties_and_sampled_rows_vs_oracle(cfg4):
    c = cfg4
    boot_np, N, n = c["boot_np"], c["N"], c["n"]
    present = np.bincount(boot_np, minlength=N) > 0
    kq = min(20, c["u"] - 1)
    short_cells = np.flatnonzero(present & (present[c["tab_idx"]].sum(1) < kq))
    short_rows = np.flatnonzero(np.isin(boot_np, short_cells))
    assert short_cells.size > 0 and c["cut"].size + short_cells.size == c["boot_stats"][1]
    rng = np.random.default_rng(18)
    if short_rows.size > 4096:
        short_rows = rng.choice(short_rows, 4096, replace=False)
    cut = c["cut"]
    if cut.size > 4096:
        cut = rng.choice(cut, 4096, replace=False)
    q = np.unique(np.concatenate([short_rows, cut, rng.choice(n, 2048, replace=False), [0, n - 1]]))
    q = q.astype(np.int32)
    X = O.gather_rows(c["pcs_np"], boot_np)
    oi, od = O.knn_queries(X, 20, q, nthreads=THREADS)
    assert np.array_equal(c["knn"][q], oi)
    np.testing.assert_allclose(c["kd"][q], od, rtol=1e-12, atol=1e-12)


@pytest.fixture(scope="module")
def cfg5(engine):
    import torch
    import bench
    dev = torch.device("cuda", 0)
    SB = 16  # bench.py's --seg-batch
    inp = bench.cfg5_inputs(torch, 100000, 30, 2000, SB, 0, dev)
    segs, off, su, idx = bench.cfg5_seg_plan(torch, inp, 0, SB)
    n = int(off[-1])
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    st = engine.knn_boot_segments_t(inp["cells"], idx, off, su, 20, knn, local_ids=False, stats=True)
    cut = engine.knn_last_fallback()
    ro = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    rl = torch.zeros(n, dtype=torch.int32, device=dev)
    cap = 700 * n  # bench.py's reservation
    nbr = torch.empty(cap, dtype=torch.int32, device=dev)
    wpk = torch.empty(cap, dtype=torch.int32, device=dev)
    ne = torch.zeros(3, dtype=torch.int64, device=dev)
    engine.snn_rows_t(knn, K_NUM, "number", ro, rl, nbr, wpk, ne)
    # the bench's pass: the row classes of all 160 segments in one call (cells: global ids)
    sb = bench.SnnBufs(torch, n, 300 * n, dev)
    info = torch.zeros(6, dtype=torch.int64, device=dev)
    sb.run(engine, knn, idx, info)
    rows = torch.empty((n, inp["dpad"]), dtype=torch.float64, device=dev)
    engine.gather_rows_rm_t(inp["cells"], inp["cells"].shape[0], inp["dpad"], idx, rows)
    torch.cuda.synchronize()
    assert int(ne.min().item()) > 0
    used = int(ro[-1].item())
    return dict(inp=inp, segs=segs, off=off, idx=idx, knn=knn.cpu().numpy(), stats=st, cut=cut,
                ro=ro.cpu().numpy(), rl=rl.cpu().numpy(), nbr=nbr[:used].cpu().numpy(),
                wpk=wpk[:used].cpu().numpy(), ne=ne.cpu().numpy(), rows=rows, rows_np=rows.cpu().numpy(),
                sb=sb, info=info.cpu().numpy())


def test_cfg5_launch_set_knn_rows_per_segment_vs_oracle(cfg5):
    import concurrent.futures as cf
    c = cfg5
    off, kn, X_all, cut = c["off"], c["knn"], c["rows_np"], c["cut"]
    nseg = len(c["segs"])
    assert nseg == 160

    def one(q):
        a, b = int(off[q]), int(off[q + 1])
        rng = np.random.default_rng(100 + q)
        cq = cut[(cut >= a) & (cut < b)] - a
        qs = np.unique(np.concatenate([cq, rng.choice(b - a, 128, replace=False), [0, b - a - 1]])).astype(np.int32)
        oi, _ = O.knn_queries(X_all[a:b], 20, qs, nthreads=1)
        loc = kn[a:b] - a  # global ids of the concatenation -> segment-local
        return bool(np.array_equal(loc[qs], oi)) and bool((loc >= 0).all() and (loc < b - a).all())

    with cf.ThreadPoolExecutor(THREADS) as ex:
        ok = list(ex.map(one, range(nseg)))
    assert all(ok), [q for q, v in enumerate(ok) if not v][:10]
    # the smallest subcluster's first segment, every row
    q0 = min(range(nseg), key=lambda q: int(off[q + 1] - off[q]))
    a, b = int(off[q0]), int(off[q0 + 1])
    oi, _ = O.knn(X_all[a:b], 20, nthreads=THREADS)
    assert np.array_equal(kn[a:b] - a, oi)


def test_cfg5_launch_set_snn_graphs_per_segment_vs_oracle(cfg5):
    """ONE SNN rows pass over the disjoint union of the 160 segments' graphs:
    each segment's rows hold only its own partners, and its graphs equal the
    oracle's over its own neighbour rows."""
    import bench
    c = cfg5
    off, kn = c["off"], c["knn"]
    tot = np.zeros(3, np.int64)
    for q in range(len(c["segs"])):
        a, b = int(off[q]), int(off[q + 1])
        got = bench.decode_union_rows(c["ro"], c["rl"], c["nbr"], c["wpk"], 3, a, b)
        loc = np.ascontiguousarray(kn[a:b] - a)
        for g, k in enumerate(K_NUM):
            ei, ej, ew = O.snn(loc, k, "number")
            gi, gj, gw = got[g]
            assert np.array_equal(gi - a, ei) and np.array_equal(gj - a, ej) and np.array_equal(gw, ew), (q, k)
            tot[g] += ei.size
    assert np.array_equal(tot, c["ne"])


def test_cfg5_launch_set_snn_classes_per_segment_vs_oracle(cfg5):
    """The bench's cfg5 SNN pass: ONE ccg_snn_classes_dev over the disjoint
    union (classes never span segments); every segment's three graphs,
    expanded from its classes, equal the oracle's."""
    c = cfg5
    off, kn, inf = c["off"], c["knn"], c["info"]
    n = int(off[-1])
    assert inf[1] == 0 and inf[3:].min() > 0
    for q in range(len(c["segs"])):
        a, b = int(off[q]), int(off[q + 1])
        got = c["sb"].decode(n, int(inf[0]), a, b)
        loc = np.ascontiguousarray(kn[a:b] - a)
        for g, k in enumerate(K_NUM):
            ref = O.snn(loc, k, "number")
            assert all(np.array_equal(x, y) for x, y in zip(got[g], ref)), (q, k)


def test_cfg5_first_bootstrap_silhouettes_per_subcluster_vs_oracle(engine, cfg5):
    import concurrent.futures as cf
    import torch
    import bench
    c = cfg5
    inp = c["inp"]
    dev = c["rows"].device
    L = 60
    for q in range(inp["nsub"]):  # segment q = (subcluster q, bootstrap 0)
        cc, j = c["segs"][q]
        assert j == 0
        a, b = int(c["off"][q]), int(c["off"][q + 1])
        Nof = inp["Nof"]
        labels = bench.synth_labels(torch, inp["popc"][Nof[cc]:Nof[cc + 1]], inp["boots_t"][cc][j], L, dev, 1000 + j,
                                    chi=20)
        cmax = int(labels.max().item())
        m_ = torch.empty(L, dtype=torch.float64, device=dev)
        nc_ = torch.empty(L, dtype=torch.int32, device=dev)
        ms_ = torch.empty(L, dtype=torch.int32, device=dev)
        engine.silhouette_cells_t(c["rows"][a:b], labels, cmax, inp["boots_t"][cc][j], inp["sizes"][cc], m_, nc_,
                                  ms_)
        torch.cuda.synchronize()
        X = c["rows_np"][a:b]
        labs = labels.cpu().numpy()
        with cf.ThreadPoolExecutor(THREADS) as ex:
            ref = list(ex.map(lambda l_: O.silhouette(X, labs[l_]), range(L)))
        got = m_.cpu().numpy()
        for l_, (_, m, C) in enumerate(ref):
            np.testing.assert_allclose(got[l_], m, rtol=1e-5)
            assert nc_[l_].item() == C


def test_cfg5_segmented_silhouettes_match_per_segment_calls(engine, cfg5):
    """The bench's ONE ccg_silhouette_segments_dev over the first batch's 160
    segments equals 160 ccg_silhouette_cells_dev calls (cluster counts and
    smallest sizes exactly, means within 1e-8: the batch's fixed-point scale
    is taken over every segment), and the per-segment calls are the ones the
    oracle test above pins."""
    import torch
    import bench
    c = cfg5
    inp = c["inp"]
    dev = c["rows"].device
    L = 60
    segs, off = c["segs"], c["off"]
    Nof = inp["Nof"]
    labels = [bench.synth_labels(torch, inp["popc"][Nof[cc]:Nof[cc + 1]], inp["boots_t"][cc][j], L, dev, 1000 + j,
                                 chi=20) for cc, j in segs]
    cmax = max(int(lb.max().item()) for lb in labels)
    plan = (segs, off, None, c["idx"])
    keys = bench.cfg5_sil_keys(torch, inp, plan, 0)
    nseg = len(segs)
    means = [torch.empty(L, dtype=torch.float64, device=dev) for _ in range(nseg)]
    ncl = [torch.empty(L, dtype=torch.int32, device=dev) for _ in range(nseg)]
    mns = [torch.empty(L, dtype=torch.int32, device=dev) for _ in range(nseg)]
    slots = 1 + max(j for _, j in segs)
    engine.silhouette_segments_t(c["rows"], off, labels, cmax, keys, slots * inp["cells"].shape[0], means, ncl, mns)
    bad = []
    for q, (cc, j) in enumerate(segs):
        a, b = int(off[q]), int(off[q + 1])
        m_ = torch.empty(L, dtype=torch.float64, device=dev)
        nc_ = torch.empty(L, dtype=torch.int32, device=dev)
        ms_ = torch.empty(L, dtype=torch.int32, device=dev)
        engine.silhouette_cells_t(c["rows"][a:b], labels[q], cmax, inp["boots_t"][cc][j], inp["sizes"][cc], m_, nc_,
                                  ms_)
        if not (torch.equal(nc_, ncl[q]) and torch.equal(ms_, mns[q])
                and torch.allclose(means[q], m_, rtol=1e-8, atol=1e-12, equal_nan=True)):
            bad.append(q)
    torch.cuda.synchronize()
    assert not bad, bad[:10]
