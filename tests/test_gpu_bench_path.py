"""Parity of the exact path bench.py times, at the size it times it (cfg3).

bench.py's step (R/consensusClust.R:391-421 + :650-692 at BASELINE cfg3:
100 000 cells x 30 PCs, n = 90 000 rows per bootstrap) runs
  ccg_gather_rows_rm_dev -> ccg_knn_table_dev (K = 48, once per step) ->
  ccg_knn_boot_table_dev (kmax = 20) -> ccg_snn_rows_dev (k = 10/15/20,
  copy nodes) -> ccg_silhouette_cells_dev (60 clusterings) ->
  ccg_select_mapback_dev -> ccg_cocluster_dev.
Each test below feeds one of those calls the bench's own synthetic inputs
(bench.synth_pcs / bench.synth_labels, bootstrap 0's draw) and compares it
with the oracle:
* the cell table: every cell the table build sent to the exact search
  (ccg_knn_last_fallback) plus 4096 sampled cells, ids bit-exact, distances
  within 1e-12;
* the bootstrap kNN from the table: every row of a cell short of kq present
  table entries, every row of a cut tie (ccg_knn_last_fallback) and 2048
  sampled rows;
* the row-major gather against the column-major gather and the oracle's;
* the SNN rows of all three graphs against the oracle's edge lists over the
  whole bootstrap (copies of cells included);
* the 60 silhouette means within 1e-5;
* the bench step's selection, map-back and co-cluster slab (sampled rows).
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
N, D, KT, KMAX = 100000, 30, 48, 20
NB = int(0.9 * N)
K_NUM = (10, 15, 20)


@pytest.fixture(scope="module")
def cfg3(engine):
    import torch
    import bench
    dev = torch.device("cuda", 0)
    pcs, pop = bench.synth_pcs(torch, N, D, 2000, 20241024 + 3, dev)
    pcs_cm = pcs.t().contiguous()
    boot_np = np.random.default_rng(123).integers(0, N, NB).astype(np.int32)  # the bench's bootstrap 0
    boot = torch.from_numpy(boot_np).to(dev)
    u = int(np.count_nonzero(np.bincount(boot_np, minlength=N)))
    tab_idx = torch.empty((N, KT), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, KT), dtype=torch.float64, device=dev)
    st = engine.knn_table_t(pcs_cm, N, D, KT, tab_idx, tab_d2, stats=True)
    tab_fb = engine.knn_last_fallback()
    assert st[1] == tab_fb.size
    rows = torch.empty((NB, D), dtype=torch.float64, device=dev)
    engine.gather_rows_rm_t(pcs, N, D, boot, rows)
    knn = torch.empty((NB, KMAX), dtype=torch.int32, device=dev)
    kd = torch.empty((NB, KMAX), dtype=torch.float64, device=dev)
    bst = engine.knn_boot_table_t(pcs_cm, N, D, boot, u, rows, KMAX, tab_idx, tab_d2, knn, out_dist=kd, stats=True)
    cut_rows = engine.knn_last_fallback()
    torch.cuda.synchronize()
    return dict(pcs=pcs, pop=pop, pcs_cm=pcs_cm, pcs_np=pcs.cpu().numpy(), boot=boot, boot_np=boot_np, u=u,
                tab_idx=tab_idx.cpu().numpy(), tab_d2=tab_d2.cpu().numpy(), tab_fb=tab_fb, rows=rows,
                knn=knn, knn_np=knn.cpu().numpy(), kd=kd.cpu().numpy(), boot_stats=bst, cut_rows=cut_rows)


def test_gather_rows_rm_equals_column_major_and_oracle(engine, cfg3):
    import torch
    c = cfg3
    alt = torch.empty_like(c["rows"])
    engine.gather_rows_t(c["pcs_cm"], N, D, c["boot"], alt)
    torch.cuda.synchronize()
    assert torch.equal(alt, c["rows"])
    assert np.array_equal(c["rows"].cpu().numpy(), O.gather_rows(c["pcs_np"], c["boot_np"]))


def test_knn_table_cfg3_fallback_and_sampled_cells_vs_oracle(cfg3):
    c = cfg3
    rng = np.random.default_rng(7)
    q = np.unique(np.concatenate([c["tab_fb"], rng.choice(N, 4096, replace=False), [0, N - 1]])).astype(np.int32)
    assert c["tab_fb"].size > 0  # the bench's table sends ~3.5k cells to the exact search: they are covered
    oi, od = O.knn_queries(c["pcs_np"], KT, q, nthreads=THREADS)
    assert np.array_equal(c["tab_idx"][q], oi)
    np.testing.assert_allclose(np.sqrt(c["tab_d2"][q]), od, rtol=1e-12, atol=1e-12)


def test_knn_boot_table_cfg3_short_cells_cut_ties_and_sampled_rows_vs_oracle(cfg3):
    c = cfg3
    boot_np = c["boot_np"]
    present = np.bincount(boot_np, minlength=N) > 0
    kq = min(KMAX, c["u"] - 1)
    # cells with fewer than kq of their K table entries in the bootstrap: the exact search among distinct cells
    short_cells = np.flatnonzero(present & (present[c["tab_idx"]].sum(1) < kq))
    short_rows = np.flatnonzero(np.isin(boot_np, short_cells))
    assert short_cells.size > 0 and c["cut_rows"].size + short_cells.size == c["boot_stats"][1]
    rng = np.random.default_rng(8)
    cut = c["cut_rows"]
    if cut.size > 8192:
        cut = rng.choice(cut, 8192, replace=False)
    q = np.unique(np.concatenate([short_rows, cut, rng.choice(NB, 2048, replace=False), [0, NB - 1]]))
    q = q.astype(np.int32)
    X = O.gather_rows(c["pcs_np"], boot_np)
    oi, od = O.knn_queries(X, KMAX, q, nthreads=THREADS)
    assert np.array_equal(c["knn_np"][q], oi)
    np.testing.assert_allclose(c["kd"][q], od, rtol=1e-12, atol=1e-12)


def _decode_rows(off, ln, nbr, wpk, ks):
    """Union-graph rows (ccg_snn_rows_dev) -> per-graph (i, j, w) NUMBER
    edge lists in (i, j) order, vectorised."""
    n = ln.size
    lens = ln.astype(np.int64)
    i = np.repeat(np.arange(n, dtype=np.int64), lens)
    start = np.repeat(off[:-1], lens)
    pos = start + (np.arange(i.size, dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens))
    j = nbr[pos]
    w = wpk.view(np.uint32)[pos]
    out = []
    for g, _ in enumerate(ks):
        b = (w >> np.uint32(8 * g)) & np.uint32(0xFF)
        m = b != 0
        out.append((i[m].astype(np.int32), j[m].astype(np.int32), b[m].astype(np.float64)))
    return out


def test_snn_rows_cfg3_all_graphs_vs_oracle(engine, cfg3):
    import torch
    c = cfg3
    dev = c["knn"].device
    off = torch.zeros(NB + 1, dtype=torch.int64, device=dev)
    ln = torch.zeros(NB, dtype=torch.int32, device=dev)
    cap = 700 * NB  # bench.py's reservation
    nbr = torch.empty(cap, dtype=torch.int32, device=dev)
    wpk = torch.empty(cap, dtype=torch.int32, device=dev)
    ne = torch.zeros(3, dtype=torch.int64, device=dev)
    engine.snn_rows_t(c["knn"], K_NUM, "number", off, ln, nbr, wpk, ne)
    torch.cuda.synchronize()
    assert int(ne.min()) > 0
    used = int(off[-1].item())
    got = _decode_rows(off.cpu().numpy(), ln.cpu().numpy(), nbr[:used].cpu().numpy(), wpk[:used].cpu().numpy(),
                       K_NUM)
    # copies of one cell (bootstrap duplicates) are present in the graph
    assert np.unique(c["boot_np"]).size < NB
    for g, k in enumerate(K_NUM):
        ref = O.snn(c["knn_np"], k, "number")
        assert int(ne[g].item()) == ref[0].size
        for a, b in zip(got[g], ref):
            assert np.array_equal(a, b)


def test_snn_classes_cfg3_all_graphs_vs_oracle(engine, cfg3):
    """The bench's SNN pass (ccg_snn_classes_dev with the bootstrap's cells):
    the class-level rows expand to exactly the oracle's three graphs over
    the whole n = 90k bootstrap."""
    import torch
    import bench
    c = cfg3
    dev = c["knn"].device
    sb = bench.SnnBufs(torch, NB, 300 * NB, dev)  # bench.py's reservation
    info = torch.zeros(6, dtype=torch.int64, device=dev)
    sb.run(engine, c["knn"], c["boot"], info)
    torch.cuda.synchronize()
    inf = info.cpu().numpy()
    u = int(inf[0])
    assert inf[1] == 0 and inf[3:].min() > 0
    assert u == np.unique(c["boot_np"]).size  # one class per distinct cell (copies of a cell, <= 11 of them)
    got = sb.decode(NB, u)
    for g, k in enumerate(K_NUM):
        ref = O.snn(c["knn_np"], k, "number")
        for a, b in zip(got[g], ref):
            assert np.array_equal(a, b)


def test_silhouette_cells_cfg3_60_bench_labelings_vs_oracle(engine, cfg3):
    import concurrent.futures as cf
    import torch
    import bench
    c = cfg3
    dev = c["knn"].device
    L = 60
    labels = bench.synth_labels(torch, c["pop"], c["boot"], L, dev, 1000)
    cmax = int(labels.max().item())
    mean = torch.empty(L, dtype=torch.float64, device=dev)
    nc = torch.empty(L, dtype=torch.int32, device=dev)
    ms = torch.empty(L, dtype=torch.int32, device=dev)
    engine.silhouette_cells_t(c["rows"], labels, cmax, c["boot"], N, mean, nc, ms)
    torch.cuda.synchronize()
    X = c["rows"].cpu().numpy()
    labs = labels.cpu().numpy()
    with cf.ThreadPoolExecutor(THREADS) as ex:  # ctypes releases the GIL
        ref = list(ex.map(lambda l_: O.silhouette(X, labs[l_]), range(L)))
    mean, nc, ms = mean.cpu().numpy(), nc.cpu().numpy(), ms.cpu().numpy()
    for l_, (_, m, C) in enumerate(ref):
        np.testing.assert_allclose(mean[l_], m, rtol=1e-5)
        assert nc[l_] == C
        assert ms[l_] == np.bincount(labs[l_])[1:][np.bincount(labs[l_])[1:] > 0].min()


def test_bench_step_selection_mapback_and_cocluster_rows_vs_oracle(engine, cfg3):
    """The bench step's tail at cfg3: 125 bootstraps' silhouettes ->
    robust selection + first-copy map-back into uint8 columns -> the
    co-cluster triangle over all N rows; choices and columns against the
    host rules and orc_mapback, sampled co/both rows against
    orc_cocluster_rows."""
    import torch
    import bench
    c = cfg3
    dev = c["knn"].device
    B, L = 125, 60
    boots_np = np.stack([np.random.default_rng(123 + b).integers(0, N, NB) for b in range(B)]).astype(np.int32)
    boots = torch.from_numpy(boots_np).to(dev)
    labels = torch.empty((B, L, NB), dtype=torch.int32, device=dev)
    for b in range(B):
        labels[b] = bench.synth_labels(torch, c["pop"], boots[b], L, dev, 1000 + b)
    cmax = int(labels.max().item())
    means = torch.empty((B, L), dtype=torch.float64, device=dev)
    nclust = torch.empty((B, L), dtype=torch.int32, device=dev)
    minsize = torch.empty((B, L), dtype=torch.int32, device=dev)
    rows = torch.empty((NB, D), dtype=torch.float64, device=dev)
    for b in range(B):
        engine.gather_rows_rm_t(c["pcs"], N, D, boots[b], rows)
        engine.silhouette_cells_t(rows, labels[b], cmax, boots[b], N, means[b], nclust[b], minsize[b])
    A = torch.zeros((B, N), dtype=torch.uint8, device=dev)
    choice = torch.empty(B, dtype=torch.int32, device=dev)
    engine.select_mapback_t("robust", labels, boots, N, A, 0, means=means, nclust=nclust, minsize=minsize,
                            out_choice=choice)
    P = N * (N - 1) // 2
    co = torch.empty(P, dtype=torch.int16, device=dev)
    both = torch.empty(P, dtype=torch.int16, device=dev)
    engine.cocluster_t(A, 0, N, co=co, both=both)
    engine.synchronize()
    means_np, nc_np, ch = means.cpu().numpy(), nclust.cpu().numpy(), choice.cpu().numpy()
    A_np = A.cpu().numpy()
    for b in range(B):
        scores = [O.robust_score(int(nc_np[b, l_]), means_np[b, l_]) for l_ in range(L)]
        assert ch[b] == O.robust_choice(scores)
    for b in (0, 1, B // 2, B - 1):
        ref = O.mapback(boots_np[b], labels[b, ch[b]].cpu().numpy(), N)
        assert np.array_equal(A_np[b].astype(np.int32), np.where(ref < 0, 0, ref))
    rng = np.random.default_rng(9)
    rsel = np.unique(np.concatenate([[0, 1, 127, 128, N // 2, N - 130, N - 2], rng.choice(N - 1, 40, replace=False)]))
    rco, rboth = O.cocluster_rows(A_np, rsel.astype(np.int32), nthreads=THREADS)
    for t, i in enumerate(rsel):
        o = i * N - i * (i + 1) // 2
        m = N - 1 - i
        gco = co[o:o + m].cpu().numpy().view(np.uint16)
        gb = both[o:o + m].cpu().numpy().view(np.uint16)
        assert np.array_equal(gco, rco[t, i + 1:]), i
        assert np.array_equal(gb, rboth[t, i + 1:]), i
