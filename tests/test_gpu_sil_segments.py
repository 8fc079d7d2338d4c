"""ccg_silhouette_segments_dev: the silhouettes of a batch of segments (an
iterate=TRUE level's (subcluster, bootstrap) pairs, R/consensusClust.R:562-566
and :664) in one launch set, against one ccg_silhouette_cells_dev call per
segment and against the oracle (orc_silhouette, 1e-5)."""
import concurrent.futures as cf

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _segments(rng, sizes, d, L, C0=2, Cstep=3):
    """Per segment: a subcluster of `size` cells (mixture in d dims), one
    bootstrap of 0.9 size rows, L labelings per cell with C rising."""
    segs = []
    for s, N in enumerate(sizes):
        centers = rng.normal(scale=3.0, size=(6, d))
        pop = rng.integers(0, 6, N)
        pcs = centers[pop] + rng.normal(size=(N, d))
        boot = rng.integers(0, N, max(2, int(0.9 * N))).astype(np.int32)
        labs = np.empty((L, boot.size), np.int32)
        for l_ in range(L):
            C = C0 + Cstep * (l_ % 8)
            lc = (pop * 3 + l_ + s) % C + 1
            flip = rng.random(N) < 0.1
            lc[flip] = rng.integers(1, C + 1, int(flip.sum()))
            labs[l_] = lc[boot]
        segs.append((pcs[boot], boot, labs, N))
    return segs


def _run_both(engine, segs, d, L):
    import torch
    cmax = max(int(s[2].max()) for s in segs)
    ncell = max(s[3] for s in segs)
    off = np.concatenate([[0], np.cumsum([s[0].shape[0] for s in segs])]).astype(np.int64)
    x = torch.from_numpy(np.concatenate([s[0] for s in segs])).cuda()
    # cell ids distinct between segments: slot x ncell + cell
    cell = torch.from_numpy(np.concatenate([s[1] + q * ncell for q, s in enumerate(segs)]).astype(np.int32)).cuda()
    labels = [torch.from_numpy(s[2]).cuda() for s in segs]
    nseg = len(segs)
    means = [torch.full((L,), -7.0, dtype=torch.float64, device="cuda") for _ in range(nseg)]
    ncl = [torch.zeros(L, dtype=torch.int32, device="cuda") for _ in range(nseg)]
    mns = [torch.zeros(L, dtype=torch.int32, device="cuda") for _ in range(nseg)]
    engine.silhouette_segments_t(x, off, labels, cmax, cell, nseg * ncell, means, ncl, mns)
    ref = []
    for q, s in enumerate(segs):
        mq = torch.empty(L, dtype=torch.float64, device="cuda")
        cq = torch.empty(L, dtype=torch.int32, device="cuda")
        sq = torch.empty(L, dtype=torch.int32, device="cuda")
        a, b = int(off[q]), int(off[q + 1])
        engine.silhouette_cells_t(x[a:b], labels[q], cmax, cell[a:b] - q * ncell, ncell, mq, cq, sq)
        ref.append((mq, cq, sq))
    torch.cuda.synchronize()
    got = [(means[q].cpu().numpy(), ncl[q].cpu().numpy(), mns[q].cpu().numpy()) for q in range(nseg)]
    ref = [tuple(t.cpu().numpy() for t in r) for r in ref]
    return got, ref


@pytest.mark.parametrize("d", [5, 15, 30])
def test_segments_match_per_segment_calls_and_oracle(engine, d):
    rng = np.random.default_rng(100 + d)
    # ragged: tiny segments (under one 128-position width tile), mid, one large
    sizes = [40, 130, 900, 2500, 61, 6000, 300]
    L = 12
    segs = _segments(rng, sizes, d, L)
    got, ref = _run_both(engine, segs, d, L)
    for q in range(len(segs)):
        gm, gc, gs = got[q]
        rm, rc, rs = ref[q]
        assert np.array_equal(gc, rc) and np.array_equal(gs, rs), q
        # the batch's fixed-point scales differ from a lone segment's (2^-30 max|x| of the batch):
        # measured up to 2.5e-9 relative
        np.testing.assert_allclose(gm, rm, rtol=1e-8, atol=1e-12)
    # every segment's means against the oracle
    jobs = [(q, l_) for q in range(len(segs)) for l_ in range(L)]
    with cf.ThreadPoolExecutor(8) as ex:
        orc = list(ex.map(lambda t: O.silhouette(segs[t[0]][0], segs[t[0]][2][t[1]])[1], jobs))
    for (q, l_), m in zip(jobs, orc):
        np.testing.assert_allclose(got[q][0][l_], m, rtol=RTOL)


def test_segments_outside_the_envelope_fall_back_per_segment(engine):
    """d > 32: the segments run one cells call each (identical results)."""
    rng = np.random.default_rng(7)
    segs = _segments(rng, [500, 800, 77], 40, 6)
    got, ref = _run_both(engine, segs, 40, 6)
    for q in range(len(segs)):
        for a, b in zip(got[q], ref[q]):
            assert np.array_equal(a, b)


def test_segments_null_outputs_and_deterministic(engine):
    """NULL output arrays are allowed; two runs give identical bits."""
    import torch
    rng = np.random.default_rng(9)
    segs = _segments(rng, [700, 1500, 90], 12, 8)
    g1, _ = _run_both(engine, segs, 12, 8)
    g2, _ = _run_both(engine, segs, 12, 8)
    for a, b in zip(g1, g2):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
    off = np.concatenate([[0], np.cumsum([s[0].shape[0] for s in segs])]).astype(np.int64)
    x = torch.from_numpy(np.concatenate([s[0] for s in segs])).cuda()
    cell = torch.from_numpy(np.concatenate([s[1] + q * 2000 for q, s in enumerate(segs)]).astype(np.int32)).cuda()
    labels = [torch.from_numpy(s[2]).cuda() for s in segs]
    engine.silhouette_segments_t(x, off, labels, int(max(s[2].max() for s in segs)), cell, 3 * 2000)
    torch.cuda.synchronize()


@pytest.mark.parametrize("d", [8, 30])
def test_width16_screen_rows_vs_oracle_near_ties(engine, d):
    """sil_width16 screens the nearest other centroid in fp16 and takes the
    chosen distances in fp64.  Random labels put every centroid near the
    global mean, so most rows see near ties between other clusters: every
    row's width must still equal the oracle's (a wrong pick inside the
    screen's error would move a width by up to ~1e-4; centroid quantisation
    moves it by ~1e-9)."""
    rng = np.random.default_rng(300 + d)
    m, L = 3000, 6
    X = rng.normal(size=(m, d)) * rng.uniform(0.5, 2.0, d) + rng.normal(scale=4.0, size=d)
    labs = np.stack([rng.integers(1, C + 1, m) for C in (3, 5, 9, 17, 33, 40)]).astype(np.int32)
    _, _, _, w = engine.silhouette(X, labs, want_width=True)
    for l_ in range(L):
        ow, om, _ = O.silhouette(X, labs[l_])
        np.testing.assert_allclose(w[l_], ow, rtol=0, atol=2e-8)
