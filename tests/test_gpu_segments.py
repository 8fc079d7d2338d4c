"""BASELINE config 5 (iterate=TRUE, R/consensusClust.R:541-567): the
bootstraps of many subclusters searched in one engine call
(ccg_knn_boot_segments[_dev]) give every bootstrap exactly the neighbours
of its own ccg_knn_boot call, and those equal the oracle's exact scan."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _sub(rng, N, d, C=5):
    centers = rng.normal(scale=3.0, size=(C, d))
    return centers[rng.integers(0, C, N)] + rng.normal(size=(N, d))


def _case(seed, sizes, dims, nb):
    rng = np.random.default_rng(seed)
    pcas = [_sub(rng, N, d) for N, d in zip(sizes, dims)]
    pcas[0][10:14] = pcas[0][3]  # distinct cells at one point (zero-distance ties between cells)
    boots = [rng.integers(0, N, (nb, int(0.9 * N))).astype(np.int32) for N in sizes]
    return pcas, boots


def test_knn_boot_segments_equal_per_bootstrap_calls_and_oracle(engine):
    pcas, boots = _case(501, [1200, 3000, 700, 2500], [5, 12, 8, 15], 3)
    got = engine.knn_boot_segments(pcas, boots, kmax=20)
    for s, (p, bb) in enumerate(zip(pcas, boots)):
        ref_i, ref_d = engine.knn_boot(p, bb, kmax=20)
        gi, gd = got[s]
        assert np.array_equal(gi, ref_i), s
        assert np.array_equal(gd, ref_d), s
        X = O.gather_rows(p, bb[0])
        oi, od = O.knn(X, 20)
        assert np.array_equal(gi[0], oi), s
        np.testing.assert_allclose(gd[0], od, rtol=1e-12, atol=1e-12)


def test_knn_boot_segments_device_global_ids_feed_one_snn_pass(engine):
    """local_ids = 0: neighbour rows of the concatenation -- the disjoint
    union of the segments' graphs -- so one ccg_snn_rows_dev pass builds every
    segment's SNN graphs; each equals the oracle's graph of its segment."""
    import torch
    pcas, boots = _case(502, [900, 1600], [6, 10], 2)
    d = 10
    Nof = np.cumsum([0] + [p.shape[0] for p in pcas])
    cells = np.zeros((Nof[-1], d))
    for s, p in enumerate(pcas):
        cells[Nof[s]:Nof[s + 1], :p.shape[1]] = p
    segs = [(s, b) for s in range(2) for b in range(2)]
    idx = np.concatenate([boots[s][b] + Nof[s] for s, b in segs]).astype(np.int32)
    off = np.cumsum([0] + [boots[s].shape[1] for s, _ in segs]).astype(np.int64)
    su = [np.unique(boots[s][b]).size for s, b in segs]
    ct = torch.from_numpy(cells).cuda()
    it = torch.from_numpy(idx).cuda()
    out = torch.empty((idx.size, 20), dtype=torch.int32, device="cuda")
    engine.knn_boot_segments_t(ct, it, off, su, 20, out, local_ids=False)
    n = idx.size
    ks = (10, 15, 20)
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    rl = torch.zeros(n, dtype=torch.int32, device="cuda")
    nbr = torch.empty(n * 400, dtype=torch.int32, device="cuda")
    wpk = torch.empty(n * 400, dtype=torch.int32, device="cuda")
    ne = torch.zeros(3, dtype=torch.int64, device="cuda")
    engine.snn_rows_t(out, ks, "number", ro, rl, nbr, wpk, ne)
    torch.cuda.synchronize()
    g = out.cpu().numpy()
    ro, rl, nbr, wpk = ro.cpu().numpy(), rl.cpu().numpy(), nbr.cpu().numpy(), wpk.cpu().numpy().view(np.uint32)
    for t, (s, b) in enumerate(segs):
        a, e = off[t], off[t + 1]
        loc = g[a:e] - a
        ref_i, _ = engine.knn_boot(pcas[s], boots[s][b], kmax=20)
        assert np.array_equal(loc, ref_i[0])
        for gi, k in enumerate(ks):
            ei, ej, w = O.snn(loc, k, "number")
            # the union graph's rows a..e restricted to graph gi
            ri, rj, rw = [], [], []
            for j in range(a, e):
                for c in range(ro[j], ro[j] + rl[j]):
                    byte = (int(wpk[c]) >> (8 * gi)) & 0xFF
                    if byte:
                        ri.append(j - a)
                        rj.append(nbr[c] - a)
                        rw.append(float(byte))
            assert np.array_equal(np.array(ri), ei) and np.array_equal(np.array(rj), ej)
            assert np.array_equal(np.array(rw), w)


def test_knn_boot_segments_rejects_small_segments(engine):
    from consensusclustr_amd._lib import CcgError
    rng = np.random.default_rng(503)
    p = _sub(rng, 400, 5)
    with pytest.raises(CcgError):
        engine.knn_boot_segments([p, p[:15]], [rng.integers(0, 400, 360), rng.integers(0, 15, 13)], kmax=20)
