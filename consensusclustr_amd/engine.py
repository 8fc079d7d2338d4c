"""Engine: a context on one GPU plus host-array and device-tensor entry points.

Host-array methods (numpy in, numpy out) call the host flavour of the C ABI,
exactly what an R ``.Call`` glue would bind.  ``*_t`` methods take torch
tensors already resident on the engine's GPU and enqueue on torch's current
stream (torch is plumbing for device memory and streams only; all compute
runs in libccg.so).
"""
import ctypes
import time

import numpy as np

from . import _lib
from ._lib import check

_vp = ctypes.c_void_p


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not (a.flags.c_contiguous or a.flags.f_contiguous):  # (the wrappers pick the layout: R's column-major
            raise ValueError(f"array of shape {a.shape} is not contiguous")  # PCs are asfortranarray)
        return a.ctypes.data_as(_vp)
    if not a.is_contiguous():  # torch tensor: a strided view would be read in the wrong order
        raise ValueError(f"tensor of shape {tuple(a.shape)} and strides {a.stride()} is not contiguous")
    return _vp(a.data_ptr())


_HIP_STREAM_LEGACY = 1  # hipStreamLegacy


def _stream():
    """torch's current stream for the library's launches.  torch's default
    stream is HIP's legacy null stream (handle 0); hipStreamLegacy is passed
    for it (the C API reads NULL the same way since ABI 7; through ABI 6 NULL
    meant the context's own non-blocking stream, unordered with torch's work
    -- the cause of round 5's illegal-address fault), so a tensor torch
    computed just before a call is complete when the library reads it, and a
    temporary freed just after a call is not reused while the library still
    reads it."""
    import torch
    h = torch.cuda.current_stream().cuda_stream
    return _vp(h if h else _HIP_STREAM_LEGACY)


class Engine:
    """One libccg context (one GPU).  Not fork-safe; one per process/device."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        self.device = device
        cfg = _lib.ccg_config(device, 0)
        ctx = _vp()
        check(self.lib.ccg_open(ctypes.byref(cfg), ctypes.byref(ctx)))
        self.ctx = ctx
        self.owned = True
        self.last_knn_stats = None

    @classmethod
    def from_ctx(cls, ctx):
        """A non-owning Engine over a context owned elsewhere (a device group's)."""
        e = cls.__new__(cls)
        e.lib = _lib.load()
        e.ctx = ctx
        e.owned = False
        e.last_knn_stats = None
        dev = ctypes.c_int()
        check(e.lib.ccg_ctx_device(ctx, ctypes.byref(dev)))
        e.device = dev.value
        return e

    def close(self):
        if self.ctx and self.owned:
            self.lib.ccg_close(self.ctx)
        self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def torch_stream(self):
        """The context's own HIP stream (ccg_stream) as a torch stream object."""
        import torch
        return torch.cuda.ExternalStream(self.lib.ccg_stream(self.ctx))

    def synchronize(self):
        """Synchronise the device; raises CcgError for a sticky device error
        (a label wider than the assignment matrix, an invalid SNN index)."""
        check(self.lib.ccg_synchronize(self.ctx))

    def check_errors(self):
        check(self.lib.ccg_check_errors(self.ctx))

    def timing(self, enable=True):
        """Enable per-kernel hipEvent timing (ccg_timing_enable)."""
        check(self.lib.ccg_timing_enable(self.ctx, 1 if enable else 0))

    def timing_read(self, which):
        """(total_ms, launches) of kernel `which` since the last read (synchronises)."""
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(self.lib.ccg_timing_read(self.ctx, _lib.CCG_KT[which], ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    # ------------------------------------------------------------ host API
    def knn_boot(self, pca, boot_idx, kmax=20, want_dist=True):
        """kNN of bootstrap rows (ccg_knn_boot).

        pca: N x d array (any order; passed column-major like an R matrix);
        boot_idx: nb x n (or n) 0-based cell indices.
        Returns idx (nb, n, kmax) int32 0-based bootstrap-row indices,
        dist (nb, n, kmax) float64 or None.
        """
        pcs = np.asfortranarray(pca, dtype=np.float64)
        N, d = pcs.shape
        bi = np.ascontiguousarray(np.atleast_2d(boot_idx), dtype=np.int32)
        nb, n = bi.shape
        out = np.empty((nb, n, kmax), np.int32)
        dist = np.empty((nb, n, kmax), np.float64) if want_dist else None
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_knn_boot(self.ctx, _ptr(pcs), N, d, _ptr(bi), n, nb, kmax, _ptr(out),
                                    _ptr(dist), ctypes.byref(st)))
        self.last_knn_stats = (st.queries, st.fallback)
        return out, dist

    def knn_segments(self, mats, kmax=20, want_dist=True):
        """Batched kNN of independent row sets (ccg_knn_segments): the
        iterate=TRUE subclusters' bootstrap matrices in one set of launches.

        mats: list of (n_s, d_s) arrays; they are zero-padded to a common d
        (padding dims do not change distances).  Returns a list of
        (idx (n_s, kmax) int32 segment-local, dist (n_s, kmax) or None).
        """
        d = max(m.shape[1] for m in mats)
        rows = np.zeros((sum(m.shape[0] for m in mats), d), np.float64)
        off = np.zeros(len(mats) + 1, np.int64)
        for s, m in enumerate(mats):
            off[s + 1] = off[s] + m.shape[0]
            rows[off[s]:off[s + 1], :m.shape[1]] = m
        n = rows.shape[0]
        out = np.empty((n, kmax), np.int32)
        dist = np.empty((n, kmax), np.float64) if want_dist else None
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_knn_segments(self.ctx, _ptr(rows), n, d, _ptr(off), len(mats), kmax, _ptr(out),
                                        _ptr(dist), ctypes.byref(st)))
        self.last_knn_stats = (st.queries, st.fallback)
        return [(out[off[s]:off[s + 1]], None if dist is None else dist[off[s]:off[s + 1]])
                for s in range(len(mats))]

    def knn_boot_segments(self, pcas, boots, kmax=20, want_dist=True):
        """The bootstrap kNN of many PC matrices in one engine call
        (ccg_knn_boot_segments): pcas a list of (N_s, d_s) matrices (zero-
        padded to a common d), boots a list of (nb_s, n_s) or (n_s,) index
        arrays into them.  Returns, per matrix, (idx (nb_s, n_s, kmax) int32
        bootstrap-row indices, dist or None): each bootstrap exactly as
        knn_boot gives it."""
        d = max(p.shape[1] for p in pcas)
        Nof = np.zeros(len(pcas) + 1, np.int64)
        for s, p in enumerate(pcas):
            Nof[s + 1] = Nof[s] + p.shape[0]
        cells = np.zeros((int(Nof[-1]), d), np.float64)
        for s, p in enumerate(pcas):
            cells[Nof[s]:Nof[s + 1], :p.shape[1]] = p
        bl = [np.atleast_2d(np.asarray(b, np.int64)) for b in boots]
        segs = [(s, b) for s, bb in enumerate(bl) for b in range(bb.shape[0])]
        off = np.zeros(len(segs) + 1, np.int64)
        for t, (s, b) in enumerate(segs):
            off[t + 1] = off[t] + bl[s].shape[1]
        idx = np.concatenate([bl[s][b] + Nof[s] for s, b in segs]).astype(np.int32)
        n = idx.size
        out = np.empty((n, kmax), np.int32)
        dist = np.empty((n, kmax), np.float64) if want_dist else None
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_knn_boot_segments(self.ctx, _ptr(cells), cells.shape[0], d, _ptr(idx), n, _ptr(off),
                                             None, len(segs), kmax, _ptr(out), _ptr(dist), ctypes.byref(st)))
        self.last_knn_stats = (st.queries, st.fallback)
        res, t = [], 0
        for s, bb in enumerate(bl):
            nb, ns = bb.shape
            a, b = off[t], off[t + nb]
            res.append((out[a:b].reshape(nb, ns, kmax),
                        None if dist is None else dist[a:b].reshape(nb, ns, kmax)))
            t += nb
        return res

    def knn_boot_segments_t(self, cells, idx, seg_off, seg_unique, kmax, out_idx, out_dist=None, local_ids=True,
                            stats=False):
        """Device flavour (ccg_knn_boot_segments_dev): cells (Ntot, d) row-major
        tensor, idx (n,) int32 tensor, seg_off / seg_unique host arrays."""
        Ntot, d = cells.shape
        off = np.ascontiguousarray(seg_off, dtype=np.int64)
        su = np.ascontiguousarray(seg_unique, dtype=np.int32)
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_knn_boot_segments_dev(self.ctx, _ptr(cells), Ntot, d, _ptr(idx), idx.numel(), _ptr(off),
                                                 _ptr(su), off.size - 1, kmax, 1 if local_ids else 0, _ptr(out_idx),
                                                 _ptr(out_dist), ctypes.byref(st), _stream()))
        self.last_knn_stats = (st.queries, st.fallback)
        return self.last_knn_stats if stats else None

    def snn(self, knn_idx, k, type="number"):
        """SNN edges i<j sorted by (i, j) with weights (ccg_snn_graphs +
        ccg_snn_graph_fetch: one device pass, decoded on the host)."""
        return self.snn_multi(knn_idx, [k], type)[0]

    def _snn_fetch(self, t, m):
        ei = np.empty(m, np.int32)
        ej = np.empty(m, np.int32)
        w = np.empty(m, np.float64)
        check(self.lib.ccg_snn_graph_fetch(self.ctx, t, _ptr(ei), _ptr(ej), _ptr(w), m))
        return ei, ej, w

    def snn_multi(self, knn_idx, ks, type="number", cell=None):
        """The graph of every k in ks (any order, repeats allowed) from one
        device pass per 4 distinct values (ccg_snn_graphs_cells: class-level
        rows for NUMBER graphs, union rows otherwise, staged on the host;
        ccg_snn_graph_fetch decodes each graph).  cell: the cell of every
        bootstrap row (copies share one; None = unknown).  Returns a list of
        (i, j, w) edge lists aligned with ks."""
        knn_idx = np.ascontiguousarray(knn_idx, dtype=np.int32)
        n, kst = knn_idx.shape
        t = {"number": _lib.CCG_SNN_NUMBER, "rank": _lib.CCG_SNN_RANK}[type]
        cl = None if cell is None else np.ascontiguousarray(cell, dtype=np.int32).ravel()
        if cl is not None and cl.size != n:  # the library reads n entries
            raise ValueError(f"snn_multi: cell has {cl.size} entries, knn_idx has {n} rows")
        uk = sorted({int(k) for k in ks})
        got = {}
        t_pass = t_fetch = 0.0
        for c0 in range(0, len(uk), 4):  # the library builds at most 4 graphs per pass
            chunk = uk[c0:c0 + 4]
            nk = len(chunk)
            ne = (ctypes.c_int64 * nk)()
            t0 = time.perf_counter()
            check(self.lib.ccg_snn_graphs_cells(self.ctx, _ptr(knn_idx), n, kst, _ptr(cl),
                                                (ctypes.c_int * nk)(*chunk), nk, t, ne))
            t1 = time.perf_counter()
            for g, k in enumerate(chunk):
                got[k] = self._snn_fetch(g, ne[g])
            t_pass += t1 - t0
            t_fetch += time.perf_counter() - t1
        # host seconds: the device pass with its copies to pinned memory, then
        # the host expansion of the class rows into the per-graph edge lists
        self.last_snn_times = (t_pass, t_fetch)
        return [got[int(k)] for k in ks]

    def scan_i64_t(self, x, out):
        """Exclusive scan (ccg_scan_i64_dev): out[:n] prefix sums of x, out[n] the total."""
        check(self.lib.ccg_scan_i64_dev(self.ctx, _ptr(x), _ptr(out), x.numel(), _stream()))

    def silhouette_cells(self, x, labels, cell, ncell, cmax=None):
        """ccg_silhouette_cells: means over bootstrap rows x whose cells are
        `cell` (copies identical), widths once per (cell, label).  Returns
        (mean[L], nclust[L], minsize[L])."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        m, d = x.shape
        lab = np.ascontiguousarray(np.atleast_2d(labels), dtype=np.int32)
        L = lab.shape[0]
        cmax = int(lab.max()) if cmax is None else cmax
        cell = np.ascontiguousarray(cell, dtype=np.int32)
        mean = np.empty(L, np.float64)
        nc = np.empty(L, np.int32)
        ms = np.empty(L, np.int32)
        check(self.lib.ccg_silhouette_cells(self.ctx, _ptr(x), m, d, _ptr(lab), L, cmax, _ptr(cell), int(ncell),
                                            _ptr(mean), _ptr(nc), _ptr(ms)))
        return mean, nc, ms

    def silhouette(self, x, labels, cmax=None, want_width=False):
        """Batched approxSilhouette means (ccg_silhouette).

        labels: (L, m) or (m,) integer codes in [1, cmax].
        Returns (mean[L], nclust[L], minsize[L], width[L, m] or None).
        """
        x = np.ascontiguousarray(x, dtype=np.float64)
        m, d = x.shape
        lab = np.ascontiguousarray(np.atleast_2d(labels), dtype=np.int32)
        L = lab.shape[0]
        if cmax is None:
            cmax = int(lab.max())
        mean = np.empty(L, np.float64)
        nc = np.empty(L, np.int32)
        ms = np.empty(L, np.int32)
        w = np.empty((L, m), np.float64) if want_width else None
        check(self.lib.ccg_silhouette(self.ctx, _ptr(x), m, d, _ptr(lab), L, cmax, _ptr(mean), _ptr(nc),
                                      _ptr(ms), _ptr(w)))
        return mean, nc, ms, w

    def cocluster(self, A, want=("co", "both", "dist")):
        """Co-clustering counts/distance (ccg_cocluster), packed R "dist" order.

        A: B x N uint8 or uint16 column-major assignment matrix (0 = not sampled).
        """
        A = np.ascontiguousarray(A)
        if A.dtype not in (np.uint8, np.uint16):
            A = A.astype(np.uint8)
        bits = 8 * A.dtype.itemsize
        B, N = A.shape
        P = N * (N - 1) // 2
        co = np.empty(P, np.uint16) if "co" in want else None
        both = np.empty(P, np.uint16) if "both" in want else None
        dist = np.empty(P, np.float64) if "dist" in want else None
        check(self.lib.ccg_cocluster(self.ctx, _ptr(A), bits, N, B, _ptr(co), _ptr(both), _ptr(dist)))
        return {"co": co, "both": both, "dist": dist}

    def consensus_knn(self, co, both, N, k):
        """dbscan::kNN(jaccardDist, k)$id equivalent (ccg_consensus_knn), 0-based."""
        co = np.ascontiguousarray(co, dtype=np.uint16)
        both = np.ascontiguousarray(both, dtype=np.uint16)
        out = np.empty((N, k), np.int32)
        rc = self.lib.ccg_consensus_knn(self.ctx, _ptr(co), _ptr(both), N, k, _ptr(out))
        if rc == _lib.CCG_ENAN:
            raise ValueError("data/distances cannot contain NAs for kNN")
        check(rc)
        return out

    def consensus_knn_assign(self, A, k):
        """The same kNN straight from the assignment matrix, fused with the
        co-clustering GEMM (ccg_consensus_knn_assign; N x N never stored)."""
        A = np.ascontiguousarray(A)
        if A.dtype not in (np.uint8, np.uint16):
            A = A.astype(np.uint8)
        B, N = A.shape
        out = np.empty((N, k), np.int32)
        rc = self.lib.ccg_consensus_knn_assign(self.ctx, _ptr(A), 8 * A.dtype.itemsize, N, B, k, _ptr(out))
        if rc == _lib.CCG_ENAN:
            raise ValueError("data/distances cannot contain NAs for kNN")
        check(rc)
        return out

    def cluster_block_sums(self, A, f, K):
        """Exact determineHierachy block sums (ccg_cluster_block_sums):
        simsum (K, K, 2) uint64 (lo, hi words of sum sim * 2^39 over pairs
        i < j with f_i = p, f_j = q, both > 0), npairs (K, K) int64."""
        A = np.ascontiguousarray(A)
        if A.dtype not in (np.uint8, np.uint16):
            A = A.astype(np.uint8)
        B, N = A.shape
        f = np.ascontiguousarray(f, dtype=np.int32)
        simsum = np.empty((K, K, 2), np.uint64)
        npairs = np.empty((K, K), np.int64)
        check(self.lib.ccg_cluster_block_sums(self.ctx, _ptr(A), 8 * A.dtype.itemsize, N, B, _ptr(f), K,
                                              _ptr(simsum), _ptr(npairs)))
        return simsum, npairs

    def contingency(self, A, f, K, C=None):
        """table(f, A[b, ]) of every bootstrap column (ccg_contingency): (B, K, C+1) int32."""
        A = np.ascontiguousarray(A)
        if A.dtype not in (np.uint8, np.uint16):
            A = A.astype(np.uint8)
        B, N = A.shape
        C = int(A.max()) if C is None else int(C)
        f = np.ascontiguousarray(f, dtype=np.int32)
        tab = np.empty((B, K, C + 1), np.int32)
        check(self.lib.ccg_contingency(self.ctx, _ptr(A), 8 * A.dtype.itemsize, N, B, _ptr(f), K, C, _ptr(tab)))
        return tab

    def pca(self, counts, sf, genes=None, cells=None, npc=50):
        """Normalisation + PCA of a cell subset (ccg_pca): log1p(counts/sf) on
        the selected genes, centred and scaled per gene, top npc components.

        counts: G x N gene-by-cell array; sf: N size factors; genes / cells:
        0-based index arrays (None = all).  Returns (x: nc x npc scores,
        sdev: npc)."""
        C = np.asfortranarray(counts, dtype=np.float64)
        G, N = C.shape
        g = np.arange(G, dtype=np.int32) if genes is None else np.ascontiguousarray(genes, dtype=np.int32)
        c = np.arange(N, dtype=np.int32) if cells is None else np.ascontiguousarray(cells, dtype=np.int32)
        sf = np.ascontiguousarray(sf, dtype=np.float64)
        if sf.size != N:  # ccg_pca reads N size factors, indexed by the global cell
            raise ValueError(f"sf has {sf.size} entries; counts has {N} cells (pass one size factor per column)")
        x = np.empty((npc, c.size), np.float64)  # column-major nc x npc
        sdev = np.empty(npc, np.float64)
        check(self.lib.ccg_pca(self.ctx, _ptr(C), G, N, _ptr(sf), _ptr(g), g.size, _ptr(c), c.size, npc, _ptr(x),
                               _ptr(sdev)))
        return x.T.copy(), sdev

    def pca_csc(self, xv, ri, cp, G, sf, genes=None, cells=None, npc=50):
        """ccg_pca on sparse counts in compressed-column form (R's dgCMatrix
        slots x, i, p; scipy.sparse.csc_matrix data, indices, indptr): G genes
        x N = len(cp) - 1 cells.  Returns (x: nc x npc, sdev)."""
        xv = np.ascontiguousarray(xv, dtype=np.float64)
        ri = np.ascontiguousarray(ri, dtype=np.int32)
        cp = np.ascontiguousarray(cp, dtype=np.int64)
        N = cp.size - 1
        g = np.arange(G, dtype=np.int32) if genes is None else np.ascontiguousarray(genes, dtype=np.int32)
        c = np.arange(N, dtype=np.int32) if cells is None else np.ascontiguousarray(cells, dtype=np.int32)
        sf = np.ascontiguousarray(sf, dtype=np.float64)
        if sf.size != N:
            raise ValueError(f"sf has {sf.size} entries; the matrix has {N} cells")
        x = np.empty((npc, c.size), np.float64)
        sdev = np.empty(npc, np.float64)
        check(self.lib.ccg_pca_csc(self.ctx, _ptr(xv), _ptr(ri), _ptr(cp), int(G), N, _ptr(sf), _ptr(g), g.size,
                                   _ptr(c), c.size, npc, _ptr(x), _ptr(sdev)))
        return x.T.copy(), sdev

    # ---------------------------------------------------------- device API
    def gather_rows_t(self, pcs_cm, N, d, idx, rows):
        """rows[i, :] = pcs[idx[i], :]; pcs_cm is a column-major (d, N) tensor."""
        check(self.lib.ccg_gather_rows_dev(self.ctx, _ptr(pcs_cm), N, d, _ptr(idx), idx.numel(),
                                           _ptr(rows), _stream()))

    def gather_rows_rm_t(self, pcs_rm, N, d, idx, rows):
        """rows[i, :] = pcs[idx[i], :] from a row-major (N, d) tensor (ccg_gather_rows_rm_dev)."""
        check(self.lib.ccg_gather_rows_rm_dev(self.ctx, _ptr(pcs_rm), N, d, _ptr(idx), idx.numel(),
                                              _ptr(rows), _stream()))

    def knn_rows_t(self, rows, kmax, out_idx, out_dist=None, stats=False):
        n, d = rows.shape
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_rows_dev(self.ctx, _ptr(rows), n, d, kmax, _ptr(out_idx), _ptr(out_dist),
                                        ctypes.byref(st) if stats else None, _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_boot_t(self, pcs_cm, N, d, idx, n_unique, rows, kmax, out_idx, out_dist=None, stats=False):
        """Device flavour of the bootstrap kNN over distinct cells
        (ccg_knn_boot_dev): pcs_cm (d, N) float64 (column-major N x d), idx (n,)
        int32 cells, n_unique = len(unique(idx)) (host int), rows (n, d) the
        gathered rows, out_idx (n, kmax) int32."""
        n = idx.numel()
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_boot_dev(self.ctx, _ptr(pcs_cm), N, d, _ptr(idx), n, int(n_unique), _ptr(rows),
                                        kmax, _ptr(out_idx), _ptr(out_dist), ctypes.byref(st) if stats else None,
                                        _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_boot_hint_t(self, pcs_cm, N, d, idx, n_unique, rows, kmax, out_idx, cell_hint, out_dist=None,
                        stats=False):
        """knn_boot_t with a warm start (ccg_knn_boot_hint_dev): cell_hint an
        (N,) float32 tensor of per-cell k-th squared distances (0 = none),
        read and updated in place.  Results do not depend on it."""
        n = idx.numel()
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_boot_hint_dev(self.ctx, _ptr(pcs_cm), N, d, _ptr(idx), n, int(n_unique), _ptr(rows),
                                             kmax, _ptr(out_idx), _ptr(out_dist), _ptr(cell_hint),
                                             ctypes.byref(st) if stats else None, _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_table_t(self, pcs_cm, N, d, K, tab_idx, tab_d2, stats=False):
        """ccg_knn_table_dev: every cell's K nearest other cells among the N
        (tab_idx (N, K) int32, tab_d2 (N, K) float64 squared distances)."""
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_table_dev(self.ctx, _ptr(pcs_cm), N, d, K, _ptr(tab_idx), _ptr(tab_d2),
                                         ctypes.byref(st) if stats else None, _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_last_fallback(self):
        """Rows the last kNN call sent to the exact search (ccg_knn_last_fallback)."""
        cnt = ctypes.c_int64(0)
        check(self.lib.ccg_knn_last_fallback(self.ctx, None, 0, ctypes.byref(cnt)))
        out = np.empty(max(cnt.value, 1), np.int32)
        check(self.lib.ccg_knn_last_fallback(self.ctx, _ptr(out), out.size, ctypes.byref(cnt)))
        return out[:cnt.value].copy()

    def knn_boot_table_t(self, pcs_cm, N, d, idx, n_unique, rows, kmax, tab_idx, tab_d2, out_idx, out_dist=None,
                         stats=False):
        """knn_boot_t from a cell table of the same PCs (ccg_knn_boot_table_dev)."""
        n = idx.numel()
        K = tab_idx.shape[1]
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_boot_table_dev(self.ctx, _ptr(pcs_cm), N, d, _ptr(idx), n, int(n_unique), _ptr(rows),
                                              kmax, _ptr(tab_idx), _ptr(tab_d2), K, _ptr(out_idx), _ptr(out_dist),
                                              ctypes.byref(st) if stats else None, _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_boots_table_t(self, N, d, idx, n_unique, rows, kmax, tab_idx, tab_d2, out_idx, out_dist=None,
                          local_ids=False, stats=False):
        """A batch of bootstraps through one set of launches
        (ccg_knn_boots_table_dev): idx (nb, n) int32 cell indices, n_unique
        nb host ints, rows (nb n, d) the gathered rows of every bootstrap,
        out_idx (nb n, kmax) -- ids of the concatenation unless local_ids."""
        nb, n = idx.shape
        nu = np.ascontiguousarray(n_unique, dtype=np.int32)
        if nu.size != nb:
            raise ValueError(f"knn_boots_table_t: {nu.size} n_unique values for {nb} bootstraps")
        if rows.shape[0] != nb * n or out_idx.shape[0] != nb * n:
            raise ValueError("knn_boots_table_t: rows / out_idx must have nb * n rows")
        K = tab_idx.shape[1]
        st = _lib.ccg_knn_stats() if stats else None
        check(self.lib.ccg_knn_boots_table_dev(self.ctx, N, d, _ptr(idx), n, nb, _ptr(nu), _ptr(rows), kmax,
                                               _ptr(tab_idx), _ptr(tab_d2), K, 1 if local_ids else 0,
                                               _ptr(out_idx), _ptr(out_dist), ctypes.byref(st) if stats else None,
                                               _stream()))
        if stats:
            self.last_knn_stats = (st.queries, st.fallback)
            return self.last_knn_stats
        return None

    def knn_segments_t(self, rows, seg_off, kmax, out_idx, out_dist=None, stats=False):
        """Device flavour: rows (n, d) tensor of concatenated segments, seg_off a
        host int64 array of nseg+1 offsets; out_idx (n, kmax) segment-local."""
        n, d = rows.shape
        off = np.ascontiguousarray(seg_off, dtype=np.int64)
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_knn_segments_dev(self.ctx, _ptr(rows), n, d, _ptr(off), off.size - 1, kmax,
                                            _ptr(out_idx), _ptr(out_dist), ctypes.byref(st), _stream()))
        self.last_knn_stats = (st.queries, st.fallback)
        return self.last_knn_stats if stats else None

    def snn_t(self, knn_idx, k, type, out_i, out_j, out_w, d_nedges):
        n, ks = knn_idx.shape
        t = {"number": _lib.CCG_SNN_NUMBER, "rank": _lib.CCG_SNN_RANK}[type]
        cap = out_i.numel() if out_i is not None else 0
        check(self.lib.ccg_snn_dev(self.ctx, _ptr(knn_idx), n, ks, k, t, _ptr(out_i), _ptr(out_j),
                                   _ptr(out_w), cap, _ptr(d_nedges), _stream()))

    def snn_multi_t(self, knn_idx, ks, type, outs, d_nedges):
        """All graphs of ks (ascending) in one pass.  outs: list of (i, j, w)
        tensors per graph (or None for count-only); d_nedges: int64 tensor (nk,)."""
        n, kst = knn_idx.shape
        nk = len(ks)
        t = {"number": _lib.CCG_SNN_NUMBER, "rank": _lib.CCG_SNN_RANK}[type]
        karr = (ctypes.c_int * nk)(*ks)
        P = _vp * nk
        oi = P(*[_ptr(o[0]) if o else None for o in outs])
        oj = P(*[_ptr(o[1]) if o else None for o in outs])
        ow = P(*[_ptr(o[2]) if o else None for o in outs])
        caps = (ctypes.c_int64 * nk)(*[o[0].numel() if o else 0 for o in outs])
        dn = P(*[_vp(d_nedges.data_ptr() + 8 * i) for i in range(nk)])
        check(self.lib.ccg_snn_multi_dev(self.ctx, _ptr(knn_idx), n, kst, karr, nk, t, oi, oj, ow, caps, dn,
                                         _stream()))

    def snn_rows_t(self, knn_idx, ks, type, row_off, row_len, nbr, wpk, d_nedges):
        """All graphs of ks as rows of the union graph (ccg_snn_rows_dev):
        row_off (n+1,) int64, row_len (n,) int32, nbr / wpk (cap,) int32 /
        uint32-as-int32 tensors, d_nedges (len(ks),) int64 (negative =
        -required capacity)."""
        n, kst = knn_idx.shape
        nk = len(ks)
        t = {"number": _lib.CCG_SNN_NUMBER, "rank": _lib.CCG_SNN_RANK}[type]
        karr = (ctypes.c_int * nk)(*ks)
        check(self.lib.ccg_snn_rows_dev(self.ctx, _ptr(knn_idx), n, kst, karr, nk, t, _ptr(row_off), _ptr(row_len),
                                        _ptr(nbr), _ptr(wpk), nbr.numel(), _ptr(d_nedges), _stream()))

    def snn_classes_t(self, knn_idx, ks, row_class, class_root, class_off, class_len, nbr, wpk, d_info, cell=None):
        """The NUMBER graphs of ks at the level of row classes
        (ccg_snn_classes_dev): row_class / class_root (n,) int32, class_off
        (n+1,) int64, class_len (n,) int32, nbr / wpk (cap,) int32 tensors,
        d_info (3 + len(ks),) int64 = [u, status, required cap, class edges per
        graph]; cell (n,) int32 tensor or None."""
        n, kst = knn_idx.shape
        nk = len(ks)
        karr = (ctypes.c_int * nk)(*ks)
        check(self.lib.ccg_snn_classes_dev(self.ctx, _ptr(knn_idx), n, kst, _ptr(cell), karr, nk, _ptr(row_class),
                                           _ptr(class_root), _ptr(class_off), _ptr(class_len), _ptr(nbr), _ptr(wpk),
                                           nbr.numel(), _ptr(d_info), _stream()))

    def snn_reserve(self, entries):
        check(self.lib.ccg_snn_reserve(self.ctx, entries))

    def silhouette_t(self, x, labels, cmax, out_mean, out_nclust, out_minsize, out_width=None):
        m, d = x.shape
        L = labels.shape[0]
        check(self.lib.ccg_silhouette_dev(self.ctx, _ptr(x), m, d, _ptr(labels), L, cmax, _ptr(out_mean),
                                          _ptr(out_nclust), _ptr(out_minsize), _ptr(out_width), _stream()))

    def silhouette_cells_t(self, x, labels, cmax, cell, ncell, out_mean, out_nclust, out_minsize):
        """ccg_silhouette_cells_dev: bootstrap rows x (m, d) whose cells are
        cell (m,) int32 in [0, ncell) (copies identical); widths once per
        (cell, label), weighted."""
        m, d = x.shape
        L = labels.shape[0]
        check(self.lib.ccg_silhouette_cells_dev(self.ctx, _ptr(x), m, d, _ptr(labels), L, cmax, _ptr(cell), ncell,
                                                _ptr(out_mean), _ptr(out_nclust), _ptr(out_minsize), _stream()))

    def silhouette_segments_t(self, x, seg_off, labels, cmax, cell, ncell, means=None, nclust=None, minsize=None):
        """ccg_silhouette_segments_dev: one launch set for a batch of segments.
        x (n, d) device rows of every segment concatenated, seg_off (nseg+1,)
        host int64 row offsets, labels: nseg device (L, m_s) int32 tensors,
        cell (n,) int32 cell ids distinct between segments, in [0, ncell);
        means / nclust / minsize: None or nseg device tensors of L values."""
        import ctypes
        n, d = x.shape
        off = np.ascontiguousarray(seg_off, dtype=np.int64)
        nseg = off.size - 1
        L = labels[0].shape[0]

        def arr(ts):
            if ts is None:
                return None
            a = (ctypes.c_void_p * nseg)(*[_ptr(t).value if t is not None else None for t in ts])
            return a
        lab = arr(labels)
        om, onc, oms = arr(means), arr(nclust), arr(minsize)
        check(self.lib.ccg_silhouette_segments_dev(
            self.ctx, _ptr(x), d, nseg, off.ctypes.data, lab, L, cmax, _ptr(cell), int(ncell),
            om, onc, oms, _stream()))

    def select_mapback_t(self, mode, labels, boot_idx, N, A, col0, means=None, nclust=None, minsize=None,
                         min_size=0, out_choice=None):
        """A: (B, N) uint8 or uint16 tensor (label width from its dtype)."""
        import torch
        nb, L, n = labels.shape
        md = {"robust": _lib.CCG_MODE_ROBUST, "granular": _lib.CCG_MODE_GRANULAR}[mode]
        bits = 8 if A.dtype == torch.uint8 else 16
        check(self.lib.ccg_select_mapback_dev(self.ctx, md, _ptr(labels), _ptr(boot_idx), n, nb, L, N,
                                              _ptr(means), _ptr(nclust), _ptr(minsize), min_size, _ptr(A), bits,
                                              col0, _ptr(out_choice), _stream()))

    def cocluster_t(self, A, r0, r1, co=None, both=None, dist=None):
        """A: (B, N) uint8 or uint16 tensor; outputs are row-slab tensors."""
        import torch
        B, N = A.shape
        bits = 8 if A.dtype == torch.uint8 else 16
        check(self.lib.ccg_cocluster_dev(self.ctx, _ptr(A), bits, N, B, r0, r1, _ptr(co), _ptr(both), _ptr(dist),
                                         _stream()))

    def consensus_knn_t(self, co, both, N, k, out_idx, d_flag):
        check(self.lib.ccg_consensus_knn_dev(self.ctx, _ptr(co), _ptr(both), N, k, _ptr(out_idx),
                                             _ptr(d_flag), _stream()))

    def sort_pairs_t(self, keys, vals, keys_out, vals_out, key_bits):
        """Stable radix sort of int32 (key, value) tensors by the low key_bits
        bits of the keys (ccg_sort_pairs_dev)."""
        check(self.lib.ccg_sort_pairs_dev(self.ctx, _ptr(keys), _ptr(keys_out), _ptr(vals), _ptr(vals_out),
                                          keys.numel(), key_bits, _stream()))

    def consensus_knn_assign_t(self, A, k, r0, r1, out_idx, d_flag):
        """Rows [r0, r1) of the consensus kNN from the (B, N) assignment tensor."""
        import torch
        B, N = A.shape
        bits = 8 if A.dtype == torch.uint8 else 16
        check(self.lib.ccg_consensus_knn_assign_dev(self.ctx, _ptr(A), bits, N, B, k, r0, r1, _ptr(out_idx),
                                                    _ptr(d_flag), _stream()))


# ----------------------------------------------------- host-only arithmetic
def cluster_block_means(simsum, npairs):
    """ccg_cluster_block_means: the K x K determineHierachy distance matrix."""
    simsum = np.ascontiguousarray(simsum, dtype=np.uint64)
    npairs = np.ascontiguousarray(npairs, dtype=np.int64)
    K = npairs.shape[0]
    out = np.empty((K, K), np.float64)
    check(_lib.load().ccg_cluster_block_means(K, _ptr(simsum), _ptr(npairs), _ptr(out)))
    return out


def pairwise_rand_ratio(tab, adjusted=True):
    """ccg_pairwise_rand_ratio: pairwiseRand(mode="ratio") from a K x (C+1) table."""
    tab = np.ascontiguousarray(tab, dtype=np.int32)
    K, W = tab.shape
    out = np.empty((K, K), np.float64)
    check(_lib.load().ccg_pairwise_rand_ratio(K, W - 1, _ptr(tab), 1 if adjusted else 0, _ptr(out)))
    return out
