"""Host community detection used by the drop-in's Leiden boundary.

The reference keeps ``igraph::cluster_leiden`` on the host (R/consensusClust.R
:656-658 via bluster, :430-433 explicitly) and so does this engine: the GPU
produces the SNN graph, the host clusters it.  python-igraph / leidenalg are
not installed in this image, so this module provides a deterministic
modularity optimiser (Louvain local moving + aggregation, resolution
parameter as in igraph's modularity objective) as the default stand-in:
``louvain`` runs libccg's host implementation (``ccg_host_louvain``, C++ on
the calling thread, GIL released), ``louvain_py`` is the same algorithm in
Python (readable, seconds per graph at 18k rows; different node order, so
its labels can differ).  Neither is bit-compatible with igraph's Leiden
(different algorithm and RNG); pass ``clusterFun=`` a callable wrapping
igraph where it is available.  A callable has the signature
``f(n, ei, ej, w, resolution, seed) -> labels`` with labels 1..C.
"""
import ctypes

import numpy as np

from . import _lib


def louvain(n, ei, ej, w, resolution=1.0, seed=0):
    """Modularity (with resolution) community detection on host threads
    (ccg_host_louvain); returns int32 labels 1..C in order of first appearance."""
    ei = np.ascontiguousarray(ei, dtype=np.int32)
    ej = np.ascontiguousarray(ej, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    if not (ei.size == ej.size == w.size):
        raise ValueError("louvain: ei, ej and w must have the same length")
    out = np.empty(int(n), np.int32)
    vp = ctypes.c_void_p
    _lib.check(_lib.load().ccg_host_louvain(int(n), ei.size, vp(ei.ctypes.data), vp(ej.ctypes.data),
                                            vp(w.ctypes.data), float(resolution), int(seed) & (2**64 - 1),
                                            vp(out.ctypes.data)))
    return out


def _csr(n, ei, ej, w):
    src = np.concatenate([ei, ej]).astype(np.int64)
    dst = np.concatenate([ej, ei]).astype(np.int64)
    ww = np.concatenate([w, w]).astype(np.float64)
    order = np.argsort(src, kind="stable")
    src, dst, ww = src[order], dst[order], ww[order]
    indptr = np.zeros(n + 1, np.int64)
    np.add.at(indptr, src + 1, 1)
    np.cumsum(indptr, out=indptr)
    return indptr, dst, ww


def _one_level(n, indptr, nbr, wts, self_w, gamma, rng):
    k = np.zeros(n)
    for i in range(n):
        k[i] = wts[indptr[i]:indptr[i + 1]].sum() + 2.0 * self_w[i]
    m2 = k.sum()
    if m2 <= 0:
        return np.arange(n), False
    comm = np.arange(n)
    tot = k.copy()
    moved_any = False
    improved = True
    sweeps = 0
    while improved and sweeps < 32:
        improved = False
        sweeps += 1
        for i in rng.permutation(n):
            ci = comm[i]
            lo, hi = indptr[i], indptr[i + 1]
            links = {}
            for t in range(lo, hi):
                c = comm[nbr[t]]
                links[c] = links.get(c, 0.0) + wts[t]
            tot[ci] -= k[i]
            best_c = ci
            best_gain = links.get(ci, 0.0) - gamma * k[i] * tot[ci] / m2
            for c, lw in links.items():
                g = lw - gamma * k[i] * tot[c] / m2
                if g > best_gain + 1e-12 or (abs(g - best_gain) <= 1e-12 and c < best_c and c != ci and g > best_gain):
                    best_gain, best_c = g, c
            tot[best_c] += k[i]
            if best_c != ci:
                comm[i] = best_c
                improved = True
                moved_any = True
    _, comm = np.unique(comm, return_inverse=True)
    return comm, moved_any


def louvain_py(n, ei, ej, w, resolution=1.0, seed=0, max_levels=16):
    """Modularity (with resolution) community detection in Python; returns labels 1..C."""
    rng = np.random.default_rng(seed)
    ei = np.asarray(ei, np.int64)
    ej = np.asarray(ej, np.int64)
    w = np.asarray(w, np.float64)
    membership = np.arange(n)
    cur_n = n
    self_w = np.zeros(n)
    for _ in range(max_levels):
        indptr, nbr, wts = _csr(cur_n, ei, ej, w)
        comm, moved = _one_level(cur_n, indptr, nbr, wts, self_w, resolution, rng)
        membership = comm[membership]
        if not moved:
            break
        # aggregate
        nc = comm.max() + 1
        new_self = np.zeros(nc)
        np.add.at(new_self, comm, self_w)
        ci, cj = comm[ei], comm[ej]
        same = ci == cj
        np.add.at(new_self, ci[same], w[same])
        a = np.minimum(ci[~same], cj[~same])
        b = np.maximum(ci[~same], cj[~same])
        if a.size:
            key = a * nc + b
            uk, inv = np.unique(key, return_inverse=True)
            nw = np.zeros(uk.size)
            np.add.at(nw, inv, w[~same])
            ei, ej, w = uk // nc, uk % nc, nw
        else:
            ei = ej = np.zeros(0, np.int64)
            w = np.zeros(0)
        self_w = new_self
        cur_n = nc
    # label ids in order of first appearance, 1-based
    _, first = np.unique(membership, return_index=True)
    order = np.argsort(first)
    remap = np.empty(order.size, np.int64)
    remap[order] = np.arange(order.size)
    return (remap[np.unique(membership, return_inverse=True)[1]] + 1).astype(np.int32)
