"""Multi-GPU sharding: a thin wrapper over libccg's device group.

The group, its RCCL communicators and the shard plan live in libccg.so
(include/ccg.h "multi-GPU", csrc/group.hip), so an R session reaches the
same multi-GPU path through .Call without PyTorch.  This module only
  * exposes the host-side plan (bootstrap blocks, row slabs),
  * hands the RCCL group id from rank 0 to the other ranks over an existing
    torch.distributed process group (one process per GPU), and
  * orders the group's HIP streams with torch's current stream.
The reference is single-node CPU (BiocParallel over bootstraps, RcppParallel
inside parDist, R/consensusClust.R:391-421).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check

_vp = ctypes.c_void_p


def row_slabs(N, G):
    """Cuts r_0=0 < ... < r_G=N of pair-balanced packed-triangle slabs
    (ccg_row_slabs: r_g ~ N(1 - sqrt(1 - g/G)), interior cuts multiples of 128)."""
    cuts = np.zeros(G + 1, np.int64)
    check(_lib.load().ccg_row_slabs(int(N), int(G), cuts.ctypes.data_as(_vp)))
    return [int(c) for c in cuts]


def rect_slabs(N, G):
    """Cuts of equal full-row slabs (ccg_rect_slabs; the consensus kNN split)."""
    cuts = np.zeros(G + 1, np.int64)
    check(_lib.load().ccg_rect_slabs(int(N), int(G), cuts.ctypes.data_as(_vp)))
    return [int(c) for c in cuts]


def boot_shard(nboots, G, rank):
    """Contiguous block [b0, b1) of bootstrap ids owned by `rank` (ccg_boot_shard)."""
    b0, b1 = ctypes.c_int64(), ctypes.c_int64()
    check(_lib.load().ccg_boot_shard(int(nboots), int(G), int(rank), ctypes.byref(b0), ctypes.byref(b1)))
    return b0.value, b1.value


def allgather_plan(counts):
    """The all-gather's collective plan (ccg_allgather_plan): (offsets,
    equal, roots) -- one ncclAllGather when every rank sends the same number
    of rows, else one ncclBroadcast per root in `roots` (rank order), root r
    sending its block at offsets[r]."""
    G = len(counts)
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    off = np.zeros(G + 1, np.int64)
    roots = np.zeros(G, np.int32)
    eq, nr = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().ccg_allgather_plan(G, cnt.ctypes.data_as(_vp), off.ctypes.data_as(_vp), ctypes.byref(eq),
                                         roots.ctypes.data_as(_vp), ctypes.byref(nr)))
    return [int(o) for o in off], bool(eq.value), [int(r) for r in roots[:nr.value]]


def slab_offset(N, r0):
    """Packed-triangle offset of row r0 (rows hold j = i+1..N-1)."""
    return r0 * N - r0 * (r0 + 1) // 2


def slab_pairs(N, r0, r1):
    """Number of packed upper-triangle entries in rows [r0, r1)."""
    return slab_offset(N, r1) - slab_offset(N, r0)


def exchange_group_id(group=None, make_id=None):
    """Rank 0 creates the RCCL id (ccg_group_unique_id, or make_id()) and
    broadcasts its bytes to every rank of the torch.distributed group."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    box = [None]
    if rank == 0:
        if make_id is None:
            buf = (ctypes.c_uint8 * _lib.GROUP_ID_BYTES)()
            check(_lib.load().ccg_group_unique_id(buf))
            box[0] = bytes(buf)
        else:
            box[0] = bytes(make_id())
    dist.broadcast_object_list(box, src=0, group=group)
    gid = box[0]
    if len(gid) != _lib.GROUP_ID_BYTES:
        raise ValueError(f"group id must be {_lib.GROUP_ID_BYTES} bytes, got {len(gid)}")
    return gid


def _ptr_array(xs):
    arr = (_vp * len(xs))()
    for i, x in enumerate(xs):
        arr[i] = None if x is None else x.data_ptr()
    return arr


class DeviceGroup:
    """A libccg device group (ccg_group): one engine context per local device
    plus RCCL communicators.  Methods take torch tensors resident on the
    local devices (lists, one per local device) and run on the contexts'
    streams, ordered after torch's current stream and before its next work."""

    def __init__(self, handle):
        self.lib = _lib.load()
        self.h = handle
        nl, nr, r0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.lib.ccg_group_info(self.h, ctypes.byref(nl), ctypes.byref(nr), ctypes.byref(r0)))
        self.nlocal, self.nranks, self.first_rank = nl.value, nr.value, r0.value
        from .engine import Engine
        self.engines = []
        for l in range(self.nlocal):
            c = _vp()
            check(self.lib.ccg_group_ctx(self.h, l, ctypes.byref(c)))
            self.engines.append(Engine.from_ctx(c))

    @classmethod
    def open(cls, devices):
        """One process driving `devices` (ccg_group_open)."""
        lib = _lib.load()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = _vp()
        check(lib.ccg_group_open(devs, len(devices), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def open_rank(cls, device, nranks, rank, gid):
        """This process's device as rank `rank` of `nranks` (ccg_group_open_rank);
        gid from exchange_group_id.  Collective: blocks until every rank joins."""
        lib = _lib.load()
        buf = (ctypes.c_uint8 * _lib.GROUP_ID_BYTES).from_buffer_copy(gid)
        h = _vp()
        check(lib.ccg_group_open_rank(int(device), int(nranks), int(rank), buf, ctypes.byref(h)))
        return cls(h)

    def close(self):
        if self.h:
            for e in self.engines:
                e.ctx = None
            self.lib.ccg_group_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def synchronize(self):
        check(self.lib.ccg_group_synchronize(self.h))

    def _enter(self):
        import torch
        for e in self.engines:
            e.torch_stream().wait_stream(torch.cuda.current_stream(e.device))

    def _leave(self):
        import torch
        for e in self.engines:
            torch.cuda.current_stream(e.device).wait_stream(e.torch_stream())

    def allgather_columns_t(self, local, counts, out):
        """ccg_allgather_columns: local[l] (counts[rank] x N uint8/uint16) ->
        out[l] (sum(counts) x N) on every local device."""
        N = out[0].shape[1]
        bits = 8 if out[0].element_size() == 1 else 16
        cnt = (ctypes.c_int64 * self.nranks)(*[int(c) for c in counts])
        self._enter()
        check(self.lib.ccg_allgather_columns(self.h, _ptr_array(local), cnt, N, bits, _ptr_array(out)))
        self._leave()

    def cocluster_sharded_t(self, A, co=None, both=None, dist=None):
        """ccg_cocluster_sharded_dev: this group's row slabs (row_slabs cuts) of
        the packed co/both/dist from the full matrices A[l] (B x N)."""
        B, N = A[0].shape
        bits = 8 if A[0].element_size() == 1 else 16
        cuts = (ctypes.c_int64 * (self.nranks + 1))()
        self._enter()
        none = [None] * self.nlocal
        check(self.lib.ccg_cocluster_sharded_dev(self.h, _ptr_array(A), bits, N, B,
                                                 _ptr_array(co or none), _ptr_array(both or none),
                                                 _ptr_array(dist or none), cuts))
        self._leave()
        return list(cuts)

    def consensus_knn_sharded_t(self, A, k, out_idx, flags):
        """ccg_consensus_knn_sharded_dev: every out_idx[l] (N x k int32) ends
        up holding the whole consensus kNN; flags[l] the OR of the NaN flags."""
        B, N = A[0].shape
        bits = 8 if A[0].element_size() == 1 else 16
        self._enter()
        check(self.lib.ccg_consensus_knn_sharded_dev(self.h, _ptr_array(A), bits, N, B, int(k),
                                                     _ptr_array(out_idx), _ptr_array(flags)))
        self._leave()

    # ------------------------------------------- host flavours (R's entry points)
    def cocluster(self, A, want=("co", "both", "dist")):
        """ccg_group_cocluster: packed co/both/dist of a host B x N matrix."""
        A = np.ascontiguousarray(A)
        B, N = A.shape
        bits = 8 if A.dtype == np.uint8 else 16
        P = N * (N - 1) // 2
        out = {}
        co = np.empty(P, np.uint16) if "co" in want else None
        both = np.empty(P, np.uint16) if "both" in want else None
        dist = np.empty(P, np.float64) if "dist" in want else None
        p = lambda a: None if a is None else a.ctypes.data_as(_vp)
        check(self.lib.ccg_group_cocluster(self.h, p(A), bits, N, B, p(co), p(both), p(dist)))
        for name, a in (("co", co), ("both", both), ("dist", dist)):
            if a is not None:
                out[name] = a
        return out

    def consensus_knn_assign(self, A, k):
        """ccg_group_consensus_knn_assign: N x k 0-based consensus kNN."""
        A = np.ascontiguousarray(A)
        B, N = A.shape
        bits = 8 if A.dtype == np.uint8 else 16
        out = np.empty((N, k), np.int32)
        check(self.lib.ccg_group_consensus_knn_assign(self.h, A.ctypes.data_as(_vp), bits, N, B, int(k),
                                                      out.ctypes.data_as(_vp)))
        return out

    def knn_boot(self, pca, boot_idx, kmax=20, want_dist=True):
        """ccg_group_knn_boot: bootstraps split over the local devices."""
        pcs = np.asfortranarray(pca, dtype=np.float64)
        N, d = pcs.shape
        bi = np.ascontiguousarray(np.atleast_2d(boot_idx), dtype=np.int32)
        nb, n = bi.shape
        idx = np.empty((nb, n, kmax), np.int32)
        dist = np.empty((nb, n, kmax), np.float64) if want_dist else None
        st = _lib.ccg_knn_stats()
        check(self.lib.ccg_group_knn_boot(self.h, pcs.ctypes.data_as(_vp), N, d, bi.ctypes.data_as(_vp), n, nb,
                                          kmax, idx.ctypes.data_as(_vp),
                                          None if dist is None else dist.ctypes.data_as(_vp), ctypes.byref(st)))
        self.last_knn_stats = (st.queries, st.fallback)
        return idx, dist
