"""Multi-GPU sharding of the bootstrap path (one process per GPU).

The reference is single-node CPU (BiocParallel workers, RcppParallel threads
in parDist, R/consensusClust.R:391-421); this is the engine's own layer:
  * bootstraps are independent -> contiguous blocks of bootstraps per rank,
    no communication for gather/kNN/SNN/silhouette/selection/map-back;
  * co-clustering needs every rank's assignment columns -> ONE all-gather of
    the uint8 columns (RCCL over xGMI via torch.distributed "nccl");
  * the co/both/dist output is the packed upper triangle, split into row
    slabs balanced by pair count, each slab owned and kept by one GPU.
"""
import math

import numpy as np


def row_slabs(N, G, align=128):
    """Row boundaries r_0=0 < ... < r_G=N of pair-balanced upper-triangle slabs.

    Slab g holds rows [r_g, r_{g+1}); row i has N-1-i pairs, so equal pair
    counts need r_g = N(1 - sqrt(1 - g/G)).  Interior cuts are rounded to
    multiples of `align` (the co-cluster tile height).
    """
    top = (N // align) * align  # interior cuts stay aligned (a cut at N would be an unaligned r0)
    cuts = [0]
    for g in range(1, G):
        r = N * (1.0 - math.sqrt(1.0 - g / G))
        r = int(round(r / align)) * align
        cuts.append(min(max(r, cuts[-1]), top))
    cuts.append(N)
    return cuts


def slab_pairs(N, r0, r1):
    """Number of packed upper-triangle entries in rows [r0, r1)."""
    def off(i):
        return i * N - i * (i + 1) // 2
    return off(r1) - off(r0)


def slab_offset(N, r0):
    return r0 * N - r0 * (r0 + 1) // 2


def boot_shard(nboots, G, rank):
    """Contiguous block [b0, b1) of bootstrap ids owned by `rank`."""
    base, rem = divmod(nboots, G)
    b0 = rank * base + min(rank, rem)
    return b0, b0 + base + (1 if rank < rem else 0)


def allgather_columns(local_cols, group=None):
    """All-gather every rank's (b_r x N) uint8 assignment columns.

    Returns the (sum_r b_r x N) matrix with rank r's columns after rank r-1's
    -- the column-major B x N layout of the C ABI.  Equal b_r (weak scaling:
    fixed bootstraps per GPU) is one all_gather_into_tensor; unequal counts
    are padded to the largest and trimmed.
    """
    import torch
    import torch.distributed as dist
    G = dist.get_world_size(group)
    b = torch.tensor([local_cols.shape[0]], dtype=torch.int64, device=local_cols.device)
    sizes = [torch.zeros_like(b) for _ in range(G)]
    dist.all_gather(sizes, b, group=group)
    sizes = [int(s.item()) for s in sizes]
    bmax = max(sizes)
    tail = tuple(local_cols.shape[1:])
    src = local_cols.contiguous()
    if src.shape[0] < bmax:
        pad = torch.zeros((bmax - src.shape[0],) + tail, dtype=src.dtype, device=src.device)
        src = torch.cat([src, pad])
    out = torch.empty((G * bmax,) + tail, dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    if all(s == bmax for s in sizes):
        return out
    return torch.cat([out[r * bmax:r * bmax + sizes[r]] for r in range(G)])


def gather_slabs_host(parts, N):
    """Concatenate per-rank packed slabs (in rank order) into the full packed array."""
    full = np.concatenate(parts)
    assert full.size == N * (N - 1) // 2
    return full


def sharded_cocluster(local_cols, N, slab_fn, group=None):
    """One rank's part of the multi-GPU co-clustering step.

    local_cols: this rank's (b_local x N) uint8 assignment columns (tensor);
    slab_fn(A, r0, r1) computes and returns this rank's packed slab of rows
    [r0, r1) from the full (G*b_local x N) matrix A (the engine's
    cocluster_t on the GPU; a CPU function in tests).  Returns
    (slab, (r0, r1), A).
    """
    import torch.distributed as dist
    G = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    A = allgather_columns(local_cols, group) if G > 1 else local_cols
    cuts = row_slabs(N, G)
    r0, r1 = cuts[rank], cuts[rank + 1]
    return slab_fn(A, r0, r1), (r0, r1), A
