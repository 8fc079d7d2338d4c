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
    cuts = [0]
    for g in range(1, G):
        r = N * (1.0 - math.sqrt(1.0 - g / G))
        r = int(round(r / align)) * align
        cuts.append(min(max(r, cuts[-1]), N))
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
    """All-gather each rank's (b_local x N) uint8 assignment columns.

    Every rank must hold the same b_local (weak scaling: fixed bootstraps per
    GPU).  Returns the (G*b_local x N) matrix with rank r's columns at rows
    [r*b_local, (r+1)*b_local) -- the column-major B x N layout of the C ABI.
    """
    import torch
    import torch.distributed as dist
    G = dist.get_world_size(group)
    out = torch.empty((G * local_cols.shape[0],) + tuple(local_cols.shape[1:]), dtype=local_cols.dtype,
                      device=local_cols.device)
    dist.all_gather_into_tensor(out, local_cols.contiguous(), group=group)
    return out


def gather_slabs_host(parts, N):
    """Concatenate per-rank packed slabs (in rank order) into the full packed array."""
    full = np.concatenate(parts)
    assert full.size == N * (N - 1) // 2
    return full
