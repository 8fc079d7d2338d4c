"""Worker for tests/test_distributed.py (gloo, CPU): the multi-GPU plan of
libccg's device group rehearsed across processes -- the group-id hand-off
from rank 0 (sharding.exchange_group_id), bootstrap blocks (ccg_boot_shard),
the rank-ordered column all-gather (emulated with gloo; on GPUs it is
ccg_allgather_columns over RCCL) and pair-balanced row slabs
(ccg_row_slabs) -- checked against the single-process oracle."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def packed_slab_numpy(A, r0, r1):
    """co/both of rows [r0, r1) of the packed upper triangle (CPU, test only)."""
    A = A.astype(np.int64)
    B, N = A.shape
    co, both = [], []
    for i in range(r0, r1):
        a = A[:, i:i + 1]
        rest = A[:, i + 1:]
        co.append(((a == rest) & (a != 0)).sum(0))
        both.append(((a != 0) & (rest != 0)).sum(0))
    if not co:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(co), np.concatenate(both)


def main(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from consensusclustr_amd.sharding import allgather_plan, boot_shard, exchange_group_id, row_slabs, slab_pairs
    import oracle as O
    # the RCCL id every rank passes to ccg_group_open_rank comes from rank 0
    gid = exchange_group_id(make_id=lambda: np.random.default_rng(99).integers(0, 256, 128, dtype=np.uint8))
    ids = [None] * world
    dist.all_gather_object(ids, gid)
    assert all(x == ids[0] for x in ids) and len(gid) == 128
    N = 300
    nboots = 10 if world != 2 else 12  # world 3: unequal blocks (broadcast plan); world 2: equal (all-gather)
    rng = np.random.default_rng(7)
    full = rng.integers(0, 6, (nboots, N)).astype(np.uint8)  # the assignment columns of all bootstraps
    spans = [boot_shard(nboots, world, r) for r in range(world)]
    b0, b1 = spans[rank]
    counts = [s[1] - s[0] for s in spans]
    # the all-gather as libccg's group issues it over RCCL (ccg_allgather_plan):
    # each rank writes its block in place into the full matrix, then one
    # all-gather (equal counts) or one broadcast per root (unequal counts)
    off, equal, roots = allgather_plan(counts)
    assert off[rank] == b0 and off[rank + 1] == b1
    A_t = torch.zeros((nboots, N), dtype=torch.uint8)
    A_t[b0:b1] = torch.from_numpy(full[b0:b1])
    if equal:
        parts = list(A_t.split(counts[0]))
        dist.all_gather(parts, A_t[b0:b1].clone())
        A_t = torch.cat(parts)
    else:
        assert roots == [r for r in range(world) if counts[r] > 0]
        for root in roots:
            blk = A_t[off[root]:off[root + 1]].contiguous()
            dist.broadcast(blk, src=root)
            A_t[off[root]:off[root + 1]] = blk
    A = A_t.numpy()
    assert np.array_equal(A, full), "all-gathered columns differ from the single-process matrix"
    cuts = row_slabs(N, world)
    r0, r1 = cuts[rank], cuts[rank + 1]
    co, both = packed_slab_numpy(A, r0, r1)
    assert co.size == slab_pairs(N, r0, r1)
    got = [None] * world
    dist.all_gather_object(got, (co, both))
    if rank == 0:
        Ao = full.astype(np.int32)
        Ao[Ao == 0] = -1
        ref = O.cocluster(Ao)
        co_all = np.concatenate([p[0] for p in got])
        both_all = np.concatenate([p[1] for p in got])
        assert np.array_equal(co_all, ref["co"].astype(np.int64)), "sharded co counts differ"
        assert np.array_equal(both_all, ref["both"].astype(np.int64)), "sharded both counts differ"
        with open(out_path, "w") as f:
            f.write("ok")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    mp.spawn(main, args=(world, port, out), nprocs=world)
