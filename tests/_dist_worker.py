"""Worker for tests/test_distributed.py (gloo, CPU): the multi-GPU sharding
plumbing -- bootstrap blocks per rank, all-gather of assignment columns,
pair-balanced row slabs -- checked against the single-process oracle."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def packed_slab_numpy(A, r0, r1):
    """co/both of rows [r0, r1) of the packed upper triangle (CPU, test only)."""
    A = A.numpy().astype(np.int64)
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
    from consensusclustr_amd.sharding import boot_shard, sharded_cocluster, slab_pairs
    import oracle as O
    N, nboots = 300, 10
    rng = np.random.default_rng(7)
    full = rng.integers(0, 6, (nboots, N)).astype(np.uint8)  # the assignment columns of all bootstraps
    b0, b1 = boot_shard(nboots, world, rank)
    local = torch.from_numpy(full[b0:b1].copy())
    (co, both), (r0, r1), A = sharded_cocluster(local, N, packed_slab_numpy)
    assert np.array_equal(A.numpy(), full), "all-gathered columns differ from the single-process matrix"
    assert co.size == slab_pairs(N, r0, r1)
    parts = [None] * world
    dist.all_gather_object(parts, (co, both))
    if rank == 0:
        Ao = full.astype(np.int32)
        Ao[Ao == 0] = -1
        ref = O.cocluster(Ao)
        co_all = np.concatenate([p[0] for p in parts])
        both_all = np.concatenate([p[1] for p in parts])
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
