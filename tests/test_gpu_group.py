"""libccg's device group (ccg_group_*, RCCL inside the library) on the GPU box.

The box has one GPU, so the groups here hold one device (ncclCommInitAll and
ncclCommInitRank with nranks 1); the multi-rank plan is rehearsed on CPU in
tests/test_distributed.py.  Each group result must equal the single-context
entry point bit for bit, and the oracle.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _assign(rng, B, N, C=7, na=0.2, dtype=np.uint8):
    A = rng.integers(1, C + 1, (B, N)).astype(dtype)
    A[rng.random((B, N)) < na] = 0
    return A


@pytest.fixture(scope="module")
def group():
    from consensusclustr_amd.sharding import DeviceGroup
    g = DeviceGroup.open([0])
    yield g
    g.close()


def test_group_info(group):
    assert (group.nlocal, group.nranks, group.first_rank) == (1, 1, 0)
    assert group.engines[0].device == 0


def test_group_cocluster_host_matches_oracle(group, engine):
    rng = np.random.default_rng(1)
    A = _assign(rng, 60, 777)
    got = group.cocluster(A)
    one = engine.cocluster(A)
    Ao = A.astype(np.int32)
    Ao[Ao == 0] = -1
    ref = O.cocluster(Ao)
    for key in ("co", "both"):
        assert np.array_equal(got[key], one[key])
        assert np.array_equal(got[key].astype(np.int64), ref[key].astype(np.int64))
    assert np.array_equal(got["dist"], one["dist"], equal_nan=True)


def test_group_sharded_dev_matches_single_context(group, engine):
    import torch
    rng = np.random.default_rng(2)
    B, N = 40, 1000
    A = _assign(rng, B, N, C=12, dtype=np.uint16)
    At = torch.from_numpy(A.astype(np.int32)).to(torch.int16).cuda()
    full = torch.zeros_like(At)
    local = full[:B]
    local.copy_(At)
    group.allgather_columns_t([local], [B], [full])  # one rank: in place
    P = N * (N - 1) // 2
    co = torch.empty(P, dtype=torch.int16, device="cuda")
    both = torch.empty_like(co)
    dist = torch.empty(P, dtype=torch.float64, device="cuda")
    cuts = group.cocluster_sharded_t([full], co=[co], both=[both], dist=[dist])
    torch.cuda.synchronize()
    assert cuts == [0, N]
    assert torch.equal(full, At)
    one = engine.cocluster(A)
    assert np.array_equal(co.cpu().numpy().view(np.uint16), one["co"])
    assert np.array_equal(both.cpu().numpy().view(np.uint16), one["both"])
    assert np.array_equal(dist.cpu().numpy(), one["dist"], equal_nan=True)


def test_group_consensus_knn_matches_oracle(group, engine):
    import torch
    rng = np.random.default_rng(3)
    B, N, k = 50, 900, 20
    A = _assign(rng, B, N, C=5, na=0.1)
    got = group.consensus_knn_assign(A, k)
    assert np.array_equal(got, engine.consensus_knn_assign(A, k))
    Ao = A.astype(np.int32)
    Ao[Ao == 0] = -1
    ref = O.consensus_knn(O.cocluster(Ao, want=("dist",))["dist"], N, k)
    assert np.array_equal(got, ref)
    # device form: every device ends with the whole matrix
    At = torch.from_numpy(A).cuda()
    out = torch.full((N, k), -1, dtype=torch.int32, device="cuda")
    flag = torch.ones(1, dtype=torch.int32, device="cuda")
    group.consensus_knn_sharded_t([At], k, [out], [flag])
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    assert np.array_equal(out.cpu().numpy(), ref)


def test_group_consensus_knn_nan_is_reported(group):
    from consensusclustr_amd._lib import CcgError
    A = np.zeros((3, 300), np.uint8)
    A[:, :150] = 1  # cells 150.. never sampled: every pair with them has both == 0
    with pytest.raises(CcgError, match="ENAN"):
        group.consensus_knn_assign(A, 5)


def test_group_knn_boot_matches_engine(group, engine):
    rng = np.random.default_rng(4)
    N, d, n, nb = 3000, 12, 2500, 3
    pcs = rng.normal(size=(N, d))
    boots = rng.integers(0, N, (nb, n)).astype(np.int32)
    gi, gd = group.knn_boot(pcs, boots, kmax=20)
    ei, ed = engine.knn_boot(pcs, boots, kmax=20)
    assert np.array_equal(gi, ei)
    assert np.array_equal(gd, ed)
    assert group.last_knn_stats[0] == nb * n


def test_group_open_rank_single(engine):
    """The one-process-per-device form: an id from ccg_group_unique_id,
    ncclCommInitRank with nranks 1, then an all-gather that is a copy."""
    import torch
    from consensusclustr_amd import _lib
    from consensusclustr_amd.sharding import DeviceGroup
    buf = (ctypes.c_uint8 * _lib.GROUP_ID_BYTES)()
    _lib.check(_lib.load().ccg_group_unique_id(buf))
    with DeviceGroup.open_rank(0, 1, 0, bytes(buf)) as g:
        assert (g.nlocal, g.nranks, g.first_rank) == (1, 1, 0)
        src = torch.arange(3 * 257, dtype=torch.int32, device="cuda").to(torch.uint8).view(3, 257)
        dst = torch.zeros_like(src)
        g.allgather_columns_t([src], [3], [dst])
        torch.cuda.synchronize()
        assert torch.equal(src, dst)


def test_group_rejects_bad_arguments():
    from consensusclustr_amd import _lib
    from consensusclustr_amd.sharding import DeviceGroup
    with pytest.raises(_lib.CcgError):
        DeviceGroup.open([0, 0])
