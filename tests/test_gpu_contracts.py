"""Library contracts that no kernel-parity test pins:

* stream ordering (round 5's illegal-address fault, gpurun_out/s4 and s5:
  ccg_silhouette_segments_dev read a temporary that torch had already freed
  and reused, because the library took torch's default stream -- handle 0 --
  for "the context's own non-blocking stream").  Since ABI 7 a NULL stream
  IS the legacy default stream: a torch op on the default stream writes an
  input after a long torch.cuda._sleep, the library call follows with a NULL
  stream (and through Engine, which passes hipStreamLegacy), the temporary
  is freed and overwritten at once; the outputs must equal the values the
  input held when the call was made;
* the single-pass scan (ccg_scan_i64_dev) at the tile counts where its
  look-back and its paths change: n = 1, 2048, 64 * 2048 + 1, 1024 * 2048
  (the last single-pass size) and 1024 * 2048 + 1 (the two-pass scan),
  in place and not, several calls in a row on one context and alternating
  between two streams (each stream has its own status words);
* the drop-in SNN graphs for a host consumer (ccg_snn_graphs_cells +
  ccg_snn_graph_fetch, what R's getClustAssignments calls) at the cfg3
  bootstrap size, n = 90 000, against the oracle.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def test_null_stream_orders_after_torch_default_stream(engine):
    import torch
    from consensusclustr_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    N, d, n = 50000, 16, 400000
    pcs = torch.from_numpy(rng.normal(size=(N, d))).to(dev)
    idx_np = rng.integers(0, N, n).astype(np.int32)
    want = pcs.cpu().numpy()[idx_np]
    src = torch.from_numpy(idx_np).to(dev)
    torch.cuda.synchronize()
    for via_engine in (False, True):
        rows = torch.zeros((n, d), dtype=torch.float64, device=dev)
        idx = torch.zeros(n, dtype=torch.int32, device=dev)  # a temporary
        torch.cuda._sleep(200_000_000)  # keep the default stream busy before the write
        idx.copy_(src)
        if via_engine:
            engine.gather_rows_rm_t(pcs, N, d, idx, rows)
        else:  # NULL stream straight through the C ABI
            rc = lib.ccg_gather_rows_rm_dev(engine.ctx, ctypes.c_void_p(pcs.data_ptr()), N, d,
                                            ctypes.c_void_p(idx.data_ptr()), n, ctypes.c_void_p(rows.data_ptr()),
                                            None)
            assert rc == 0
        del idx  # freed while the call may still be queued: the next allocation reuses the block
        junk = torch.full((n,), N - 1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        assert np.array_equal(rows.cpu().numpy(), want), via_engine
        del junk


def test_silhouette_segments_input_written_on_default_stream(engine):
    """The call that faulted in round 5, with its labels written by torch on
    the default stream just before it and freed just after."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(4)
    segs = [3000, 1800, 2500]
    off = np.concatenate([[0], np.cumsum(segs)]).astype(np.int64)
    d, L, C = 15, 6, 9
    cells = [rng.integers(0, 4000, m) for m in segs]
    base = rng.normal(size=(4000, d))
    x = torch.from_numpy(np.concatenate([base[c] for c in cells])).to(dev)
    cell = torch.from_numpy(np.concatenate([c + 4000 * s for s, c in enumerate(cells)]).astype(np.int32)).to(dev)
    lab_np = [rng.integers(1, C + 1, (L, m)).astype(np.int32) for m in segs]
    for s, c in enumerate(cells):  # copies of a cell share a label (Leiden gives copies one label)
        first = {}
        for r, v in enumerate(c):
            first.setdefault(int(v), r)
        lab_np[s] = np.ascontiguousarray(lab_np[s][:, [first[int(v)] for v in c]])
    ref = []
    for s in range(len(segs)):
        X = base[cells[s]]
        ref.append([O.silhouette(X, lab_np[s][l_])[1] for l_ in range(L)])
    src = [torch.from_numpy(a).to(dev) for a in lab_np]
    means = [torch.empty(L, dtype=torch.float64, device=dev) for _ in segs]
    torch.cuda.synchronize()
    labs = [torch.zeros_like(a) for a in src]
    torch.cuda._sleep(200_000_000)
    for a, b in zip(labs, src):
        a.copy_(b)
    engine.silhouette_segments_t(x, off, labs, C, cell, 4000 * len(segs), means)
    del labs
    junk = [torch.full_like(a, C) for a in src]
    torch.cuda.synchronize()
    for s in range(len(segs)):
        np.testing.assert_allclose(means[s].cpu().numpy(), ref[s], rtol=1e-5)
    del junk
    with pytest.raises(ValueError):  # a strided view would be read in the wrong order: refused
        engine.silhouette_segments_t(x, off, [a.t().contiguous().t() for a in src], C, cell, 4000 * len(segs), means)


def test_pinned_ring_wait_is_accounted_and_reset(engine):
    """CCG_KT_HOST_RING_WAIT: more staged uploads than the ring has slots,
    queued behind a busy GPU, block the host on the oldest slot; the wait is
    reported once and then reset (bench.py's host_ring_wait_ms_per_step)."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    segs = [300, 200]
    off = np.concatenate([[0], np.cumsum(segs)]).astype(np.int64)
    x = torch.from_numpy(rng.normal(size=(sum(segs), 4))).to(dev)
    cell = torch.arange(sum(segs), dtype=torch.int32, device=dev)
    labs = [torch.from_numpy(rng.integers(1, 4, (2, m)).astype(np.int32)).to(dev) for m in segs]
    means = [torch.empty(2, dtype=torch.float64, device=dev) for _ in segs]
    engine.silhouette_segments_t(x, off, labs, 3, cell, sum(segs), means)
    torch.cuda.synchronize()
    ref = [m.clone() for m in means]
    engine.timing_read("host_ring_wait")  # (reset)
    torch.cuda._sleep(300_000_000)
    for _ in range(80):  # > CCG_PIN_RING (8) uploads on the legacy stream behind the sleep
        engine.silhouette_segments_t(x, off, labs, 3, cell, sum(segs), means)
    torch.cuda.synchronize()
    ms, waits = engine.timing_read("host_ring_wait")
    assert waits >= 1 and ms > 0.0
    assert engine.timing_read("host_ring_wait") == (0.0, 0)
    for a, b in zip(means, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [1, 2048, 64 * 2048 + 1, 1024 * 2048, 1024 * 2048 + 1])
def test_scan_tile_counts_in_place_and_repeated(engine, n):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(n)
    for rep in range(3):
        x = rng.integers(0, 1 << 40, n, dtype=np.int64) if rep == 2 else rng.integers(0, 1000, n, dtype=np.int64)
        if rep == 1:
            x[:] = 0
        want = np.concatenate([[0], np.cumsum(x)])
        xt = torch.from_numpy(x).to(dev)
        out = torch.empty(n + 1, dtype=torch.int64, device=dev)
        engine.scan_i64_t(xt, out)
        buf = torch.empty(n + 1, dtype=torch.int64, device=dev)  # in place: out aliases in
        buf[:n] = xt
        engine.scan_i64_t(buf[:n], buf)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want), rep
        assert np.array_equal(buf.cpu().numpy(), want), rep


def test_scan_reports_values_outside_its_range(engine):
    """The status words pack 62-bit values: a prefix at or past 2^62 sets the
    sticky error instead of wrapping silently."""
    import torch
    from consensusclustr_amd import CcgError
    x = torch.zeros(3 * 2048, dtype=torch.int64, device="cuda:0")
    x[2048] = 1 << 62  # tile 1's sum
    out = torch.empty(x.numel() + 1, dtype=torch.int64, device="cuda:0")
    engine.scan_i64_t(x, out)
    with pytest.raises(CcgError):
        engine.synchronize()
    engine.synchronize()  # (the error is taken once)


def test_scan_alternating_streams_one_context(engine):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    n = 700 * 2048 + 5
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    xs = [torch.from_numpy(rng.integers(0, 1 << 20, n, dtype=np.int64)).to(dev) for _ in range(6)]
    outs = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(6)]
    torch.cuda.synchronize()
    for i, (x, o) in enumerate(zip(xs, outs)):  # back to back, no ordering between the two streams
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            engine.scan_i64_t(x, o)
    torch.cuda.synchronize()
    for x, o in zip(xs, outs):
        xn = x.cpu().numpy()
        assert np.array_equal(o.cpu().numpy(), np.concatenate([[0], np.cumsum(xn)]))


def test_snn_drop_in_host_decoder_at_cfg3_size(engine):
    """Engine.snn_multi (ccg_snn_graphs_cells + ccg_snn_graph_fetch: the
    product's host decoder both drop-ins use) on the bench's first cfg3
    bootstrap, n = 90 000 rows with their cells, against orc_snn."""
    import time
    import torch
    import bench
    dev = torch.device("cuda", 0)
    N, d, n = 100000, 30, 90000
    pcs, _ = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, dev)
    boot_np = np.random.default_rng(123).integers(0, N, n).astype(np.int32)
    rows = torch.empty((n, d), dtype=torch.float64, device=dev)
    boot = torch.from_numpy(boot_np).to(dev)
    engine.gather_rows_rm_t(pcs, N, d, boot, rows)
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    u = int(np.unique(boot_np).size)
    engine.knn_boot_t(pcs.t().contiguous(), N, d, boot, u, rows, 20, knn)
    torch.cuda.synchronize()
    kn = knn.cpu().numpy()
    t0 = time.perf_counter()
    graphs = engine.snn_multi(kn, [10, 15, 20], "number", cell=boot_np)
    wall = time.perf_counter() - t0
    for (gi, gj, gw), k in zip(graphs, (10, 15, 20)):
        ei, ej, ew = O.snn(kn, k, "number")
        assert np.array_equal(gi, ei) and np.array_equal(gj, ej) and np.array_equal(gw, ew), k
    t_pass, t_fetch = engine.last_snn_times
    print(f"snn_multi n={n}: device pass + staging {1e3 * t_pass:.1f} ms, host decode {1e3 * t_fetch:.1f} ms, "
          f"wall {1e3 * wall:.1f} ms, edges {[g[0].size for g in graphs]}")
    with pytest.raises(ValueError):
        engine.snn_multi(kn, [10], "number", cell=boot_np[:-1])
