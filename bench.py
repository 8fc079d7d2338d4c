#!/usr/bin/env python
"""Benchmark: bootstraps/sec (kNN+SNN+co-cluster) at 100k cells on 1..8 MI355X.

One step = per GPU, B bootstraps of the robust consensusClust path
(R/consensusClust.R:391-408 + :650-692) -- gather of the bootstrap rows, exact
kNN at k=20 (k=10/15 are prefixes), SNN "number" graphs for k = 10, 15, 20,
silhouette scores of the 60 clusterings, selection + map-back to the
uint8 assignment column -- then the all-gather of every rank's columns and
this rank's row slab of the co-clustering counts (:411-421) over all
G*B columns.  Host Leiden is excluded (north_star): the 60 clusterings per
bootstrap are synthetic labels derived from the true populations with 5%
flips, generated on the device before timing.  Inputs are resident in HBM
when the timed region starts.  Weak scaling: B bootstraps per GPU per step
(default 125 -> 1000 bootstraps = BASELINE config 3 at 8 GPUs).

Usage: python bench.py [--gpus N --steps K --warmup W].  With --gpus N > 1
and no WORLD_SIZE in the environment, this process (which never touches the
GPU) starts N ranks through torch.distributed.run (127.0.0.1) and exits with
their status; under torch.distributed.run (WORLD_SIZE set) each rank drives
one GPU, RCCL ("nccl") for the all-gather.  --launcher-check runs only the
rank wiring (gloo, no GPU) and prints the world the ranks saw.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "bootstraps/sec (kNN+SNN+co-cluster) at 100k cells, 1/2/4/8 MI355X"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak
PEAK_F16_TFLOPS = 2500.0   # dense fp16/bf16 MFMA (the screen's v_mfma_f32_32x32x16_f16)
PEAK_I8_TOPS = 5000.0      # dense int8 MFMA (2x bf16 dense 2.5 PF)
PEAK_HBM_GBS = 8000.0
PEAK_F64_TFLOPS = 78.6     # dense fp64 MFMA (MI355X spec; not in the guide)
K_NUM = (10, 15, 20)
N_RES = 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cells", type=int, default=100000)
    ap.add_argument("--pcs", type=int, default=30)
    ap.add_argument("--genes", type=int, default=2000)
    ap.add_argument("--boots-per-gpu", type=int, default=125)
    ap.add_argument("--boot-size", type=float, default=0.9)
    ap.add_argument("--cpu-sample-rows", type=int, default=6000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=3,
                    help="bootstraps in flight per GPU (one engine context + HIP stream each)")
    ap.add_argument("--pipeline", default="",
                    help="NK,NS: stage-split schedule instead of --streams: NK kNN streams feed NS "
                         "SNN+silhouette streams through a ring of bootstrap buffers")
    ap.add_argument("--knn-path", choices=["table", "screen"], default="table",
                    help="table: one cell table per step (ccg_knn_table_dev) filtered per bootstrap; "
                         "screen: a screen per bootstrap (warm-started)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="HIP hardware queues for this process (0: the runtime's default)")
    ap.add_argument("--table-k", type=int, default=48,
                    help="cell-table length K (<= 48): cells with fewer than 20 of their K nearest cells in a "
                         "bootstrap take the exact search")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r03.json"))
    ap.add_argument("--launcher-check", action="store_true",
                    help="only start the ranks, all-gather their ids over gloo and print them (no GPU)")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """Parent of a multi-GPU run: start one rank per GPU and return their exit
    status.  Nothing here initialises the GPU (no torch.cuda call), so no GPU
    state is inherited or replaced; rank 0's JSON line is passed through."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launcher_check(args):
    """Each rank joins a gloo group and all-gathers (rank, LOCAL_RANK); rank 0
    prints what the ranks saw.  Exercises exactly the wiring the bench uses."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    mine = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0"))], dtype=torch.int64)
    seen = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(seen, mine)
    else:
        seen = [mine]
    if world > 1 and world != args.gpus:
        raise SystemExit(f"world size {world} != --gpus {args.gpus}")
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": [s.tolist() for s in seen], "backend": "gloo"}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def synth_pcs(torch, N, d, G, seed, dev):
    """NB counts (12 populations, log-normal base means, 10% DE genes, size
    factors, theta=5) -> shifted log -> scale -> randomized PCA.  Identical on
    every rank (same seed)."""
    torch.manual_seed(seed)
    C = 12
    pop = torch.randint(0, C, (N,), device=dev)
    base = torch.exp(torch.randn(G, device=dev) * 1.5 - 1.0)
    de = (torch.rand(G, device=dev) < 0.1).float()
    lfc = torch.randn(C, G, device=dev) * de
    mu = base[None, :] * torch.pow(2.0, lfc)
    sf = torch.exp(torch.randn(N, device=dev) * 0.3)
    theta = 5.0
    x = torch.empty(N, G, device=dev)
    for a in range(0, N, 20000):  # chunked to bound temporaries
        b = min(N, a + 20000)
        mean = mu[pop[a:b]] * sf[a:b, None]
        lam = torch.distributions.Gamma(torch.full_like(mean, theta), theta / mean).sample()
        cnt = torch.poisson(lam)
        x[a:b] = torch.log1p(cnt / sf[a:b, None])
    x -= x.mean(0)
    x /= x.std(0).clamp_min(1e-8)
    U, S, _ = torch.pca_lowrank(x, q=d, center=False, niter=3)
    pcs = (U * S).double()
    del x
    return pcs, pop


def synth_labels(torch, pop, boot, L, dev, seed):
    """60 clusterings of one bootstrap: C rising with resolution (2..40),
    permuted true populations, 5% uniform flips; codes 1..C.  Labels are
    drawn per cell and gathered to the bootstrap rows: a cell's copies are
    identical points with the same neighbours, which community detection puts
    in one community."""
    g = torch.Generator(device=dev).manual_seed(seed)
    N = pop.numel()
    li = torch.arange(L, device=dev)
    ki = (li // N_RES)[:, None]
    Cl = (2 + (38 * (li % N_RES)) // (N_RES - 1))[:, None]
    lab = (pop[None, :] * 7 + ki) % Cl + 1
    flip = torch.rand(L, N, device=dev, generator=g) < 0.05
    rnd = (torch.rand(L, N, device=dev, generator=g) * Cl).long() + 1
    return torch.where(flip, rnd, lab).to(torch.int32)[:, boot.long()].contiguous()


def _cpu_boot_worker(a):
    """One bootstrap's per-bootstrap CPU work (kNN k=20, SNN k=10/15/20, 6
    silhouettes) on a single core, as one BiocParallel MulticoreParam worker
    runs getClustAssignments.  Returns its seconds."""
    X, seed = a
    sys.path.insert(0, ROOT)
    import oracle as O
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    idx, _ = O.knn(X, 20, nthreads=1)
    t1 = time.perf_counter()
    for k in K_NUM:
        O.snn(idx, k, "number")
    t2 = time.perf_counter()
    for l_ in rng.integers(1, 21, (6, X.shape[0])).astype(np.int32):  # 6 of the 60 clusterings, C ~ 20
        O.silhouette(X, l_)
    t3 = time.perf_counter()
    return t1 - t0, t2 - t1, t3 - t2


def cpu_baseline(pcs_np, B, n, N, d, sample_rows, seed=0):
    """The CPU restatement (oracle/, C) timed bootstrap-parallel on the host's
    cores, as the reference fans bootstraps over bplapply(MulticoreParam):
    `cores` single-threaded workers each run one bootstrap sample of
    `sample_rows` rows concurrently (so memory contention is included); the
    per-bootstrap seconds are extrapolated to n rows (kNN n^2, SNN and
    silhouette n, 60 clusterings) and divided over the cores.  The co-cluster
    runs OpenMP over the same cores on 2000 cells, extrapolated by N^2."""
    import multiprocessing as mp
    import oracle as O
    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    rng = np.random.default_rng(seed)
    ns = min(sample_rows, n)
    samples = [(O.gather_rows(pcs_np, rng.integers(0, N, ns).astype(np.int32)), seed + w) for w in range(cores)]
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_cpu_boot_worker, samples)
    t_knn = float(np.mean([r[0] for r in res])) * (n / ns) ** 2
    t_snn = float(np.mean([r[1] for r in res])) * (n / ns)
    t_sil = float(np.mean([r[2] for r in res])) * (60 / 6) * (n / ns)
    Nc = 2000
    A = rng.integers(1, 13, (B, Nc)).astype(np.int32)
    A[rng.random((B, Nc)) < 0.35] = -1
    t0 = time.perf_counter()
    O.cocluster(A, nthreads=cores, want=("co", "both"))
    t_coc = (time.perf_counter() - t0) * (N * (N - 1) / (Nc * (Nc - 1)))
    t_step = B * (t_knn + t_snn + t_sil) / cores + t_coc
    return {
        "value": B / t_step,
        "unit": "bootstraps/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle (C) bootstrap-parallel: {cores} single-threaded workers, one {ns}-row bootstrap each "
                   f"(kNN x (n/{ns})^2, SNN k=10/15/20 x n/{ns}, silhouette of 6 clusterings x 10 x n/{ns}), "
                   f"per-bootstrap core-seconds knn {t_knn:.1f}, snn {t_snn:.2f}, silhouette {t_sil:.2f}; "
                   f"co-cluster OpenMP x{cores} on {B} columns x {Nc} cells x (N/{Nc})^2 = {t_coc:.1f} s per step"),
    }


def visible_gpus():
    """Devices this process could use.  torch.cuda.device_count() does not
    initialise the GPU on this image, so the launcher may call it before it
    starts the ranks."""
    import torch
    return torch.cuda.device_count()


def main():
    args = parse()
    if not args.launcher_check and "WORLD_SIZE" not in os.environ:
        have = visible_gpus()
        if have < args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} requested but {have} GPU(s) are visible\n")
            sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.launcher_check:
        return launcher_check(args)
    # The result is ONE JSON line on stdout.  Native libraries print banners
    # to fd 1 (RCCL announces its version on communicator init), so fd 1 goes
    # to stderr for the run and the JSON line is written to the saved stdout.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.hw_queues > 0:  # hardware queues per process (read at HIP initialisation)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 16))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
        if world != args.gpus:
            raise SystemExit(f"world size {world} != --gpus {args.gpus}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ranks_seen = [world]
    if world > 1:  # the ranks RCCL actually connected: (rank, device) of each
        mine = torch.tensor([rank, local], dtype=torch.int64, device=dev)
        got = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(got, mine)
        ranks_seen = [g.tolist() for g in got]

    from consensusclustr_amd import Engine
    from consensusclustr_amd.sharding import DeviceGroup, exchange_group_id, row_slabs, slab_pairs

    # libccg's device group: this rank's context + an RCCL communicator over
    # all ranks (the all-gather and the slab split run inside libccg)
    if world > 1:
        grp = DeviceGroup.open_rank(local, world, rank, exchange_group_id())
    else:
        grp = DeviceGroup.open([local])
    S = max(1, args.streams)
    NK = NS = 0
    if args.pipeline:
        NK, NS = (max(1, int(v)) for v in args.pipeline.split(","))
        S = NK + NS
    engs = [grp.engines[0]] + [Engine(local) for _ in range(S - 1)]  # own workspaces per in-flight bootstrap
    eng = engs[0]
    N, d, B = args.cells, args.pcs, args.boots_per_gpu
    n = int(args.boot_size * N)
    L = len(K_NUM) * N_RES
    G = world

    # ---------------- inputs, resident in HBM before timing
    pcs, pop = synth_pcs(torch, N, d, args.genes, 20241024 + 3, dev)
    pcs_cm = pcs.t().contiguous()  # (d, N): column-major N x d like an R matrix
    bids = [rank * B + j for j in range(B)]
    boots_np = np.stack([np.random.default_rng(123 + b).integers(0, N, n) for b in bids]).astype(np.int32)
    boots = torch.from_numpy(boots_np).to(dev)
    # distinct cells per bootstrap (R: length(unique(idx))), passed to the
    # distinct-cell kNN; host input like the indices themselves
    uniq = [int(np.count_nonzero(np.bincount(b, minlength=N))) for b in boots_np]
    # per-cell k-th distances certified by earlier bootstraps of the same PCs:
    # the screen's warm start (ccg_knn_boot_hint_dev; results do not depend on
    # it), shared by the streams
    hint = torch.zeros(N, dtype=torch.float32, device=dev)
    # the cell table (ccg_knn_table_dev): every cell's KT nearest other cells,
    # recomputed inside every timed step, then filtered per bootstrap
    KT = args.table_k
    use_table = args.knn_path == "table"
    tab_idx = torch.empty((N, KT), dtype=torch.int32, device=dev)
    tab_d2 = torch.empty((N, KT), dtype=torch.float64, device=dev)

    def boot_knn(e, j, rows_j, knn_j):
        if use_table:
            e.knn_boot_table_t(pcs_cm, N, d, boots[j], uniq[j], rows_j, 20, tab_idx, tab_d2, knn_j)
        else:
            e.knn_boot_hint_t(pcs_cm, N, d, boots[j], uniq[j], rows_j, 20, knn_j, hint)

    labels = torch.empty((B, L, n), dtype=torch.int32, device=dev)
    for j in range(B):
        labels[j] = synth_labels(torch, pop, boots[j], L, dev, 1000 + bids[j])
    cmax = int(labels.max().item())

    RING = NK + NS + 1 if NK else S  # bootstrap buffers (gathered rows, kNN) in flight
    rows_s = [torch.empty((n, d), dtype=torch.float64, device=dev) for _ in range(RING)]
    knn_s = [torch.empty((n, 20), dtype=torch.int32, device=dev) for _ in range(RING)]
    rows, knn = rows_s[0], knn_s[0]
    rcap = 700 * n  # SNN row entries (items per node ~ 560 at cfg3); grown once after the warmup if short

    def alloc_snn(rcap):
        # per stream: the union-graph rows of ccg_snn_rows_dev (row offsets, lengths, partners, packed weights)
        return [(torch.zeros(n + 1, dtype=torch.int64, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),
                 torch.empty(rcap, dtype=torch.int32, device=dev), torch.empty(rcap, dtype=torch.int32, device=dev))
                for _ in range(S)]
    snn_out = alloc_snn(rcap)
    if os.environ.get("CCG_BENCH_TORCH_STREAMS"):
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    else:
        streams = [e.torch_stream() for e in engs]  # each context's own non-blocking HIP stream
    nedges = torch.zeros((B, len(K_NUM)), dtype=torch.int64, device=dev)
    means = torch.empty((B, L), dtype=torch.float64, device=dev)
    nclust = torch.empty((B, L), dtype=torch.int32, device=dev)
    minsize = torch.empty((B, L), dtype=torch.int32, device=dev)
    choice = torch.empty(B, dtype=torch.int32, device=dev)
    A_full = torch.zeros((G * B, N), dtype=torch.uint8, device=dev)  # all ranks' columns
    A_local = A_full[rank * B:(rank + 1) * B]  # this rank's block, all-gathered in place
    cuts = row_slabs(N, G)
    r0, r1 = cuts[rank], cuts[rank + 1]
    P = max(slab_pairs(N, r0, r1), 1)
    co = torch.empty(P, dtype=torch.int16, device=dev)      # uint16 counts (viewed as int16)
    both = torch.empty(P, dtype=torch.int16, device=dev)

    ev_k = [torch.cuda.Event() for _ in range(B)]
    ev_s = [torch.cuda.Event() for _ in range(B)]

    def step_pipeline():
        # stage split: kNN streams (MFMA-bound screen) run ahead of the
        # SNN + silhouette streams (issue/LDS-bound) by up to RING bootstraps,
        # so the two kinds of work always share the GPU
        cur = torch.cuda.current_stream()
        if use_table:
            eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
        for st_ in streams:
            st_.wait_stream(cur)
        for j in range(B):
            slot, ks, ss = j % RING, j % NK, NK + j % NS
            with torch.cuda.stream(streams[ks]):
                if j >= RING:
                    streams[ks].wait_event(ev_s[j - RING])  # the slot's previous bootstrap is consumed
                engs[ks].gather_rows_rm_t(pcs, N, d, boots[j], rows_s[slot])
                boot_knn(engs[ks], j, rows_s[slot], knn_s[slot])
                ev_k[j].record(streams[ks])
            with torch.cuda.stream(streams[ss]):
                streams[ss].wait_event(ev_k[j])
                engs[ss].snn_rows_t(knn_s[slot], K_NUM, "number", *snn_out[ss - NK], nedges[j])
                engs[ss].silhouette_cells_t(rows_s[slot], labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
                ev_s[j].record(streams[ss])
        for st_ in streams:
            cur.wait_stream(st_)
        eng.select_mapback_t("robust", labels, boots, N, A_local, 0, means=means, nclust=nclust,
                             minsize=minsize, out_choice=choice)
        grp.allgather_columns_t([A_local], [B] * G, [A_full])
        grp.cocluster_sharded_t([A_full], co=[co], both=[both])

    host_t = [0.0]  # host time spent enqueueing the bootstrap loop (the launches are asynchronous)

    def step():
        if NK:
            return step_pipeline()
        th = time.perf_counter()
        # S bootstraps in flight: bootstrap j runs on stream j % S with its own
        # engine context (workspaces), so one bootstrap's latency-bound SNN
        # build overlaps another's MFMA-bound kNN screen
        cur = torch.cuda.current_stream()
        if use_table:  # one table per step: every bootstrap of the step filters it
            eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
        for st_ in streams:
            st_.wait_stream(cur)
        for j in range(B):
            si = j % S
            e = engs[si]
            with torch.cuda.stream(streams[si]):
                e.gather_rows_rm_t(pcs, N, d, boots[j], rows_s[si])
                boot_knn(e, j, rows_s[si], knn_s[si])
                e.snn_rows_t(knn_s[si], K_NUM, "number", *snn_out[si], nedges[j])
                e.silhouette_cells_t(rows_s[si], labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
        host_t[0] += time.perf_counter() - th
        for st_ in streams:
            cur.wait_stream(st_)
        eng.select_mapback_t("robust", labels, boots, N, A_local, 0, means=means, nclust=nclust,
                             minsize=minsize, out_choice=choice)
        grp.allgather_columns_t([A_local], [B] * G, [A_full])
        grp.cocluster_sharded_t([A_full], co=[co], both=[both])

    def barrier():
        if G > 1:
            dist.barrier()

    # ---------------- warmup (also sizes the SNN edge buffers)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    short = int(nedges.min().item())
    if short < 0:  # rows did not fit: -short entries needed; grow once and redo the warmup
        rcap = int(-short * 1.25)
        snn_out = alloc_snn(rcap)
        step()
        torch.cuda.synchronize()
        if int(nedges.min().item()) < 0:
            raise RuntimeError(f"SNN row capacity too small: {rcap}")
    need = nedges.max(0).values.tolist()
    eng.gather_rows_rm_t(pcs, N, d, boots[0], rows)
    fb = eng.knn_boot_hint_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, knn, hint, stats=True)  # certification statistics
    fb_cold = eng.knn_boot_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, knn, stats=True)
    fb_tab_build = eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2, stats=True)
    fb_tab = eng.knn_boot_table_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, tab_idx, tab_d2, knn, stats=True)

    # ---------------- timed region (library timers off: their event records
    # cost host time on every launch group)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_t[0] = 0.0
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    host_ms = host_t[0] / args.steps * 1000
    # kernel-time breakdown: one more (untimed) step with the library's
    # hipEvent timers on
    for e in engs:
        e.timing(True)
        for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
            e.timing_read(w)
    step()
    torch.cuda.synchronize()
    kt = {}
    for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
        r = [e.timing_read(w) for e in engs]
        kt[w] = (sum(x[0] for x in r), sum(x[1] for x in r))
    for e in engs:
        e.timing(False)
    # host cost of one bootstrap's launches on an idle GPU (no queue back-pressure)
    host_idle = []
    for j in range(min(B, 6)):
        torch.cuda.synchronize()
        th = time.perf_counter()
        with torch.cuda.stream(streams[0]):
            eng.gather_rows_rm_t(pcs, N, d, boots[j], rows_s[0])
            boot_knn(eng, j, rows_s[0], knn_s[0])
            eng.snn_rows_t(knn_s[0], K_NUM, "number", *snn_out[0], nedges[j])
            eng.silhouette_cells_t(rows_s[0], labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
        host_idle.append(time.perf_counter() - th)
        torch.cuda.synchronize()
    host_idle_ms = 1000 * float(np.median(host_idle))
    # roofline of the kNN screens, measured in isolation (one launch at a
    # time, nothing else on the GPU), since in the timed region they overlap
    # other bootstraps' kernels: the per-step cell-table screen over all N
    # cells, and (for comparison) the per-bootstrap screen over the u
    # distinct cells, warm-started and cold
    eng.timing(True)
    eng.timing_read("knn_screen")
    eng.timing_read("knn_total")
    for _ in range(3):
        eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
    iso_table = eng.timing_read("knn_screen")
    iso_table_total = eng.timing_read("knn_total")
    for j in range(min(B, 8)):
        eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
        eng.knn_boot_table_t(pcs_cm, N, d, boots[j], uniq[j], rows, 20, tab_idx, tab_d2, knn)
    iso_boot_table = eng.timing_read("knn_total")
    for j in range(min(B, 8)):  # as in the screen path: warm-started by earlier bootstraps
        eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
        eng.knn_boot_hint_t(pcs_cm, N, d, boots[j], uniq[j], rows, 20, knn, hint)
    u_iso = float(np.mean(uniq[:min(B, 8)]))  # the screen searches the distinct cells
    iso_screen = eng.timing_read("knn_screen")
    iso_screen_total = eng.timing_read("knn_total")
    for j in range(min(B, 8)):  # cold: no hint (the first bootstrap of a run)
        eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
        eng.knn_boot_t(pcs_cm, N, d, boots[j], uniq[j], rows, 20, knn)
    iso_cold = eng.timing_read("knn_screen")
    # SNN and silhouette per bootstrap, in isolation (one stream, nothing else
    # on the GPU): the per-bootstrap rooflines below
    eng.timing_read("snn")
    eng.timing_read("silhouette")
    nis = min(B, 4)
    for j in range(nis):
        eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
        boot_knn(eng, j, rows, knn)
        eng.snn_rows_t(knn, K_NUM, "number", *snn_out[0], nedges[j])
        eng.silhouette_cells_t(rows, labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
    iso_snn = eng.timing_read("snn")
    iso_sil = eng.timing_read("silhouette")
    torch.cuda.synchronize()
    iso_edges = nedges[:nis].sum(0).tolist()  # per graph, over the nis bootstraps
    iso_npres = int(nclust[:nis].sum().item())  # sum over the bootstraps' labelings of present clusters
    eng.timing(False)
    if G > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()

    value = G * B * args.steps / el
    avg = lambda r: r[0] / max(r[1], 1)  # noqa: E731
    ms_screen = avg(iso_screen)
    ms_table = avg(iso_table)
    # SURVEY 8(d)'s kNN F = 2 n^2 d: for the cell-table screen over the N
    # cells, per bootstrap screen over the u distinct cells it searches
    flops_table = 2.0 * N * N * d
    flops = 2.0 * u_iso * u_iso * d
    achieved = flops / (ms_screen * 1e-3) / 1e12
    achieved_table = flops_table / (ms_table * 1e-3) / 1e12
    # the screen runs on the fp16 MFMA pipe: 3 products (hi.hi, hi.lo, lo.hi)
    # per 16-dim block, d padded to 16*ceil(d/16)
    kpad = 16 * ((d + 15) // 16)
    mfma_exec = 3 * 2.0 * u_iso * u_iso * kpad
    mfma_exec_table = 3 * 2.0 * N * N * kpad
    # co-cluster roofline: OPS = 2 * P * (sum_b C_b + B) over this rank's slab
    colC = int(A_full.max(dim=1).values.to(torch.int64).sum().item())  # sum_b C_b over all ranks' columns
    coc_ops = 2.0 * P * (colC + G * B)
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            traffic = json.load(f).get("knn_screen_bytes_per_launch")
    per_step = {w: round(v[0], 3) for w, v in kt.items()}  # the one timer step
    roof_screen = {
        "kernel": "knn_screen16_kernel<2,20,28> per bootstrap (fp16 hi/lo split, v_mfma_f32_32x32x16_f16)",
        "bound": "mfma",
        "achieved": round(achieved, 2),
        "peak": PEAK_F16_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_F16_TFLOPS, 4),
        "traffic": traffic,
        "algorithmic_per_launch": f"2*u^2*d = {flops:.3e} flop (u={u_iso:.0f} distinct cells of the n={n} "
                                  f"bootstrap rows, d={d}), SURVEY 8(d) over the rows the screen searches",
        "avg_launch_ms": round(ms_screen, 4),
        "avg_launch_ms_cold": round(avg(iso_cold), 4),
        "cold_note": "the same launches without the warm start (no certified distances from earlier bootstraps)",
        "knn_total_ms_per_boot": round(avg(iso_screen_total), 4),
        "avg_launch_ms_note": f"{iso_screen[1]} launches timed in isolation after the timed region",
        "mfma_flops_executed_per_launch": mfma_exec,
        "mfma_pipe_frac": round(mfma_exec / (ms_screen * 1e-3) / 1e12 / PEAK_F16_TFLOPS, 4),
    }
    roof_table = {
        "kernel": "knn_screen16_kernel<2,32,56> cell table over all N cells, once per step "
                  "(fp16 hi/lo split, v_mfma_f32_32x32x16_f16)",
        "bound": "mfma",
        "achieved": round(achieved_table, 2),
        "peak": PEAK_F16_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved_table / PEAK_F16_TFLOPS, 4),
        "traffic": None,
        "algorithmic_per_launch": f"2*N^2*d = {flops_table:.3e} flop (N={N} cells, d={d}, K={KT} neighbours "
                                  "each), SURVEY 8(d)'s 2 n^2 d over the cells the table searches",
        "avg_launch_ms": round(ms_table, 4),
        "table_total_ms": round(avg(iso_table_total), 4),
        "table_fallback_cells": int(fb_tab_build[1]),
        "knn_total_ms_per_boot_from_table": round(avg(iso_boot_table), 4),
        "boot_fallback_last_boot": int(fb_tab[1]),
        "avg_launch_ms_note": f"{iso_table[1]} launches timed in isolation after the timed region; one per step "
                              f"serves the step's {B} bootstraps",
        "mfma_flops_executed_per_launch": mfma_exec_table,
        "mfma_pipe_frac": round(mfma_exec_table / (ms_table * 1e-3) / 1e12 / PEAK_F16_TFLOPS, 4),
    }
    coc_ms = kt["cocluster"][0] / max(kt["cocluster"][1], 1)
    coc_traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            coc_traffic = json.load(f).get("cocluster_bytes_per_launch_B125")
    roof_coc = {
        "kernel": "cof_tile_kernel (one-hot int8 co/both GEMM, v_mfma_i32_32x32x32_i8), this rank's row slab",
        "bound": "mfma",
        "achieved": round(coc_ops / (coc_ms * 1e-3) / 1e12, 2),
        "peak": PEAK_I8_TOPS,
        "unit": "TOP/s",
        "frac": round(coc_ops / (coc_ms * 1e-3) / 1e12 / PEAK_I8_TOPS, 4),
        "traffic": coc_traffic,
        "algorithmic_per_launch": f"2*P*(sum C_b + B) = {coc_ops:.3e} int8 ops (P={P} pairs in this slab, "
                                  f"sum C_b={colC}, B={G * B}), SURVEY 8(d); one launch per step",
        "avg_launch_ms": round(coc_ms, 4),
        "avg_launch_ms_note": "library hipEvent timer on the launch stream, the timer step after the timed region",
        "output_bytes_per_launch": 4 * P,
    }
    # SNN rows (bytes = sum_K (n K 4 + E_K 16) per bootstrap) and
    # silhouette (fp64 MFMA widths: 2 d u sum_l C_l over the distinct cells),
    # per bootstrap in isolation
    snn_ms = iso_snn[0] / max(iso_snn[1], 1)
    sil_ms = iso_sil[0] / max(iso_sil[1], 1)
    snn_bytes = sum(n * k * 4 for k in K_NUM) + 16 * sum(iso_edges) / max(nis, 1)
    sil_flop = 2.0 * d * u_iso * iso_npres / max(nis, 1)
    roof_snn = {
        "kernel": "SNN union-graph rows (ccg_snn_rows_dev: host lists, bitonic build tiers, copy rows)",
        "bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
        "achieved": round(snn_bytes / (snn_ms * 1e-3) / 1e9, 1),
        "frac": round(snn_bytes / (snn_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "traffic": None,
        "algorithmic_per_launch": f"sum_K (n K 4 + E_K 16) = {snn_bytes:.3e} B per bootstrap (E_K the edges of "
                                  f"graph K), SURVEY 8(d)",
        "ms_per_boot": round(snn_ms, 4),
    }
    roof_sil = {
        "kernel": "silhouette of the 60 clusterings (ccg_silhouette_cells_dev; widths on v_mfma_f64_16x16x4f64)",
        "bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_F64_TFLOPS,
        "achieved": round(sil_flop / (sil_ms * 1e-3) / 1e12, 2),
        "frac": round(sil_flop / (sil_ms * 1e-3) / 1e12 / PEAK_F64_TFLOPS, 4),
        "traffic": None,
        "algorithmic_per_launch": f"2 d u sum_l C_l = {sil_flop:.3e} flop per bootstrap (x.mu of the u distinct "
                                  f"cells against every present centroid of the 60 labelings)",
        "ms_per_boot": round(sil_ms, 4),
    }
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "bootstraps/s",
        "n_gpus": G,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1000, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "dtype_detail": ("kNN order exact in f64 (cell table over all cells once per step: fp16 hi/lo x3 MFMA "
                         "screen, f32 accumulate, f64 certify; per bootstrap the table's present entries, exact "
                         "f64 search for cells short of kq, exact f64 expansion to rows); " if use_table else
                         "kNN order exact in f64 (distinct cells: fp16 hi/lo x3 MFMA screen, f32 accumulate, "
                         "f64 certify, exact f64 expansion to rows; screen warm-started by earlier bootstraps' "
                         "certified distances); ") +
                        "silhouette f64 with fixed-point sums; co-cluster int8 MFMA, int32 counts",
        "data": "synthetic: NB counts (12 populations, 2000 genes) -> PCA; synthetic clusterings in place of host Leiden",
        "config": {
            "workload": "BASELINE cfg3 shapes: 100k cells x 30 PCs, robust mode, kNum 10/15/20 x 20 resolutions; "
                        f"{B} bootstraps per GPU per step ({G * B} total) + co-cluster row slab over all columns",
            "cells": N, "pcs": d, "bootstrap_rows": n, "distinct_cells_mean": round(float(np.mean(uniq)), 1),
            "boots_per_gpu": B, "clusterings_per_boot": L,
            "parallelism": f"bootstraps x{G}, co-cluster row slabs x{G}", "streams_per_gpu": S,
            "knn_path": args.knn_path,
        },
        "roofline": roof_coc,
        "roofline_note": "the co-cluster GEMM is the largest single launch of a step; the per-bootstrap "
                         "stages follow (kNN table screen once per step, SNN, silhouette)",
        "roofline_knn_table" if use_table else "roofline_knn_screen": (roof_table if use_table else roof_screen),
        "roofline_knn_screen_path" if use_table else "roofline_knn_table_path": (roof_screen if use_table else roof_table),
        "roofline_snn": roof_snn,
        "roofline_silhouette": roof_sil,
        "kernel_ms_per_step": per_step,
        "kernel_ms_per_step_note": "library hipEvent timers over one extra step after the timed region "
                                   "(bootstraps overlap, so kernel times sum to more than the step)",
        "host_enqueue_ms_per_step": round(host_ms, 3),
        "host_launch_ms_per_boot_idle_gpu": round(host_idle_ms, 3),
        "cocluster_avg_ms": round(coc_ms, 3),
        "knn_fallback_rows_last_boot": int(fb[1]),
        "knn_fallback_rows_last_boot_cold": int(fb_cold[1]),
        "snn_edges_max_per_boot": [int(e) for e in need],
    }
    if rank == 0 and G == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pcs.cpu().numpy(), B, n, N, d, args.cpu_sample_rows)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    for e in engs[1:]:
        e.close()
    grp.close()
    if G > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
