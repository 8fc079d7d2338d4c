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

Workloads (--workload; the default cfg3 line is the metric line):
  cfg3    : the metric -- 100k cells x 30 PCs, 125 bootstraps per GPU per step,
            robust, the co-cluster row slab of this rank over all ranks' columns;
  cfg3job : cfg3 as one whole 1-GPU job: 1000 bootstraps per step and one
            co-cluster over the 1000 columns;
  cfg2    : 20k cells x 20 PCs, 500 bootstraps, robust, one whole 1-GPU job;
  cfg4    : 250k cells x 30 PCs, granular (60 map-back columns per bootstrap,
            no silhouettes, :688): one GPU's share of the 8-GPU job -- 125
            bootstraps and rank 0's pair-balanced slab of the 60 000-column
            co-cluster (the other ranks' columns are synthetic copies);
  cfg5    : iterate=TRUE on 100k cells: every subcluster (5k-20k cells, d_c
            5-15 PCs) of one level through the batched segment kNN
            (ccg_knn_boot_segments_dev), one SNN pass over the disjoint union,
            one segmented silhouette launch set (ccg_silhouette_segments_dev),
            map-back and per-subcluster co-clusters.

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
# BASELINE.json configs: shapes per workload (weak scaling: bootstraps per GPU)
WORKLOADS = {
    "cfg3": dict(cells=100000, pcs=30, boots_per_gpu=125, mode="robust", emul_ranks=0, cmax=40, boot_batch=8,
                 batch_streams=3),
    "cfg3job": dict(cells=100000, pcs=30, boots_per_gpu=1000, mode="robust", emul_ranks=0, cmax=40, boot_batch=8,
                    batch_streams=3),
    "cfg2": dict(cells=20000, pcs=20, boots_per_gpu=500, mode="robust", emul_ranks=0, cmax=40, boot_batch=32,
                 batch_streams=3),
    "cfg4": dict(cells=250000, pcs=30, boots_per_gpu=125, mode="granular", emul_ranks=8, cmax=60, boot_batch=8,
                 batch_streams=3),
    "cfg5": dict(cells=100000, pcs=30, boots_per_gpu=125, mode="robust", emul_ranks=0, cmax=40),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg3")
    ap.add_argument("--cells", type=int, default=None)
    ap.add_argument("--pcs", type=int, default=None)
    ap.add_argument("--genes", type=int, default=2000)
    ap.add_argument("--boots-per-gpu", type=int, default=None)
    ap.add_argument("--check", action="store_true",
                    help="with the CPU baseline leg: also check one bootstrap's outputs against the oracle "
                         "(on by default with the CPU baseline)")
    ap.add_argument("--boot-size", type=float, default=0.9)
    ap.add_argument("--cpu-sample-rows", type=int, default=6000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=0,
                    help="bootstraps in flight per GPU (one engine context + HIP stream each); 0 = auto: 4 (one per "
                         "hardware queue, GPU_MAX_HW_QUEUES=4) for bootstraps of >= 50k rows, 3 below, 2 for cfg5. "
                         "Round 5: cfg3 2/3/4/5/6/8 -> 987/1156/1200/1085/1142/1210 bootstraps/s; cfg2 (18k-row "
                         "bootstraps, host-bound) 2/3/4 -> 3828/4385/3774; cfg5 2/3/4 -> 1062/1025/967")
    ap.add_argument("--seg-batch", type=int, default=16,
                    help="cfg5: bootstraps of every subcluster per segmented launch set")
    ap.add_argument("--boot-batch", type=int, default=0,
                    help="table path: bootstraps per launch set (ccg_knn_boots_table_dev, one SNN class pass over "
                         "the batch's disjoint union, one ccg_silhouette_segments_dev); 1 = one bootstrap per launch "
                         "set (the round-5 step); 0 = auto")
    ap.add_argument("--knn-path", choices=["table", "screen"], default="table",
                    help="table: one cell table per step (ccg_knn_table_dev) filtered per bootstrap; "
                         "screen: a screen per bootstrap (warm-started)")
    ap.add_argument("--split-sil", type=int, default=0,
                    help="launch sets: the silhouettes of set t on a stream (and context) of their own, after the "
                         "set's gather and beside its kNN + SNN (they depend on the rows only), so the MFMA/VALU-bound "
                         "widths overlap the latency-bound SNN (round 6, cfg3: boot phase 87.4 ms against 87.8 -- the GPU "
                         "is already full); 0 = one stream per set (default)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="HIP hardware queues for this process (0: the runtime's default)")
    ap.add_argument("--launch", choices=["auto", "graph", "eager"], default="auto",
                    help="graph: the step's bootstrap phase (table, every bootstrap's gather, kNN, SNN, silhouette "
                         "on the S streams) is captured once after the warmup as one HIP graph and replayed per step; "
                         "eager: launched from the host every step; auto: graph when a bootstrap has >= 50k rows "
                         "(round 5, 4 streams: cfg3 graph 1187 / eager 1041 bootstraps/s; cfg2, 18k-row "
                         "bootstraps x 500 per step, graph 2799 / eager 3658 -- the replay of ~20k graph nodes "
                         "costs more host time than launching them)")
    ap.add_argument("--table-k", type=int, default=48,
                    help="cell-table length K (<= 48): cells with fewer than 20 of their K nearest cells in a "
                         "bootstrap take the exact search")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"))
    ap.add_argument("--launcher-check", action="store_true",
                    help="only start the ranks, all-gather their ids over gloo and print them (no GPU)")
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for k in ("cells", "pcs", "boots_per_gpu"):
        if getattr(a, k) is None:
            setattr(a, k, w[k])
    return a


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
    # the per-rank phase report of a real run, over the same gather (gloo, CPU
    # tensors): a host-timed stand-in step per rank
    t0 = time.perf_counter()
    float(np.linalg.norm(np.random.default_rng(rank).random((256, 256)) @ np.eye(256)))
    step_ms = 1000 * (time.perf_counter() - t0)
    rep = per_rank_report(torch, dist, world, {"step_ms": step_ms, "boot_phase_ms": step_ms})
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": [s.tolist() for s in seen], "backend": "gloo",
                          "per_rank": rep}), flush=True)
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


def synth_labels(torch, pop, boot, L, dev, seed, chi=40):
    """60 clusterings of one bootstrap: C rising with resolution (2..chi),
    permuted true populations, 5% uniform flips; codes 1..C.  Labels are
    drawn per cell and gathered to the bootstrap rows: a cell's copies are
    identical points with the same neighbours, which community detection puts
    in one community."""
    g = torch.Generator(device=dev).manual_seed(seed)
    N = pop.numel()
    li = torch.arange(L, device=dev)
    ki = (li // N_RES)[:, None]
    Cl = (2 + ((chi - 2) * (li % N_RES)) // (N_RES - 1))[:, None]
    lab = (pop[None, :] * 7 + ki) % Cl + 1
    flip = torch.rand(L, N, device=dev, generator=g) < 0.05
    rnd = (torch.rand(L, N, device=dev, generator=g) * Cl).long() + 1
    return torch.where(flip, rnd, lab).to(torch.int32)[:, boot.long()].contiguous()


def _cpu_boot_worker(a):
    """One bootstrap's per-bootstrap CPU work (kNN k=20, SNN k=10/15/20, and
    in robust mode 6 silhouettes) on a single core, as one BiocParallel
    MulticoreParam worker runs getClustAssignments.  Returns its seconds."""
    X, seed, n_sil = a
    sys.path.insert(0, ROOT)
    import oracle as O
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    idx, _ = O.knn(X, 20, nthreads=1)
    t1 = time.perf_counter()
    for k in K_NUM:
        O.snn(idx, k, "number")
    t2 = time.perf_counter()
    for l_ in rng.integers(1, 21, (n_sil, X.shape[0])).astype(np.int32):  # n_sil of the 60 clusterings, C ~ 20
        O.silhouette(X, l_)
    t3 = time.perf_counter()
    return t1 - t0, t2 - t1, t3 - t2


def cpu_baseline(pcs_np, B, n, N, d, sample_rows, seed=0, robust=True, coc_cols=None, coc_pairs=None,
                 seg_rows=None):
    """The CPU restatement (oracle/, C) timed bootstrap-parallel on the host's
    cores, as the reference fans bootstraps over bplapply(MulticoreParam):
    `cores` single-threaded workers each run one bootstrap sample of
    `sample_rows` rows concurrently (so memory contention is included); the
    per-bootstrap seconds are extrapolated to n rows (kNN n^2, SNN and
    silhouette n, 60 clusterings; granular mode scores none) and divided over
    the cores.  The co-cluster runs OpenMP over the same cores on 2000 cells
    x min(B, 1000) columns, extrapolated by pairs and columns.  seg_rows
    (cfg5): the per-bootstrap work is the sum over subclusters of n_s rows."""
    import multiprocessing as mp
    import oracle as O
    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    rng = np.random.default_rng(seed)
    ns = min(sample_rows, n)
    n_sil = 6 if robust else 0
    samples = [(O.gather_rows(pcs_np, rng.integers(0, N, ns).astype(np.int32)), seed + w, n_sil)
               for w in range(cores)]
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_cpu_boot_worker, samples)
    segs = [n] if seg_rows is None else list(seg_rows)
    k1 = float(np.mean([r[0] for r in res]))
    k2 = float(np.mean([r[1] for r in res]))
    k3 = float(np.mean([r[2] for r in res]))
    t_knn = sum(k1 * (m / ns) ** 2 for m in segs)
    t_snn = sum(k2 * (m / ns) for m in segs)
    t_sil = sum(k3 * (60 / 6) * (m / ns) for m in segs) if robust else 0.0
    Nc = 2000
    Bc = B if coc_cols is None else coc_cols
    Bs = min(Bc, 1000)
    P = N * (N - 1) / 2 if coc_pairs is None else coc_pairs
    A = rng.integers(1, 13, (Bs, Nc)).astype(np.int32)
    A[rng.random((Bs, Nc)) < 0.35] = -1
    t0 = time.perf_counter()
    O.cocluster(A, nthreads=cores, want=("co", "both"))
    t_coc = (time.perf_counter() - t0) * (P / (Nc * (Nc - 1) / 2)) * (Bc / Bs)
    t_step = B * (t_knn + t_snn + t_sil) / cores + t_coc
    return {
        "value": B / t_step,
        "unit": "bootstraps/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle (C) bootstrap-parallel: {cores} single-threaded workers, one {ns}-row bootstrap each "
                   f"(kNN x (n/{ns})^2, SNN k=10/15/20 x n/{ns}" +
                   (f", silhouette of 6 clusterings x 10 x n/{ns}" if robust else ", no silhouettes (granular)") +
                   (f"; summed over {len(segs)} subclusters of {min(segs)}-{max(segs)} rows" if seg_rows else "") +
                   f"), per-bootstrap core-seconds knn {t_knn:.1f}, snn {t_snn:.2f}, silhouette {t_sil:.2f}; "
                   f"co-cluster OpenMP x{cores} on {Bs} columns x {Nc} cells, x (pairs {P:.3g} / sample pairs) x "
                   f"(columns {Bc} / {Bs}) = {t_coc:.1f} s per step"),
    }


def cpu_baseline_check(eng, torch, pcs, pcs_cm, boot, u, labels0, tab, cmax, robust, A_full=None, co=None,
                       both=None, r0=0, r1=0, sample=256, batch=None):
    """Part of the cpu_baseline leg: the oracle as the CHECKER of one timed
    bootstrap.  Bootstrap 0 runs again through the step's calls (gather, kNN
    from the cell table, SNN rows, silhouette) into fresh buffers; sampled kNN
    rows (plus every row the fast paths sent to the exact search) must be
    bit-exact, all three SNN graphs must equal the oracle's edge lists, the
    60 silhouette means must agree within 1e-5, and sampled rows of the
    step's co/both slab must equal orc_cocluster_rows.  batch (the batched
    step): the step's first launch set runs again -- ccg_knn_boots_table_dev,
    one class-level SNN pass over the batch, one ccg_silhouette_segments_dev
    -- and its first bootstrap is checked as above, plus sampled kNN rows of
    its last bootstrap."""
    import concurrent.futures as cf
    import oracle as O
    N, d = pcs.shape
    n = boot.numel()
    dev = pcs.device
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    out = {}
    L = labels0.shape[0]
    rng = np.random.default_rng(5)
    if batch is not None:
        nbb = batch["idx"].shape[0]
        m = nbb * n
        rows = torch.empty((m, d), dtype=torch.float64, device=dev)
        knn = torch.empty((m, 20), dtype=torch.int32, device=dev)
        eng.gather_rows_rm_t(pcs, N, d, batch["idx"].reshape(-1), rows)
        eng.knn_boots_table_t(N, d, batch["idx"], batch["uniq"], rows, 20, tab[0], tab[1], knn)
        cut_all = eng.knn_last_fallback()
        sb = SnnBufs(torch, m, 400 * m, dev)
        info = torch.zeros(3 + len(K_NUM), dtype=torch.int64, device=dev)
        sb.run(eng, knn, batch["keys"], info, n=m)
        ms = [torch.empty(L, dtype=torch.float64, device=dev) for _ in range(nbb)]
        if robust:
            eng.silhouette_segments_t(rows, np.arange(nbb + 1, dtype=np.int64) * n, batch["labels"], cmax,
                                      batch["keys"], nbb * N, ms)
        torch.cuda.synchronize()
        mean = ms[0]
        # the batch's last bootstrap: sampled kNN rows and its cut-tie rows (ids of the concatenation)
        a = (nbb - 1) * n
        XL = rows[a:].cpu().numpy()
        cl = cut_all[cut_all >= a] - a
        ql = np.unique(np.concatenate([cl[:2048], rng.choice(n, min(sample, n), replace=False)])).astype(np.int32)
        oi, _ = O.knn_queries(XL, 20, ql, nthreads=threads)
        out["batch_bootstraps"] = int(nbb)
        out["knn_last_boot_rows_checked"] = int(ql.size)
        out["knn_last_boot_exact"] = bool(np.array_equal(knn[a:].cpu().numpy()[ql] - a, oi))
        cut = cut_all[cut_all < n]
        rows, knn = rows[:n], knn[:n]
    else:
        rows = torch.empty((n, d), dtype=torch.float64, device=dev)
        knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
        eng.gather_rows_rm_t(pcs, N, d, boot, rows)
        if tab is not None:
            eng.knn_boot_table_t(pcs_cm, N, d, boot, u, rows, 20, tab[0], tab[1], knn)
        else:
            eng.knn_boot_t(pcs_cm, N, d, boot, u, rows, 20, knn)
        cut = eng.knn_last_fallback()
        sb = SnnBufs(torch, n, 400 * n, dev)
        info = torch.zeros(3 + len(K_NUM), dtype=torch.int64, device=dev)
        sb.run(eng, knn, boot, info)
        mean = torch.empty(L, dtype=torch.float64, device=dev)
        ncl = torch.empty(L, dtype=torch.int32, device=dev)
        mns = torch.empty(L, dtype=torch.int32, device=dev)
        if robust:
            eng.silhouette_cells_t(rows, labels0, cmax, boot, N, mean, ncl, mns)
        torch.cuda.synchronize()
    X = rows.cpu().numpy()
    kn = knn.cpu().numpy()
    q = np.unique(np.concatenate([cut[:4096], rng.choice(n, min(sample, n), replace=False)])).astype(np.int32)
    oi, _ = O.knn_queries(X, 20, q, nthreads=threads)
    out["knn_rows_checked"] = int(q.size)
    out["knn_exact"] = bool(np.array_equal(kn[q], oi))
    inf = info.cpu().numpy()
    ok = int(inf[1]) == 0 and int(inf[3:].min()) >= 0
    out["snn_classes"] = int(inf[0])
    if ok:
        got = sb.decode(sb.n if batch is not None else n, int(inf[0]), 0, n)
        for g, k in enumerate(K_NUM):
            ei, ej, ew = O.snn(kn, k, "number")
            ok = ok and np.array_equal(got[g][0], ei) and np.array_equal(got[g][1], ej) and \
                np.array_equal(got[g][2], ew)
    out["snn_graphs_exact"] = bool(ok)
    if robust:
        labs = labels0.cpu().numpy()
        with cf.ThreadPoolExecutor(threads) as ex:
            ref = list(ex.map(lambda l_: O.silhouette(X, labs[l_])[1], range(L)))
        got = mean.cpu().numpy()
        rel = np.abs(got - np.asarray(ref)) / np.maximum(np.abs(np.asarray(ref)), 1e-300)
        out["silhouette_max_rel_err"] = float(rel.max())
        out["silhouette_within_1e-5"] = bool(rel.max() <= 1e-5)
    if A_full is not None and A_full.numel() <= (1 << 31):
        An = A_full.cpu().numpy()
        rsel = np.unique(np.clip(np.array([r0, r0 + 1, (r0 + r1) // 2, r1 - 2]), r0, r1 - 2)).astype(np.int32)
        rco, rb = O.cocluster_rows(An, rsel, nthreads=threads)
        good = True
        for t, i_ in enumerate(rsel):
            o = int(i_) * N - int(i_) * (int(i_) + 1) // 2 - (r0 * N - r0 * (r0 + 1) // 2)
            m_ = N - 1 - int(i_)
            good = good and np.array_equal(co[o:o + m_].cpu().numpy().view(np.uint16), rco[t, i_ + 1:]) and \
                np.array_equal(both[o:o + m_].cpu().numpy().view(np.uint16), rb[t, i_ + 1:])
        out["cocluster_rows_checked"] = int(rsel.size)
        out["cocluster_exact"] = bool(good)
    out["ok"] = all(v for k_, v in out.items() if isinstance(v, bool))
    return out


def workload_text(name, N, d, B, G, emul):
    if name == "cfg3":
        return ("BASELINE cfg3 shapes: 100k cells x 30 PCs, robust mode, kNum 10/15/20 x 20 resolutions; "
                f"{B} bootstraps per GPU per step ({G * B} total) + co-cluster row slab over all columns "
                "(at 1 GPU: one rank's share of the 8-GPU job; the whole 1000-bootstrap job on one GPU is "
                "--workload cfg3job)")
    if name == "cfg3job":
        return (f"BASELINE cfg3 as one whole job: {N} cells x {d} PCs, robust, {B * G} bootstraps per step, "
                "one co-cluster over all their columns")
    if name == "cfg2":
        return f"BASELINE cfg2: {N} cells x {d} PCs, robust, {B * G} bootstraps, whole job incl. co-cluster"
    if name == "cfg4":
        return (f"BASELINE cfg4 granular, one GPU's share of the {emul or G}-GPU job: {N} cells x {d} PCs, {B} "
                f"bootstraps (60 map-back columns each, C 2..60, no silhouettes, :688) + this rank's pair-balanced "
                f"row slab of the {(emul or G) * B * 60}-column co-cluster"
                + (" (the other ranks' columns synthetic)" if emul else ""))
    return name


CFG5_SIZES = [5000, 6000, 7000, 8000, 9000, 10000, 11000, 12000, 12000, 20000]


def cfg5_inputs(torch, N, d, genes, B, rank, dev):
    """BASELINE cfg5's level: N cells in 10 subclusters of 5k-20k cells with
    pcNum d_c = 5..15 (the :356 rule's range), their PC matrices stacked
    row-major and zero-padded to the largest d_c, and B bootstraps of every
    subcluster (default_rng(123 + b): the same stream seed for every
    subcluster, as the forwarded BPPARAM gives, :562-566)."""
    pcs, pop = synth_pcs(torch, N, d, genes, 20241024 + 5, dev)
    sizes = list(CFG5_SIZES)
    sizes[-1] += N - sum(sizes)
    nsub = len(sizes)
    dcs = [5 + (10 * c) // (nsub - 1) for c in range(nsub)]
    dpad = max(dcs)
    perm = torch.from_numpy(np.random.default_rng(55).permutation(N)).to(dev)
    Nof = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    cells = torch.zeros((N, dpad), dtype=torch.float64, device=dev)  # the subclusters' PCs stacked, zero-padded
    for c in range(nsub):
        cells[Nof[c]:Nof[c + 1], :dcs[c]] = pcs[perm[Nof[c]:Nof[c + 1]], :dcs[c]]
    ns = [int(0.9 * m) for m in sizes]
    bids = [rank * B + j for j in range(B)]
    boots = [[np.random.default_rng(123 + b).integers(0, sizes[c], ns[c]).astype(np.int32) for b in bids]
             for c in range(nsub)]
    uniq = [[int(np.count_nonzero(np.bincount(x, minlength=sizes[c]))) for x in boots[c]] for c in range(nsub)]
    boots_t = [torch.from_numpy(np.stack(boots[c])).to(dev) for c in range(nsub)]  # (B, n_c) local cells
    return dict(pcs=pcs, pop=pop, popc=pop[perm], sizes=sizes, nsub=nsub, dcs=dcs, dpad=dpad, Nof=Nof, cells=cells,
                ns=ns, bids=bids, boots=boots, uniq=uniq, boots_t=boots_t)


def cfg5_seg_plan(torch, inp, b0, b1):
    """Segments (subcluster c, bootstrap j) of bootstraps [b0, b1) of every
    subcluster: their row offsets, distinct-cell counts and the rows' global
    cell ids (block start + local cell)."""
    segs = [(c, j) for j in range(b0, b1) for c in range(inp["nsub"])]
    off = np.concatenate([[0], np.cumsum([inp["ns"][c] for c, _ in segs])]).astype(np.int64)
    su = np.array([inp["uniq"][c][j] for c, j in segs], np.int32)
    idx = torch.cat([inp["boots_t"][c][j] + int(inp["Nof"][c]) for c, j in segs])
    return segs, off, su, idx


def cfg5_sil_keys(torch, inp, plan, b0):
    """Cell keys of a batch's rows for ccg_silhouette_segments_dev: distinct
    between segments -- global cell id + (bootstrap slot) x N (segments of one
    subcluster's bootstraps share global ids); ncell = slots x N."""
    segs, off, _, idx = plan
    slot = torch.from_numpy(np.repeat(np.array([j - b0 for _, j in segs], np.int32), np.diff(off))).to(idx.device)
    return (idx + slot * int(inp["cells"].shape[0])).to(torch.int32)


def decode_union_rows(off, ln, nbr, wpk, nk, r0=0, r1=None):
    """Union-graph rows (ccg_snn_rows_dev) of rows [r0, r1) -> per-graph
    (i, j, w) NUMBER edge lists in (i, j) order (numpy, vectorised)."""
    r1 = ln.size if r1 is None else r1
    lens = ln[r0:r1].astype(np.int64)
    i = np.repeat(np.arange(r0, r1, dtype=np.int64), lens)
    start = np.repeat(off[r0:r1], lens)
    pos = start + (np.arange(i.size, dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens))
    j = nbr[pos]
    w = wpk.view(np.uint32)[pos]
    out = []
    for g in range(nk):
        b = (w >> np.uint32(8 * g)) & np.uint32(0xFF)
        m = b != 0
        out.append((i[m], j[m].astype(np.int64), b[m].astype(np.float64)))
    return out


def decode_class_rows(row_class, u, off, ln, nbr, wpk, ks, c0=0):
    """Class-level rows (ccg_snn_classes_dev) -> per-graph row-level
    (i, j, w) NUMBER edge lists sorted by (i, j) (numpy): rows x of class C
    and y of class H get w(C, H); two rows of one class get k + 1.  c0: the
    first class of a slice (row_class, off, ln relative to it; partners are
    global ordinals)."""
    row_class = np.asarray(row_class, np.int64)
    n = row_class.size
    m = np.bincount(row_class, minlength=u).astype(np.int64)
    order = np.argsort(row_class, kind="stable")  # rows of each class, ascending
    ms = np.concatenate([[0], np.cumsum(m)])
    lens = ln[:u].astype(np.int64)
    C = np.repeat(np.arange(u, dtype=np.int64), lens)
    pos = np.repeat(off[:u], lens) + (np.arange(C.size, dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens))
    H = nbr[pos].astype(np.int64) - c0
    W = wpk.view(np.uint32)[pos]
    out = []
    # pairs inside a class
    mi = m[m > 1]
    ci = np.flatnonzero(m > 1)
    for g, k in enumerate(ks):
        b = (W >> np.uint32(8 * g)) & np.uint32(0xFF)
        sel = b != 0
        Cg, Hg, wg = C[sel], H[sel], b[sel].astype(np.float64)
        cnt = m[Cg] * m[Hg]
        e = np.repeat(np.arange(Cg.size), cnt)
        kk = np.arange(e.size, dtype=np.int64) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        mh = m[Hg][e]
        x = order[ms[Cg[e]] + kk // mh]
        y = order[ms[Hg[e]] + kk % mh]
        wv = wg[e]
        # intra-class pairs x < y, weight k + 1
        pc = mi * (mi - 1) // 2
        ei = np.repeat(np.arange(ci.size), pc)
        t = np.arange(ei.size, dtype=np.int64) - np.repeat(np.cumsum(pc) - pc, pc)
        # t -> (a, b) with a < b inside the class (m <= 15: small tables)
        a_ = np.zeros(ei.size, np.int64)
        b_ = np.zeros(ei.size, np.int64)
        for mm in np.unique(mi):
            pa, pb = np.triu_indices(int(mm), 1)
            s_ = mi[ei] == mm
            a_[s_], b_[s_] = pa[t[s_]], pb[t[s_]]
        xi = order[ms[ci[ei]] + a_]
        yi = order[ms[ci[ei]] + b_]
        I = np.concatenate([np.minimum(x, y), np.minimum(xi, yi)])
        J = np.concatenate([np.maximum(x, y), np.maximum(xi, yi)])
        Wt = np.concatenate([wv, np.full(xi.size, float(k + 1))])
        o = np.lexsort((J, I))
        out.append((I[o], J[o], Wt[o]))
    return out


class SnnBufs:
    """Output buffers of one in-flight SNN pass at the level of row classes
    (ccg_snn_classes_dev: the kernels both drop-ins run through
    ccg_snn_graphs_cells): row -> class, class roots, the class rows
    (capacity-based offsets, lengths, partner classes, packed per-graph
    weights)."""

    def __init__(self, torch, n, cap, dev):
        self.n, self.cap = n, cap
        self.row_class = torch.zeros(n, dtype=torch.int32, device=dev)
        self.class_root = torch.zeros(n, dtype=torch.int32, device=dev)
        self.off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        self.ln = torch.zeros(n, dtype=torch.int32, device=dev)
        self.nbr = torch.empty(cap, dtype=torch.int32, device=dev)
        self.wpk = torch.empty(cap, dtype=torch.int32, device=dev)

    def run(self, e, knn, cell, info, n=None):
        """info: (3 + len(K_NUM),) int64 tensor row -- [u, status, required
        capacity, class edges per graph (negative: capacity too small)]."""
        n = self.n if n is None else n
        e.snn_classes_t(knn, K_NUM, self.row_class[:n], self.class_root[:n], self.off[:n + 1], self.ln[:n], self.nbr,
                        self.wpk, info, cell=cell)

    def decode(self, n, u, r0=0, r1=None):
        """Row-level graphs of rows [r0, r1) (a segment: its classes are a
        contiguous ordinal range, rows and partners relative to r0)."""
        r1 = n if r1 is None else r1
        used = int(self.off[n].item())
        rc = self.row_class[r0:r1].cpu().numpy().astype(np.int64)
        c0, c1 = (int(rc[0]), int(rc.max()) + 1) if r0 > 0 or r1 < n else (0, u)
        return decode_class_rows(rc - c0, c1 - c0, self.off[c0:c1 + 1].cpu().numpy(), self.ln[c0:c1].cpu().numpy(),
                                 self.nbr[:used].cpu().numpy(), self.wpk[:used].cpu().numpy(), K_NUM, c0=c0)


def cfg5_check(eng, torch, inp, labels, cmax, plan, sample=512, b0=0):
    """cfg5's cpu_baseline check leg: the oracle as the checker of the first
    segmented launch set.  The batch runs again through the step's calls
    (ccg_knn_boot_segments_dev with global ids, ONE row-class SNN pass over
    the disjoint union, ONE ccg_silhouette_segments_dev); for three
    segments (the smallest and the largest subcluster's first bootstrap and
    the batch's last segment) sampled kNN rows plus every exact-search row
    must equal orc_knn_queries on the segment's rows (segment-local ids), the
    segment's three SNN graphs must equal orc_snn of its neighbour rows, and
    its 60 silhouette means must agree with orc_silhouette within 1e-5."""
    import concurrent.futures as cf
    import oracle as O
    segs, off, su, idx = plan
    dev = idx.device
    n = int(off[-1])
    dpad = inp["dpad"]
    knn = torch.empty((n, 20), dtype=torch.int32, device=dev)
    eng.knn_boot_segments_t(inp["cells"], idx, off, su, 20, knn, local_ids=False)
    cut = eng.knn_last_fallback()
    sb = SnnBufs(torch, n, 300 * n, dev)
    info = torch.zeros(3 + len(K_NUM), dtype=torch.int64, device=dev)
    sb.run(eng, knn, idx, info)
    rows = torch.empty((n, dpad), dtype=torch.float64, device=dev)
    eng.gather_rows_rm_t(inp["cells"], inp["cells"].shape[0], dpad, idx, rows)
    nsub = inp["nsub"]
    pick = sorted({0, max(range(nsub), key=lambda c: inp["sizes"][c]), len(segs) - 1})
    L = labels[0].shape[1]
    sil = [torch.empty(L, dtype=torch.float64, device=dev) for _ in segs]
    slots = 1 + max(j for _, j in segs) - b0
    eng.silhouette_segments_t(rows, off, [labels[c][j] for c, j in segs], cmax, cfg5_sil_keys(torch, inp, plan, b0),
                              slots * inp["cells"].shape[0], sil)
    torch.cuda.synchronize()
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    kn = knn.cpu().numpy()
    X_all = rows.cpu().numpy()
    inf = info.cpu().numpy()
    ok_snn = int(inf[1]) == 0 and int(inf[3:].min()) >= 0
    rng = np.random.default_rng(11)
    out = {"segments_checked": [], "knn_rows_checked": 0}
    knn_ok, snn_ok, rel_max = True, ok_snn, 0.0
    for q in pick:
        c, j = segs[q]
        a, b = int(off[q]), int(off[q + 1])
        X = X_all[a:b]
        loc = kn[a:b] - a
        cq = cut[(cut >= a) & (cut < b)] - a
        qs = np.unique(np.concatenate([cq[:2048], rng.choice(b - a, min(sample, b - a), replace=False),
                                       [0, b - a - 1]])).astype(np.int32)
        oi, _ = O.knn_queries(X, 20, qs, nthreads=threads)
        knn_ok = knn_ok and bool(np.array_equal(loc[qs], oi))
        out["knn_rows_checked"] += int(qs.size)
        if ok_snn:
            graphs = sb.decode(n, int(inf[0]), a, b)  # the segment's classes (a contiguous range)
            for g, k in enumerate(K_NUM):
                ei, ej, ew = O.snn(np.ascontiguousarray(loc), k, "number")
                gi, gj, gw = graphs[g]
                snn_ok = snn_ok and np.array_equal(gi, ei) and np.array_equal(gj, ej) and np.array_equal(gw, ew)
        labs = labels[c][j].cpu().numpy()
        with cf.ThreadPoolExecutor(threads) as ex:
            ref = np.asarray(list(ex.map(lambda l_: O.silhouette(X, labs[l_])[1], range(L))))
        g_ = sil[q].cpu().numpy()
        rel_max = max(rel_max, float((np.abs(g_ - ref) / np.maximum(np.abs(ref), 1e-300)).max()))
        out["segments_checked"].append([int(c), int(j), b - a])
    out["knn_exact"] = bool(knn_ok)
    out["snn_graphs_exact"] = bool(snn_ok)
    out["silhouette_max_rel_err"] = rel_max
    out["silhouette_within_1e-5"] = bool(rel_max <= 1e-5)
    out["ok"] = all(v for v in out.values() if isinstance(v, bool))
    return out


def run_cfg5(args, torch, dist, grp, engs, dev, world, rank, json_fd, ranks_seen):
    """BASELINE cfg5: one iterate=TRUE level on 100k cells (R/consensusClust.R:
    541-567).  The cells fall into 10 subclusters of 5k-20k cells with pcNum
    d_c = 5..15 (the :356 rule's range); each subcluster's bootstrap loop
    (:391-400, :650-692) runs B bootstraps.  A step batches `--seg-batch`
    bootstraps of EVERY subcluster per launch set: the segmented distinct-cell
    kNN (ccg_knn_boot_segments_dev, one segment per (subcluster, bootstrap),
    neighbour ids of the concatenation), ONE SNN rows pass over the disjoint
    union of all the batch's graphs, ONE ccg_silhouette_segments_dev for the
    60 clusterings of every segment; per subcluster the selection + map-back
    and its co-cluster
    triangle.  The subclusters' PC matrices are slices of synthetic PCs (the
    per-subset PCA, f4, is timed on its own)."""
    eng = engs[0]
    S = len(engs)
    N, B, G = args.cells, args.boots_per_gpu, world
    L = len(K_NUM) * N_RES
    inp = cfg5_inputs(torch, N, args.pcs, args.genes, B, rank, dev)
    pcs, sizes, nsub, dcs, dpad = inp["pcs"], inp["sizes"], inp["nsub"], inp["dcs"], inp["dpad"]
    Nof, cells, popc, ns, bids = inp["Nof"], inp["cells"], inp["popc"], inp["ns"], inp["bids"]
    uniq, boots_t = inp["uniq"], inp["boots_t"]
    labels = [torch.empty((B, L, ns[c]), dtype=torch.int32, device=dev) for c in range(nsub)]
    for c in range(nsub):
        for j in range(B):
            labels[c][j] = synth_labels(torch, popc[Nof[c]:Nof[c + 1]], boots_t[c][j], L, dev, 1000 + bids[j], chi=20)
    cmax = max(int(lb.max().item()) for lb in labels)
    SB = max(1, min(args.seg_batch, B))
    batches = [(b0, min(B, b0 + SB)) for b0 in range(0, B, SB)]

    def seg_plan(b0, b1):
        return cfg5_seg_plan(torch, inp, b0, b1)

    plans = [seg_plan(b0, b1) for b0, b1 in batches]
    skeys = [cfg5_sil_keys(torch, inp, p, b0) for p, (b0, _) in zip(plans, batches)]
    nmax = max(int(p[1][-1]) for p in plans)
    rows_s = [torch.empty((nmax, dpad), dtype=torch.float64, device=dev) for _ in range(S)]
    knn_s = [torch.empty((nmax, 20), dtype=torch.int32, device=dev) for _ in range(S)]
    rcap = 300 * nmax
    snn_s = [SnnBufs(torch, nmax, rcap, dev) for _ in range(S)]
    snn_info = torch.zeros((len(batches), 3 + len(K_NUM)), dtype=torch.int64, device=dev)
    means = [torch.empty((B, L), dtype=torch.float64, device=dev) for _ in range(nsub)]
    nclust = [torch.empty((B, L), dtype=torch.int32, device=dev) for _ in range(nsub)]
    minsize = [torch.empty((B, L), dtype=torch.int32, device=dev) for _ in range(nsub)]
    A = [torch.zeros((B, sizes[c]), dtype=torch.uint8, device=dev) for c in range(nsub)]
    P = [sizes[c] * (sizes[c] - 1) // 2 for c in range(nsub)]
    co = [torch.empty(P[c], dtype=torch.int16, device=dev) for c in range(nsub)]
    both = [torch.empty(P[c], dtype=torch.int16, device=dev) for c in range(nsub)]
    streams = [e.torch_stream() for e in engs]

    def run_batch(t, si):
        segs, off, su, idx = plans[t]
        e = engs[si]
        n = int(off[-1])
        rows, knn = rows_s[si][:n], knn_s[si][:n]
        e.knn_boot_segments_t(cells, idx, off, su, 20, knn, local_ids=False)
        snn_s[si].run(e, knn, idx, snn_info[t], n=n)  # the classes of every segment in one pass
        e.gather_rows_rm_t(cells, N, dpad, idx, rows)
        # every segment's 60 silhouettes in one launch set
        e.silhouette_segments_t(rows, off, [labels[c][j] for c, j in segs], cmax, skeys[t], SB * N,
                                [means[c][j] for c, j in segs], [nclust[c][j] for c, j in segs],
                                [minsize[c][j] for c, j in segs])

    def step(evs=None):
        def mark(name):
            if evs is not None:
                evs[name] = torch.cuda.Event(enable_timing=True)
                evs[name].record()
        cur = torch.cuda.current_stream()
        mark("start")
        for st_ in streams:
            st_.wait_stream(cur)
        for t in range(len(batches)):
            si = t % S
            with torch.cuda.stream(streams[si]):
                run_batch(t, si)
        for st_ in streams:
            cur.wait_stream(st_)
        mark("boots_done")
        for c in range(nsub):
            eng.select_mapback_t("robust", labels[c], boots_t[c], sizes[c], A[c], 0, means=means[c],
                                 nclust=nclust[c], minsize=minsize[c])
        mark("selected")
        mark("gathered")  # (one GPU per level: no all-gather)
        for c in range(nsub):
            eng.cocluster_t(A[c], 0, sizes[c], co=co[c], both=both[c])
        mark("slab_done")

    def barrier():
        if G > 1:
            dist.barrier()

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if int(snn_info[:, 3:].min().item()) < 0:
        raise RuntimeError(f"SNN row capacity too small: {rcap}")
    if int(snn_info[:, 1].max().item()) != 0:
        raise RuntimeError("ccg_snn_classes_dev: the class contract failed")
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    # kernel times (library timers) over one more step, then the segmented kNN in isolation
    for e in engs:
        e.timing(True)
        for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
            e.timing_read(w)
    evs = {}
    step(evs)
    torch.cuda.synchronize()
    phase = {"step_ms": el / args.steps * 1000,  # this rank's own timed steps (value uses the max over ranks)
             "boot_phase_ms": evs["start"].elapsed_time(evs["boots_done"]),
             "select_mapback_ms": evs["boots_done"].elapsed_time(evs["selected"]),
             "allgather_ms": evs["selected"].elapsed_time(evs["gathered"]),
             "slab_ms": evs["gathered"].elapsed_time(evs["slab_done"])}
    per_rank = per_rank_report(torch, dist, G, phase, dev)
    kt = {}
    for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
        r = [e.timing_read(w) for e in engs]
        kt[w] = (sum(x[0] for x in r), sum(x[1] for x in r))
    for e in engs:
        e.timing(False)
    eng.timing(True)
    eng.timing_read("knn_screen")
    eng.timing_read("knn_total")
    fbk = 0
    with torch.cuda.stream(streams[0]):
        for t in range(len(batches)):
            segs, off, su, idx = plans[t]
            n = int(off[-1])
            fbk += eng.knn_boot_segments_t(cells, idx, off, su, 20, knn_s[0][:n], local_ids=False, stats=True)[1]
    iso_scr = eng.timing_read("knn_screen")
    iso_tot = eng.timing_read("knn_total")
    eng.timing(False)
    per_rank = per_rank_report(torch, dist, G, {"step_ms": el / args.steps * 1000}, dev)
    if G > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = tt.item()
    value = G * B * args.steps / el
    # the screen's algorithmic work: 2 u_s^2 d_c per segment (the distinct cells it searches)
    flops = sum(2.0 * uniq[c][j] ** 2 * dcs[c] for c in range(nsub) for j in range(B))
    scr_ms = iso_scr[0]
    roof = {
        "kernel": "knn_screen16_kernel over every (subcluster, bootstrap) segment's distinct cells "
                  "(ccg_knn_boot_segments_dev; fp16 hi/lo split, v_mfma_f32_32x32x16_f16)",
        "bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_F16_TFLOPS,
        "achieved": round(flops / (scr_ms * 1e-3) / 1e12, 2),
        "frac": round(flops / (scr_ms * 1e-3) / 1e12 / PEAK_F16_TFLOPS, 4),
        "traffic": None,
        "algorithmic_per_launch": f"sum over segments of 2 u_s^2 d_c = {flops:.3e} flop per step over "
                                  f"{iso_scr[1]} launches ({nsub} subclusters x {B} bootstraps)",
        "avg_launch_ms": round(scr_ms / max(iso_scr[1], 1), 4),
        "knn_total_ms_per_step": round(iso_tot[0], 3),
        "exact_search_rows_per_step": int(fbk),
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
        "dtype_detail": "kNN order exact in f64 (segmented distinct-cell screen: fp16 hi/lo x3 MFMA, f64 certify, "
                        "exact f64 expansion); silhouette f64 fixed-point sums; co-cluster int8 MFMA",
        "data": "synthetic: NB counts (12 populations, 2000 genes) -> PCA, subclusters = random cell blocks of "
                "5k-20k cells with the first d_c PCs; synthetic clusterings (C 2..20) in place of host Leiden",
        "config": {
            "workload": f"BASELINE cfg5: one iterate=TRUE level on {N} cells -- {nsub} subclusters "
                        f"({min(sizes)}-{max(sizes)} cells, pcNum {min(dcs)}-{max(dcs)}), {B} bootstraps of every "
                        f"subcluster per GPU per step (value = level bootstraps/s; x{nsub} subcluster-bootstraps), "
                        f"{SB} bootstraps x {nsub} subclusters per segmented launch set",
            "name": "cfg5", "cells": N, "subcluster_cells": sizes, "subcluster_pcs": dcs, "boots_per_gpu": B,
            "segments_per_launch": SB * nsub, "streams_per_gpu": S,
        },
        "subcluster_bootstraps_per_s": round(value * nsub, 3),
        "per_rank": per_rank,
        "roofline": roof,
        "kernel_ms_per_step": {w: round(v[0], 3) for w, v in kt.items()},
        "kernel_launches_per_step": {w: int(v[1]) for w, v in kt.items()},
    }
    if rank == 0 and G == 1 and not args.no_cpu_baseline:
        dm = int(round(float(np.mean(dcs))))
        out["cpu_baseline"] = cpu_baseline(pcs[:, :dm].contiguous().cpu().numpy(), B, max(ns), N, dm,
                                           args.cpu_sample_rows, coc_cols=B, coc_pairs=float(sum(P)),
                                           seg_rows=ns)
        out["cpu_baseline"]["check"] = cfg5_check(eng, torch, inp, labels, cmax, plans[0])
    elif rank == 0 and args.check:
        out["cpu_baseline"] = {"check": cfg5_check(eng, torch, inp, labels, cmax, plans[0])}
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    for e in engs[1:]:
        e.close()
    grp.close()
    if G > 1:
        dist.destroy_process_group()


def group_ranks_seen(torch, dist, world, rank, local, grp, dev):
    """[torch rank, HIP device, nranks and first rank of libccg's device
    group (ccg_group_info)] of every rank, gathered over the process group:
    the ranks libccg's RCCL communicator actually joined."""
    mine = torch.tensor([rank, local, grp.nranks, grp.first_rank], dtype=torch.int64, device=dev)
    if world == 1:
        return [mine.tolist()]
    got = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    return [g.tolist() for g in got]


PHASES = ("step_ms", "boot_phase_ms", "select_mapback_ms", "allgather_ms", "slab_ms")


def per_rank_report(torch, dist, world, values, dev=None):
    """Every rank's PHASES values (ms) gathered to all ranks: a list of
    dicts in rank order (the whole-job value is the max step; these say
    where each rank spent it)."""
    t = torch.tensor([float(values.get(k, float("nan"))) for k in PHASES], dtype=torch.float64,
                     device=dev if dev is not None else "cpu")
    if world > 1:
        got = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(got, t)
    else:
        got = [t]
    return [dict({"rank": r}, **{k: round(float(v), 3) for k, v in zip(PHASES, g.tolist())})
            for r, g in enumerate(got)]


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

    from consensusclustr_amd import Engine
    from consensusclustr_amd.sharding import DeviceGroup, exchange_group_id, row_slabs, slab_pairs

    # libccg's device group: this rank's context + an RCCL communicator over
    # all ranks (the all-gather and the slab split run inside libccg)
    if world > 1:
        grp = DeviceGroup.open_rank(local, world, rank, exchange_group_id())
    else:
        grp = DeviceGroup.open([local])
    # what libccg's own communicator saw (ccg_group_info), per rank:
    # [torch rank, device, the group's nranks, the group's first rank]
    ranks_seen = group_ranks_seen(torch, dist, world, rank, local, grp, dev)
    W = WORKLOADS[args.workload]
    # bootstraps per launch set (table path): one set of launches for the
    # batch's kNN, SNN and silhouettes (round 6)
    NBB = args.boot_batch if args.boot_batch > 0 else W.get("boot_batch", 16)
    if args.knn_path != "table":
        NBB = 1
    if args.streams > 0:
        S = args.streams
    elif args.workload == "cfg5":
        S = 2
    elif NBB > 1:
        S = W.get("batch_streams", 2)
    else:
        S = 4 if int(args.boot_size * (args.cells or W["cells"])) >= 50000 else 3
    if args.workload == "cfg5":
        return run_cfg5(args, torch, dist, grp, [grp.engines[0]] + [Engine(local) for _ in range(S - 1)], dev, world,
                        rank, json_fd, ranks_seen)
    robust = W["mode"] == "robust"
    emul = W["emul_ranks"] if world == 1 else 0  # one GPU's share of an emul-rank job (synthetic other columns)
    engs = [grp.engines[0]] + [Engine(local) for _ in range(S - 1)]  # own workspaces per in-flight bootstrap
    eng = engs[0]
    N, d, B = args.cells, args.pcs, args.boots_per_gpu
    n = int(args.boot_size * N)
    L = len(K_NUM) * N_RES
    G = world
    Gc = emul or G  # ranks whose columns the co-cluster counts
    cpr = B if robust else B * L  # assignment columns per rank per step (granular: all 60, :688)

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
        labels[j] = synth_labels(torch, pop, boots[j], L, dev, 1000 + bids[j], chi=W["cmax"])
    cmax = int(labels.max().item())

    NBB = max(1, min(NBB, B))
    batched = NBB > 1
    batches = [(b0, min(B, b0 + NBB)) for b0 in range(0, B, NBB)]
    nrow = NBB * n  # rows of a launch set
    RING = S  # launch-set buffers (gathered rows, kNN) in flight
    rows_s = [torch.empty((nrow, d), dtype=torch.float64, device=dev) for _ in range(RING)]
    knn_s = [torch.empty((nrow, 20), dtype=torch.int32, device=dev) for _ in range(RING)]
    rows, knn = rows_s[0][:n], knn_s[0][:n]
    rcap = 300 * nrow  # SNN class-row entries (items per class ~ 190 at cfg3); grown once after the warmup if short

    def alloc_snn(rcap):
        # per stream: the class-level rows of ccg_snn_classes_dev
        return [SnnBufs(torch, nrow, rcap, dev) for _ in range(S)]
    snn_out = alloc_snn(rcap)
    if os.environ.get("CCG_BENCH_TORCH_STREAMS"):
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    else:
        streams = [e.torch_stream() for e in engs]  # each context's own non-blocking HIP stream
    # [u, status, cap, class edges] per bootstrap, or per launch set (batched)
    snn_info = torch.zeros((len(batches) if batched else B, 3 + len(K_NUM)), dtype=torch.int64, device=dev)
    means = torch.empty((B, L), dtype=torch.float64, device=dev)
    nclust = torch.empty((B, L), dtype=torch.int32, device=dev)
    minsize = torch.empty((B, L), dtype=torch.int32, device=dev)
    # launch sets: bootstrap j's rows are slot (j - b0) of its set; its cells
    # get the keys slot N + cell (SNN classes and silhouette cells stay apart
    # between the set's bootstraps); everything a launch needs is built here,
    # before timing
    vkeys = boots + (torch.tensor([j - (j // NBB) * NBB for j in range(B)], dtype=torch.int32,
                                  device=dev) * N)[:, None]
    sets = [dict(idx=boots[b0:b1], flat=boots[b0:b1].reshape(-1), keys=vkeys[b0:b1].reshape(-1),
                 uniq=np.array(uniq[b0:b1], np.int32), m=(b1 - b0) * n,
                 off=np.arange(b1 - b0 + 1, dtype=np.int64) * n, ncell=(b1 - b0) * N,
                 labels=[labels[j] for j in range(b0, b1)], means=[means[j] for j in range(b0, b1)],
                 nclust=[nclust[j] for j in range(b0, b1)], minsize=[minsize[j] for j in range(b0, b1)])
            for b0, b1 in batches]

    # --split-sil: the silhouettes of a set on their own stream and context
    # (a context's workspaces serve one stream at a time), ordered after the
    # set's gather; the next set on the same buffers waits for them
    split = batched and robust and args.split_sil > 0
    engs_sil = [Engine(local) for _ in range(S)] if split else []
    streams_sil = [e.torch_stream() for e in engs_sil]
    ev_g = [torch.cuda.Event() for _ in range(S)]
    ev_s = [torch.cuda.Event() for _ in range(S)]

    def run_set_split(si, t):
        c = sets[t]
        m = c["m"]
        r, k = rows_s[si][:m], knn_s[si][:m]
        e, es = engs[si], engs_sil[si]
        with torch.cuda.stream(streams[si]):
            streams[si].wait_event(ev_s[si])  # set t - S's silhouettes have read the rows
            e.gather_rows_rm_t(pcs, N, d, c["flat"], r)
            ev_g[si].record(streams[si])
            e.knn_boots_table_t(N, d, c["idx"], c["uniq"], r, 20, tab_idx, tab_d2, k)
            snn_out[si].run(e, k, c["keys"], snn_info[t], n=m)
        with torch.cuda.stream(streams_sil[si]):
            streams_sil[si].wait_event(ev_g[si])
            es.silhouette_segments_t(r, c["off"], c["labels"], cmax, c["keys"], c["ncell"], c["means"],
                                     c["nclust"], c["minsize"])
            ev_s[si].record(streams_sil[si])

    def run_set(e, si, t, info=None):
        # one launch set: gather, kNN from the table, SNN classes, silhouettes of its bootstraps
        c = sets[t]
        m = c["m"]
        r, k = rows_s[si][:m], knn_s[si][:m]
        e.gather_rows_rm_t(pcs, N, d, c["flat"], r)
        e.knn_boots_table_t(N, d, c["idx"], c["uniq"], r, 20, tab_idx, tab_d2, k)
        snn_out[si].run(e, k, c["keys"], snn_info[t] if info is None else info, n=m)
        if robust:  # granular mode scores no clustering (:688)
            e.silhouette_segments_t(r, c["off"], c["labels"], cmax, c["keys"], c["ncell"], c["means"], c["nclust"],
                                    c["minsize"])
    choice = torch.empty(B, dtype=torch.int32, device=dev)
    A_full = torch.zeros((Gc * cpr, N), dtype=torch.uint8, device=dev)  # all ranks' columns
    A_local = A_full[rank * cpr:(rank + 1) * cpr]  # this rank's block, all-gathered in place
    cuts = row_slabs(N, Gc)
    r0, r1 = cuts[rank], cuts[rank + 1]
    P = max(slab_pairs(N, r0, r1), 1)
    co = torch.empty(P, dtype=torch.int16, device=dev)      # uint16 counts (viewed as int16)
    both = torch.empty(P, dtype=torch.int16, device=dev)


    def mark(evs, k):
        # phase events on torch's current stream (the tail's calls order their
        # context streams after it and it after them), the timer step only
        if evs is not None:
            evs[k] = torch.cuda.Event(enable_timing=True)
            evs[k].record()

    def step_tail(evs=None):
        # selection + map-back into this rank's columns, the all-gather, this rank's co/both slab
        mark(evs, "boots_done")
        if robust:
            eng.select_mapback_t("robust", labels, boots, N, A_local, 0, means=means, nclust=nclust,
                                 minsize=minsize, out_choice=choice)
        else:
            eng.select_mapback_t("granular", labels, boots, N, A_local, 0)
        mark(evs, "selected")
        if emul:  # one rank of an emul-rank job: the other ranks' columns are already in place
            mark(evs, "gathered")
            eng.cocluster_t(A_full, r0, r1, co=co, both=both)
        else:
            grp.allgather_columns_t([A_local], [cpr] * G, [A_full])
            mark(evs, "gathered")
            grp.cocluster_sharded_t([A_full], co=[co], both=[both])
        mark(evs, "slab_done")

    host_t = [0.0]  # host time spent enqueueing the bootstrap loop (the launches are asynchronous)

    def boot_phase():
        # S bootstraps in flight: bootstrap j runs on stream j % S with its own
        # engine context (workspaces), so one bootstrap's latency-bound SNN
        # build overlaps another's MFMA-bound kNN screen
        cur = torch.cuda.current_stream()
        if use_table:  # one table per step: every bootstrap of the step filters it
            eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2)
        for st_ in streams + streams_sil:
            st_.wait_stream(cur)
        if batched and split:
            for t in range(len(batches)):
                run_set_split(t % S, t)
        elif batched:
            for t in range(len(batches)):
                si = t % S
                with torch.cuda.stream(streams[si]):
                    run_set(engs[si], si, t)
        else:
            for j in range(B):
                si = j % S
                e = engs[si]
                with torch.cuda.stream(streams[si]):
                    e.gather_rows_rm_t(pcs, N, d, boots[j], rows_s[si][:n])
                    boot_knn(e, j, rows_s[si][:n], knn_s[si][:n])
                    snn_out[si].run(e, knn_s[si][:n], boots[j], snn_info[j], n=n)
                    if robust:  # granular mode scores no clustering (:688)
                        e.silhouette_cells_t(rows_s[si][:n], labels[j], cmax, boots[j], N, means[j], nclust[j],
                                             minsize[j])
        for st_ in streams + streams_sil:
            cur.wait_stream(st_)

    graph = [None]  # the captured bootstrap phase (--launch graph)

    def step(evs=None, eager=False):
        mark(evs, "start")
        th = time.perf_counter()
        if graph[0] is not None and not eager:
            graph[0].replay()  # every kernel of the phase runs again; only the host launch work is gone
        else:
            boot_phase()
        host_t[0] += time.perf_counter() - th
        step_tail(evs)

    def barrier():
        if G > 1:
            dist.barrier()

    # ---------------- warmup (also sizes the SNN edge buffers)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    short = int(snn_info[:, 3:].min().item())
    if short < 0:  # rows did not fit: -short entries needed; grow once and redo the warmup
        rcap = int(-short * 1.25)
        snn_out = alloc_snn(rcap)
        step()
        torch.cuda.synchronize()
        if int(snn_info[:, 3:].min().item()) < 0:
            raise RuntimeError(f"SNN row capacity too small: {rcap}")
    if int(snn_info[:, 1].max().item()) != 0:  # (cannot happen for bootstrap copies under the kNN contract)
        raise RuntimeError("ccg_snn_classes_dev: the class contract failed; the row-level pass would be needed")
    need = snn_info[:, 3:].max(0).values.tolist()
    if emul:  # the other ranks' column blocks: this rank's columns with the cells rotated (same label counts)
        for k in range(1, emul):
            A_full[k * cpr:(k + 1) * cpr] = torch.roll(A_local, shifts=k * 7919, dims=1)
        torch.cuda.synchronize()
    eng.gather_rows_rm_t(pcs, N, d, boots[0], rows)
    fb = eng.knn_boot_hint_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, knn, hint, stats=True)  # certification statistics
    fb_cold = eng.knn_boot_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, knn, stats=True)
    fb_tab_build = eng.knn_table_t(pcs_cm, N, d, KT, tab_idx, tab_d2, stats=True)
    fb_tab = eng.knn_boot_table_t(pcs_cm, N, d, boots[0], uniq[0], rows, 20, tab_idx, tab_d2, knn, stats=True)

    # --launch graph: capture the bootstrap phase once, after every untimed
    # call above (the warmup and the statistics calls sized every workspace:
    # the graph's baked pointers stay valid); the replay is checked against an
    # eager step's outputs before timing
    launch_note = "eager"
    # (launch sets upload small host tables -- segment offsets, label and
    # output pointers -- and issue ~80 launches per set: eager)
    use_graph = args.launch == "graph" or (args.launch == "auto" and n >= 50000 and not batched)
    if use_graph and not W.get("no_graph"):
        try:
            torch.cuda.synchronize()
            ref_means = means.clone()
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream(device=dev)
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.graph(g, stream=cs):
                boot_phase()
            torch.cuda.synchronize()
            means.fill_(-9.0)
            g.replay()
            torch.cuda.synchronize()
            if robust and not torch.equal(means, ref_means):
                raise RuntimeError("graph replay differs from the eager step")
            graph[0] = g
            launch_note = "hipgraph"
        except Exception as ex:  # (capture unsupported here: stay eager and say why)
            graph[0] = None
            launch_note = f"eager (graph capture failed: {type(ex).__name__}: {str(ex)[:160]})"
            torch.cuda.synchronize()
    # ---------------- timed region (library timers off: their event records
    # cost host time on every launch group)
    barrier()
    torch.cuda.synchronize()
    ring_engs = list({id(e): e for e in [eng] + engs + engs_sil}.values())
    for e in ring_engs:
        e.timing_read("host_ring_wait")  # (reset: host-side accounting, always on)
    t0 = time.perf_counter()
    host_t[0] = 0.0
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    host_ms = host_t[0] / args.steps * 1000
    ring_ms = sum(e.timing_read("host_ring_wait")[0] for e in ring_engs) / args.steps
    # kernel-time breakdown: one more (untimed) step with the library's
    # hipEvent timers on
    for e in engs + engs_sil:
        e.timing(True)
        for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
            e.timing_read(w)
    evs = {}
    step(evs, eager=True)  # (the library timers need the host calls)
    torch.cuda.synchronize()
    phase = {"step_ms": el / args.steps * 1000,  # this rank's own timed steps (value uses the max over ranks)
             "boot_phase_ms": evs["start"].elapsed_time(evs["boots_done"]),
             "select_mapback_ms": evs["boots_done"].elapsed_time(evs["selected"]),
             "allgather_ms": evs["selected"].elapsed_time(evs["gathered"]),
             "slab_ms": evs["gathered"].elapsed_time(evs["slab_done"])}
    per_rank = per_rank_report(torch, dist, G, phase, dev)
    kt = {}
    for w in ("knn_screen", "knn_total", "snn", "silhouette", "cocluster"):
        r = [e.timing_read(w) for e in engs + engs_sil]
        kt[w] = (sum(x[0] for x in r), sum(x[1] for x in r))
    for e in engs + engs_sil:
        e.timing(False)
    # host cost of one bootstrap's launches on an idle GPU (no queue
    # back-pressure): one launch set divided by its bootstraps when batched
    host_idle = []
    iso_info = torch.zeros(3 + len(K_NUM), dtype=torch.int64, device=dev)
    for j in range(min(len(batches) if batched else B, 6)):
        torch.cuda.synchronize()
        th = time.perf_counter()
        with torch.cuda.stream(streams[0]):
            if batched:
                run_set(eng, 0, j, iso_info)
            else:
                eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
                boot_knn(eng, j, rows, knn)
                snn_out[0].run(eng, knn, boots[j], iso_info, n=n)
                if robust:
                    eng.silhouette_cells_t(rows, labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
        host_idle.append((time.perf_counter() - th) / (sets[j]["m"] // n if batched else 1))
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
    iso_set_table = None
    if batched:  # the launch set's kNN (ccg_knn_boots_table_dev), per bootstrap
        c0 = sets[0]
        eng.gather_rows_rm_t(pcs, N, d, c0["flat"], rows_s[0][:c0["m"]])
        for _ in range(2):
            eng.knn_boots_table_t(N, d, c0["idx"], c0["uniq"], rows_s[0][:c0["m"]], 20, tab_idx, tab_d2,
                                  knn_s[0][:c0["m"]])
        t_, c_ = eng.timing_read("knn_total")
        iso_set_table = (t_, c_ * (c0["m"] // n))
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
    if batched:  # one launch set (its SNN pass and its silhouette launch set), per bootstrap
        nis = sets[0]["m"] // n
        iso_infos = torch.zeros((1, 3 + len(K_NUM)), dtype=torch.int64, device=dev)
        run_set(eng, 0, 0, iso_infos[0])
        iso_snn = eng.timing_read("snn")
        iso_sil = eng.timing_read("silhouette")
        iso_snn, iso_sil = (iso_snn[0], iso_snn[1] * nis), (iso_sil[0], iso_sil[1] * nis)
    else:
        nis = min(B, 4)
        iso_infos = torch.zeros((nis, 3 + len(K_NUM)), dtype=torch.int64, device=dev)
        for j in range(nis):
            eng.gather_rows_rm_t(pcs, N, d, boots[j], rows)
            boot_knn(eng, j, rows, knn)
            snn_out[0].run(eng, knn, boots[j], iso_infos[j], n=n)
            if robust:
                eng.silhouette_cells_t(rows, labels[j], cmax, boots[j], N, means[j], nclust[j], minsize[j])
        iso_snn = eng.timing_read("snn")
        iso_sil = eng.timing_read("silhouette")
    torch.cuda.synchronize()
    iso_edges = iso_infos[:, 3:].sum(0).tolist()  # class edges per graph, over the nis bootstraps
    iso_classes = float(iso_infos[:, 0].double().sum().item()) / nis
    iso_npres = int(nclust[:nis].sum().item())  # sum over the bootstraps' labelings of present clusters
    # the drop-in's host side of the SNN (R: igraph::make_graph of each graph,
    # :656-658): ccg_snn_graphs_cells (device pass + copy to pinned memory)
    # and the host expansion of the class rows (ccg_snn_graph_fetch), for
    # bootstrap 0 through Engine.snn_multi; outside value
    eng.gather_rows_rm_t(pcs, N, d, boots[0], rows)
    boot_knn(eng, 0, rows, knn)
    torch.cuda.synchronize()
    kn0 = knn.cpu().numpy()
    b0np = boots_np[0]
    eng.snn_multi(kn0, K_NUM, "number", cell=b0np)  # (warm: pinned staging sized)
    eng.snn_multi(kn0, K_NUM, "number", cell=b0np)
    host_snn = eng.last_snn_times
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
    coc_ops = 2.0 * P * (colC + Gc * cpr)
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
        "knn_total_ms_per_boot_from_table": round(avg(iso_set_table if batched else iso_boot_table), 4),
        "knn_total_ms_per_boot_from_table_one_boot_per_call": round(avg(iso_boot_table), 4),
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
    if args.workload != "cfg3":
        coc_traffic = None  # the committed PMC traffic is the cfg3 (N = 100k, B = 125) launch
    roof_coc = {
        "kernel": "cof_tile_kernel (one-hot int8 co/both GEMM, v_mfma_i32_32x32x32_i8), this rank's row slab",
        "bound": "mfma",
        "achieved": round(coc_ops / (coc_ms * 1e-3) / 1e12, 2),
        "peak": PEAK_I8_TOPS,
        "unit": "TOP/s",
        "frac": round(coc_ops / (coc_ms * 1e-3) / 1e12 / PEAK_I8_TOPS, 4),
        "traffic": coc_traffic,
        "algorithmic_per_launch": f"2*P*(sum C_b + B) = {coc_ops:.3e} int8 ops (P={P} pairs in this slab, "
                                  f"sum C_b={colC}, B={Gc * cpr}), SURVEY 8(d); one launch per step",
        "avg_launch_ms": round(coc_ms, 4),
        "avg_launch_ms_note": "library hipEvent timer on the launch stream, the timer step after the timed region",
        "output_bytes_per_launch": 4 * P,
    }
    # SNN (the rows pass the drop-ins run too: ccg_snn_graphs = these kernels
    # + a host decode) and silhouette (fp64 MFMA widths: 2 d u sum_l C_l over
    # the distinct cells), per bootstrap in isolation.  SNN bytes are what the
    # pass reads and writes as its interface: the kNN rows in, the union-graph
    # rows out (8 B per union edge: partner + packed per-graph values), the row
    # lengths and offsets and the per-graph edge offsets; SURVEY 8(d)'s
    # per-graph (i, j, w) lists (16 B per edge per graph) are no longer
    # formed on the device.
    snn_ms = iso_snn[0] / max(iso_snn[1], 1)
    sil_ms = iso_sil[0] / max(iso_sil[1], 1)
    nk_ = len(K_NUM)
    e_union = iso_edges[-1] / max(nis, 1)  # class edges of the largest k's graph = the union
    snn_bytes = (n * max(K_NUM) * 4 + 8 * e_union + 4 * n + 4 * iso_classes + 8 * (n + 1) + 4 * n +
                 nk_ * (n + 1) * 8)
    snn_traffic = None
    if os.path.exists(args.traffic_json) and args.workload == "cfg3":
        with open(args.traffic_json) as f:
            snn_traffic = json.load(f).get("snn_bytes_per_boot")
    sil_flop = 2.0 * d * u_iso * iso_npres / max(nis, 1)
    if not robust:
        sil_ms = 0.0
    roof_snn = {
        "kernel": "SNN graphs at the level of row classes (ccg_snn_classes_dev; the same kernels "
                  "ccg_snn_graphs_cells runs for the R and Python drop-ins before the host expands the rows)",
        "bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
        "achieved": round(snn_bytes / (snn_ms * 1e-3) / 1e9, 1),
        "frac": round(snn_bytes / (snn_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "traffic": snn_traffic,
        "algorithmic_per_launch": f"n kmax 4 (kNN in) + 8 E_class + 4 n + 4 u + 8 (n+1) + 4 n + 8 nk (n+1) (class "
                                  f"rows, row->class, roots, offsets, lengths, per-graph offsets out) = "
                                  f"{snn_bytes:.3e} B per bootstrap (u = {iso_classes:.0f} classes, "
                                  f"E_class = {e_union:.0f})",
        "survey_8d_note": "SURVEY 8(d)'s sum_K (n K 4 + E_K 16) counts per-graph (i, j, w) row lists, which "
                          "neither the bench nor the drop-ins write on the device (the host expands the classes)",
        "ms_per_boot": round(snn_ms, 4),
    }
    sil_traffic = None
    if os.path.exists(args.traffic_json) and args.workload == "cfg3":
        with open(args.traffic_json) as f:
            sil_traffic = json.load(f).get("silhouette_bytes_per_boot")
    roof_sil = {
        "kernel": "silhouette of the 60 clusterings (ccg_silhouette_cells_dev: the nearest other centroid "
                  "screened on v_mfma_f32_32x32x16_f16, the own and nearest distances exact in fp64; cluster "
                  "sums by int64 LDS atomics)",
        "bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_F16_TFLOPS,
        "achieved": round(sil_flop / (sil_ms * 1e-3) / 1e12, 2) if robust else None,
        "frac": round(sil_flop / (sil_ms * 1e-3) / 1e12 / PEAK_F16_TFLOPS, 4) if robust else None,
        "traffic": sil_traffic,
        "traffic_note": "HBM bytes per bootstrap over the stage's kernels (profiles/traffic_r06.json); the "
                        "stage is bound by VALU issue (the screen's min tracking, the exact fp64 distances) "
                        "and the sums' LDS atomics, not by either peak",
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
            "workload": workload_text(args.workload, N, d, B, G, emul),
            "name": args.workload,
            "mode": W["mode"], "assignment_columns": Gc * cpr, "slab_rows": [int(r0), int(r1)],
            "cells": N, "pcs": d, "bootstrap_rows": n, "distinct_cells_mean": round(float(np.mean(uniq)), 1),
            "boots_per_gpu": B, "clusterings_per_boot": L,
            "parallelism": f"bootstraps x{G}, co-cluster row slabs x{G}", "streams_per_gpu": S,
            "knn_path": args.knn_path, "silhouette_streams": len(streams_sil),
        },
        "roofline": roof_coc,
        "roofline_note": "the co-cluster GEMM is the largest single launch of a step; the per-bootstrap "
                         "stages follow (kNN table screen once per step, SNN, silhouette)",
        "roofline_knn_table" if use_table else "roofline_knn_screen": (roof_table if use_table else roof_screen),
        "roofline_knn_screen_path" if use_table else "roofline_knn_table_path": (roof_screen if use_table else roof_table),
        "roofline_snn": roof_snn,
        "roofline_silhouette": roof_sil if robust else None,
        "kernel_ms_per_step": per_step,
        "kernel_ms_per_step_note": "library hipEvent timers over one extra step after the timed region "
                                   "(bootstraps overlap, so kernel times sum to more than the step)",
        "per_rank": per_rank,
        "per_rank_note": "step_ms: each rank's own timed-region step (value uses the max over ranks); the "
                         "phases come from torch-stream events in the extra timer step: the bootstrap loop, "
                         "selection + map-back, the RCCL all-gather of the assignment columns, this rank's "
                         "co/both row slab",
        "launch": launch_note,
        "host_enqueue_ms_per_step": round(host_ms, 3),
        "host_ring_wait_ms_per_step": round(ring_ms, 3),
        "host_launch_ms_per_step": round(host_ms - ring_ms, 3),
        "host_enqueue_note": "host time in the step's launch loop; of it, host_ring_wait is time blocked on the "
                             "pinned upload ring (the host is that many launch sets ahead of the GPU: "
                             "back-pressure), host_launch the rest (issuing work)",
        "host_launch_ms_per_boot_idle_gpu": round(host_idle_ms, 3),
        "boots_per_launch_set": NBB,
        "launch_sets_per_step": len(batches) if batched else B,
        "host_snn_pass_ms_per_boot": round(1e3 * host_snn[0], 2),
        "host_snn_decode_ms_per_boot": round(1e3 * host_snn[1], 2),
        "host_snn_note": "the drop-in's host consumer path for one bootstrap (Engine.snn_multi: ccg_snn_graphs_cells "
                         "= device class pass + copy of the class rows to pinned memory, then ccg_snn_graph_fetch "
                         "expanding them into the three (i, j, w) edge lists on host threads); outside value",
        "cocluster_avg_ms": round(coc_ms, 3),
        "knn_fallback_rows_last_boot": int(fb[1]),
        "knn_fallback_rows_last_boot_cold": int(fb_cold[1]),
        ("snn_class_edges_max_per_launch_set" if batched else "snn_class_edges_max_per_boot"): [int(e) for e in need],
    }
    if rank == 0 and G == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pcs.cpu().numpy(), B, n, N, d, args.cpu_sample_rows, robust=robust,
                                           coc_cols=Gc * cpr, coc_pairs=P)
        out["cpu_baseline"]["check"] = cpu_baseline_check(
            eng, torch, pcs, pcs_cm, boots[0], uniq[0], labels[0], (tab_idx, tab_d2) if use_table else None, cmax,
            robust, A_full, co, both, int(r0), int(r1),
            batch=dict(idx=sets[0]["idx"], uniq=sets[0]["uniq"], keys=sets[0]["keys"], labels=sets[0]["labels"])
            if batched else None)
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
