"""Micro-benchmark of ccg_knn_rows_dev at BASELINE cfg3 shapes (n=90000, d=30).

Times the screen kernel and the whole kNN with the library's hipEvent timers:
by default the bench's path (ccg_knn_boot_dev: the bootstrap's distinct
cells, then the expansion to rows); KM_MODE=rows searches all n rows
(ccg_knn_rows_dev).
Data: one 90k-row bootstrap of bench.py's synthetic NB-count PCs (KM_DATA=gauss:
a 12-component Gaussian mixture instead).
Variants are separate builds of libccg (tools/build_variant.sh, --lib);
run each in its own process.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import _lib  # noqa: E402
if len(sys.argv) > 2 and sys.argv[1] == "--lib":  # tools only: time a variant build of libccg
    import ctypes
    _lib.LIB_PATH = os.path.abspath(sys.argv[2])
    _raw = ctypes.CDLL(_lib.LIB_PATH)  # a variant may predate newer exports: bind what it has
    _lib.SIGNATURES = {k: v for k, v in _lib.SIGNATURES.items() if hasattr(_raw, k)}
import bench  # noqa: E402
from consensusclustr_amd import Engine  # noqa: E402


def main():
    n, d, reps = int(os.environ.get("KM_N", 90000)), int(os.environ.get("KM_D", 30)), 5
    eng = Engine(0)
    if os.environ.get("KM_DATA") == "gauss":
        rng = np.random.default_rng(0)
        centers = rng.normal(scale=3.0, size=(12, d))
        X = centers[rng.integers(0, 12, n)] + rng.normal(size=(n, d))
        rows = torch.from_numpy(X).cuda()
    else:
        N = int(n / 0.9)
        pcs, _ = bench.synth_pcs(torch, N, d, 2000, 20241024 + 3, torch.device("cuda", 0))
        boot = torch.from_numpy(np.random.default_rng(123).integers(0, N, n).astype(np.int32)).cuda()
        rows = torch.empty((n, d), dtype=torch.float64, device="cuda")
        eng.gather_rows_t(pcs.t().contiguous(), N, d, boot, rows)
    idx = torch.empty((n, 20), dtype=torch.int32, device="cuda")
    boot_mode = os.environ.get("KM_MODE", "boot") == "boot" and os.environ.get("KM_DATA") != "gauss"
    if boot_mode:  # the bench's path: the bootstrap's distinct cells (ccg_knn_boot_dev)
        pcs_cm = pcs.t().contiguous()
        u = int(torch.unique(boot).numel())

        def run(stats=False):
            return eng.knn_boot_t(pcs_cm, N, d, boot, u, rows, 20, idx, stats=stats)
    else:
        u = n

        def run(stats=False):
            return eng.knn_rows_t(rows, 20, idx, stats=stats)
    run()
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("knn_screen")
    eng.timing_read("knn_total")
    for _ in range(reps):
        run()
    scr = eng.timing_read("knn_screen")
    tot = eng.timing_read("knn_total")
    st = run(stats=True)
    out = {"lib": os.path.basename(_lib.LIB_PATH), "mode": "boot" if boot_mode else "rows", "n": n, "u": u,
           "screen_ms": scr[0] / scr[1], "knn_total_ms": tot[0] / tot[1], "fallback": st[1]}
    lib = _lib.load()
    if hasattr(lib, "ccg_debug_knn_stamps"):  # a -DKNN_STAMPS=1 variant: per-wave cycle attribution
        import ctypes
        buf = (ctypes.c_ulonglong * 12)()
        lib.ccg_debug_knn_stamps(buf)  # reset
        run()
        torch.cuda.synchronize()
        lib.ccg_debug_knn_stamps(buf)
        waves = max(1, buf[11])
        names = ["dma_issue", "tile_mfma_max", "enqueue", "flush", "union", "vmcnt_wait", "barrier",
                 "n_tiles_with_candidates", "n_flushes", "n_flush_rounds", "n_tiles"]
        out["stamps_cycles_per_wave"] = {k: buf[i] / waves for i, k in enumerate(names)}
        out["stamps_waves"] = waves
    print(json.dumps(out))


if __name__ == "__main__":
    main()
