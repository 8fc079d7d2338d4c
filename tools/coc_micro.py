"""Micro-benchmark of the co-clustering kernel (ccg_cocluster_dev) at bench shapes.

N cells x B columns of uint8 labels (C per column uniform in [CM_CLO, CM_CHI],
10% unsampled), the full upper triangle (one GPU, r0 = 0, r1 = N), co + both
outputs.  Reports the kernel time (library hipEvent timer) and the
algorithmic int8 MFMA rate 2 * P * (sum_b C_b + B) / t.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusclustr_amd import _lib  # noqa: E402
if len(sys.argv) > 2 and sys.argv[1] == "--lib":  # tools only: time a variant build of libccg
    _lib.LIB_PATH = os.path.abspath(sys.argv[2])
from consensusclustr_amd import Engine  # noqa: E402


def main():
    N = int(os.environ.get("CM_N", 100000))
    B = int(os.environ.get("CM_B", 125))
    clo, chi = int(os.environ.get("CM_CLO", 2)), int(os.environ.get("CM_CHI", 40))
    reps = 3
    rng = np.random.default_rng(0)
    C = rng.integers(clo, chi + 1, B)
    A = (rng.integers(0, 1 << 30, (B, N)) % C[:, None] + 1).astype(np.uint8)
    A[rng.random((B, N)) < 0.1] = 0
    eng = Engine(0)
    At = torch.from_numpy(A).cuda()
    P = N * (N - 1) // 2
    co = torch.empty(P, dtype=torch.int16, device="cuda")
    both = torch.empty(P, dtype=torch.int16, device="cuda")
    eng.cocluster_t(At, 0, N, co=co, both=both)
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_read("cocluster")
    for _ in range(reps):
        eng.cocluster_t(At, 0, N, co=co, both=both)
    ms, cnt = eng.timing_read("cocluster")
    ms /= cnt
    ops = 2.0 * P * (int(C.sum()) + B)
    w = (torch.arange(P, device="cuda") % 1009).to(torch.int64)
    digest = [int(co.to(torch.int64).sum()), int(both.to(torch.int64).sum()), int((co.to(torch.int64) * w).sum()),
              int((both.to(torch.int64) * w).sum())]  # compares library variants
    print(json.dumps({"N": N, "B": B, "sumC": int(C.sum()), "coc_ms": ms, "tops": ops / (ms * 1e-3) / 1e12,
                      "frac_of_5000": ops / (ms * 1e-3) / 5e15, "out_GBs": 4.0 * P / (ms * 1e-3) / 1e9,
                      "digest": digest}))


if __name__ == "__main__":
    main()
