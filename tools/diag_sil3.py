"""Diagnostic: per-row widths of ccg_silhouette on the ragged synthetic
segments of tests/test_gpu_sil_segments.py against orc_silhouette, and the
distinct-cell means against the oracle means."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import diag_sil2 as D  # noqa: E402


def main():
    from consensusclustr_amd import Engine
    import test_gpu_sil_segments as T
    eng = Engine(0)
    for d in (5, 30):
        rng = np.random.default_rng(100 + d)
        segs = T._segments(rng, [40, 130, 900, 2500, 61, 6000, 300], d, 12)
        for q, (X, boot, labs, N) in enumerate(segs):
            D.check(eng, X, labs, f"d{d} seg{q}", boot=boot, ncell=N)
        D.log(f"d{d} done")
    eng.close()


if __name__ == "__main__":
    main()
