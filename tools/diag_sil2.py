"""Diagnostic: per-row silhouette widths of ccg_silhouette (want_width)
against orc_silhouette on the null-statistic and getClustAssignments inputs
of tests/test_gpu_pipeline.py, and the distinct-cell means against both.
Prints the labelings whose widths deviate and their worst rows."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def check(eng, X, lab, tag, boot=None, ncell=None):
    import oracle as O
    mean, ncl, mns, w = eng.silhouette(X, lab, want_width=True)
    cm = None
    if boot is not None:
        cm, _, _ = eng.silhouette_cells(X, lab, boot, ncell)
    for l_ in range(lab.shape[0]):
        ow, om, C = O.silhouette(X, lab[l_])
        dw = np.abs(np.nan_to_num(w[l_]) - np.nan_to_num(ow))
        bad = np.nonzero(dw > 2e-8)[0]
        cmsg = "" if cm is None else f" cells {cm[l_]:.9f} (d {cm[l_] - om:.2e})"
        if bad.size or abs(mean[l_] - om) > 1e-9 * max(1.0, abs(om)) or (cm is not None and abs(cm[l_] - om) > 1e-8):
            log(f"{tag} l={l_} C={C} cmax={lab[l_].max()} mean {mean[l_]:.9f} oracle {om:.9f}{cmsg} "
                f"rows>2e-8: {bad.size} max {dw.max():.3e}")
            for i in bad[:4]:
                log(f"   row {i} lab {lab[l_][i]} w {w[l_][i]:.12f} oracle {ow[i]:.12f}")


def main():
    from consensusclustr_amd import Engine
    import oracle as O
    import test_gpu_pipeline as T
    from consensusclustr_amd.consensus import NULL_RES_RANGE
    eng = Engine(0)
    rng = np.random.default_rng(77)
    nulls = [rng.normal(size=(int(n), d)) for n, d in [(600, 5), (750, 5), (420, 8), (900, 3)]]
    for t, X in enumerate(nulls):
        idx, _ = O.knn(X, max(T.KNUM))
        labs = []
        for k in T.KNUM:
            ei, ej, w = O.snn(idx, k, "number")
            for res in NULL_RES_RANGE:
                labs.append(T.components(X.shape[0], ei, ej, w, float(res), 123))
        check(eng, X, np.stack(labs).astype(np.int32), f"null{t}")
        log(f"null{t} done")
    pca = T._pcs()
    boots = T._boots()
    for b in (0, 9, 18):
        X = O.gather_rows(pca, boots[b])
        idx, _ = O.knn(X, max(T.KNUM))
        labs = []
        for k in T.KNUM:
            ei, ej, w = O.snn(idx, k, "number")
            for res in T.RES:
                labs.append(T.components(X.shape[0], ei, ej, w, float(res), 123))
        check(eng, X, np.stack(labs).astype(np.int32), f"boot{b}", boot=boots[b], ncell=pca.shape[0])
        log(f"boot{b} done")
    eng.close()


if __name__ == "__main__":
    main()
