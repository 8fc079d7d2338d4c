"""Normalisation + PCA of a cell subset (ccg_pca; R/consensusClust.R:287,
:339, :369, :790) against numpy's exact eigen-decomposition of the same
standardised matrix.  prcomp_irlba is approximate (tol 1e-5) and its signs
follow a random start, so the contract is the exact PCA with each
component's largest-|loading| gene positive."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _counts(rng, G, N, pops=4):
    base = rng.lognormal(-0.5, 1.2, G)
    fc = np.exp(rng.normal(0, 1.0, (pops, G)) * (rng.random((pops, G)) < 0.15))
    lab = rng.integers(0, pops, N)
    sf = rng.lognormal(0, 0.3, N)
    mu = base[None, :] * fc[lab] * sf[:, None]
    return rng.poisson(mu).T.astype(np.float64), sf  # G x N


def _reference(counts, sf, genes, cells, npc):
    Y = np.log1p(counts[np.ix_(genes, cells)] / sf[cells][None, :]).T  # cells x genes
    Z = (Y - Y.mean(0)) / Y.std(0, ddof=1)
    C = Z.T @ Z / (Z.shape[0] - 1)
    w, V = np.linalg.eigh(C)
    w, V = w[::-1][:npc], V[:, ::-1][:, :npc]
    for j in range(npc):
        if V[np.argmax(np.abs(V[:, j])), j] < 0:
            V[:, j] = -V[:, j]
    return Z @ V, np.sqrt(w), w


@pytest.mark.parametrize("G,N,ng,nc,npc", [(300, 900, 200, 700, 20), (120, 400, 120, 400, 10),
                                         (300, 900, 200, 700, 80)])  # p = 96: the host Cholesky
def test_pca_matches_exact_eigendecomposition(engine, G, N, ng, nc, npc):
    rng = np.random.default_rng(G + nc)
    counts, sf = _counts(rng, G, N)
    genes = np.sort(rng.choice(G, ng, replace=False)).astype(np.int32)
    cells = rng.choice(N, nc, replace=False).astype(np.int32)
    keep = counts[np.ix_(genes, cells)].std(1) > 0
    genes = genes[keep]
    x, sdev = engine.pca(counts, sf, genes, cells, npc)
    xr, sr, w = _reference(counts, sf, genes, cells, npc)
    assert x.shape == (cells.size, npc)
    assert np.allclose(sdev, sr, rtol=1e-10, atol=0)
    for j in range(npc):  # vectors are determined where the eigenvalue is separated
        gap = min(abs(w[j] - w[j - 1]) if j else np.inf, abs(w[j] - w[j + 1]) if j + 1 < npc else np.inf) / w[0]
        if gap > 1e-3:
            assert np.linalg.norm(x[:, j] - xr[:, j]) <= 1e-6 * np.linalg.norm(xr[:, j]), j


def test_pca_zero_variance_gene_is_reported(engine):
    from consensusclustr_amd._lib import CcgError
    rng = np.random.default_rng(5)
    counts, sf = _counts(rng, 50, 200)
    counts[7] = 0.0
    with pytest.raises(CcgError, match="ENAN"):
        engine.pca(counts, sf, None, None, 5)


def test_subset_pcs_find_rule_and_scale(engine):
    """pcNum = 'find': 50 components, then the :356 rule, at a subcluster's size."""
    from consensusclustr_amd.consensus import choose_pc_num, subset_pcs
    rng = np.random.default_rng(9)
    counts, sf = _counts(rng, 2000, 6000, pops=6)
    genes = np.flatnonzero(counts.std(1) > 0)[:1500].astype(np.int32)
    t0 = time.perf_counter()
    pcs, sdev = subset_pcs(counts, sf, genes, None, "find", 0.2, engine)
    dt = time.perf_counter() - t0
    print(f"ccg_pca 1500 genes x 6000 cells, 50 PCs: {dt:.2f} s")
    assert pcs.shape == (6000, choose_pc_num(sdev, 0.2))
    assert np.all(np.diff(sdev) <= 0)


def _csc(counts):
    from scipy.sparse import csc_matrix
    m = csc_matrix(counts)
    m.sort_indices()
    return m.data, m.indices, m.indptr


def test_pca_sparse_counts_equal_dense(engine):
    """ccg_pca_csc (dgCMatrix slots; R/consensusClust.R:273-288 normalises
    sparse counts) gives the dense path's PCs bit for bit."""
    rng = np.random.default_rng(21)
    counts, sf = _counts(rng, 300, 900)
    genes = np.flatnonzero(counts.std(1) > 0)[::2].astype(np.int32)
    cells = np.sort(rng.choice(900, 600, replace=False)).astype(np.int32)
    genes = genes[counts[np.ix_(genes, cells)].std(1) > 0]
    xd, sd = engine.pca(counts, sf, genes, cells, 15)
    xs, ss = engine.pca_csc(*_csc(counts), counts.shape[0], sf, genes, cells, 15)
    assert np.array_equal(sd, ss)
    assert np.array_equal(xd, xs)
    xr, sr, _ = _reference(counts, sf, genes, cells, 15)
    assert np.allclose(ss, sr, rtol=1e-10, atol=0)


def test_pca_sparse_rejects_bad_input_and_zero_variance(engine):
    from consensusclustr_amd._lib import CcgError
    rng = np.random.default_rng(22)
    counts, sf = _counts(rng, 60, 200)
    counts[3] = 0.0
    xv, ri, cp = _csc(counts)
    with pytest.raises(CcgError, match="ENAN"):
        engine.pca_csc(xv, ri, cp, 60, sf, None, None, 5)
    with pytest.raises(CcgError, match="selected twice"):
        engine.pca_csc(xv, ri, cp, 60, sf, np.array([1, 2, 2, 4], np.int32), None, 2)


def test_pca_production_shape_sparse(engine):
    """BASELINE cfg3's producer shape: 2000 genes x 100 000 cells, 50 PCs, from
    sparse NB-like counts (timed; tools/pca_micro.py profiles it)."""
    from scipy.sparse import random as sprandom
    rng = np.random.default_rng(23)
    G, N = 2000, 100000
    m = sprandom(G, N, density=0.08, format="csc", random_state=23, dtype=np.float64)
    m.data = np.ceil(m.data * 6.0)
    sf = rng.lognormal(0, 0.3, N)
    t0 = time.perf_counter()
    x, sdev = engine.pca_csc(m.data, m.indices, m.indptr, G, sf, None, None, 50)
    dt = time.perf_counter() - t0
    print(f"ccg_pca_csc 2000 genes x 100000 cells, 50 PCs: {dt:.2f} s")
    assert x.shape == (N, 50) and np.all(np.diff(sdev) <= 0) and np.all(np.isfinite(x))
    assert abs(np.var(x[:, 0], ddof=1) - sdev[0] ** 2) <= 1e-8 * sdev[0] ** 2
    # the whole spectrum against numpy's exact eigenvalues of the same
    # correlation matrix (sparse Y^T Y; a flat spectrum: lambda_50 / lambda_66
    # = 1.007, the case the Chebyshev filter exists for)
    Y = m.multiply(1.0 / sf[None, :]).tocsc()
    Y.data = np.log1p(Y.data)
    Yt = Y.T.tocsr()
    mu = np.asarray(Yt.mean(axis=0)).ravel()
    cov = ((Yt.T @ Yt).toarray() - N * np.outer(mu, mu)) / (N - 1)
    sd = np.sqrt(np.diag(cov))
    w = np.linalg.eigvalsh(cov / np.outer(sd, sd))[::-1][:50]
    assert np.allclose(sdev, np.sqrt(w), rtol=1e-9, atol=0)
    assert dt < 1.0
