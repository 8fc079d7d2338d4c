/*
 * ccg_r.c -- the .Call glue a consensusClustR maintainer adds to reach
 * libccg.so (include/ccg.h, ABI version 6) from R.  Build with the package:
 *   src/Makevars:  PKG_CPPFLAGS = -I$(CCG_HOME)/include
 *                  PKG_LIBS     = -L$(CCG_HOME)/consensusclustr_amd -lccg -Wl,-rpath,$(CCG_HOME)/consensusclustr_amd
 * (R is not installed in the image this repository is built in, so this file
 * is written against the R C API and include/ccg.h but not compiled here;
 * tests/test_r_glue.py checks that every libccg call below matches a
 * declaration in ccg.h and that every entry point is registered.)
 *
 * Conventions
 *  - Every libccg call returns a status; on failure the glue copies
 *    ccg_last_error() and calls Rf_error only after the C frames returned
 *    (no longjmp through libccg).
 *  - R indices are 1-based, libccg's 0-based; the glue converts.
 *  - The assignment matrix is R's N x B integer matrix (cells x bootstraps,
 *    NA coded -1 as after R/consensusClust.R:408).  Its column-major memory
 *    is exactly libccg's layout (bootstrap b's N labels contiguous), so the
 *    glue only narrows it to uint8/uint16 with -1 -> 0.
 *  - A context ("ccg_ctx") or a device group ("ccg_group") lives in an
 *    external pointer with a finalizer.  Entry points marked "ctx|group"
 *    accept either; a group spreads the work over its GPUs.
 *  - HIP is not fork-safe: open the engine in the R main process, never in
 *    MulticoreParam workers (the engine replaces bplapply's fan-out).
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <stdint.h>
#include <string.h>

#include "ccg.h"

/* ------------------------------------------------------------ plumbing -- */
static char g_msg[1024];

static void fail(const char* what, int rc) {
    /* copy first: ccg_last_error() is thread-local storage of libccg */
    snprintf(g_msg, sizeof(g_msg), "%s failed (%d): %s", what, rc, ccg_last_error());
    Rf_error("%s", g_msg);
}

#define CALL(what, expr)          \
    do {                          \
        int rc_ = (expr);         \
        if (rc_ != CCG_OK) fail(what, rc_); \
    } while (0)

static SEXP tag_ctx(void) { return Rf_install("ccg_ctx"); }
static SEXP tag_group(void) { return Rf_install("ccg_group"); }

static void ctx_finalizer(SEXP p) {
    ccg_ctx* c = (ccg_ctx*)R_ExternalPtrAddr(p);
    if (c) {
        ccg_close(c);
        R_ClearExternalPtr(p);
    }
}

static void group_finalizer(SEXP p) {
    ccg_group* g = (ccg_group*)R_ExternalPtrAddr(p);
    if (g) {
        ccg_group_close(g);
        R_ClearExternalPtr(p);
    }
}

/* The engine behind an external pointer: a context, or a group (then *ctx is
 * the group's first context, for entry points without a group flavour). */
static void engine_of(SEXP e, ccg_ctx** ctx, ccg_group** grp) {
    if (TYPEOF(e) != EXTPTRSXP || !R_ExternalPtrAddr(e)) Rf_error("not an open ccg engine");
    *ctx = NULL;
    *grp = NULL;
    if (R_ExternalPtrTag(e) == tag_group()) {
        *grp = (ccg_group*)R_ExternalPtrAddr(e);
        CALL("ccg_group_ctx", ccg_group_ctx(*grp, 0, ctx));
    } else if (R_ExternalPtrTag(e) == tag_ctx()) {
        *ctx = (ccg_ctx*)R_ExternalPtrAddr(e);
    } else {
        Rf_error("not a ccg engine");
    }
}

/* R's N x B integer assignment matrix (-1 = NA) -> uint8 or uint16 codes.
 * Returns label_bits; the buffer is R_alloc'ed (freed at the end of .Call). */
static int narrow_assignments(SEXP A, void** out) {
    const R_xlen_t len = XLENGTH(A);
    const int* a = INTEGER(A);
    int mx = 0;
    for (R_xlen_t t = 0; t < len; ++t) {
        if (a[t] == NA_INTEGER || a[t] < -1 || a[t] == 0) Rf_error("assignment codes must be -1 or 1..65535");
        if (a[t] > mx) mx = a[t];
    }
    if (mx > 65535) Rf_error("cluster codes above 65535 are not supported");
    if (mx <= 255) {
        uint8_t* b = (uint8_t*)R_alloc(len, 1);
        for (R_xlen_t t = 0; t < len; ++t) b[t] = (uint8_t)(a[t] < 0 ? 0 : a[t]);
        *out = b;
        return 8;
    }
    uint16_t* b = (uint16_t*)R_alloc(len, 2);
    for (R_xlen_t t = 0; t < len; ++t) b[t] = (uint16_t)(a[t] < 0 ? 0 : a[t]);
    *out = b;
    return 16;
}

/* n x k 0-based row-major (libccg) -> n x k 1-based R matrix */
static SEXP knn_matrix(const int32_t* idx, int64_t n, int k) {
    SEXP m = PROTECT(Rf_allocMatrix(INTSXP, (int)n, k));
    int* o = INTEGER(m);
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < k; ++j) o[i + (R_xlen_t)j * n] = idx[i * k + j] + 1;
    UNPROTECT(1);
    return m;
}

/* n x ks 1-based R matrix -> n x ks 0-based row-major */
static int32_t* knn_from_r(SEXP knn, int64_t* n, int* ks) {
    *n = Rf_nrows(knn);
    *ks = Rf_ncols(knn);
    int32_t* kn = (int32_t*)R_alloc((size_t)(*n) * (*ks), sizeof(int32_t));
    const int* v = INTEGER(knn);
    for (int64_t i = 0; i < *n; ++i)
        for (int j = 0; j < *ks; ++j) kn[i * (*ks) + j] = v[i + (R_xlen_t)j * (*n)] - 1;
    return kn;
}

/* ----------------------------------------------------------- lifecycle -- */
SEXP ccg_r_open(SEXP device) {
    ccg_config cfg = {Rf_asInteger(device), 0};
    ccg_ctx* c = NULL;
    CALL("ccg_open", ccg_open(&cfg, &c));
    SEXP p = PROTECT(R_MakeExternalPtr(c, tag_ctx(), R_NilValue));
    R_RegisterCFinalizerEx(p, ctx_finalizer, TRUE);
    UNPROTECT(1);
    return p;
}

SEXP ccg_r_group_open(SEXP devices) {
    ccg_group* g = NULL;
    CALL("ccg_group_open", ccg_group_open(INTEGER(devices), Rf_length(devices), &g));
    SEXP p = PROTECT(R_MakeExternalPtr(g, tag_group(), R_NilValue));
    R_RegisterCFinalizerEx(p, group_finalizer, TRUE);
    UNPROTECT(1);
    return p;
}

SEXP ccg_r_close(SEXP e) {
    if (TYPEOF(e) == EXTPTRSXP && R_ExternalPtrAddr(e)) {
        if (R_ExternalPtrTag(e) == tag_group()) group_finalizer(e);
        else ctx_finalizer(e);
    }
    return R_NilValue;
}

SEXP ccg_r_abi_version(void) { return Rf_ScalarInteger(ccg_abi_version()); }

/* ---------------------------------------------------------------- kNN -- */
/* ctx|group.  pca: N x d double matrix; boot: n x nb integer matrix of
 * 1-based row indices (one column per bootstrap, R's sample(...) draws);
 * returns a list of nb n x kmax 1-based neighbour matrices (bootstrap-row
 * indices), attribute "fallback" = rows that took the exact path.  Each
 * bootstrap is searched over its distinct cells and expanded back to rows
 * (ccg_knn_boot); a group splits the bootstraps over its GPUs
 * (ccg_group_knn_boot).  getClustAssignments alone passes its distinct rows
 * as pca and the row -> cell map as boot. */
SEXP ccg_r_knn_boot(SEXP e, SEXP pca, SEXP boot, SEXP kmax) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = Rf_nrows(pca), n = Rf_nrows(boot);
    const int d = Rf_ncols(pca), nb = Rf_ncols(boot), k = Rf_asInteger(kmax);
    int32_t* bi = (int32_t*)R_alloc((size_t)n * nb, sizeof(int32_t));
    const int* b = INTEGER(boot);
    for (R_xlen_t t = 0; t < (R_xlen_t)n * nb; ++t) bi[t] = b[t] - 1; /* column b = bootstrap b: already nb x n row-major */
    int32_t* idx = (int32_t*)R_alloc((size_t)n * nb * k, sizeof(int32_t));
    ccg_knn_stats st;
    if (grp) CALL("ccg_group_knn_boot", ccg_group_knn_boot(grp, REAL(pca), N, d, bi, n, nb, k, idx, NULL, &st));
    else CALL("ccg_knn_boot", ccg_knn_boot(ctx, REAL(pca), N, d, bi, n, nb, k, idx, NULL, &st));
    SEXP out = PROTECT(Rf_allocVector(VECSXP, nb));
    for (int t = 0; t < nb; ++t) SET_VECTOR_ELT(out, t, knn_matrix(idx + (size_t)t * n * k, n, k));
    Rf_setAttrib(out, Rf_install("fallback"), Rf_ScalarReal((double)st.fallback));
    UNPROTECT(1);
    return out;
}

/* iterate=TRUE subclusters / null simulations: list of n_s x d_s matrices,
 * searched together; returns a list of n_s x kmax 1-based segment-local
 * neighbour matrices. */
SEXP ccg_r_knn_segments(SEXP e, SEXP mats, SEXP kmax) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int ns = Rf_length(mats), k = Rf_asInteger(kmax);
    int d = 0;
    int64_t* off = (int64_t*)R_alloc(ns + 1, sizeof(int64_t));
    off[0] = 0;
    for (int s = 0; s < ns; ++s) {
        SEXP m = VECTOR_ELT(mats, s);
        off[s + 1] = off[s] + Rf_nrows(m);
        if (Rf_ncols(m) > d) d = Rf_ncols(m);
    }
    double* rows = (double*)R_alloc((size_t)off[ns] * d, sizeof(double)); /* row-major, zero-padded dims */
    for (int s = 0; s < ns; ++s) {
        SEXP m = VECTOR_ELT(mats, s);
        const int r = Rf_nrows(m), c = Rf_ncols(m);
        const double* v = REAL(m);
        for (int i = 0; i < r; ++i)
            for (int j = 0; j < d; ++j) rows[(off[s] + i) * d + j] = j < c ? v[i + (R_xlen_t)j * r] : 0.0;
    }
    int32_t* idx = (int32_t*)R_alloc((size_t)off[ns] * k, sizeof(int32_t));
    ccg_knn_stats st;
    CALL("ccg_knn_segments", ccg_knn_segments(ctx, rows, off[ns], d, off, ns, k, idx, NULL, &st));
    SEXP out = PROTECT(Rf_allocVector(VECSXP, ns));
    for (int s = 0; s < ns; ++s) SET_VECTOR_ELT(out, s, knn_matrix(idx + off[s] * k, off[s + 1] - off[s], k));
    UNPROTECT(1);
    return out;
}

/* iterate=TRUE, one level (BASELINE config 5): pcas a list of N_s x d_s
 * matrices (the level's subclusters), boots a list of n_s x nb 1-based index
 * matrices (one column per bootstrap, like ccg_r_knn_boot).  Every bootstrap
 * of every subcluster in ONE call (ccg_knn_boot_segments); returns a list
 * (per subcluster) of lists (per bootstrap) of n_s x kmax 1-based
 * neighbour matrices, each equal to ccg_r_knn_boot's. */
SEXP ccg_r_knn_boot_segments(SEXP e, SEXP pcas, SEXP boots, SEXP kmax) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int nsub = Rf_length(pcas), k = Rf_asInteger(kmax);
    if (Rf_length(boots) != nsub) Rf_error("one bootstrap matrix per PC matrix");
    int d = 0;
    int64_t Ntot = 0, n = 0;
    int nseg = 0;
    int64_t* Nof = (int64_t*)R_alloc((size_t)nsub + 1, sizeof(int64_t));
    Nof[0] = 0;
    for (int s = 0; s < nsub; ++s) {
        SEXP p = VECTOR_ELT(pcas, s), b = VECTOR_ELT(boots, s);
        if (Rf_ncols(p) > d) d = Rf_ncols(p);
        Nof[s + 1] = Nof[s] + Rf_nrows(p);
        nseg += Rf_ncols(b);
        n += (int64_t)Rf_nrows(b) * Rf_ncols(b);
    }
    Ntot = Nof[nsub];
    double* cells = (double*)R_alloc((size_t)Ntot * d, sizeof(double)); /* row-major, zero-padded dims */
    int32_t* idx = (int32_t*)R_alloc((size_t)n, sizeof(int32_t));
    int64_t* off = (int64_t*)R_alloc((size_t)nseg + 1, sizeof(int64_t));
    off[0] = 0;
    int q = 0;
    for (int s = 0; s < nsub; ++s) {
        SEXP p = VECTOR_ELT(pcas, s), b = VECTOR_ELT(boots, s);
        const int r = Rf_nrows(p), c = Rf_ncols(p), ns = Rf_nrows(b), nb = Rf_ncols(b);
        const double* v = REAL(p);
        for (int i = 0; i < r; ++i)
            for (int j = 0; j < d; ++j) cells[(Nof[s] + i) * d + j] = j < c ? v[i + (R_xlen_t)j * r] : 0.0;
        for (int t = 0; t < nb; ++t, ++q) {
            for (int i = 0; i < ns; ++i) idx[off[q] + i] = (int32_t)(INTEGER(b)[i + (R_xlen_t)t * ns] - 1 + Nof[s]);
            off[q + 1] = off[q] + ns;
        }
    }
    int32_t* out = (int32_t*)R_alloc((size_t)n * k, sizeof(int32_t));
    ccg_knn_stats st;
    CALL("ccg_knn_boot_segments", ccg_knn_boot_segments(ctx, cells, Ntot, d, idx, n, off, NULL, nseg, k, out, NULL,
                                                        &st));
    SEXP res = PROTECT(Rf_allocVector(VECSXP, nsub));
    q = 0;
    for (int s = 0; s < nsub; ++s) {
        SEXP b = VECTOR_ELT(boots, s);
        const int ns = Rf_nrows(b), nb = Rf_ncols(b);
        SEXP lst = PROTECT(Rf_allocVector(VECSXP, nb));
        for (int t = 0; t < nb; ++t, ++q) SET_VECTOR_ELT(lst, t, knn_matrix(out + off[q] * k, ns, k));
        SET_VECTOR_ELT(res, s, lst);
        UNPROTECT(1);
    }
    UNPROTECT(1);
    return res;
}

/* ---------------------------------------------------------------- SNN -- */
/* One graph of the staged rows of the last ccg_snn_graphs call as
 * list(from, to, weight), 1-based, from < to: R allocates the vectors at the
 * exact edge count and the library decodes straight into them. */
static SEXP fetch_edge_list(ccg_ctx* ctx, int t, int64_t ne) {
    SEXP from = PROTECT(Rf_allocVector(INTSXP, ne));
    SEXP to = PROTECT(Rf_allocVector(INTSXP, ne));
    SEXP wt = PROTECT(Rf_allocVector(REALSXP, ne));
    int rc = ccg_snn_graph_fetch(ctx, t, INTEGER(from), INTEGER(to), REAL(wt), ne);
    if (rc != CCG_OK) {
        UNPROTECT(3);
        fail("ccg_snn_graph_fetch", rc);
    }
    for (int64_t q = 0; q < ne; ++q) {
        INTEGER(from)[q] += 1;
        INTEGER(to)[q] += 1;
    }
    SEXP res = PROTECT(Rf_allocVector(VECSXP, 3));
    SET_VECTOR_ELT(res, 0, from);
    SET_VECTOR_ELT(res, 1, to);
    SET_VECTOR_ELT(res, 2, wt);
    SEXP nm = PROTECT(Rf_allocVector(STRSXP, 3));
    SET_STRING_ELT(nm, 0, Rf_mkChar("from"));
    SET_STRING_ELT(nm, 1, Rf_mkChar("to"));
    SET_STRING_ELT(nm, 2, Rf_mkChar("weight"));
    Rf_setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(5);
    return res;
}

/* knn: n x ks 1-based; first k columns used; type 0 = "number", 1 = "rank".
 * Returns list(from, to, weight), 1-based, from < to.  One device pass
 * (ccg_snn_graphs), decoded on the host. */
SEXP ccg_r_snn(SEXP e, SEXP knn, SEXP k, SEXP type) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    int64_t n;
    int ks;
    int32_t* kn = knn_from_r(knn, &n, &ks);
    int kk = Rf_asInteger(k);
    int64_t ne = 0;
    CALL("ccg_snn_graphs", ccg_snn_graphs(ctx, kn, n, ks, &kk, 1, Rf_asInteger(type), &ne));
    return fetch_edge_list(ctx, 0, ne);
}

/* Every graph of kNum (ccg_snn_graphs_cells: one device pass per 4 values):
 * knn n x kst 1-based, ks the distinct k values in ascending order, cell the
 * 1-based cell of every bootstrap row (copies share one; NULL = unknown);
 * returns a list (one per k) of list(from, to, weight), 1-based, from < to. */
SEXP ccg_r_snn_multi(SEXP e, SEXP knn, SEXP ks, SEXP type, SEXP cell) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    int64_t n;
    int kst;
    int32_t* kn = knn_from_r(knn, &n, &kst);
    const int nk = Rf_length(ks);
    if (nk < 1) Rf_error("ccg_r_snn_multi: no values of k");
    int32_t* cl = NULL;
    if (cell != R_NilValue) {
        if (Rf_length(cell) != n) Rf_error("ccg_r_snn_multi: cell must have one entry per row");
        cl = (int32_t*)R_alloc((size_t)n, sizeof(int32_t));
        for (int64_t r = 0; r < n; ++r) cl[r] = INTEGER(cell)[r] - 1;
    }
    SEXP out = PROTECT(Rf_allocVector(VECSXP, nk));
    for (int c0 = 0; c0 < nk; c0 += 4) {  /* the library builds up to 4 graphs per pass */
        const int m = nk - c0 < 4 ? nk - c0 : 4;
        int kv[4];
        int64_t ne[4] = {0, 0, 0, 0};
        for (int t = 0; t < m; ++t) kv[t] = INTEGER(ks)[c0 + t];
        int rc = ccg_snn_graphs_cells(ctx, kn, n, kst, cl, kv, m, Rf_asInteger(type), ne);
        if (rc != CCG_OK) {
            UNPROTECT(1);
            fail("ccg_snn_graphs_cells", rc);
        }
        for (int t = 0; t < m; ++t) SET_VECTOR_ELT(out, c0 + t, fetch_edge_list(ctx, t, ne[t]));
    }
    UNPROTECT(1);
    return out;
}

/* --------------------------------------------------------- silhouette -- */
/* mean(approxSilhouette(x, labels[, l])[, 3], na.rm = TRUE) for every column
 * l of an m x L integer matrix of codes 1..cmax (factor codes).  Returns
 * list(mean, nclust, minsize). */
SEXP ccg_r_silhouette(SEXP e, SEXP x, SEXP labels) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t m = Rf_nrows(x);
    const int d = Rf_ncols(x);
    if (Rf_nrows(labels) != m) Rf_error("labels must have one row per row of x");
    const int L = Rf_ncols(labels);
    const int* lab = INTEGER(labels);
    int cmax = 1;
    for (R_xlen_t t = 0; t < (R_xlen_t)m * L; ++t) {
        if (lab[t] == NA_INTEGER || lab[t] < 1) Rf_error("labels must be codes >= 1");
        if (lab[t] > cmax) cmax = lab[t];
    }
    /* column l of an m x L matrix is contiguous: exactly the L x m layout */
    SEXP mean = PROTECT(Rf_allocVector(REALSXP, L));
    SEXP ncl = PROTECT(Rf_allocVector(INTSXP, L));
    SEXP mns = PROTECT(Rf_allocVector(INTSXP, L));
    int rc = ccg_silhouette(ctx, REAL(x), m, d, lab, L, cmax, REAL(mean), INTEGER(ncl), INTEGER(mns), NULL);
    if (rc != CCG_OK) {
        UNPROTECT(3);
        fail("ccg_silhouette", rc);
    }
    SEXP res = PROTECT(Rf_allocVector(VECSXP, 3));
    SET_VECTOR_ELT(res, 0, mean);
    SET_VECTOR_ELT(res, 1, ncl);
    SET_VECTOR_ELT(res, 2, mns);
    SEXP nm = PROTECT(Rf_allocVector(STRSXP, 3));
    SET_STRING_ELT(nm, 0, Rf_mkChar("mean"));
    SET_STRING_ELT(nm, 1, Rf_mkChar("nclust"));
    SET_STRING_ELT(nm, 2, Rf_mkChar("minsize"));
    Rf_setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(5);
    return res;
}

/* The same means for the bootstrap matrix x = pca[sample(...), ] whose rows
 * repeat cells: cell = match(rownames(x), unique(rownames(x))) (1-based), so
 * widths are computed once per (cell, label) (ccg_silhouette_cells). */
SEXP ccg_r_silhouette_cells(SEXP e, SEXP x, SEXP labels, SEXP cell) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t m = Rf_nrows(x);
    const int d = Rf_ncols(x);
    if (Rf_nrows(labels) != m || XLENGTH(cell) != m) Rf_error("labels and cell need one row per row of x");
    const int L = Rf_ncols(labels);
    const int* lab = INTEGER(labels);
    int cmax = 1;
    for (R_xlen_t t = 0; t < (R_xlen_t)m * L; ++t) {
        if (lab[t] == NA_INTEGER || lab[t] < 1) Rf_error("labels must be codes >= 1");
        if (lab[t] > cmax) cmax = lab[t];
    }
    int32_t* c0 = (int32_t*)R_alloc((size_t)m, sizeof(int32_t));
    int ncell = 1;
    for (int64_t r = 0; r < m; ++r) {
        c0[r] = INTEGER(cell)[r] - 1;
        if (c0[r] + 1 > ncell) ncell = c0[r] + 1;
    }
    SEXP mean = PROTECT(Rf_allocVector(REALSXP, L));
    SEXP ncl = PROTECT(Rf_allocVector(INTSXP, L));
    SEXP mns = PROTECT(Rf_allocVector(INTSXP, L));
    int rc = ccg_silhouette_cells(ctx, REAL(x), m, d, lab, L, cmax, c0, ncell, REAL(mean), INTEGER(ncl),
                                  INTEGER(mns));
    if (rc != CCG_OK) {
        UNPROTECT(3);
        fail("ccg_silhouette_cells", rc);
    }
    SEXP res = PROTECT(Rf_allocVector(VECSXP, 3));
    SET_VECTOR_ELT(res, 0, mean);
    SET_VECTOR_ELT(res, 1, ncl);
    SET_VECTOR_ELT(res, 2, mns);
    SEXP nm = PROTECT(Rf_allocVector(STRSXP, 3));
    SET_STRING_ELT(nm, 0, Rf_mkChar("mean"));
    SET_STRING_ELT(nm, 1, Rf_mkChar("nclust"));
    SET_STRING_ELT(nm, 2, Rf_mkChar("minsize"));
    Rf_setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(5);
    return res;
}

/* ------------------------------------------------------ co-clustering -- */
/* ctx|group.  1 - parDist(A, customDist) (:411-421) as the numeric vector of
 * a "dist" object (R's storage order); attributes are set in R. */
SEXP ccg_r_cocluster_dist(SEXP e, SEXP A) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = Rf_nrows(A), B = Rf_ncols(A);
    void* a;
    const int bits = narrow_assignments(A, &a);
    SEXP d = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)(N * (N - 1) / 2)));
    int rc = grp ? ccg_group_cocluster(grp, a, bits, N, B, NULL, NULL, REAL(d))
                 : ccg_cocluster(ctx, a, bits, N, B, NULL, NULL, REAL(d));
    if (rc != CCG_OK) {
        UNPROTECT(1);
        fail("ccg_cocluster", rc);
    }
    UNPROTECT(1);
    return d;
}

/* ctx|group.  kNN(jaccardDist, k)$id (:425) straight from A (the N x N
 * distance is never stored).  N x k 1-based. */
SEXP ccg_r_consensus_knn(SEXP e, SEXP A, SEXP k) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = Rf_nrows(A), B = Rf_ncols(A);
    const int kk = Rf_asInteger(k);
    void* a;
    const int bits = narrow_assignments(A, &a);
    int32_t* idx = (int32_t*)R_alloc((size_t)N * kk, sizeof(int32_t));
    int rc = grp ? ccg_group_consensus_knn_assign(grp, a, bits, N, B, kk, idx)
                 : ccg_consensus_knn_assign(ctx, a, bits, N, B, kk, idx);
    if (rc == CCG_ENAN) Rf_error("data/distances cannot contain NAs for kNN"); /* dbscan's stop() */
    if (rc != CCG_OK) fail("ccg_consensus_knn_assign", rc);
    return knn_matrix(idx, N, kk);
}

/* determineHierachy(as.matrix(jaccardDist), f, return = "distance")
 * (:463, :699-721): f = integer codes 1..K in unique(assignments) order.
 * Returns the K x K matrix (diagonal 0, dimnames set in R). */
SEXP ccg_r_block_dist(SEXP e, SEXP A, SEXP f, SEXP K) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = Rf_nrows(A), B = Rf_ncols(A);
    const int kk = Rf_asInteger(K);
    void* a;
    const int bits = narrow_assignments(A, &a);
    int32_t* f0 = (int32_t*)R_alloc((size_t)N, sizeof(int32_t));
    for (int64_t i = 0; i < N; ++i) f0[i] = INTEGER(f)[i] - 1;
    uint64_t* s = (uint64_t*)R_alloc((size_t)2 * kk * kk, sizeof(uint64_t));
    int64_t* np = (int64_t*)R_alloc((size_t)kk * kk, sizeof(int64_t));
    CALL("ccg_cluster_block_sums", ccg_cluster_block_sums(ctx, a, bits, N, B, f0, kk, s, np));
    SEXP out = PROTECT(Rf_allocMatrix(REALSXP, kk, kk));
    double* tmp = (double*)R_alloc((size_t)kk * kk, sizeof(double));
    CALL("ccg_cluster_block_means", ccg_cluster_block_means(kk, s, np, tmp));
    for (int p = 0; p < kk; ++p)
        for (int q = 0; q < kk; ++q) REAL(out)[p + (R_xlen_t)q * kk] = tmp[(R_xlen_t)p * kk + q];
    UNPROTECT(1);
    return out;
}

/* Bootstrap stability (:470-481): for every column b of A, pairwiseRand(
 * f[mask], A[mask, b], mode = "ratio", adjusted) with f = codes 1..K in
 * factor-level order.  Returns the list of K_b x K_b ratio matrices (K_b =
 * levels present in the bootstrap), which R stacks as the reference does. */
SEXP ccg_r_stability(SEXP e, SEXP A, SEXP f, SEXP K, SEXP adjusted) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = Rf_nrows(A), B = Rf_ncols(A);
    const int kk = Rf_asInteger(K), adj = Rf_asLogical(adjusted);
    void* a;
    const int bits = narrow_assignments(A, &a);
    int C = 0;
    for (R_xlen_t t = 0; t < XLENGTH(A); ++t)
        if (INTEGER(A)[t] > C) C = INTEGER(A)[t];
    int32_t* f0 = (int32_t*)R_alloc((size_t)N, sizeof(int32_t));
    for (int64_t i = 0; i < N; ++i) f0[i] = INTEGER(f)[i] - 1;
    const size_t W = (size_t)C + 1;
    int32_t* tab = (int32_t*)R_alloc((size_t)B * kk * W, sizeof(int32_t));
    CALL("ccg_contingency", ccg_contingency(ctx, a, bits, N, B, f0, kk, C, tab));
    SEXP out = PROTECT(Rf_allocVector(VECSXP, B));
    int32_t* sub = (int32_t*)R_alloc((size_t)kk * W, sizeof(int32_t));
    double* r = (double*)R_alloc((size_t)kk * kk, sizeof(double));
    for (int64_t b = 0; b < B; ++b) {
        const int32_t* t = tab + (size_t)b * kk * W;
        int kb = 0;
        for (int p = 0; p < kk; ++p) {
            int64_t sampled = 0;
            for (size_t c = 1; c < W; ++c) sampled += t[(size_t)p * W + c];
            if (sampled) memcpy(sub + (size_t)(kb++) * W, t + (size_t)p * W, sizeof(int32_t) * W);
        }
        CALL("ccg_pairwise_rand_ratio", ccg_pairwise_rand_ratio(kb, C, sub, adj, r));
        SEXP m = PROTECT(Rf_allocMatrix(REALSXP, kb, kb));
        /* bluster's pairwiseRand(mode = "ratio") fills the lower triangle only */
        for (int p = 0; p < kb; ++p)
            for (int q = 0; q < kb; ++q) REAL(m)[p + (R_xlen_t)q * kb] = q > p ? NA_REAL : r[(size_t)p * kb + q];
        SET_VECTOR_ELT(out, b, m);
        UNPROTECT(1);
    }
    UNPROTECT(1);
    return out;
}

/* ------------------------------------------------ normalisation + PCA -- */
/* The PC matrix of a cell subset (:287, :339, :369, :790): counts G x N
 * double matrix (dense), sf size factors (N), genes / cells 1-based index
 * vectors, npc components.  Returns list(x = ncells x npc, sdev).  A gene
 * with zero variance raises the error the reference's tryCatch(prcomp_irlba)
 * turns into NA (:368-378). */
SEXP ccg_r_pca(SEXP e, SEXP counts, SEXP sf, SEXP genes, SEXP cells, SEXP npc) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t G = Rf_nrows(counts), N = Rf_ncols(counts), nc = XLENGTH(cells);
    const int ng = Rf_length(genes), k = Rf_asInteger(npc);
    int32_t* g0 = (int32_t*)R_alloc((size_t)ng, sizeof(int32_t));
    int32_t* c0 = (int32_t*)R_alloc((size_t)nc, sizeof(int32_t));
    for (int t = 0; t < ng; ++t) g0[t] = INTEGER(genes)[t] - 1;
    for (int64_t t = 0; t < nc; ++t) c0[t] = INTEGER(cells)[t] - 1;
    SEXP x = PROTECT(Rf_allocMatrix(REALSXP, (int)nc, k));
    SEXP sd = PROTECT(Rf_allocVector(REALSXP, k));
    int rc = ccg_pca(ctx, REAL(counts), G, N, REAL(sf), g0, ng, c0, nc, k, REAL(x), REAL(sd));
    if (rc != CCG_OK) {
        UNPROTECT(2);
        fail("ccg_pca", rc);
    }
    SEXP res = PROTECT(Rf_allocVector(VECSXP, 2));
    SET_VECTOR_ELT(res, 0, x);
    SET_VECTOR_ELT(res, 1, sd);
    SEXP nm = PROTECT(Rf_allocVector(STRSXP, 2));
    SET_STRING_ELT(nm, 0, Rf_mkChar("x"));
    SET_STRING_ELT(nm, 1, Rf_mkChar("sdev"));
    Rf_setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(4);
    return res;
}

/* The same from a dgCMatrix's slots (x, i, p; 0-based row indices, p of
 * length N + 1), so the genes x cells matrix is never densified in R
 * (R/consensusClust.R:273-288 keeps counts sparse).  genes must be distinct. */
SEXP ccg_r_pca_csc(SEXP e, SEXP xv, SEXP ri, SEXP cp, SEXP G, SEXP sf, SEXP genes, SEXP cells, SEXP npc) {
    ccg_ctx* ctx;
    ccg_group* grp;
    engine_of(e, &ctx, &grp);
    const int64_t N = XLENGTH(cp) - 1, nc = XLENGTH(cells), nG = (int64_t)Rf_asReal(G);
    const int ng = Rf_length(genes), k = Rf_asInteger(npc);
    if (N < 1 || XLENGTH(sf) != N) Rf_error("ccg_r_pca_csc: one size factor per column is required");
    int64_t* p64 = (int64_t*)R_alloc((size_t)N + 1, sizeof(int64_t));
    for (int64_t c = 0; c <= N; ++c) p64[c] = INTEGER(cp)[c];
    int32_t* g0 = (int32_t*)R_alloc((size_t)ng, sizeof(int32_t));
    int32_t* c0 = (int32_t*)R_alloc((size_t)nc, sizeof(int32_t));
    for (int t = 0; t < ng; ++t) g0[t] = INTEGER(genes)[t] - 1;
    for (int64_t t = 0; t < nc; ++t) c0[t] = INTEGER(cells)[t] - 1;
    SEXP x = PROTECT(Rf_allocMatrix(REALSXP, (int)nc, k));
    SEXP sd = PROTECT(Rf_allocVector(REALSXP, k));
    int rc = ccg_pca_csc(ctx, REAL(xv), INTEGER(ri), p64, nG, N, REAL(sf), g0, ng, c0, nc, k, REAL(x), REAL(sd));
    if (rc != CCG_OK) {
        UNPROTECT(2);
        fail("ccg_pca_csc", rc);
    }
    SEXP res = PROTECT(Rf_allocVector(VECSXP, 2));
    SET_VECTOR_ELT(res, 0, x);
    SET_VECTOR_ELT(res, 1, sd);
    SEXP nm = PROTECT(Rf_allocVector(STRSXP, 2));
    SET_STRING_ELT(nm, 0, Rf_mkChar("x"));
    SET_STRING_ELT(nm, 1, Rf_mkChar("sdev"));
    Rf_setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(4);
    return res;
}

/* ------------------------------------------------------- registration -- */
static const R_CallMethodDef call_methods[] = {
    {"ccg_r_open", (DL_FUNC)&ccg_r_open, 1},
    {"ccg_r_group_open", (DL_FUNC)&ccg_r_group_open, 1},
    {"ccg_r_close", (DL_FUNC)&ccg_r_close, 1},
    {"ccg_r_abi_version", (DL_FUNC)&ccg_r_abi_version, 0},
    {"ccg_r_knn_boot", (DL_FUNC)&ccg_r_knn_boot, 4},
    {"ccg_r_knn_segments", (DL_FUNC)&ccg_r_knn_segments, 3},
    {"ccg_r_knn_boot_segments", (DL_FUNC)&ccg_r_knn_boot_segments, 4},
    {"ccg_r_snn", (DL_FUNC)&ccg_r_snn, 4},
    {"ccg_r_snn_multi", (DL_FUNC)&ccg_r_snn_multi, 5},
    {"ccg_r_silhouette", (DL_FUNC)&ccg_r_silhouette, 3},
    {"ccg_r_silhouette_cells", (DL_FUNC)&ccg_r_silhouette_cells, 4},
    {"ccg_r_cocluster_dist", (DL_FUNC)&ccg_r_cocluster_dist, 2},
    {"ccg_r_consensus_knn", (DL_FUNC)&ccg_r_consensus_knn, 3},
    {"ccg_r_block_dist", (DL_FUNC)&ccg_r_block_dist, 4},
    {"ccg_r_stability", (DL_FUNC)&ccg_r_stability, 5},
    {"ccg_r_pca", (DL_FUNC)&ccg_r_pca, 6},
    {"ccg_r_pca_csc", (DL_FUNC)&ccg_r_pca_csc, 9},
    {NULL, NULL, 0}};

void R_init_consensusClustR(DllInfo* dll) {
    R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
    R_useDynamicSymbols(dll, FALSE);
}
