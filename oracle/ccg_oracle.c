/*
 * ccg_oracle.c -- CPU restatement of consensusClust's bootstrap hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * engine (consensusclustr_amd/csrc).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path never
 * calls it and has no CPU fallback.
 *
 * PARITY UNPINNED: the reference (AndyCGraham/consensusClustR) is R-only, has
 * no tests / golden vectors, and R + Bioconductor are absent from this image,
 * so nothing here could be checked against outputs of the reference itself.
 * The semantics below restate the reference source where it defines them
 * (R/consensusClust.R) and the third-party algorithms it calls (bluster,
 * BiocNeighbors, dbscan; versions unpinned in DESCRIPTION:15-33) from their
 * published descriptions.  The hand-derived known-answer tests in
 * tests/golden/ pin the restatement against the reference's own code text.
 *
 * Semantics (file:line refer to /root/reference/R/consensusClust.R):
 *  - orc_gather_rows : pca[sample(...), ]                            :394
 *  - orc_knn         : bluster::clusterRows -> BiocNeighbors::findKNN :656-658
 *                      exact Euclidean, self excluded by row identity,
 *                      order = (fp64 squared distance summed unfused in
 *                      dimension order, then row index).  Distances are
 *                      sqrt of that sum.
 *  - orc_snn         : bluster::neighborsToSNNGraph(type="number")    :656
 *                      and (type="rank")                              :426
 *                      (bluster build_snn_number / build_snn_rank)
 *  - orc_silhouette  : bluster::approxSilhouette(x, clusters)[,3] and
 *                      mean(..., na.rm=TRUE)                     :447,:518,:664
 *                      long-double accumulation as R's colMeans/colSums/
 *                      sum/mean do on x86-64.
 *  - orc_mapback     : assignments[match(cellOrder, names(assignments))] :673
 *  - orc_cocluster   : customDist + 1 - parDist(...)             :411-421
 *                      overlap/U held in float, float division, widened to
 *                      double, D = 1 - sim; packed as R's "dist" (lower
 *                      triangle by columns == upper triangle by rows).
 *  - orc_consensus_knn: dbscan::kNN(jaccardDist, k)$id            :425
 *                      per-row stable order() of the distance row with the
 *                      diagonal set to +Inf; NaN distances are an error.
 *  - orc_knn_queries : orc_knn restricted to selected query rows (same
 *                      semantics; for parity checks at BASELINE sizes where
 *                      the full O(n^2 d) scan would take too long).
 *  - orc_cocluster_rows: customDist counts for selected rows i against every
 *                      j (full rows, j = i included), from the engine's
 *                      encoding of clustAssignments (:404-408): uint8/uint16
 *                      codes with 0 = NA.
 *  - orc_block_means : determineHierachy(as.matrix(jaccardDist), f,
 *                      return="distance")                      :463, :699-721
 *                      mean(distanceMatrix[c1, c2], na.rm=TRUE) with R's
 *                      two-pass long-double mean, once per unordered pair.
 *  - orc_contingency : table(ref, alt) per bootstrap column -- the counting
 *                      inside bluster::pairwiseRand(ref, alt)      :473-474
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_OK 0
#define ORC_EINVAL -1
#define ORC_ENOMEM -2
#define ORC_ENAN -3
#define ORC_ECAP -4

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

/* pcs: N x d column-major (an R numeric matrix).  X: n x d row-major. */
int orc_gather_rows(const double* pcs, int64_t N, int d, const int32_t* idx,
                    int64_t n, double* X) {
    for (int64_t i = 0; i < n; ++i) {
        int64_t r = idx[i];
        if (r < 0 || r >= N) return ORC_EINVAL;
        for (int k = 0; k < d; ++k) X[i * d + k] = pcs[(int64_t)k * N + r];
    }
    return ORC_OK;
}

/* Unfused fp64 squared distance in dimension order (x86-64 baseline has no
 * FMA; the volatile store keeps the compiler from contracting). */
static inline double sqdist(const double* a, const double* b, int d) {
    double s = 0.0;
    for (int k = 0; k < d; ++k) {
        volatile double t = a[k] - b[k];
        volatile double t2 = t * t;
        s = s + t2;
    }
    return s;
}

/* Exact kNN among the rows of X (self excluded), K <= n-1. */
int orc_knn(const double* X, int64_t n, int d, int K, int32_t* out_idx,
            double* out_dist, int nthreads) {
    if (K < 1 || K > n - 1 || d < 1) return ORC_EINVAL;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel
    {
        double* bd = (double*)malloc(sizeof(double) * (size_t)K);
        int32_t* bi = (int32_t*)malloc(sizeof(int32_t) * (size_t)K);
        if (!bd || !bi) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 16)
            for (int64_t i = 0; i < n; ++i) {
                int cnt = 0;
                const double* xi = X + i * d;
                for (int64_t j = 0; j < n; ++j) {
                    if (j == i) continue;
                    double s = sqdist(xi, X + j * d, d);
                    /* j ascending, so an equal distance never displaces an
                     * earlier (lower-index) entry: strict '<' keeps
                     * (distance, index) order. */
                    if (cnt == K && !(s < bd[K - 1])) continue;
                    int p = (cnt < K) ? cnt++ : K - 1;
                    while (p > 0 && s < bd[p - 1]) {
                        bd[p] = bd[p - 1];
                        bi[p] = bi[p - 1];
                        --p;
                    }
                    bd[p] = s;
                    bi[p] = (int32_t)j;
                }
                for (int t = 0; t < K; ++t) {
                    out_idx[i * K + t] = bi[t];
                    if (out_dist) out_dist[i * K + t] = sqrt(bd[t]);
                }
            }
        }
        free(bd);
        free(bi);
    }
    return err ? ORC_ENOMEM : ORC_OK;
}

/* The same search for the nq rows qidx[] only: out rows t = 0..nq-1. */
int orc_knn_queries(const double* X, int64_t n, int d, int K, const int32_t* qidx, int64_t nq,
                    int32_t* out_idx, double* out_dist, int nthreads) {
    if (K < 1 || K > n - 1 || d < 1) return ORC_EINVAL;
    for (int64_t t = 0; t < nq; ++t)
        if (qidx[t] < 0 || qidx[t] >= n) return ORC_EINVAL;
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel
    {
        double* bd = (double*)malloc(sizeof(double) * (size_t)K);
        int32_t* bi = (int32_t*)malloc(sizeof(int32_t) * (size_t)K);
        if (!bd || !bi) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 4)
            for (int64_t t = 0; t < nq; ++t) {
                const int64_t i = qidx[t];
                int cnt = 0;
                const double* xi = X + i * d;
                for (int64_t j = 0; j < n; ++j) {
                    if (j == i) continue;
                    double s = sqdist(xi, X + j * d, d);
                    if (cnt == K && !(s < bd[K - 1])) continue;
                    int p = (cnt < K) ? cnt++ : K - 1;
                    while (p > 0 && s < bd[p - 1]) {
                        bd[p] = bd[p - 1];
                        bi[p] = bi[p - 1];
                        --p;
                    }
                    bd[p] = s;
                    bi[p] = (int32_t)j;
                }
                for (int u = 0; u < K; ++u) {
                    out_idx[t * K + u] = bi[u];
                    if (out_dist) out_dist[t * K + u] = sqrt(bd[u]);
                }
            }
        }
        free(bd);
        free(bi);
    }
    return err ? ORC_ENOMEM : ORC_OK;
}

/* ---- SNN graphs (bluster build_snn_number / build_snn_rank) ----------- */
typedef struct {
    int32_t i, j;
    double w;
} orc_edge;

static int edge_cmp(const void* a, const void* b) {
    const orc_edge* x = (const orc_edge*)a;
    const orc_edge* y = (const orc_edge*)b;
    if (x->i != y->i) return x->i < y->i ? -1 : 1;
    if (x->j != y->j) return x->j < y->j ? -1 : 1;
    return 0;
}

/* knn: n x kstride row-major 0-based neighbour lists (self excluded); the
 * first k columns are used.  type 0 = "number", 1 = "rank".
 * Output: edges (i<j) sorted by (i, j).  If cap is too small the function
 * returns ORC_ECAP with *nedges set to the required count. */
int orc_snn(const int32_t* knn, int64_t n, int kstride, int k, int type,
            int64_t* nedges, int32_t* out_i, int32_t* out_j, double* out_w,
            int64_t cap) {
    if (k < 1 || k > kstride || (type != 0 && type != 1)) return ORC_EINVAL;
    /* hosts[x] = list of (rank, host) with x in knn(host) at 1-based rank. */
    int64_t* hcount = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    if (!hcount) return ORC_ENOMEM;
    for (int64_t h = 0; h < n; ++h)
        for (int t = 0; t < k; ++t) {
            int32_t x = knn[h * kstride + t];
            if (x < 0 || x >= n) {
                free(hcount);
                return ORC_EINVAL;
            }
            hcount[x + 1]++;
        }
    for (int64_t x = 0; x < n; ++x) hcount[x + 1] += hcount[x];
    int32_t* hhost = (int32_t*)malloc(sizeof(int32_t) * (size_t)(hcount[n] + 1));
    int32_t* hrank = (int32_t*)malloc(sizeof(int32_t) * (size_t)(hcount[n] + 1));
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int32_t* score = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
    int32_t* added = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    if (!hhost || !hrank || !fill || !score || !added) {
        free(hcount); free(hhost); free(hrank); free(fill); free(score); free(added);
        return ORC_ENOMEM;
    }
    memcpy(fill, hcount, sizeof(int64_t) * (size_t)n);
    /* bluster walks neighbour columns outer, cells inner: host lists are in
     * (rank, host) order.  Only the set matters for the result. */
    for (int t = 0; t < k; ++t)
        for (int64_t h = 0; h < n; ++h) {
            int32_t x = knn[h * kstride + t];
            int64_t p = fill[x]++;
            hhost[p] = (int32_t)h;
            hrank[p] = t + 1;
        }
    int64_t ne = 0;
    int64_t ecap = 1024;
    orc_edge* edges = (orc_edge*)malloc(sizeof(orc_edge) * (size_t)ecap);
    if (!edges) {
        free(hcount); free(hhost); free(hrank); free(fill); free(score); free(added);
        return ORC_ENOMEM;
    }
    for (int64_t j = 0; j < n; ++j) {
        int nadd = 0;
        for (int i = 0; i <= k; ++i) {
            int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
            for (int64_t p = hcount[cur]; p < hcount[cur + 1]; ++p) {
                int32_t other = hhost[p];
                if (other < j) {
                    if (type == 0) {
                        if (score[other] == 0) added[nadd++] = other;
                        score[other] += 1;
                    } else {
                        int32_t r = hrank[p] + i;
                        if (score[other] == 0) {
                            score[other] = r;
                            added[nadd++] = other;
                        } else if (score[other] > r) {
                            score[other] = r;
                        }
                    }
                }
            }
            if (cur < j) {
                if (type == 0) {
                    if (score[cur] == 0) added[nadd++] = cur;
                    score[cur] += 1;
                } else {
                    if (score[cur] == 0) {
                        score[cur] = i;
                        added[nadd++] = cur;
                    } else if (score[cur] > i) {
                        score[cur] = i;
                    }
                }
            }
        }
        for (int a = 0; a < nadd; ++a) {
            int32_t other = added[a];
            double w;
            if (type == 0)
                w = (double)score[other];
            else {
                w = (double)k - 0.5 * (double)score[other];
                if (w < 1e-6) w = 1e-6;
            }
            score[other] = 0;
            if (ne == ecap) {
                ecap *= 2;
                orc_edge* e2 = (orc_edge*)realloc(edges, sizeof(orc_edge) * (size_t)ecap);
                if (!e2) {
                    free(edges); free(hcount); free(hhost); free(hrank); free(fill);
                    free(score); free(added);
                    return ORC_ENOMEM;
                }
                edges = e2;
            }
            edges[ne].i = other; /* other < j */
            edges[ne].j = (int32_t)j;
            edges[ne].w = w;
            ++ne;
        }
    }
    qsort(edges, (size_t)ne, sizeof(orc_edge), edge_cmp);
    *nedges = ne;
    int rc = ORC_OK;
    if (ne > cap) {
        rc = ORC_ECAP;
    } else {
        for (int64_t e = 0; e < ne; ++e) {
            out_i[e] = edges[e].i;
            out_j[e] = edges[e].j;
            out_w[e] = edges[e].w;
        }
    }
    free(edges); free(hcount); free(hhost); free(hrank); free(fill); free(score); free(added);
    return rc;
}

/* ---- approxSilhouette (bluster) + mean(na.rm=TRUE) -------------------- */
static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

/* X: m x d row-major; labels: m cluster codes (any int32 values).
 * width (nullable): m silhouette widths; *mean_out = mean(width, na.rm=TRUE).
 * Returns the number of clusters (>0) or a negative error. */
int orc_silhouette(const double* X, int64_t m, int d, const int32_t* labels,
                   double* width, double* mean_out) {
    if (m < 1 || d < 1) return ORC_EINVAL;
    int32_t* u = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
    if (!u) return ORC_ENOMEM;
    memcpy(u, labels, sizeof(int32_t) * (size_t)m);
    qsort(u, (size_t)m, sizeof(int32_t), cmp_i32);
    int64_t C = 0;
    for (int64_t i = 0; i < m; ++i)
        if (i == 0 || u[i] != u[i - 1]) u[C++] = u[i];
    double* cen = (double*)malloc(sizeof(double) * (size_t)(C * d));
    double* var = (double*)malloc(sizeof(double) * (size_t)C);
    int32_t* code = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
    double* selfd = (double*)malloc(sizeof(double) * (size_t)m);
    double* othd = (double*)malloc(sizeof(double) * (size_t)m);
    double* w = width ? width : (double*)malloc(sizeof(double) * (size_t)m);
    if (!cen || !var || !code || !selfd || !othd || !w) {
        free(u); free(cen); free(var); free(code); free(selfd); free(othd);
        if (!width) free(w);
        return ORC_ENOMEM;
    }
    for (int64_t i = 0; i < m; ++i) {
        int64_t lo = 0, hi = C - 1;
        while (lo < hi) {
            int64_t mid = (lo + hi) / 2;
            if (u[mid] < labels[i]) lo = mid + 1; else hi = mid;
        }
        code[i] = (int32_t)lo;
    }
    for (int64_t c = 0; c < C; ++c) {
        int64_t nc = 0;
        for (int64_t i = 0; i < m; ++i) nc += (code[i] == c);
        /* centroid <- colMeans(xcurrent) */
        for (int k = 0; k < d; ++k) {
            long double s = 0.0L;
            for (int64_t i = 0; i < m; ++i)
                if (code[i] == c) s += X[i * d + k];
            s /= (long double)nc;
            cen[c * d + k] = (double)s;
        }
        /* clust.var <- sum(colMeans(sweep(xcurrent, 2, centroid)^2)) */
        long double tot = 0.0L;
        for (int k = 0; k < d; ++k) {
            long double s = 0.0L;
            for (int64_t i = 0; i < m; ++i)
                if (code[i] == c) {
                    double t = X[i * d + k] - cen[c * d + k];
                    double t2 = t * t;
                    s += t2;
                }
            s /= (long double)nc;
            tot += (double)s;
        }
        var[c] = (double)tot;
    }
    for (int64_t i = 0; i < m; ++i) {
        selfd[i] = INFINITY;
        othd[i] = INFINITY;
    }
    for (int64_t c = 0; c < C; ++c) {
        for (int64_t i = 0; i < m; ++i) {
            /* D <- sqrt(colSums((tx - averaged[[c]])^2) + clust.var[c]) */
            long double s = 0.0L;
            for (int k = 0; k < d; ++k) {
                double t = X[i * d + k] - cen[c * d + k];
                double t2 = t * t;
                s += t2;
            }
            double Dc = sqrt((double)s + var[c]);
            if (code[i] == c)
                selfd[i] = Dc;
            else if (Dc < othd[i])
                othd[i] = Dc;
        }
    }
    for (int64_t i = 0; i < m; ++i) {
        if (C > 1) {
            double mx = othd[i] > selfd[i] ? othd[i] : selfd[i];
            /* pmax: NaN if either is NaN */
            if (isnan(othd[i]) || isnan(selfd[i])) mx = NAN;
            w[i] = (othd[i] - selfd[i]) / mx;
        } else {
            w[i] = 0.0;
        }
    }
    if (mean_out) {
        long double s = 0.0L;
        int64_t cnt = 0;
        for (int64_t i = 0; i < m; ++i)
            if (!isnan(w[i])) {
                s += w[i];
                ++cnt;
            }
        if (cnt == 0) {
            *mean_out = NAN;
        } else {
            s /= (long double)cnt;
            if (isfinite((double)s)) {
                long double t = 0.0L;
                for (int64_t i = 0; i < m; ++i)
                    if (!isnan(w[i])) t += (w[i] - s);
                s += t / (long double)cnt;
            }
            *mean_out = (double)s;
        }
    }
    free(u); free(cen); free(var); free(code); free(selfd); free(othd);
    if (!width) free(w);
    return (int)C;
}

/* ---- map-back (first copy wins; unsampled -> -1) ---------------------- */
int orc_mapback(const int32_t* idx, int64_t n, const int32_t* labels_n,
                int64_t N, int32_t* out) {
    for (int64_t c = 0; c < N; ++c) out[c] = -1;
    /* match(cellOrder, names): first occurrence in sample order */
    for (int64_t p = n - 1; p >= 0; --p) {
        int32_t c = idx[p];
        if (c < 0 || c >= N) return ORC_EINVAL;
        out[c] = labels_n[p];
    }
    return ORC_OK;
}

/* ---- co-clustering distance (customDist) ------------------------------ */
/* A: B x N column-major labels (R's clustAssignments after cbind), -1 = NA.
 * co / both (nullable): packed upper triangle by rows (== R "dist" order),
 * N(N-1)/2 entries.  dist (nullable): 1 - (double)((float)co/(float)U). */
int orc_cocluster(const int32_t* A, int64_t N, int64_t B, uint32_t* co,
                  uint32_t* both, double* dist, int nthreads) {
    if (N < 1 || B < 1) return ORC_EINVAL;
    set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t i = 0; i < N; ++i) {
        int64_t base = i * N - i * (i + 1) / 2 - i - 1;
        for (int64_t j = i + 1; j < N; ++j) {
            uint32_t ov = 0, un = 0;
            for (int64_t b = 0; b < B; ++b) {
                int32_t a = A[b * N + i], c = A[b * N + j];
                ov += (a == c) & (a != -1);
                un += (a != -1) & (c != -1);
            }
            int64_t o = base + j;
            if (co) co[o] = ov;
            if (both) both[o] = un;
            if (dist) {
                float overlap = (float)ov, U = (float)un;
                volatile float q = overlap / U;
                double jac = (double)q;
                dist[o] = 1.0 - jac;
            }
        }
    }
    return ORC_OK;
}

/* ---- consensus kNN on the co-clustering distance (dbscan::kNN(dist)) -- */
/* dist: packed as above.  Per row i: order() of d[i, ] with d[i,i] = Inf,
 * stable (ties by ascending column index); first k ids. */
int orc_consensus_knn(const double* dist, int64_t N, int k, int32_t* out_idx,
                      int nthreads) {
    if (k < 1 || k > N - 1) return ORC_EINVAL;
    int64_t P = N * (N - 1) / 2;
    for (int64_t p = 0; p < P; ++p)
        if (isnan(dist[p])) return ORC_ENAN; /* anyNA(x) -> stop() */
    set_threads(nthreads);
    int err = 0;
#pragma omp parallel
    {
        double* bd = (double*)malloc(sizeof(double) * (size_t)k);
        int32_t* bi = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
        if (!bd || !bi) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 16)
            for (int64_t i = 0; i < N; ++i) {
                int cnt = 0;
                for (int64_t j = 0; j < N; ++j) {
                    double s;
                    if (j == i) {
                        s = INFINITY;
                    } else {
                        int64_t a = i < j ? i : j, b = i < j ? j : i;
                        s = dist[a * N - a * (a + 1) / 2 + b - a - 1];
                    }
                    if (cnt == k && !(s < bd[k - 1])) continue;
                    int p = (cnt < k) ? cnt++ : k - 1;
                    while (p > 0 && s < bd[p - 1]) {
                        bd[p] = bd[p - 1];
                        bi[p] = bi[p - 1];
                        --p;
                    }
                    bd[p] = s;
                    bi[p] = (int32_t)j;
                }
                for (int t = 0; t < k; ++t) out_idx[i * k + t] = bi[t];
            }
        }
        free(bd);
        free(bi);
    }
    return err ? ORC_ENOMEM : ORC_OK;
}

/* ---- customDist counts for selected full rows ------------------------- */
/* A: B x N column-major codes, uint8 (label_bits 8) or uint16 (16), 0 = NA.
 * For each of the nr rows rows[t]: co[t*N + j] = #{b: A_bi == A_bj != 0},
 * both[t*N + j] = #{b: A_bi != 0, A_bj != 0} for every j (j = i included). */
int orc_cocluster_rows(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* rows, int64_t nr,
                       uint32_t* co, uint32_t* both, int nthreads) {
    if (N < 1 || B < 1 || (label_bits != 8 && label_bits != 16)) return ORC_EINVAL;
    for (int64_t t = 0; t < nr; ++t)
        if (rows[t] < 0 || rows[t] >= N) return ORC_EINVAL;
    set_threads(nthreads);
    const uint8_t* A8 = (const uint8_t*)A;
    const uint16_t* A16 = (const uint16_t*)A;
    const int64_t JB = 4096;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t j0 = 0; j0 < N; j0 += JB) {
        const int64_t j1 = j0 + JB < N ? j0 + JB : N;
        for (int64_t t = 0; t < nr; ++t) {
            uint32_t* cr = co + t * N;
            uint32_t* br = both + t * N;
            for (int64_t j = j0; j < j1; ++j) cr[j] = br[j] = 0;
            const int64_t i = rows[t];
            for (int64_t b = 0; b < B; ++b) {
                if (label_bits == 8) {
                    const uint8_t* col = A8 + b * N;
                    const uint8_t a = col[i];
                    if (!a) continue;
                    for (int64_t j = j0; j < j1; ++j) {
                        cr[j] += col[j] == a;
                        br[j] += col[j] != 0;
                    }
                } else {
                    const uint16_t* col = A16 + b * N;
                    const uint16_t a = col[i];
                    if (!a) continue;
                    for (int64_t j = j0; j < j1; ++j) {
                        cr[j] += col[j] == a;
                        br[j] += col[j] != 0;
                    }
                }
            }
        }
    }
    return ORC_OK;
}

/* ---- consensus kNN of selected rows, straight from A ------------------ */
/* dbscan::kNN(jaccardDist, k)$id (R/consensusClust.R:421-425) for the rows
 * rows[0..nr) only, without the N x N distance: per row i the full co/both row
 * (the customDist counts of :411-418), D_ij = 1 - (double)((float)co/(float)U)
 * (fp32 quotient, :416), d[i,i] = Inf, stable order() (ties by ascending j),
 * first k ids.  nan_row[t] = 1 if row i has a pair with U = 0 (dbscan stop()s
 * on anyNA).  A: B x N column-major codes, uint8/uint16, 0 = NA. */
int orc_consensus_knn_rows(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* rows, int64_t nr,
                           int k, int32_t* out_idx, int32_t* nan_row, int nthreads) {
    if (N < 2 || B < 1 || k < 1 || k > N - 1 || (label_bits != 8 && label_bits != 16)) return ORC_EINVAL;
    for (int64_t t = 0; t < nr; ++t)
        if (rows[t] < 0 || rows[t] >= N) return ORC_EINVAL;
    set_threads(nthreads);
    const uint8_t* A8 = (const uint8_t*)A;
    const uint16_t* A16 = (const uint16_t*)A;
    int err = 0;
#pragma omp parallel
    {
        uint32_t* cr = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)N);
        uint32_t* br = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)N);
        double* bd = (double*)malloc(sizeof(double) * (size_t)k);
        int32_t* bi = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
        if (!cr || !br || !bd || !bi) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 1)
            for (int64_t t = 0; t < nr; ++t) {
                const int64_t i = rows[t];
                memset(cr, 0, sizeof(uint32_t) * (size_t)N);
                memset(br, 0, sizeof(uint32_t) * (size_t)N);
                for (int64_t b = 0; b < B; ++b) {
                    if (label_bits == 8) {
                        const uint8_t* col = A8 + b * N;
                        const uint8_t a = col[i];
                        if (!a) continue;
                        for (int64_t j = 0; j < N; ++j) {
                            cr[j] += col[j] == a;
                            br[j] += col[j] != 0;
                        }
                    } else {
                        const uint16_t* col = A16 + b * N;
                        const uint16_t a = col[i];
                        if (!a) continue;
                        for (int64_t j = 0; j < N; ++j) {
                            cr[j] += col[j] == a;
                            br[j] += col[j] != 0;
                        }
                    }
                }
                int cnt = 0, nan = 0;
                for (int64_t j = 0; j < N; ++j) {
                    double s;
                    if (j == i) {
                        s = INFINITY;
                    } else if (br[j] == 0) {
                        nan = 1;
                        continue;
                    } else {
                        float overlap = (float)cr[j], U = (float)br[j];
                        volatile float q = overlap / U;
                        s = 1.0 - (double)q;
                    }
                    if (cnt == k && !(s < bd[k - 1])) continue;
                    int p = (cnt < k) ? cnt++ : k - 1;
                    while (p > 0 && s < bd[p - 1]) {
                        bd[p] = bd[p - 1];
                        bi[p] = bi[p - 1];
                        --p;
                    }
                    bd[p] = s;
                    bi[p] = (int32_t)j;
                }
                for (int q = 0; q < k; ++q) out_idx[t * k + q] = q < cnt ? bi[q] : -1;
                if (nan_row) nan_row[t] = nan;
            }
        }
        free(cr);
        free(br);
        free(bd);
        free(bi);
    }
    return err ? ORC_ENOMEM : ORC_OK;
}

/* ---- determineHierachy block means (R/consensusClust.R:699-721) -------- */
/* dist packed as orc_cocluster.  f: N cluster positions 0..K-1 in
 * unique(assignments) order.  out (K x K, row-major): diagonal 0 (the matrix
 * starts at 0 and the diagonal is never written, :702-704); for p < q
 * (clust1 = p visited first, :707-716) out[p][q] = out[q][p] =
 * mean(distanceMatrix[which(f == p), which(f == q)], na.rm = TRUE): the
 * submatrix in column-major order, NaN dropped, R's mean (long-double sum,
 * divide, one long-double correction pass; summary.c).  Empty -> NaN. */
int orc_block_means(const double* dist, int64_t N, const int32_t* f, int K, double* out, int nthreads) {
    if (N < 1 || K < 1) return ORC_EINVAL;
    for (int64_t i = 0; i < N; ++i)
        if (f[i] < 0 || f[i] >= K) return ORC_EINVAL;
    int64_t* cnt = (int64_t*)calloc((size_t)K, sizeof(int64_t));
    int64_t* start = (int64_t*)calloc((size_t)K + 1, sizeof(int64_t));
    int64_t* members = (int64_t*)malloc(sizeof(int64_t) * (size_t)N);
    if (!cnt || !start || !members) {
        free(cnt); free(start); free(members);
        return ORC_ENOMEM;
    }
    for (int64_t i = 0; i < N; ++i) cnt[f[i]]++;
    for (int c = 0; c < K; ++c) start[c + 1] = start[c] + cnt[c];
    for (int c = 0; c < K; ++c) cnt[c] = 0;
    for (int64_t i = 0; i < N; ++i) members[start[f[i]] + cnt[f[i]]++] = i;  /* which(): ascending */
    for (int64_t t = 0; t < (int64_t)K * K; ++t) out[t] = 0.0;
    set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int p = 0; p < K; ++p)
        for (int q = 0; q < K; ++q) {
            if (q <= p) continue;
            const int64_t* rp = members + start[p];
            const int64_t* rq = members + start[q];
            const int64_t np_ = start[p + 1] - start[p], nq = start[q + 1] - start[q];
#define ORC_D(i, j) dist[((i) < (j) ? (i) : (j)) * N - ((i) < (j) ? (i) : (j)) * (((i) < (j) ? (i) : (j)) + 1) / 2 + \
                         ((i) < (j) ? (j) : (i)) - ((i) < (j) ? (i) : (j)) - 1]
            long double s = 0.0L;
            int64_t n = 0;
            for (int64_t b = 0; b < nq; ++b)      /* columns: clust2 samples */
                for (int64_t a = 0; a < np_; ++a) {  /* rows: clust1 samples */
                    double v = ORC_D(rp[a], rq[b]);
                    if (isnan(v)) continue;
                    s += v;
                    ++n;
                }
            double m;
            if (n == 0) {
                m = NAN;
            } else {
                s /= (long double)n;
                if (isfinite((double)s)) {
                    long double t = 0.0L;
                    for (int64_t b = 0; b < nq; ++b)
                        for (int64_t a = 0; a < np_; ++a) {
                            double v = ORC_D(rp[a], rq[b]);
                            if (!isnan(v)) t += (v - s);
                        }
                    s += t / (long double)n;
                }
                m = (double)s;
            }
#undef ORC_D
            out[(int64_t)p * K + q] = m;
            out[(int64_t)q * K + p] = m;
        }
    free(cnt); free(start); free(members);
    return ORC_OK;
}

/* ---- contingency tables of each bootstrap column vs a clustering ------ */
/* A: B x N codes (uint8/uint16, 0 = NA); f: N reference positions 0..K-1.
 * tab[(b*K + p)*(C+1) + a] = #{i : f_i = p, A_bi = a}, a = 0..C. */
int orc_contingency(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* f, int K, int C,
                    int32_t* tab) {
    if (N < 1 || B < 1 || K < 1 || C < 0 || (label_bits != 8 && label_bits != 16)) return ORC_EINVAL;
    memset(tab, 0, sizeof(int32_t) * (size_t)(B * K * (C + 1)));
    for (int64_t b = 0; b < B; ++b)
        for (int64_t i = 0; i < N; ++i) {
            int a = label_bits == 8 ? ((const uint8_t*)A)[b * N + i] : ((const uint16_t*)A)[b * N + i];
            if (a > C || f[i] < 0 || f[i] >= K) return ORC_EINVAL;
            tab[(b * K + f[i]) * (C + 1) + a]++;
        }
    return ORC_OK;
}
