/* Memory-safety check of the CPU oracle (test infrastructure, not product).
 *
 * Built with -fsanitize=address,undefined together with ccg_oracle.c
 * (`make -C oracle asan`, run by tests/test_oracle_asan.py).  Calls every
 * orc_* entry point on small seeded inputs and on the edge shapes the
 * parity tests use (one row, K = n - 1, all-NA columns, 8- and 16-bit
 * codes, the SNN capacity query), with every buffer malloc'd to its exact
 * size, so an out-of-bounds read or write, a use after free or undefined
 * arithmetic aborts the run.  Exit status 0 = every call returned the
 * expected status. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_gather_rows(const double* pcs, int64_t N, int d, const int32_t* idx, int64_t n, double* X);
int orc_knn(const double* X, int64_t n, int d, int K, int32_t* out_idx, double* out_dist, int nthreads);
int orc_knn_queries(const double* X, int64_t n, int d, int K, const int32_t* qidx, int64_t nq,
                    int32_t* out_idx, double* out_dist, int nthreads);
int orc_snn(const int32_t* knn, int64_t n, int kstride, int k, int type, int64_t* nedges, int32_t* out_i,
            int32_t* out_j, double* out_w, int64_t cap);
int orc_silhouette(const double* X, int64_t m, int d, const int32_t* labels, double* width, double* mean_out);
int orc_mapback(const int32_t* idx, int64_t n, const int32_t* labels_n, int64_t N, int32_t* out);
int orc_cocluster(const int32_t* A, int64_t N, int64_t B, uint32_t* co, uint32_t* both, double* dist,
                  int nthreads);
int orc_consensus_knn(const double* dist, int64_t N, int k, int32_t* out_idx, int nthreads);
int orc_cocluster_rows(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* rows, int64_t nr,
                       uint32_t* co, uint32_t* both, int nthreads);
int orc_consensus_knn_rows(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* rows,
                           int64_t nr, int k, int32_t* out_idx, int32_t* nan_row, int nthreads);
int orc_block_means(const double* dist, int64_t N, const int32_t* f, int K, double* out, int nthreads);
int orc_contingency(const void* A, int label_bits, int64_t N, int64_t B, const int32_t* f, int K, int C,
                    int32_t* tab);

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 16);
}
static double rndu(void) { return (rnd() & 0xFFFFFF) / 16777216.0; }

static int failures = 0;
#define EXPECT(call, want)                                                       \
    do {                                                                         \
        int rc_ = (call);                                                        \
        if (rc_ != (want)) {                                                     \
            fprintf(stderr, "%s:%d %s -> %d (want %d)\n", __FILE__, __LINE__,    \
                    #call, rc_, (want));                                         \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "out of memory\n"); exit(2); }
    return p;
}

/* kNN -> SNN (both weightings, capacity query then fill) -> silhouette and
 * map-back, for n rows in d dimensions with K neighbours. */
static void chain(int64_t N, int64_t n, int d, int K, int ncl) {
    double* pcs = xmalloc(sizeof(double) * N * d);
    for (int64_t t = 0; t < N * d; ++t) pcs[t] = (double)(rnd() % 7) + rndu();  /* some ties */
    int32_t* idx = xmalloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; ++i) idx[i] = (int32_t)(rnd() % N);
    double* X = xmalloc(sizeof(double) * n * d);
    EXPECT(orc_gather_rows(pcs, N, d, idx, n, X), 0);
    if (K >= 1 && K < n) {
        int32_t* ki = xmalloc(sizeof(int32_t) * n * K);
        double* kd = xmalloc(sizeof(double) * n * K);
        EXPECT(orc_knn(X, n, d, K, ki, kd, 2), 0);
        int64_t nq = n / 2 + 1;
        int32_t* q = xmalloc(sizeof(int32_t) * nq);
        for (int64_t t = 0; t < nq; ++t) q[t] = (int32_t)(rnd() % n);
        int32_t* qi = xmalloc(sizeof(int32_t) * nq * K);
        double* qd = xmalloc(sizeof(double) * nq * K);
        EXPECT(orc_knn_queries(X, n, d, K, q, nq, qi, qd, 2), 0);
        for (int type = 0; type < 2; ++type)
            for (int k = 1; k <= K; k += (K > 2 ? K / 2 : 1)) {
                int64_t ne = 0;
                int rc = orc_snn(ki, n, K, k, type, &ne, NULL, NULL, NULL, 0);
                if (rc != 0 && rc != -4) EXPECT(rc, 0);
                int32_t* ei = xmalloc(sizeof(int32_t) * ne);
                int32_t* ej = xmalloc(sizeof(int32_t) * ne);
                double* w = xmalloc(sizeof(double) * ne);
                EXPECT(orc_snn(ki, n, K, k, type, &ne, ei, ej, w, ne), 0);
                free(ei); free(ej); free(w);
            }
        free(q); free(qi); free(qd); free(ki); free(kd);
    }
    int32_t* lab = xmalloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; ++i) lab[i] = 1 + (int32_t)(rnd() % ncl);
    double* wid = xmalloc(sizeof(double) * n);
    double mean = 0;
    EXPECT(orc_silhouette(X, n, d, lab, wid, &mean) >= 0 ? 0 : -1, 0);
    EXPECT(orc_silhouette(X, n, d, lab, NULL, &mean) >= 0 ? 0 : -1, 0);
    int32_t* mb = xmalloc(sizeof(int32_t) * N);
    EXPECT(orc_mapback(idx, n, lab, N, mb), 0);
    free(mb); free(wid); free(lab); free(X); free(idx); free(pcs);
}

/* co-clustering, consensus kNN (from the packed distances and from the
 * assignments), block means and contingency for B bootstraps of N cells. */
static void consensus(int64_t N, int64_t B, int C, double na_frac) {
    int32_t* A = xmalloc(sizeof(int32_t) * B * N);
    uint8_t* A8 = xmalloc(B * N);
    uint16_t* A16 = xmalloc(sizeof(uint16_t) * B * N);
    for (int64_t t = 0; t < B * N; ++t) {
        int a = rndu() < na_frac ? -1 : (int)(rnd() % C);
        A[t] = a;
        A8[t] = (uint8_t)(a + 1);
        A16[t] = (uint16_t)(a + 1);
    }
    const int64_t P = N * (N - 1) / 2;
    uint32_t* co = xmalloc(sizeof(uint32_t) * P);
    uint32_t* both = xmalloc(sizeof(uint32_t) * P);
    double* dist = xmalloc(sizeof(double) * P);
    EXPECT(orc_cocluster(A, N, B, co, both, dist, 2), 0);
    EXPECT(orc_cocluster(A, N, B, NULL, NULL, dist, 2), 0);
    int has_nan = 0;
    for (int64_t t = 0; t < P; ++t) has_nan |= both[t] == 0;
    const int k = N > 4 ? 3 : (int)N - 1;
    if (k >= 1) {
        int32_t* ko = xmalloc(sizeof(int32_t) * N * k);
        EXPECT(orc_consensus_knn(dist, N, k, ko, 2), has_nan ? -3 : 0);
        free(ko);
    }
    const int64_t nr = N / 3 + 1;
    int32_t* rows = xmalloc(sizeof(int32_t) * nr);
    for (int64_t t = 0; t < nr; ++t) rows[t] = (int32_t)(rnd() % N);
    uint32_t* rco = xmalloc(sizeof(uint32_t) * nr * N);
    uint32_t* rboth = xmalloc(sizeof(uint32_t) * nr * N);
    EXPECT(orc_cocluster_rows(A8, 8, N, B, rows, nr, rco, rboth, 2), 0);
    EXPECT(orc_cocluster_rows(A16, 16, N, B, rows, nr, rco, rboth, 2), 0);
    if (k >= 1) {
        int32_t* out = xmalloc(sizeof(int32_t) * nr * k);
        int32_t* nan = xmalloc(sizeof(int32_t) * nr);
        EXPECT(orc_consensus_knn_rows(A8, 8, N, B, rows, nr, k, out, nan, 2), 0);
        EXPECT(orc_consensus_knn_rows(A16, 16, N, B, rows, nr, k, out, nan, 2), 0);
        free(out); free(nan);
    }
    const int K = N > 3 ? 3 : 1;
    int32_t* f = xmalloc(sizeof(int32_t) * N);
    for (int64_t i = 0; i < N; ++i) f[i] = (int32_t)(i % K);
    double* bm = xmalloc(sizeof(double) * K * K);
    EXPECT(orc_block_means(dist, N, f, K, bm, 2), 0);
    int32_t* tab = xmalloc(sizeof(int32_t) * B * K * (C + 1));
    EXPECT(orc_contingency(A8, 8, N, B, f, K, C, tab), 0);
    EXPECT(orc_contingency(A16, 16, N, B, f, K, C, tab), 0);
    free(tab); free(bm); free(f); free(rco); free(rboth); free(rows);
    free(co); free(both); free(dist); free(A); free(A8); free(A16);
}

int main(void) {
    chain(200, 180, 6, 10, 5);
    chain(40, 40, 3, 39, 2);   /* K = n - 1 */
    chain(30, 2, 4, 1, 1);     /* two rows, one cluster */
    chain(5, 1, 2, 0, 1);      /* one row: no kNN */
    consensus(70, 12, 6, 0.2);
    consensus(33, 3, 2, 0.0);
    consensus(2, 1, 1, 0.0);   /* one pair */
    consensus(9, 4, 3, 0.9);   /* mostly NA: never co-sampled pairs */
    if (failures) {
        fprintf(stderr, "%d unexpected status codes\n", failures);
        return 1;
    }
    printf("oracle asan check: ok\n");
    return 0;
}
