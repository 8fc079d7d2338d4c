/*
 * ccg.h -- C ABI of libccg.so, the MI355X (gfx950) engine for the bootstrap
 * hot path of consensusClust (AndyCGraham/consensusClustR).
 *
 * Plain C: pointers, sizes and an opaque context.  No C++ or PyTorch types
 * cross this boundary.  Every function returns CCG_OK (0) or a negative
 * CCG_E* code; ccg_last_error() then returns a thread-local message.  No
 * function throws or longjmps across the ABI.
 *
 * Two flavours of each entry point:
 *   - host-pointer functions (ccg_knn_boot, ccg_snn, ...): what an R .Call
 *     glue binds.  They copy in, run, copy out and
 *     synchronise.
 *   - device-pointer functions (*_dev): inputs/outputs already in HBM,
 *     enqueued on `stream` (a hipStream_t).  NULL is HIP's legacy default
 *     stream of the current device (hipStreamLegacy; torch's default stream),
 *     as for any HIP library: the call is ordered after the caller's earlier
 *     work on that stream and on every blocking stream, so an input written
 *     just before the call is complete when the library reads it.  (Through
 *     ABI 6, NULL meant the context's own non-blocking stream.)  The
 *     context's device must be current.  No host synchronisation unless
 *     stated.
 *   - one stream at a time per context: a context's workspaces are shared
 *     by its calls, so calls on one context must not run concurrently on
 *     different streams (order them, or open one context per stream -- what
 *     bench.py does for its bootstraps in flight).  The single-pass scan
 *     keeps separate state per stream (up to 8), so a violation corrupts
 *     data but cannot hang the GPU.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   ccg_knn_boot / ccg_knn_rows_dev : BiocNeighbors::findKNN as reached by
 *       bluster::clusterRows(pca, SNNGraphParam(k, type="number"))
 *       R/consensusClust.R:656-658, on pca[sample(...), ] (:394).
 *   ccg_snn (type NUMBER)           : bluster::neighborsToSNNGraph(type="number")
 *       inside SNNGraphParam (:656-658).
 *   ccg_snn (type RANK)             : bluster::neighborsToSNNGraph(knn, type="rank")
 *       (:426).
 *   ccg_silhouette                  : mean(bluster::approxSilhouette(x, cl)[,3],
 *       na.rm=TRUE) (:447, :518, :664).
 *   ccg_select_mapback_dev          : robust selection rank(ties="first")
 *       (:684-686) + assignments[match(cellOrder, names)] (:673) + NA -> -1
 *       (:408, encoded as 0) + do.call(cbind) (:404, :688).
 *   ccg_cocluster                   : the RcppXPtrUtils customDist plugin passed
 *       to parallelDist::parDist(method="custom") and 1 - parDist(...)
 *       (:411-421).
 *   ccg_consensus_knn[_assign]      : dbscan::kNN(jaccardDist, k)$id (:425).
 *
 *   ccg_cluster_block_sums          : determineHierachy(as.matrix(jaccardDist), ...)
 *       block means (:463, :699-721).
 *   ccg_contingency                 : the counting of bluster::pairwiseRand
 *       (:470-474).
 *   ccg_pca / ccg_pca_csc           : shifted_log_transform + prcomp_irlba
 *       (:287, :339, :369, :790), dense or dgCMatrix counts.
 *
 * Errors found by a kernel on the device (a label wider than the assignment
 * matrix, an invalid SNN neighbour index) are sticky in the context and are
 * returned by the next ccg_synchronize / ccg_check_errors call.
 */
#ifndef CCG_H
#define CCG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCG_ABI_VERSION 7

#define CCG_OK 0
#define CCG_EINVAL (-1)  /* bad argument / shape */
#define CCG_ENOMEM (-2)  /* device allocation failed */
#define CCG_EHIP (-3)    /* HIP runtime error */
#define CCG_ECAP (-4)    /* caller buffer too small; required size reported */
#define CCG_ENAN (-5)    /* NaN distance where the reference stop()s */
#define CCG_ERANGE (-6)  /* label out of supported range */

#define CCG_SNN_NUMBER 0
#define CCG_SNN_RANK 1

#define CCG_MODE_ROBUST 0
#define CCG_MODE_GRANULAR 1

typedef struct ccg_ctx ccg_ctx;

typedef struct ccg_config {
    int device; /* HIP device ordinal */
    int flags;  /* reserved, 0 */
} ccg_config;

/* kNN certification statistics for the last ccg_knn_* call. */
typedef struct ccg_knn_stats {
    int64_t queries;   /* rows searched */
    int64_t fallback;  /* rows that needed the exact fp64 rescan */
} ccg_knn_stats;

int ccg_abi_version(void);
const char* ccg_last_error(void);
int ccg_open(const ccg_config* cfg, ccg_ctx** out);
int ccg_close(ccg_ctx* ctx);
/* Synchronises the device; returns the sticky device error if one was
 * raised since the last check (CCG_ERANGE / CCG_EINVAL), else CCG_OK. */
int ccg_synchronize(ccg_ctx* ctx);
int ccg_check_errors(ccg_ctx* ctx);
/* The context's default stream (hipStream_t). */
void* ccg_stream(ccg_ctx* ctx);
/* The HIP device ordinal the context runs on. */
int ccg_ctx_device(const ccg_ctx* ctx, int* device);

/* ---------------------------------------------------------------- kNN -- */
/* Exact Euclidean kNN of every bootstrap row among the other rows of the
 * same bootstrap (duplicated cells are distinct points at distance 0).
 * Order: ascending fp64 squared distance summed unfused in dimension order,
 * ties by ascending bootstrap-row index.  k = 10, 15 lists are prefixes of
 * the kmax list.
 *   pcs      : N x d float64, COLUMN-major (R matrix layout), d <= 64
 *   boot_idx : nb x n int32, 0-based cell indices (R's sample() - 1)
 *   out_idx  : nb x n x kmax int32, 0-based bootstrap-row indices
 *   out_dist : nb x n x kmax float64 (sqrt of the squared distance) or NULL
 * Requires 1 <= kmax <= min(32, n-1), n < 2^30. */
int ccg_knn_boot(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                 const int32_t* boot_idx, int64_t n, int nb, int kmax,
                 int32_t* out_idx, double* out_dist, ccg_knn_stats* stats);

/* Gather bootstrap rows: rows[i][k] = pcs_colmajor[k*N + idx[i]]. */
int ccg_gather_rows_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                        const int32_t* idx, int64_t n, double* rows,
                        void* stream);

/* The same from a ROW-major N x d copy of the PCs (pcs_rm[c*d + k]): each
 * row is d contiguous doubles, so the gather reads whole rows instead of one
 * 8-byte word per column-major line (a caller drawing many bootstraps of one
 * PC matrix transposes it once). */
int ccg_gather_rows_rm_dev(ccg_ctx* ctx, const double* pcs_rm, int64_t N, int d,
                           const int32_t* idx, int64_t n, double* rows,
                           void* stream);

/* kNN among the rows of a row-major n x d float64 matrix (device).
 * stats may be NULL; when given, the call synchronises to fill it. */
int ccg_knn_rows_dev(ccg_ctx* ctx, const double* rows, int64_t n, int d,
                     int kmax, int32_t* out_idx, double* out_dist,
                     ccg_knn_stats* stats, void* stream);

/* kNN of the bootstrap rows pcs[idx[i], ] among each other -- the contract
 * of ccg_knn_rows_dev on the gathered matrix, bit for bit -- computed over
 * the bootstrap's distinct cells (duplicated cells are copies at distance 0;
 * about 59% of the rows are distinct at cfg3, so the search does ~0.35 of
 * the n^2 work), then expanded back to rows in (d2, row index) order.
 *   pcs      : N x d float64 COLUMN-major (device; rows must be pcs[idx, ] --
 *              the distinct cells' coordinates are copied from rows)
 *   idx      : n int32 0-based cell indices (device; R's sample() - 1)
 *   n_unique : the number of distinct values in idx (host; R:
 *              length(unique(idx))), or -1 to count them on the device (one
 *              stream synchronisation).  A wrong value -- or an index outside
 *              [0, N) -- sets the sticky device error (CCG_EINVAL at the next
 *              ccg_synchronize / ccg_check_errors); outputs are then undefined.
 *   rows     : the gathered n x d rows (ccg_gather_rows_dev; read by the exact
 *              fallback for rows whose kmax-th entry is a tie the distinct-cell
 *              list may cut)
 * Requires 1 <= kmax <= min(32, n-1), 2 <= n < 2^30, d <= 63. */
int ccg_knn_boot_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                     const int32_t* idx, int64_t n, int n_unique,
                     const double* rows, int kmax, int32_t* out_idx,
                     double* out_dist, ccg_knn_stats* stats, void* stream);

/* ccg_knn_boot_dev with a warm start: cell_hint (device, N floats, in/out)
 * holds per cell a squared distance -- 0 = none -- that the cell's kq-th
 * nearest distinct cell is expected within (kq = min(kmax, n_unique - 1)).
 * The screen starts each hinted query with that radius (plus 15%) as its
 * rejection threshold instead of nothing, and on return every searched cell's
 * entry holds its certified kq-th distance for the next bootstrap of the same
 * PC matrix.  Results are bit-identical with any hint values: a hint that is
 * too tight only sends the row to the exact fallback.  Concurrent calls may
 * share one array (a raced entry is still a valid hint). */
int ccg_knn_boot_hint_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                          const int32_t* idx, int64_t n, int n_unique,
                          const double* rows, int kmax, int32_t* out_idx,
                          double* out_dist, float* cell_hint,
                          ccg_knn_stats* stats, void* stream);

/* Cell table: the K nearest OTHER cells of every one of the N cells, in
 * (fp64 squared distance, cell index) order -- the kNN contract over the N
 * cells -- with the certified squared distances.  Computed once per PC
 * matrix; every bootstrap of the same PCs then filters it
 * (ccg_knn_boot_table_dev) instead of searching.  (R/consensusClust.R:394
 * draws every bootstrap from the same cells; :656-658 searches each.)
 *   pcs     : N x d float64 COLUMN-major (device)
 *   tab_idx : N x K int32 (device), tab_d2: N x K float64 (device)
 * Requires 1 <= K <= min(48, N-1), 2 <= N < 2^30, d <= 63. */
int ccg_knn_table_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                      int K, int32_t* tab_idx, double* tab_d2,
                      ccg_knn_stats* stats, void* stream);

/* ccg_knn_boot_dev from a cell table of the same pcs (ccg_knn_table_dev):
 * each distinct cell's kq = min(kmax, n_unique - 1) nearest distinct cells
 * are the first kq entries of its table row that the bootstrap holds; a cell
 * with fewer than kq such entries among its K is searched exactly among the
 * bootstrap's distinct cells.  Bit-identical to ccg_knn_boot_dev.  With a
 * presence rate p = n_unique / N, a cell needs the exact search when fewer
 * than kq of its K table entries are present (Binomial(K, p) < kq: about
 * 0.6% of the cells at p = 0.59, K = 48, kq = 20).  stats->fallback counts
 * those cells plus the rows of cut ties. */
int ccg_knn_boot_table_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                           const int32_t* idx, int64_t n, int n_unique,
                           const double* rows, int kmax,
                           const int32_t* tab_idx, const double* tab_d2, int K,
                           int32_t* out_idx, double* out_dist,
                           ccg_knn_stats* stats, void* stream);

/* A batch of nb bootstraps of the same PCs through ONE set of launches of
 * ccg_knn_boot_table_dev's path (the bootstrap loop of R/consensusClust.R:
 * 391-400 with :656-658's findKNN on each pca[sample(...), ]): every
 * bootstrap gets ccg_knn_boot_table_dev's result, bit for bit.
 *   idx      : device, nb x n int32 cell indices (bootstrap s = idx[s n ..
 *              (s+1) n), R's sample() - 1)
 *   n_unique : HOST, nb values: each bootstrap's length(unique(idx_s)), each
 *              >= kmax + 1 (a wrong value sets the sticky device error)
 *   rows     : device, (nb n) x d row-major: the gathered rows of every
 *              bootstrap (ccg_gather_rows_rm_dev on the whole idx)
 *   tab_idx / tab_d2 / K : the cell table of the same pcs (ccg_knn_table_dev)
 *   local_ids: 1 = out_idx holds each bootstrap's own row indices (0 .. n-1),
 *              0 = rows of the concatenation (s n + i: the disjoint union of
 *              the nb graphs, ready for one ccg_snn_classes_dev pass)
 *   out_idx  : device, (nb n) x kmax; out_dist optional (nb n) x kmax
 * Requires 1 <= nb <= 64, nb n < 2^30, nb N < 2^31 - 1, kmax <= 32.  No host
 * synchronisation (unless stats).  ccg_knn_last_fallback then returns the
 * rows of cut ties (ids of the concatenation). */
int ccg_knn_boots_table_dev(ccg_ctx* ctx, int64_t N, int d, const int32_t* idx, int64_t n, int nb,
                            const int* n_unique, const double* rows, int kmax,
                            const int32_t* tab_idx, const double* tab_d2, int K, int local_ids,
                            int32_t* out_idx, double* out_dist, ccg_knn_stats* stats,
                            void* stream);

/* The bootstrap kNN of many small PC matrices in one set of launches:
 * iterate=TRUE (R/consensusClust.R:541-567, BASELINE config 5) re-runs the
 * bootstrap loop (:391-400) on every subcluster of a level.  One segment =
 * one bootstrap of one subcluster; every segment gets ccg_knn_boot_dev's
 * result (the distinct-cell search, bit for bit), all segments together:
 *   cells      : Ntot x d float64 ROW-major (device): the subclusters' PC
 *                matrices stacked (zero-pad a smaller pcNum: padding dims do
 *                not change distances)
 *   idx        : n int32 (device): segment s's rows are idx[seg_off[s] ..
 *                seg_off[s+1]), each a row of `cells` (its subcluster's block;
 *                R's sample() - 1 plus the block start)
 *   seg_off    : HOST, nseg + 1 offsets (0 .. n)
 *   seg_unique : HOST, nseg: the distinct values of each segment (R:
 *                length(unique(...))); each must be >= kmax + 1
 *   local_ids  : 1 = out_idx holds segment-local bootstrap-row indices
 *                (ccg_knn_boot_dev's), 0 = rows of the concatenation (the
 *                disjoint union graph, ready for one ccg_snn_rows_dev call)
 * Requires nseg * Ntot < 2^31 (split larger batches).  Synchronises the stream
 * before returning (a small host plan is uploaded). */
int ccg_knn_boot_segments_dev(ccg_ctx* ctx, const double* cells, int64_t Ntot, int d,
                              const int32_t* idx, int64_t n, const int64_t* seg_off,
                              const int* seg_unique, int nseg, int kmax, int local_ids,
                              int32_t* out_idx, double* out_dist, ccg_knn_stats* stats,
                              void* stream);
/* Host flavour (cells, idx, outputs host; segment-local ids); seg_unique may
 * be NULL (counted on the host). */
int ccg_knn_boot_segments(ccg_ctx* ctx, const double* cells, int64_t Ntot, int d,
                          const int32_t* idx, int64_t n, const int64_t* seg_off,
                          const int* seg_unique, int nseg, int kmax, int32_t* out_idx,
                          double* out_dist, ccg_knn_stats* stats);

/* Diagnostics: the rows that the last kNN call on this context sent to the
 * exact fp64 search -- certification failures of ccg_knn_rows_dev /
 * ccg_knn_table_dev (cells, for the table), and in the bootstrap paths the
 * rows whose kmax-th entry was a tie the distinct-cell list may cut (not the
 * distinct cells searched exactly for lack of table entries).  *count gets
 * their number, the first min(count, cap) go to rows (host).  Synchronises
 * the device.  Lets a test check exactly the rows the fast paths did not
 * settle. */
int ccg_knn_last_fallback(ccg_ctx* ctx, int32_t* rows, int64_t cap, int64_t* count);

/* Batched kNN over independent segments: the iterate=TRUE subclustering
 * (R/consensusClust.R:541-566, BASELINE config 5) runs one bootstrap loop per
 * subcluster; their (small) bootstrap matrices are searched in ONE set of
 * launches.  rows: the segments' row-major n_s x d matrices concatenated
 * (n = sum n_s rows, one common d -- zero-pad smaller pcNum; padding dims do
 * not change distances).  seg_off: HOST array of nseg+1 row offsets (0 ..
 * n).  Each row's neighbours are searched within its own segment only and
 * returned as segment-local 0-based indices, in the same order and tie
 * contract as ccg_knn_rows_dev.  Requires n_s >= kmax + 1 for every segment.
 * rows / out_idx / out_dist are device pointers; the call uploads a small
 * plan and synchronises `stream` before returning. */
int ccg_knn_segments_dev(ccg_ctx* ctx, const double* rows, int64_t n, int d,
                         const int64_t* seg_off, int nseg, int kmax,
                         int32_t* out_idx, double* out_dist,
                         ccg_knn_stats* stats, void* stream);
/* Host flavour of ccg_knn_segments_dev (all pointers host). */
int ccg_knn_segments(ccg_ctx* ctx, const double* rows, int64_t n, int d,
                     const int64_t* seg_off, int nseg, int kmax,
                     int32_t* out_idx, double* out_dist, ccg_knn_stats* stats);

/* ---------------------------------------------------------------- SNN -- */
/* Shared-nearest-neighbour graph from the first k columns of an n x kstride
 * int32 0-based neighbour matrix (self excluded).  Edges i < j sorted by
 * (i, j).  NUMBER: w = |N+(i) & N+(j)|, N+(x) = {x} u knn(x).  RANK:
 * w = max(k - r/2, 1e-6), r = min over shared s of rank_i(s) + rank_j(s),
 * self rank 0, neighbours 1..k.
 * Host flavour: if cap < required, returns CCG_ECAP with *nedges = required
 * (call with cap = 0 to size; the graph stays staged for
 * ccg_snn_graph_fetch(ctx, 0, ...)). */
int ccg_snn(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, int k,
            int type, int32_t* out_i, int32_t* out_j, double* out_w,
            int64_t cap, int64_t* nedges);

/* Device flavour: writes min(E, cap) edges and E to *d_nedges (device
 * int64); no host synchronisation.  If E > cap the caller re-runs with a
 * larger cap; a negative *d_nedges means the row reservation
 * (ccg_snn_reserve) was too small. */
int ccg_snn_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride,
                int k, int type, int32_t* out_i, int32_t* out_j,
                double* out_w, int64_t cap, int64_t* d_nedges, void* stream);

/* Several graphs in one pass: ks[0..nk) ascending (nk <= 4, ks <= 32) -- the
 * kNum loop of getClustAssignments (:653) over one kmax neighbour matrix.
 * Graph t goes to out_i[t]/out_j[t]/out_w[t] (capacity caps[t]); its edge
 * count to *d_nedges[t] (device int64). */
int ccg_snn_multi_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n,
                      int kstride, const int* ks, int nk, int type,
                      int32_t* const* out_i, int32_t* const* out_j,
                      double* const* out_w, const int64_t* caps,
                      int64_t* const* d_nedges, void* stream);

/* Host flavour of ccg_snn_multi_dev (knn, outputs and caps host; nedges a
 * host array of nk counts): ccg_snn_graphs + ccg_snn_graph_fetch of every
 * graph.  If some caps[t] < nedges[t] (call with caps all 0 to size) returns
 * CCG_ECAP with every nedges[t] set and no edges copied; the graphs stay
 * staged, so a caller may fetch them (ccg_snn_graph_fetch) instead of calling
 * again. */
int ccg_snn_multi(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride,
                  const int* ks, int nk, int type, int32_t* const* out_i,
                  int32_t* const* out_j, double* const* out_w, const int64_t* caps,
                  int64_t* nedges);

/* The kNum graphs for a HOST consumer (igraph::make_graph + cluster_leiden,
 * R/consensusClust.R:656-658): ONE device pass -- for NUMBER graphs the
 * kernels of ccg_snn_classes_dev below (class-level rows), for RANK graphs or
 * an input that breaks the class contract those of ccg_snn_rows_dev (union
 * rows) -- then the rows (8 B per class / union edge: partner + packed
 * per-graph values), each graph's per-row offsets and the row -> class map
 * are copied to pinned host memory owned by the context, and nedges[t]
 * (host, nk entries) receives graph ks[t]'s row-level edge count.  No edge
 * list is formed on the device.  ks ascending, nk <= 4, ks <= 32.
 * Synchronises. */
int ccg_snn_graphs(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks, int nk, int type,
                   int64_t* nedges);
/* ccg_snn_graphs for bootstrap rows whose copies are known: cell (host, n
 * entries, may be NULL) names each row's cell (R: match(rownames(pca),
 * unique(rownames(pca))) - 1); only rows of one cell join a row class (see
 * ccg_snn_classes_dev).  ccg_snn_graphs is this with cell = NULL. */
int ccg_snn_graphs_cells(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                         const int* ks, int nk, int type, int64_t* nedges);
/* Graph t (0 <= t < nk) of the last ccg_snn_graphs call on this context,
 * decoded on the host from the staged rows (no device work): edges i < j
 * sorted by (i, j), weights as ccg_snn.  Any output may be NULL; cap < the
 * edge count returns CCG_ECAP.  May be called any number of times until the
 * next ccg_snn_graphs / ccg_snn / ccg_snn_multi call. */
int ccg_snn_graph_fetch(ccg_ctx* ctx, int t, int32_t* out_i, int32_t* out_j, double* out_w, int64_t cap);

/* The same graphs as rows (CSR of the union graph = the largest k, built in
 * one pass): row j = partners p > j of node j in ascending order,
 * nbr[row_off[j] .. row_off[j] + row_len[j]) with wpk = per-graph packed
 * values (byte t: NUMBER count / RANK rank sum r of graph ks[t]; absent =
 * 0 / 0xFF; weight = count or max(ks[t] - r/2, 1e-6)).  Row capacities are
 * the node's item counts, so row_off (device int64, n+1) is capacity-based
 * and row_len (device int32, n) gives the used length.  d_nedges[t] (device
 * int64, nk entries) receives graph t's edge count, or -(required row
 * capacity) when it exceeds cap (rows are then not written; rerun with a
 * larger cap).  No host synchronisation.  This is the compact form a caller
 * hands to host clustering (8 B per union edge instead of 16 B per edge per
 * graph). */
int ccg_snn_rows_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride,
                     const int* ks, int nk, int type, int64_t* row_off,
                     int32_t* row_len, int32_t* nbr, uint32_t* wpk, int64_t cap,
                     int64_t* d_nedges, void* stream);
/* The NUMBER graphs of a bootstrap at the level of ROW CLASSES: the rows
 * chained by equal N+ sets (every k of ks; the copies of a cell, whose kNN
 * lists list each other first and then the same rows) form a class, and
 *   w_k(x, y) = sum over classes c of min(t_x(c), t_y(c)),
 * t_x(c) = the rows of c in N+_k(x) -- a prefix of c's rows in row order,
 * because copies of one point sit at equal distance from every row, ordered
 * by row index (the kNN contract).  So the graph of the classes carries every
 * row-level weight: rows x of class C and y of class H get w(C, H), two rows of
 * one class get k + 1.  One pass builds it; nothing row-level is written.
 *   cell      : device, n entries or NULL: only rows of one cell share a class
 *   row_class : device int32 n: class ordinal of every row (classes are
 *               numbered in the order of their lowest row)
 *   class_root: device int32 n (u used): lowest row of every class
 *   class_off : device int64 n + 1: capacity-based row offsets over class
 *               ordinals (entries from u on are empty); class_len: used lengths;
 *               nbr / wpk: partners H > C in ascending order with per-graph
 *               packed weights (byte t = w of graph ks[t], 0 = no edge),
 *               written when class_off[n] <= cap
 *   d_info    : device int64, 3 + nk: u, status (0: valid; 1: the input breaks
 *               the class contract -- a class's rows out of row order in some
 *               list -- use ccg_snn_rows_dev), required row capacity, then per
 *               graph its class-edge count (or -(required capacity) when it
 *               exceeds cap: rows not written).
 * Requires ks ascending, nk <= 4, ks[0] <= 14.  No host synchronisation.
 * ccg_snn_graphs(_cells) runs these kernels for a host consumer and expands
 * the rows on the host. */
int ccg_snn_classes_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                        const int* ks, int nk, int32_t* row_class, int32_t* class_root, int64_t* class_off,
                        int32_t* class_len, int32_t* nbr, uint32_t* wpk, int64_t cap, int64_t* d_info,
                        void* stream);

/* Row entries the per-graph functions reserve in the context workspace
 * (0 = the default 40 n (kmax+1)); ccg_snn grows it on demand, the _dev
 * functions report -(required) in d_nedges instead. */
int ccg_snn_reserve(ccg_ctx* ctx, int64_t entries);

/* --------------------------------------------------------- silhouette -- */
/* mean(approxSilhouette(x, labels_l)[,3], na.rm=TRUE) for L label vectors
 * over the same m x d float64 row-major matrix.  labels: L x m int32 codes
 * in [1, cmax], cmax <= 2^24 (workspace grows with L x cmax x d).  Outputs (length L): mean width (NaN if every
 * width is NaN), number of distinct clusters, smallest cluster size.
 * out_width (L x m) may be NULL. */
int ccg_silhouette(ccg_ctx* ctx, const double* x, int64_t m, int d,
                   const int32_t* labels, int L, int cmax, double* out_mean,
                   int32_t* out_nclust, int32_t* out_minsize,
                   double* out_width);
int ccg_silhouette_dev(ccg_ctx* ctx, const double* x, int64_t m, int d,
                       const int32_t* labels, int L, int cmax,
                       double* out_mean, int32_t* out_nclust,
                       int32_t* out_minsize, double* out_width, void* stream);

/* The same means for bootstrap rows that repeat cells: cell[r] (device, m
 * entries in [0, ncell)) names row r's cell -- R's sample() indices -- and
 * rows of one cell must be identical (bootstrap copies).  Widths are
 * computed once per (cell, label) and weighted by the number of copies
 * sharing it; cluster sums, counts and the mean are over every row, as in
 * ccg_silhouette_dev (same fixed-point reductions, so deterministic).  No
 * per-row widths. */
int ccg_silhouette_cells_dev(ccg_ctx* ctx, const double* x, int64_t m, int d,
                             const int32_t* labels, int L, int cmax,
                             const int32_t* cell, int64_t ncell, double* out_mean,
                             int32_t* out_nclust, int32_t* out_minsize, void* stream);

/* A batch of segments in one launch set (an iterate=TRUE level scores every
 * subcluster's bootstraps, R/consensusClust.R:562-566 and :664): segment s
 * is rows [seg_off[s], seg_off[s+1]) of x (device, seg_off[nseg] x d,
 * row-major), labelled by labels[s] (device, L x m_s int32 codes in
 * [1, cmax]); cell (device, seg_off[nseg] entries in [0, ncell)) names each
 * row's cell and must differ between rows of different segments (e.g. slot
 * x ncell_per_slot + cell).  seg_off and the pointer arrays labels,
 * out_mean, out_nclust, out_minsize (nseg entries each, each entry a device
 * pointer to L values or NULL; the arrays themselves may be NULL) are host
 * memory.  Results equal nseg calls of ccg_silhouette_cells_dev (the
 * fixed-point scales are taken over the whole batch).  Segments must be
 * non-empty.  Replaces: bluster::approxSilhouette at R/consensusClust.R:664
 * per (subcluster, bootstrap). */
int ccg_silhouette_segments_dev(ccg_ctx* ctx, const double* x, int d, int nseg,
                                const int64_t* seg_off, const int32_t* const* labels,
                                int L, int cmax, const int32_t* cell, int64_t ncell,
                                double* const* out_mean, int32_t* const* out_nclust,
                                int32_t* const* out_minsize, void* stream);

/* Host flavour of ccg_silhouette_cells_dev (all pointers host): what an R
 * getClustAssignments calls with the bootstrap matrix pca[sample(...), ] and
 * cell = match(rownames, unique(rownames)) - 1. */
int ccg_silhouette_cells(ccg_ctx* ctx, const double* x, int64_t m, int d,
                         const int32_t* labels, int L, int cmax, const int32_t* cell,
                         int64_t ncell, double* out_mean, int32_t* out_nclust,
                         int32_t* out_minsize);

/* ----------------------------------------------- selection + map-back -- */
/* For nb bootstraps with L clusterings each (labels nb x L x n int32,
 * codes 1..2^label_bits - 1), map labels back to the N cells (first copy in
 * sample order wins; unsampled -> 0) and write columns of the column-major
 * assignment matrix A (B x N, uint8 for label_bits 8, uint16 for 16) starting
 * at column col0.
 *   ROBUST  : one column per bootstrap, the clustering chosen by the
 *             per-bootstrap score rules (:662-670) and rank(ties="first")
 *             (:685-686) from means/nclust/minsize (nb x L);
 *             out_choice (nb, nullable) receives the chosen index.
 *   GRANULAR: L columns per bootstrap (:688).
 * A label outside [1, 2^label_bits - 1] is stored as 0 and raises the sticky
 * CCG_ERANGE (reported by ccg_synchronize / ccg_check_errors). */
int ccg_select_mapback_dev(ccg_ctx* ctx, int mode, const int32_t* labels,
                           const int32_t* boot_idx, int64_t n, int nb, int L,
                           int64_t N, const double* means,
                           const int32_t* nclust, const int32_t* minsize,
                           int min_size, void* A, int label_bits, int64_t col0,
                           int32_t* out_choice, void* stream);

/* ------------------------------------------------------- co-clustering -- */
/* A: the assignment matrix as R holds it (N cells x B bootstraps,
 * column-major: bootstrap b's N labels are contiguous at A + b*N), uint8
 * (label_bits 8) or uint16 (label_bits 16) codes, 0 = not sampled (R's -1),
 * 1.. = cluster code.
 * B <= 65535 (uint16 counts; columns are accumulated in chunks of 16383).
 * For the rows [r0, r1) of the packed upper triangle (row i holds
 * j = i+1..N-1; this is exactly the order of R's "dist" object) writes
 *   co   : #{b : A_bi == A_bj != 0}         (uint16)
 *   both : #{b : A_bi != 0 and A_bj != 0}   (uint16)
 *   dist : 1 - (double)((float)co / (float)both)  (NaN when both == 0)
 * Any output may be NULL.  Slab element (i, j) lives at
 * i*N - i*(i+1)/2 + (j-i-1) - (r0*N - r0*(r0+1)/2).
 * r0 must be a multiple of 128 (CCG_COCLUSTER_ROW_ALIGN) unless r0 == r1.
 * label_bits 16 synchronises the stream once (slot-table sizing). */
#define CCG_COCLUSTER_ROW_ALIGN 128
int ccg_cocluster(ccg_ctx* ctx, const void* A, int label_bits, int64_t N,
                  int64_t B, uint16_t* co, uint16_t* both, double* dist);
int ccg_cocluster_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N,
                      int64_t B, int64_t r0, int64_t r1, uint16_t* co,
                      uint16_t* both, double* dist, void* stream);

/* --------------------------------------------------- consensus kNN -- */
/* kNN on the co-clustering distance from packed (full, r0 = 0) co/both:
 * per row, ascending distance with ties by ascending column index, self
 * excluded.  Returns CCG_ENAN if any pair has both == 0 (dbscan stop()s). */
int ccg_consensus_knn(ccg_ctx* ctx, const uint16_t* co, const uint16_t* both,
                      int64_t N, int k, int32_t* out_idx);
int ccg_consensus_knn_dev(ccg_ctx* ctx, const uint16_t* co,
                          const uint16_t* both, int64_t N, int k,
                          int32_t* out_idx, int32_t* d_nan_flag, void* stream);
/* The same kNN straight from the assignment matrix, fused with the
 * co-clustering GEMM: rows [r0, r1) (r0 a multiple of 128) are processed in
 * sub-slabs whose full rows of (co, both) live only in a bounded workspace
 * (<= 4 GB), so the N x N matrix is never stored.  out_idx rows r0..r1-1 of
 * an N x k int32 matrix (0-based).  *d_nan_flag (device) is set to 1 if any
 * pair in those rows was never co-sampled. */
int ccg_consensus_knn_assign(ccg_ctx* ctx, const void* A, int label_bits,
                             int64_t N, int64_t B, int k, int32_t* out_idx);
int ccg_consensus_knn_assign_dev(ccg_ctx* ctx, const void* A, int label_bits,
                                 int64_t N, int64_t B, int k, int64_t r0,
                                 int64_t r1, int32_t* out_idx,
                                 int32_t* d_nan_flag, void* stream);

/* ------------------------------------- cluster distances and stability -- */
/* determineHierachy(as.matrix(jaccardDist), f, return="distance")
 * (R/consensusClust.R:463, :585, :621, :699-721) without the N x N matrix.
 * f: N cluster positions in [0, K) (device for _dev).  For every packed pair
 * i < j with both_ij > 0 (NaN pairs are dropped, na.rm=TRUE):
 *   simsum[2 (f_i K + f_j) + {0, 1}] += sim_ij * 2^39 as a 128-bit (lo, hi)
 *       integer, sim_ij = (float)co_ij / (float)both_ij (exact: every such
 *       ratio is a multiple of 2^-39);
 *   npairs[f_i K + f_j] += 1.
 * The sums are exact, so merging clusters is adding entries.  N < 2^24. */
int ccg_cluster_block_sums(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                           const int32_t* f, int K, uint64_t* simsum, int64_t* npairs);
int ccg_cluster_block_sums_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                               const int32_t* f, int K, uint64_t* simsum, int64_t* npairs, void* stream);
/* Host-only: the K x K determineHierachy matrix from the sums: diagonal 0,
 * out[p][q] = mean of D = 1 - sim over the pairs between p and q (both
 * orientations), NaN if there are none. */
int ccg_cluster_block_means(int K, const uint64_t* simsum, const int64_t* npairs, double* out);
/* Contingency of every bootstrap column against a clustering -- the counting
 * inside bluster::pairwiseRand(f[mask], A[, b][mask]) (:470-474):
 * tab[(b K + p)(C + 1) + a] = #{i : f_i = p, A_bi = a}, a = 0..C (0 = not
 * sampled).  A label above C raises the sticky CCG_ERANGE. */
int ccg_contingency(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, const int32_t* f,
                    int K, int C, int32_t* tab);
int ccg_contingency_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                        const int32_t* f, int K, int C, int32_t* tab, void* stream);
/* Host-only: pairwiseRand(mode="ratio", adjusted) from one K x (C+1) table
 * (column 0 ignored): diagonal = fraction of the pairs inside ref cluster p
 * that share an alt cluster, off-diagonal = fraction of the pairs across p
 * and q that alt splits; adjusted: (obs - E) / (total - E) with E under
 * random alt labels.  0/0 -> NaN. */
int ccg_pairwise_rand_ratio(int K, int C, const int32_t* tab, int adjusted, double* out);

/* ---------------------------------------------- normalisation + PCA -- */
/* The producer of a (sub)cluster's PC matrix (R/consensusClust.R:287, :339,
 * :369, :790; iterate=TRUE re-runs it per cluster):
 *   norm = log1p(counts[genes, cells] / sf[cells])   shifted_log_transform
 *                                                     with pseudo_count 1
 *   pca  = prcomp_irlba(t(norm), npc, center = rowMeans2(norm),
 *                       scale = rowSds(norm))
 * counts: G x N column-major doubles (R's gene x cell matrix); sf: N size
 * factors; genes: ng 0-based rows (the variable features); cells: nc 0-based
 * columns.  Outputs: x (nc x npc, column-major = pca$x) and sdev (npc,
 * descending; a HOST array in both flavours).  The PCA is exact (subspace
 * iteration to a 1e-11 relative eigen-residual; irlba stops at 1e-5).  Each
 * component's sign puts its largest-|loading| gene positive (irlba's signs
 * follow its random start).  CCG_ENAN if a selected gene has zero variance
 * among the cells (prcomp_irlba fails there; the reference then returns one
 * cluster, :371-378).  Requires 1 <= npc < min(ng, nc). */
int ccg_pca(ccg_ctx* ctx, const double* counts, int64_t G, int64_t N, const double* sf,
            const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc, double* x,
            double* sdev);
int ccg_pca_dev(ccg_ctx* ctx, const double* counts, int64_t G, int64_t N, const double* sf,
                const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc, double* x,
                double* sdev, void* stream);
/* The same from sparse counts as R's dgCMatrix holds them (compressed
 * columns; R/consensusClust.R:273-288 normalises sparse matrices): column c's
 * nonzeros are xv[cp[c] .. cp[c+1]) at gene rows ri[] (0-based, cp has N+1
 * entries, cp[0] = 0).  genes must be distinct.  The dense G x N matrix is
 * never formed; only the selected genes x cells are, on the device.  The
 * device flavour takes gpos (G entries: the position of each gene in the
 * selection, or -1) instead of genes. */
int ccg_pca_csc(ccg_ctx* ctx, const double* xv, const int32_t* ri, const int64_t* cp, int64_t G, int64_t N,
                const double* sf, const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc,
                double* x, double* sdev);
int ccg_pca_csc_dev(ccg_ctx* ctx, const double* xv, const int32_t* ri, const int64_t* cp, int64_t G, int64_t N,
                    const double* sf, const int32_t* gpos, int ng, const int32_t* cells, int64_t nc, int npc,
                    double* x, double* sdev, void* stream);

/* ------------------------------------------------------------ multi-GPU -- */
/* A device group: one context (stream + workspaces) per device and one RCCL
 * communicator per device over xGMI.  The reference runs bootstraps on
 * BiocParallel workers and parDist on RcppParallel threads of one node
 * (R/consensusClust.R:391-421); the group is that fan-out across GPUs:
 *   bootstraps  -> contiguous blocks per rank (ccg_boot_shard), no traffic;
 *   co-cluster  -> one all-gather of the assignment columns, then row slabs
 *                  of the packed triangle balanced by pair count
 *                  (ccg_row_slabs), each kept by its device;
 *   consensus kNN -> equal full-row slabs (ccg_rect_slabs), then an
 *                  all-gather of the N x k neighbour matrix.
 * Arrays indexed by "local device" l have one entry per device this process
 * drives (ccg_group_info nlocal); rank of local l = first_rank + l. */
#define CCG_GROUP_ID_BYTES 128
typedef struct ccg_group ccg_group;

/* Host-only planning (no device work): cuts[0..G] with cuts[0] = 0,
 * cuts[G] = N and interior cuts multiples of CCG_COCLUSTER_ROW_ALIGN.
 * ccg_row_slabs: cut g ~ N (1 - sqrt(1 - g/G)) (equal packed-triangle pairs);
 * ccg_rect_slabs: cut g ~ N g / G (equal full rows). */
int ccg_row_slabs(int64_t N, int G, int64_t* cuts);
int ccg_rect_slabs(int64_t N, int G, int64_t* cuts);
/* Bootstrap block [*b0, *b1) of `rank` among G (sizes differ by <= 1). */
int ccg_boot_shard(int64_t nboots, int G, int rank, int64_t* b0, int64_t* b1);

/* Host-only plan of the all-gathers (ccg_allgather_columns and the row
 * all-gather of ccg_consensus_knn_sharded_dev): offsets[0..nranks] = the
 * exclusive prefix of counts (rank r's rows land at offsets[r]); *equal = 1
 * when every count is equal (one ncclAllGather, *nroots = 0), else 0 with
 * roots[0..*nroots) = the ranks with counts > 0 in rank order, each the root
 * of one ncclBroadcast of its block (all in one RCCL group).  roots may be
 * NULL (count only). */
int ccg_allgather_plan(int nranks, const int64_t* counts, int64_t* offsets, int* equal, int* roots, int* nroots);
/* One process, several devices (ncclCommInitAll over `devices`). */
int ccg_group_open(const int* devices, int ndev, ccg_group** out);
/* One process per device: rank 0 calls ccg_group_unique_id, the caller
 * broadcasts the CCG_GROUP_ID_BYTES bytes to every rank (any channel), then
 * every rank calls ccg_group_open_rank (collective; blocks until all join). */
int ccg_group_unique_id(uint8_t* id);
int ccg_group_open_rank(int device, int nranks, int rank, const uint8_t* id, ccg_group** out);
int ccg_group_close(ccg_group* g);
int ccg_group_info(const ccg_group* g, int* nlocal, int* nranks, int* first_rank);
/* The engine context of local device `local` (owned by the group). */
int ccg_group_ctx(ccg_group* g, int local, ccg_ctx** out);
/* ccg_synchronize on every local context; first sticky error wins. */
int ccg_group_synchronize(ccg_group* g);

/* All-gather of assignment columns (device pointers, enqueued on each local
 * context's stream, no host synchronisation).  Rank r contributes counts[r]
 * bootstrap columns of N labels (local_A[l]: counts[first_rank+l] x N, each
 * column contiguous); every local device receives the sum(counts) x N matrix
 * A[l] with rank r's columns after rank r-1's.  local_A[l] may alias its own
 * block of A[l].  counts: host array of nranks entries. */
int ccg_allgather_columns(ccg_group* g, const void* const* local_A, const int64_t* counts, int64_t N,
                          int label_bits, void* const* A);
/* Each local device computes its rank's row slab [cuts[r], cuts[r+1]) of the
 * packed co/both/dist (ccg_row_slabs cuts) from its full copy A[l]; slab
 * layout as ccg_cocluster_dev with r0 = cuts[r].  co/both/dist may be NULL
 * (or hold NULL entries).  cuts (host, nranks+1) may be NULL. */
int ccg_cocluster_sharded_dev(ccg_group* g, const void* const* A, int label_bits, int64_t N, int64_t B,
                              uint16_t* const* co, uint16_t* const* both, double* const* dist,
                              int64_t* cuts);
/* Fused consensus kNN over the group: each device computes rows
 * [cuts[r], cuts[r+1]) (ccg_rect_slabs) of its N x k out_idx[l], then the
 * rows are all-gathered so every device holds the whole matrix, and
 * d_nan_flag[l] (device int32) holds the OR over ranks. */
int ccg_consensus_knn_sharded_dev(ccg_group* g, const void* const* A, int label_bits, int64_t N, int64_t B,
                                  int k, int32_t* const* out_idx, int32_t* const* d_nan_flag);
/* Host flavours for a single-process group (nlocal == nranks): A is uploaded
 * once and broadcast over xGMI; outputs as ccg_cocluster /
 * ccg_consensus_knn_assign / ccg_knn_boot (bootstraps split over devices). */
int ccg_group_cocluster(ccg_group* g, const void* A, int label_bits, int64_t N, int64_t B, uint16_t* co,
                        uint16_t* both, double* dist);
int ccg_group_consensus_knn_assign(ccg_group* g, const void* A, int label_bits, int64_t N, int64_t B, int k,
                                   int32_t* out_idx);
int ccg_group_knn_boot(ccg_group* g, const double* pcs, int64_t N, int d, const int32_t* boot_idx, int64_t n,
                       int nb, int kmax, int32_t* out_idx, double* out_dist, ccg_knn_stats* stats);

/* --------------------------------------------------------- utilities -- */
/* Stable radix sort of n (int32 key, int32 value) pairs by the low key_bits
 * bits of the keys (device pointers; outputs must not alias the inputs): the
 * grouping step of the distinct-cell kNN (rows by cell) and of the SNN host
 * lists (kNN entries by neighbour), exported for testing and reuse.
 * Requires 0 <= key_bits <= 31, n < 2^31. */
int ccg_sort_pairs_dev(ccg_ctx* ctx, const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                       int32_t* vals_out, int64_t n, int key_bits, void* stream);

/* Exclusive scan of n int64 values (device pointers; out has n + 1 entries,
 * out[n] = the total; out may alias in): the single-pass look-back scan the
 * library's counting sorts and SNN offsets use (up to 2^21 values in one
 * launch, the two-pass scan beyond), exported for testing.  Values and their
 * partial sums must lie in [0, 2^62); in the single-pass range a tile sum or
 * total outside it sets the sticky device error (CCG_ERANGE at the next
 * ccg_synchronize). */
int ccg_scan_i64_dev(ccg_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, void* stream);

/* ------------------------------------------------------ kernel timing -- */
/* Device time of selected kernels, measured with hipEvents recorded on the
 * stream each kernel is launched on (used by bench.py for the live roofline).
 * Disabled by default; enabling adds two event records per timed launch. */
#define CCG_KT_KNN_SCREEN 0   /* the fp16 hi/lo MFMA screening kernel of ccg_knn_* */
#define CCG_KT_KNN_TOTAL 1    /* prep + screen + certify + fallback */
#define CCG_KT_SNN 2          /* whole ccg_snn_dev call */
#define CCG_KT_SILHOUETTE 3   /* whole ccg_silhouette_dev call */
#define CCG_KT_COCLUSTER 4    /* the co-cluster tile kernel */
#define CCG_KT_COUNT 5
/* Not a kernel: host milliseconds spent blocked on the pinned upload ring
 * (a full ring means the host is CCG_PIN_RING uploads ahead of the GPU:
 * back-pressure, not launch cost) and the number of such waits since the
 * last read.  Always accounted (no ccg_timing_enable needed). */
#define CCG_KT_HOST_RING_WAIT 100
int ccg_timing_enable(ccg_ctx* ctx, int enable);
/* Synchronises, returns the summed milliseconds and launch count of kernel
 * `which` since the last read, and resets that counter. */
int ccg_timing_read(ccg_ctx* ctx, int which, double* total_ms, int64_t* launches);

/* ------------------------------------------ host clustering stand-in -- */
/* Louvain community detection (modularity with igraph's resolution-scaled
 * gain, local moving + aggregation) of an undirected weighted edge list, on
 * the calling host thread; no device, no context.  The Python drop-in's
 * stand-in for igraph::cluster_leiden (R/consensusClust.R:656-658 via
 * bluster, :430-433), which R keeps.  Not igraph's algorithm: labels differ
 * from igraph's.  Edges (ei[e], ej[e]) with ei != ej in [0, n), weights >= 0;
 * labels[n] receives 1..C in order of first appearance.  Thread-safe. */
int ccg_host_louvain(int64_t n, int64_t ne, const int32_t* ei, const int32_t* ej, const double* w,
                     double resolution, uint64_t seed, int32_t* labels);

#ifdef __cplusplus
}
#endif
#endif /* CCG_H */
