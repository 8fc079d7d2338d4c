// Internal declarations of libccg.so (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <vector>
#include <stdint.h>
#include <stddef.h>

#include "../../include/ccg.h"

// Workspace slots owned by a context.  Each slot grows on demand; growth
// synchronises the context stream before freeing the old buffer.
enum ccg_ws_slot {
    WS_ROWS64 = 0,   // gathered bootstrap rows, float64 [n][d]
    WS_REFS32,       // screening image, float32 [npad][2*KS]
    WS_CAND_IDX,     // screening candidates [n][2][KP]
    WS_CAND_THR,     // screening thresholds [n][2]
    WS_MISC,         // small scalars (mnorm, fail counter, ...)
    WS_FAIL_LIST,    // rows that failed certification [n]
    WS_SNN_A,        // SNN host counts / offsets
    WS_SNN_B,        // SNN host lists
    WS_SNN_C,        // SNN per-node bounds / offsets
    WS_SNN_D,        // SNN scratch edges
    WS_SNN_E,        // SNN per-node counts / flags
    WS_SNN_F,        // SNN sorted per-node partner rows (scratch)
    WS_SNN_G,        // SNN host back-pointers and per-node splits
    WS_SNN_H,        // SNN node size classes (scan)
    WS_SIL_A,        // silhouette accumulators
    WS_SIL_B,        // silhouette centroids
    WS_SIL_Q,        // silhouette fixed-point rows (x and x^2)
    WS_SIL_C,        // silhouette distinct-cell tables (first rows, representatives, weights, exceptions)
    WS_KB_A,         // distinct-cell kNN: sorted (cell, row) pairs, heads, tables
    WS_KB_B,         // distinct-cell kNN: distinct rows and their kNN
    WS_COC_A,        // co-cluster column tables
    WS_COC_B,        // co-cluster fused-path slot tables
    WS_COC_C,        // co-cluster partial counts between column chunks / consensus row slab
    WS_MAP_A,        // map-back first-position scratch
    WS_HOST_A,       // host-API staging 1
    WS_HOST_B,       // host-API staging 2
    WS_HOST_C,       // host-API staging 3
    WS_HOST_D,       // host-API staging 4
    WS_HOST_E,       // host-API staging 5
    WS_SCAN,         // scan block sums
    WS_ORDER,        // kNN spatial ordering (bucket histogram, permutation)
    WS_FB_D,         // kNN fallback per-range lists (keys)
    WS_FB_I,         // kNN fallback per-range lists (ids)
    WS_SEGS,         // kNN batched-segment plan (offsets, blocks, positions)
    WS_SORT,         // device radix sort temporary storage
    WS_SNN_ROWS,     // SNN per-node partner rows (padded CSR of the per-graph API)
    WS_HIER,         // cluster block sums: co/both row sub-slab
    WS_PCA,          // PCA: standardised cells x genes, covariance, subspace blocks
    WS_COC_D,        // consensus kNN candidate path: the row-permuted assignment matrix
    WS_COC_E,        // consensus kNN candidate path: per-row candidate lists
    WS_COC_F,        // consensus kNN candidate path: thresholds, counters, flags
    WS_COC_G,        // co-cluster fragment-entry matrix of a column chunk (slots x rows bytes)
    WS_HINT,         // kNN: per-cell threshold hints shared by the bootstraps of one host call
    WS_TAB_ROWS,     // kNN cell table: the PCs row-major (certify / fallback rows)
    WS_TAB_MAP,      // kNN cell table: cell -> distinct-cell id of a bootstrap (-1: absent)
    WS_TAB,          // kNN cell table of a host call (ccg_knn_boot): ids then squared distances
    WS_FX_A,         // kNN exact search of failed rows: radii, candidate counts, overflow list
    WS_FX_B,         // kNN exact search of failed rows: candidate (d2, row) buffers
    WS_SEG_ROWS,     // batched bootstrap segments: the gathered rows of every segment
    WS_SEG_TAB,      // batched bootstrap segments: row and distinct-cell segment offsets
    WS_KB_C,         // distinct-cell kNN: per-cell counts / offsets / cursors / cell -> distinct id (counting grouping)
    WS_SIL_IMG,      // silhouette: per-labeling LDS images of the fp16-screen width kernel
    WS_SIL_SEG,      // silhouette segments: offsets, tile starts, label and output pointers
    WS_FX_C,         // kNN segmented exact search: the compacted failed list, radii, segment offsets
    WS_KBT,          // kNN bootstrap batches: segment offsets (distinct cells, rows), per-segment fail counts
    WS_NSLOTS
};

struct ccg_timer_rec {
    int which;
    hipEvent_t start, stop;
};

// Sticky device error bits (ccg_ctx::d_err): kernels that find invalid input
// they cannot report synchronously OR a bit in; the next ccg_synchronize /
// ccg_check_errors / host-flavour call turns it into a status code.
#define CCG_DERR_LABEL_RANGE 1  // map-back: a label exceeds the assignment matrix's label width
#define CCG_DERR_SNN_INDEX 2    // SNN: neighbour index out of range or self
#define CCG_DERR_CLUSTER_INDEX 4  // block sums / contingency: cluster position outside [0, K)
#define CCG_DERR_KNN_UNIQUE 8     // ccg_knn_boot_dev: n_unique differs from the distinct cells of idx
#define CCG_DERR_SCAN_RANGE 16    // ccg_scan_i64: a tile sum or prefix outside [0, 2^62) (the status-word packing)

#ifndef CCG_PIN_RING
// a launch set uploads its tables here: the host runs at most this many
// uploads ahead of the GPU.  Measured (round 6): 8 against 16 / 32 / 64
// slots -- cfg3 and cfg2 within noise, cfg5 1056-1088 against 990-1046
// bootstraps/s (a host far ahead fills one stream's queue and blocks there
// while the other stream runs dry).
#define CCG_PIN_RING 8
#endif
#define CCG_SCAN_SLOTS 8  // streams with their own single-pass scan state per context

struct ccg_ctx {
    int device;
    hipStream_t stream;
    int* d_err;  // device word of CCG_DERR_* bits
    int64_t snn_row_reserve;  // SNN row entries reserved by the per-graph API (0 = default)
    void* snn_stage;          // host-staged SNN rows of the last ccg_snn_graphs call (snn.hip)
    void* ws[WS_NSLOTS];
    size_t ws_bytes[WS_NSLOTS];
    ccg_knn_stats last_stats;
    void* fx_zeroed;  // kNN radius search: the WS_FX_A buffer whose counters were zeroed at allocation
    void* kb_zeroed;  // kNN row grouping: the WS_KB_C buffer whose counts / cursors are zero for N = kb_zero_n
    int64_t kb_zero_n;
    // kNN: the exact-search row list of the last call and its count (device; ccg_knn_last_fallback)
    const int* last_fail_list;
    const int* last_fail_count;
    // pinned staging ring for host tables copied inside asynchronous entry
    // points (ccg_h2d_staged): the caller's host memory may be gone before
    // the copy runs
    void* pin_buf[CCG_PIN_RING];
    size_t pin_bytes[CCG_PIN_RING];
    hipEvent_t pin_ev[CCG_PIN_RING];
    int pin_next;
    double pin_wait_ms;    // host time blocked on ring slots (ccg_timing_read CCG_KT_HOST_RING_WAIT)
    int64_t pin_waits;
    // single-pass scan state (ccg_scan_i64): per-tile status words and the
    // finished-tile count, zero between calls (the kernel's last tile clears
    // them); one slice per stream the context has scanned on (CCG_SCAN_SLOTS),
    // so scans enqueued on two streams never share status words
    void* d_scan;
    hipStream_t scan_stream[CCG_SCAN_SLOTS];
    int scan_nstreams;
    // kernel timing (ccg_timing_*)
    int timing;
    ccg_timer_rec* timers;   // pool, grows
    int ntimers, cap_timers, used_timers;
};

// Record a timing start/stop around a launch on stream st (no-ops when
// timing is disabled).  Returns a handle for ccg_timer_stop or -1.
int ccg_timer_start(ccg_ctx* ctx, int which, hipStream_t st);
void ccg_timer_stop(ccg_ctx* ctx, int handle, hipStream_t st);

// Copy bytes of host memory to device dst on stream st through a pinned
// staging slot of the context (the source may be freed when this returns;
// a pageable source would be read by the DMA after that).  Waits only when
// the slot's previous copy, CCG_PIN_RING uses ago, has not run yet.
int ccg_h2d_staged(ccg_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t st);

void ccg_set_error(const char* fmt, ...);
int ccg_hip_fail(hipError_t e, const char* what, const char* file, int line);

#define CCG_HIP(x)                                                        \
    do {                                                                  \
        hipError_t ccg_e_ = (x);                                          \
        if (ccg_e_ != hipSuccess)                                         \
            return ccg_hip_fail(ccg_e_, #x, __FILE__, __LINE__);          \
    } while (0)

#define CCG_REQUIRE(cond, ...)                                            \
    do {                                                                  \
        if (!(cond)) {                                                    \
            ccg_set_error(__VA_ARGS__);                                   \
            return CCG_EINVAL;                                            \
        }                                                                 \
    } while (0)

// Frees the host staging of ccg_snn_graphs (ccg_close).
void ccg_snn_stage_free(ccg_ctx* ctx);

// Reads and clears ctx->d_err (synchronising the device); returns CCG_OK or
// the status code of the first error bit with the message set.
int ccg_take_device_error(ccg_ctx* ctx);

// Returns a device buffer of at least `bytes` for `slot` (nullptr on OOM,
// with the error message set).
void* ccg_ws(ccg_ctx* ctx, int slot, size_t bytes);

// The stream a _dev entry point enqueues on.  NULL is HIP's legacy default
// stream (hipStreamLegacy) of the current device, as for any HIP library:
// ordered after every earlier call on that stream and every blocking stream
// (torch's default stream is that stream), so an input written just before a
// call is complete when the library reads it and a temporary freed just
// after is not reused while it still runs.  (Through round 5 NULL meant the
// context's own non-blocking stream, unordered with the caller's work.)  The
// host flavours pass ctx->stream explicitly.
static inline hipStream_t ccg_pick_stream(ccg_ctx* ctx, void* s) {
    (void)ctx;
    return s ? (hipStream_t)s : hipStreamLegacy;
}

// Exclusive scan of int64 values on device: out[i] = sum_{t<i} in[i]; the
// total goes to out[n].  in may alias out.  Uses WS_SCAN.
// ccg_scan_i64's single pass: up to SCAN_LB_MAX tiles; its state (status
// words, finished count) in ctx->d_scan
#define SCAN_LB_MAX 1024
#define SCAN_LB_BYTES (SCAN_LB_MAX * 8 + 64)  // one stream's slice of ctx->d_scan
int ccg_scan_i64(ccg_ctx* ctx, const int64_t* in, int64_t* out, int64_t n,
                 hipStream_t st);

// Stable device radix sort of (key, value) int32 pairs on the low key_bits
// bits of the keys (sort.hip; temporary storage in WS_SORT).
int ccg_sort_pairs_i32(ccg_ctx* ctx, const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                       int32_t* vals_out, int64_t n, int key_bits, hipStream_t st);

__host__ __device__ static inline int64_t ccg_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
