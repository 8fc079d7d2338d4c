// Exact brute-force kNN of bootstrap rows on gfx950.
//
// Reference path: bluster::clusterRows(pca, SNNGraphParam(k, ...)) ->
// BiocNeighbors::findKNN (R/consensusClust.R:656-658) on the bootstrap
// matrix pca[sample(...), ] (:394).  Contract (DESIGN.md "kNN"): exact
// Euclidean neighbours, self excluded by row identity, ordered by the fp64
// squared distance summed unfused in dimension order, ties by row index.
//
// Stages, all on the device:
//   1. order + prep : Morton order of the leading PCs; rows scaled by 2^e and
//                     split into fp16 hi/lo images (knn_prep16_kernel).
//   2. screen       : three v_mfma_f32_32x32x16_f16 per 16 dims compute
//                     v = x.y - |y|^2/2 for a 32-query x 32-reference tile per
//                     wave; each lane keeps the KP best references of its
//                     half-tile in registers (knn_screen16_kernel).
//   3. certify      : one wave per query recomputes the 2*KP candidates in
//                     fp64, bitonic-sorts them by (d2, j) across lanes and
//                     proves with a rigorous error bound that no excluded
//                     reference can enter the top k; rows that cannot be
//                     proven go to
//   4. fallback     : exact fp64 scan of all references for that row.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ccg_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define KNN_KP 20          // candidates kept per half-lane for kmax <= 20
#define KNN_KP_BIG 32      // ... for 20 < kmax <= 32 (2*KP <= 64 lanes in certify)
#define KNN_TAB_K 48       // cell tables (ccg_knn_table_dev): up to 48 neighbours from KP = 32 lists
#define KNN_TABLE_MIN_BOOTS 8  // ccg_knn_boot: a cell table for calls of at least this many bootstraps
#ifndef KNN_TMARGIN
#define KNN_TMARGIN 8      // screen threshold: rank KP + KNN_TMARGIN of the two half-lists' union
#endif
#define KNN_QPB 128        // queries per 256-thread block (4 waves x 32)
#define KNN_FB_K 48        // fallback list length (>= kmax)
#ifndef KNN_FB_S
#define KNN_FB_S 64        // max reference ranges per failed row
#endif
#define KNN_FB_SLOTS 65536 // min scratch lists (failed rows x ranges)
#define KNN_FB_UNITS 448   // target (failed row, range) blocks
#ifndef KNN_EXPAND_CELLS
#define KNN_EXPAND_CELLS 1  // tools only: 0 = the per-row expansion for every row (A/B)
#endif
#ifndef KNN_EXPAND_RADIUS
#define KNN_EXPAND_RADIUS 1  // tools only: 0 = cut ties by the per-thread-list search (A/B)
#endif
#define KNN_FB_GRID 128    // fallback grids (grid-stride loops; usually 0-30 rows fail, and a
                           // 1024-block launch of exiting blocks alone cost ~30 us)

// Error budget of the fp16 hi/lo screen (DESIGN.md "kNN certification bound"):
// relative part in units of the fp32 ulp (2^-24) times (2|x| + sqrt(dK))^2 --
// 3 x 16*KSTEPS products accumulated in fp32 -- plus an absolute part from
// the hi/lo representation floor: hi/lo parts below KNN_F16_FLOOR (the
// smallest normal fp16) are flushed to zero in prep, so every scaled value
// carries an absolute error of at most 2^-14 whatever the hardware's fp16
// denormal mode.
#define KNN_ERR_ULPS_F16 1024.0
#define KNN_F16_FLOOR 0x1p-14

// --------------------------------------------------------------- gather --
// (column-major source: LPR lanes per output row, a lane per dimension --
// coalesced row writes, no per-element 64-bit division)
template <int LPR>
__global__ __launch_bounds__(256) void gather_rows_kernel(const double* __restrict__ pcs, int64_t N, int d,
                                                          const int32_t* __restrict__ idx, int64_t n,
                                                          double* __restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    if (i >= n) return;
    const int c = idx[i];
    for (int k = threadIdx.x & (LPR - 1); k < d; k += LPR) rows[i * d + k] = pcs[(int64_t)k * N + c];
}

// --------------------------------------------------------------- screen --
// Insert (v, id) into a descending register list (v > lv[KP-1] assumed) by
// "position + shift": the keep-flags c_t = !(v > lv[t]) are independent
// compares, and each slot is then a two-level select
// (keep / take v / take the left neighbour), so the dependency depth is 3
// instead of the KP-long compare-swap chain of list_insert.
template <int KP>
__device__ __forceinline__ void list_insert_par(float (&lv)[KP], int (&li)[KP], float v, int id) {
    bool keep[KP];
#pragma unroll
    for (int t = 0; t < KP; ++t) keep[t] = !(v > lv[t]);  // slot t keeps its entry (ties keep the old one)
#pragma unroll
    for (int t = KP - 1; t >= 1; --t) {
        const float sv = keep[t - 1] ? v : lv[t - 1];
        const int si = keep[t - 1] ? id : li[t - 1];
        lv[t] = keep[t] ? lv[t] : sv;
        li[t] = keep[t] ? li[t] : si;
    }
    lv[0] = keep[0] ? lv[0] : v;
    li[0] = keep[0] ? li[0] : id;
}

// R-th largest (R = KP + KNN_TMARGIN; kmax + KNN_TMARGIN for the cell
// tables' kmax > KP) of the union of this half-lane's list
// and its partner's (lane ^ 32), both sorted descending: max over splits i
// of min(mine[i-1], other[R-1-i]).  The partner's entries arrive by
// v_permlane32_swap (no LDS).  Every ref either half has rejected or evicted
// is <= this value, so it is a valid rejection threshold for both halves and
// tighter than max(thr_h0, thr_h1) (about rank 2*KP of the union); the
// margin of KNN_TMARGIN ranks above k keeps certification (excl - E > dK)
// provable.
template <int KP, int R>
__device__ __forceinline__ float union_kth(const float (&lv)[KP]) {
    static_assert(R >= KP && R <= 2 * KP, "union rank out of range");
    const bool lo = (threadIdx.x & 32) == 0;
    float t = -INFINITY;
#pragma unroll
    for (int i = R - KP; i <= KP; ++i) {
        // i from mine (lv[i-1]), R - i from the partner (its lv[R-1-i])
        const unsigned x = __float_as_uint(lv[R - 1 - i]);
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        const float b = __uint_as_float(lo ? r[1] : r[0]);
        t = fmaxf(t, i == 0 ? b : fminf(lv[i - 1], b));
    }
    return t;
}

// ------------------------------------------------- fp16 hi/lo screen --
// Each value x (scaled by sigma = 2^e so max|x| < 2^12) is split into
// fp16 hi = rn(x) and lo = rn(x - hi); x.y ~ hi.hi + hi.lo + lo.hi with
// |error| <= ~2^-22 |x||y| per product plus fp32 accumulation, i.e. fp32-class
// accuracy from three v_mfma_f32_32x32x16_f16 per 16 dims.  The reference
// norm term rides in dimension d (the first padding dimension): the image
// holds -|y|^2/2 / 2^KNN_NORM_SHIFT there (hi/lo split like any value) and the
// query side 2^KNN_NORM_SHIFT, so the MFMA chain alone yields
// v = x.y - |y|^2/2 from a zero accumulator (16 * KSTEPS >= d + 1).
// Row image (64*KSTEPS bytes): for lane-half h in {0,1}: KSTEPS hi chunks
// then KSTEPS lo chunks of 8 halves (dims 16s + 8h .. +7), so a lane reads
// one contiguous 32*KSTEPS-byte run.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// LDS staging of the reference image: chunks of knn_chunk(KSTEPS) refs
// (chunk / 32 MFMA tiles per barrier) in knn_nbuf(KSTEPS) buffers (prefetch
// distance nbuf - 1).  128-ref chunks in 2 buffers halve the barriers of 64 x 3
// at the same LDS (3 blocks per CU); d > 31 rows are twice as wide and keep
// 64 x 3 so that 2 blocks still fit.
__host__ __device__ constexpr int knn_chunk(int ksteps) { return ksteps == 4 ? 64 : 128; }
__host__ __device__ constexpr int knn_nbuf(int ksteps) { return ksteps == 4 ? 3 : 2; }
static inline int knn_ksteps(int d) { return d + 1 <= 16 ? 1 : (d + 1 <= 32 ? 2 : 4); }  // d dims + the norm dim
#ifndef KNN_NO_MORTON
#define KNN_NO_MORTON 0     // tools only: screen in input order (no Morton bucketing)
#endif
#ifndef KNN_QCAP
#define KNN_QCAP 8          // per-lane insertion queue slots (flush before a half tile that could overflow)
#endif
#ifndef KNN_PAIR
#define KNN_PAIR 0          // two tiles per step (two MFMA chains in flight)
#endif
#define KNN_NORM_SHIFT 15   // the query's norm-dimension value 2^15 (exact in fp16)
#ifndef KNN_HINT_MARGIN
#define KNN_HINT_MARGIN 0.15  // relative slack on a hinted squared distance (see ccg_knn_boot_hint_dev)
#endif
#define KNN_PAD_NORM (-65504.0f)  // padding rows: below every real value (|v| < 1.6e9 < 2^31)

__device__ __forceinline__ int knn_scale_exp(const unsigned* maxabs_bits) {
    const float m = __uint_as_float(*maxabs_bits);
    if (!(m > 0.f)) return 0;
    return 12 - (ilogbf(m) + 1);  // max|x| * 2^e < 2^12, so |y|^2/2 / 2^15 < 2^14 for d <= 63
}

__device__ __forceinline__ void knn_split16(double xs, _Float16& hi, _Float16& lo) {
    // parts below the smallest normal fp16 are flushed here, explicitly,
    // so the certification floor (KNN_F16_FLOOR) holds in any denorm mode
    // (the fp32 values are pinned in registers: without that the compiler
    // folds double -> float -> half into a ~40-instruction software
    // conversion; with it, v_cvt_f32_f64 + v_cvt_f16_f32, the same rounding)
    float f = (float)xs;
    asm volatile("" : "+v"(f));
    hi = (_Float16)f;
    if (fabs((double)(float)hi) < KNN_F16_FLOOR) hi = (_Float16)0.0f;
    float r = (float)(xs - (double)(float)hi);
    asm volatile("" : "+v"(r));
    lo = (_Float16)r;
    if (fabs((double)(float)lo) < KNN_F16_FLOOR) lo = (_Float16)0.0f;
}

template <int KSTEPS>
__global__ void knn_prep16_kernel(const double* __restrict__ rows, int64_t n, int64_t npad, int d,
                                  const unsigned* __restrict__ maxabs_bits, const int* __restrict__ perm,
                                  uint4* __restrict__ img, double* __restrict__ inv_scale2,
                                  const float* __restrict__ row_hint, float* __restrict__ pos_t0) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // position in spatial order
    if (r >= npad) return;
    const int64_t src = r < n ? (perm ? perm[r] : r) : -1;  // -1: padding position (segment padding or r >= n)
    const bool valid = src >= 0;
    const int e = knn_scale_exp(maxabs_bits);
    if (r == 0) *inv_scale2 = ldexp(1.0, -2 * e);
    _Float16 hv[KSTEPS * 32];  // [h][hi s..][lo s..] flattened below
    double nr = 0.0;
    for (int k = 0; k < d; ++k) {
        const double x = valid ? rows[src * d + k] : 0.0;
        nr += x * x;
    }
    if (pos_t0) {
        // the screen's initial rejection threshold from the row's hint (a
        // squared distance its kq-th nearest distinct row is expected within):
        // v = x.y - |y|^2/2 > t0  <=>  |x - y|^2 < hint (scaled by 2^2e)
        const float hint = valid && row_hint ? row_hint[src] : 0.0f;
        pos_t0[r] = hint > 0.0f ? (float)(0.5 * ldexp(nr - (double)hint * (1.0 + KNN_HINT_MARGIN), 2 * e))
                                : -INFINITY;
    }
#pragma unroll
    for (int k = 0; k < KSTEPS * 16; ++k) {
        double xs = 0.0;
        if (k < d) xs = valid ? ldexp(rows[src * d + k], e) : 0.0;
        else if (k == d) xs = valid ? -0.5 * ldexp(nr, 2 * e - KNN_NORM_SHIFT) : (double)KNN_PAD_NORM;
        _Float16 hi, lo;
        knn_split16(xs, hi, lo);
        const int s = k / 16, h = (k % 16) / 8, j = k % 8;
        hv[h * (KSTEPS * 16) + s * 8 + j] = hi;
        hv[h * (KSTEPS * 16) + KSTEPS * 8 + s * 8 + j] = lo;
    }
    uint4* out = img + r * (KSTEPS * 4);
#pragma unroll
    for (int c = 0; c < KSTEPS * 4; ++c) out[c] = *reinterpret_cast<const uint4*>(&hv[c * 8]);
}

template <int KSTEPS>
__device__ __forceinline__ int swz_chunk(int row, int c) {
    // rows of 64*KSTEPS bytes; spread the 16-B chunk over the 256-B bank row
    if constexpr (KSTEPS == 1) return c ^ ((row >> 2) & 3);
    else if constexpr (KSTEPS == 2) return c ^ ((row >> 1) & 7);
    else return c ^ (row & 15);
}

// ---------------------------------------------------- spatial ordering --
// Order rows by a Morton code of their leading KNN_MORTON_DIMS coordinates
// (the leading PCs), KNN_MORTON_BITS bits each, so that rows close in space
// sit in nearby chunks: the screen's thresholds tighten within the first
// chunks it scans.  Any permutation is correct; only screening speed depends
// on it.  Codes of <= 15 bits are bucketed by a counting sort; longer codes
// are radix-sorted (key, row) pairs.
#ifndef KNN_MORTON_DIMS
#define KNN_MORTON_DIMS 3
#endif
#ifndef KNN_MORTON_BITS
#define KNN_MORTON_BITS 5
#endif
#define KNN_MD KNN_MORTON_DIMS
static_assert(KNN_MORTON_DIMS * KNN_MORTON_BITS <= 31 && KNN_MORTON_DIMS <= 24, "Morton code too long");
__device__ __forceinline__ unsigned f2ord(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// max|x| (fp32 bits, rounded up) and the ordered-float bounds of the leading
// KNN_MD coordinates in one coalesced pass; block-level reduction so each
// block issues 1 + 2 KNN_MD atomics (a per-wave atomic on one word serialises
// at ~13 ns each).  bnd: [0, KNN_MD) minima, [KNN_MD, 2 KNN_MD) maxima.
__global__ __launch_bounds__(256) void knn_rowstats_kernel(const double* __restrict__ rows, int64_t n, int d,
                                                           unsigned* __restrict__ maxabs_bits,
                                                           unsigned* __restrict__ bnd) {
    constexpr int NV = 1 + 2 * KNN_MD;
    __shared__ unsigned red[4][NV];
    unsigned v[NV];
    v[0] = 0u;
#pragma unroll
    for (int i = 0; i < KNN_MD; ++i) {
        v[1 + i] = 0xffffffffu;
        v[1 + KNN_MD + i] = 0u;
    }
    const int64_t tot = n * d;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const int kstep = (int)(S % d);
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int k = (int)(t % d);
    for (; t < tot; t += S) {
        const double x = rows[t];
        float f = (float)fabs(x);
        f = nextafterf(f, INFINITY);
        v[0] = max(v[0], __float_as_uint(f));
        const unsigned o = f2ord((float)x);
#pragma unroll
        for (int i = 0; i < KNN_MD; ++i)
            if (k == i) {
                v[1 + i] = min(v[1 + i], o);
                v[1 + KNN_MD + i] = max(v[1 + KNN_MD + i], o);
            }
        k += kstep;
        if (k >= d) k -= d;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        unsigned a = v[i];
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned b = (unsigned)__shfl_xor((int)a, o, 64);
            a = (i >= 1 && i <= KNN_MD) ? min(a, b) : max(a, b);
        }
        if (lane == 0) red[wv][i] = a;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int i = threadIdx.x;
        unsigned a = red[0][i];
        for (int w = 1; w < 4; ++w) a = (i >= 1 && i <= KNN_MD) ? min(a, red[w][i]) : max(a, red[w][i]);
        if (i == 0) atomicMax(maxabs_bits, a);
        else if (i <= KNN_MD) { if (i - 1 < d) atomicMin(&bnd[i - 1], a); }
        else if (i - 1 - KNN_MD < d) atomicMax(&bnd[i - 1], a);
    }
}

__device__ __forceinline__ unsigned morton_key(const double* __restrict__ x, int d,
                                               const unsigned* __restrict__ bnd) {
    const int nd = d < KNN_MD ? d : KNN_MD;
    unsigned code = 0;
    for (int k = 0; k < nd; ++k) {
        const float lo = ord2f(bnd[k]), hi = ord2f(bnd[KNN_MD + k]);
        const float span = hi - lo;
        float t = span > 0.f ? ((float)x[k] - lo) / span : 0.f;
        t = fminf(fmaxf(t, 0.f), 0.999999f);
        const unsigned qv = (unsigned)(t * (float)(1u << KNN_MORTON_BITS));
        for (int b = 0; b < KNN_MORTON_BITS; ++b) code |= ((qv >> b) & 1u) << (KNN_MD * b + k);
    }
    return code;
}

__global__ void knn_bucket_count_kernel(const double* __restrict__ rows, int64_t n, int d,
                                        const unsigned* __restrict__ bnd, int64_t* __restrict__ hist) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    atomicAdd((unsigned long long*)&hist[morton_key(rows + r * d, d, bnd)], 1ull);
}

__global__ void knn_bucket_scatter_kernel(const double* __restrict__ rows, int64_t n, int d,
                                          const unsigned* __restrict__ bnd, int64_t* __restrict__ cursor,
                                          int* __restrict__ perm) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const unsigned key = morton_key(rows + r * d, d, bnd);
    const int64_t pos = (int64_t)atomicAdd((unsigned long long*)&cursor[key], 1ull);
    perm[pos] = (int)r;
}

// One launch for knn_run's small initialisations: misc (max|x| bits, fail
// count, 1/sigma^2, the distinct-cell expansion's fail count), the coordinate bounds (minima all-ones, maxima zero) and
// the Morton bucket histogram (hist may be null).
__global__ void knn_init_kernel(unsigned* __restrict__ misc, unsigned* __restrict__ bnd,
                                int64_t* __restrict__ hist, int64_t nhist) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 8) misc[t] = 0u;  // [4]: ccg_knn_boot_dev's expansion fail count
    if (t < 2 * KNN_MD) bnd[t] = t < KNN_MD ? 0xffffffffu : 0u;
    if (hist)
        for (int64_t i = t; i < nhist; i += (int64_t)gridDim.x * blockDim.x) hist[i] = 0;
}

// (Morton key, row) pairs for the radix-sorted order of long codes
__global__ void knn_morton_keys_kernel(const double* __restrict__ rows, int64_t n, int d,
                                       const unsigned* __restrict__ bnd, int32_t* __restrict__ keys,
                                       int32_t* __restrict__ ids) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    keys[r] = (int32_t)morton_key(rows + r * d, d, bnd);
    ids[r] = (int32_t)r;
}

__device__ __forceinline__ int knn_chunk_at(int k, int c0, int Lc, int Rc, int Mc) {
    if (k == 0) return c0;
    if (k <= 2 * Mc) return (k & 1) ? c0 + (k + 1) / 2 : c0 - k / 2;
    const int m = k - 2 * Mc;
    return Rc > Lc ? c0 + Mc + m : c0 - Mc - m;
}

// 16-byte LDS-DMA: lane l's 16 bytes from sbase + voff land at LDS byte
// address lds + 16*l (sbase and lds wave-uniform).
__device__ __forceinline__ void glds16(const void* sbase, unsigned voff, unsigned lds) {
    int keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds))
        : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own
// 4 MB L2).  Give XCD x a contiguous range of query blocks: neighbouring
// blocks scan nearly the same chunk sequence a few steps apart, so each
// staged chunk is fetched into an XCD's L2 once and re-read from there.
// A bijection on [0, G) for any G; only speed depends on it.
__device__ __forceinline__ int xcd_block(int bid, int G) {
    const int q = G >> 3, r = G & 7, x = bid & 7, i = bid >> 3;
    return x * q + min(x, r) + i;
}

// s_waitcnt vmcnt(N) for a compile-time N (the LDS-DMA is issued as inline
// asm, so the compiler does not track it).
template <int N>
__device__ __forceinline__ void knn_wait_vmcnt() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else static_assert(N == 0, "unsupported vmcnt");
}

#ifndef KNN_WPE
#define KNN_WPE 3           // screen waves per SIMD the register budget is sized for
#endif
template <int KSTEPS, int KP, int R, int WPE = KNN_WPE, int QC = KNN_QCAP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void knn_screen16_kernel(
    const uint4* __restrict__ img, int n, int nchunks, int d, int* __restrict__ cand_idx,
    float* __restrict__ cand_thr, const int4* __restrict__ blk, const float* __restrict__ pos_t0) {
    constexpr int C16 = KSTEPS * 4;                 // 16-B chunks per row
    constexpr int ROWB = KSTEPS * 64;               // bytes per row
    constexpr int KNN_CHUNK = knn_chunk(KSTEPS);
    constexpr int KNN_NBUF = knn_nbuf(KSTEPS);
    constexpr int STAGE = KNN_CHUNK * ROWB;         // bytes of one stage
    constexpr int LOADS = (KNN_CHUNK * C16) / 256;  // LDS-DMA instructions per thread per stage
    // ALL of the kernel's LDS is this one array (the staging buffers, then the
    // queues): with a second __shared__ object beside the LDS-DMA target,
    // hipcc waits vmcnt(0) before the first ds_read of every tile, which
    // serialises the staging with the compute.
    __shared__ __attribute__((aligned(16))) unsigned char smem[KNN_NBUF * STAGE + 4 * (QC + 1) * 64 * 8];
#define lds(bb_) (smem + (bb_) * STAGE)
    // Per-lane insertion queues (slot-major [slot][lane]; slot QC is spare).
    // Candidates above the running threshold are queued per tile and inserted
    // in batches: a flush costs max-queue-length insertion rounds for the
    // whole wave instead of one round per (tile, register) any lane touched.
    uint2* const qbw = reinterpret_cast<uint2*>(smem + KNN_NBUF * STAGE) + (threadIdx.x >> 6) * (QC + 1) * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int bx = xcd_block(blockIdx.x, gridDim.x);
    // the block's reference chunks [cl, ch), query limit qhi (= the last valid
    // reference position + 1): the whole image, or (batched segments) its own
    int cl = 0, ch = nchunks, qhi = n;
    if (blk) {
        const int4 bi = blk[bx];
        cl = bi.x;
        ch = bi.y;
        qhi = bi.z;
    }
    const int q0 = bx * KNN_QPB + wave * 32;
    const int q = q0 + col;
    const int qrow = q < qhi ? q : qhi - 1;

    h8 qh[KSTEPS], ql[KSTEPS];
    {
        const uint4* qp = img + (int64_t)qrow * C16 + h * 2 * KSTEPS;
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            uint4 a = qp[s], b = qp[KSTEPS + s];
            // retire the loads here: hipcc does not see the asm DMA in the
            // chunk loop and would otherwise put its waits for these (which
            // then drain the DMA too) in front of the loop's MFMAs
            asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
            qh[s] = *reinterpret_cast<h8*>(&a);
            ql[s] = *reinterpret_cast<h8*>(&b);
        }
        // the query side of the norm dimension d is 2^KNN_NORM_SHIFT (exact, no lo part)
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (16 * s + 8 * h + e == d) {
                    qh[s][e] = (_Float16)(float)(1 << KNN_NORM_SHIFT);
                    ql[s][e] = (_Float16)0.0f;
                }
    }
    float lv[KP];
    int li[KP];
#pragma unroll
    for (int t = 0; t < KP; ++t) {
        lv[t] = -INFINITY;
        li[t] = -1;
    }
    float thr = -INFINITY;

    // Staging by LDS-DMA (global_load_lds_dwordx4): the LDS image is written
    // lane-linearly, so the row swizzle goes on the per-lane SOURCE address
    // (swz_chunk is an involution) and the same swizzle on the fragment reads.
#define KNN_STAGE_GLDS(bb, cidx)                                                                   \
    do {                                                                                           \
        const unsigned char* src_ = reinterpret_cast<const unsigned char*>(img) +                 \
                                    (int64_t)(cidx) * (KNN_CHUNK * ROWB);                          \
        _Pragma("unroll") for (int i_ = 0; i_ < LOADS; ++i_) {                                     \
            const int p_ = i_ * 256 + tid;                                                         \
            const int row_ = p_ / C16, cs_ = p_ % C16;                                             \
            glds16(src_, (unsigned)(row_ * ROWB + swz_chunk<KSTEPS>(row_, cs_) * 16),             \
                   lds_addr(lds(bb) + (i_ * 256 + wave * 64) * 16));                              \
        }                                                                                          \
    } while (0)
    // Rows are in spatial (Morton) order, so scan ref chunks outward from the
    // block's own position: near neighbours arrive first, the threshold tightens
    // within a few tiles and later tiles rarely insert (the order only changes
    // speed; certification makes the result exact for any order).
    const int c0 = min((int)(bx * KNN_QPB) / KNN_CHUNK, ch - 1);
    const int Lc = c0 - cl, Rc = ch - 1 - c0, Mc = min(Lc, Rc);
    const int nck = ch - cl;
#define chunk_at(kk_) knn_chunk_at((kk_), c0, Lc, Rc, Mc)
    // rejection threshold (see below); a hinted row starts at its hint's
    // threshold, which every later T keeps as a floor (T0 is itself a valid
    // rejection threshold for both halves, so certification stays exact)
    const float T0 = pos_t0 ? pos_t0[qrow] : -INFINITY;
    float T = T0;
    int qc = 0;           // this lane's queued candidates
    bool tdirty = false;  // lists changed since T was last set to the union threshold
#define KNN_FLUSH()                                                                   \
    do {                                                                              \
        for (int i_ = 0; __any(i_ < qc); ++i_) {                                      \
            if (i_ < qc) {                                                            \
                const uint2 e_ = qbw[i_ * 64 + lane];                                 \
                const float v_ = __uint_as_float(e_.x);                               \
                if (v_ > T) {                                                         \
                    list_insert_par<KP>(lv, li, v_, (int)e_.y);                       \
                    thr = lv[KP - 1];                                                 \
                    T = fmaxf(T, thr);                                                \
                }                                                                     \
            }                                                                         \
        }                                                                             \
        qc = 0;                                                                       \
        tdirty = true;                                                                \
    } while (0)
    // Pipeline: chunks k+1 and k+2 are in flight while chunk k is computed; at
    // the top of iteration k the wave waits for its own part of chunk k
    // (vmcnt: the younger chunk k+1 may stay outstanding), the barrier makes
    // every wave's part visible and frees buffer (k+2) % 3 (last read in k-1).
    static_assert(KNN_NBUF == 2 || KNN_NBUF == 3, "2 or 3 staging buffers");
    KNN_STAGE_GLDS(0, chunk_at(0));
    if (KNN_NBUF == 3 && nck > 1) KNN_STAGE_GLDS(1, chunk_at(1));
    for (int k = 0; k < nck; ++k) {
        const int b = k % KNN_NBUF;
        const int c = chunk_at(k);
        if constexpr (knn_nbuf(KSTEPS) == 3) {
            if (k + 1 < nck) knn_wait_vmcnt<LOADS>();
            else knn_wait_vmcnt<0>();
        } else {
            knn_wait_vmcnt<0>();
        }
        __syncthreads();
        if (k + KNN_NBUF - 1 < nck) KNN_STAGE_GLDS((k + KNN_NBUF - 1) % KNN_NBUF, chunk_at(k + KNN_NBUF - 1));
        // After the MFMA chain of a tile (accumulator ACC_, first ref RB_):
        // self / padding masking, the tile maximum, and -- when some lane's
        // value beats its threshold -- the branch-free enqueue (per half-tile
        // of 8 registers: flush first if its candidates could overflow a
        // queue).  After a flush both halves move to the union threshold;
        // between flushes T only rises.
#define KNN_TILE_TEST(ACC_)                                                                 \
    float vmax = ACC_[0];                                                                   \
    _Pragma("unroll") for (int reg = 1; reg < 16; ++reg) vmax = fmaxf(vmax, ACC_[reg]);     \
    if (__any(vmax > T))
#define KNN_TILE_POST(ACC_, RB_)                                                            \
    do {                                                                                    \
        const int rbase = (RB_);                                                            \
        if (rbase == q0 || rbase + 32 > qhi) { /* diagonal tile (self) or padding refs */   \
            _Pragma("unroll") for (int reg = 0; reg < 16; ++reg) {                          \
                const int r = rbase + (reg & 3) + 8 * (reg >> 2) + 4 * h;                   \
                if (r == q || r >= qhi) ACC_[reg] = -INFINITY;                              \
            }                                                                               \
        }                                                                                   \
        KNN_TILE_TEST(ACC_) {                                                               \
            _Pragma("unroll") for (int hh = 0; hh < 2; ++hh) {                              \
                int c8 = 0;                                                                 \
                _Pragma("unroll") for (int reg = 8 * hh; reg < 8 * hh + 8; ++reg) c8 += ACC_[reg] > T ? 1 : 0; \
                if (__any(qc + c8 > QC)) KNN_FLUSH();                                       \
                _Pragma("unroll") for (int reg = 8 * hh; reg < 8 * hh + 8; ++reg) {         \
                    const float v = ACC_[reg];                                              \
                    qbw[qc * 64 + lane] =                                                   \
                        make_uint2(__float_as_uint(v), rbase + (reg & 3) + 8 * (reg >> 2) + 4 * h); \
                    qc += v > T ? 1 : 0;                                                    \
                }                                                                           \
            }                                                                               \
        }                                                                                   \
        if (tdirty) {                                                                       \
            T = fmaxf(T0, union_kth<KP, R>(lv));                                            \
            tdirty = false;                                                                 \
        }                                                                                   \
    } while (0)
        static_assert(QC >= 8, "queue must hold a half tile");
#define KNN_LOAD_A(AH_, AL_, ROW_)                                                                  \
    _Pragma("unroll") for (int s = 0; s < KSTEPS; ++s) {                                            \
        uint4 a_ = *reinterpret_cast<const uint4*>(                                                 \
            lds(b) + (ROW_) * ROWB + swz_chunk<KSTEPS>((ROW_), h * 2 * KSTEPS + s) * 16);           \
        uint4 b_ = *reinterpret_cast<const uint4*>(                                                 \
            lds(b) + (ROW_) * ROWB + swz_chunk<KSTEPS>((ROW_), h * 2 * KSTEPS + KSTEPS + s) * 16);  \
        AH_[s] = *reinterpret_cast<h8*>(&a_);                                                       \
        AL_[s] = *reinterpret_cast<h8*>(&b_);                                                       \
    }
#if KNN_PAIR
        // two tiles per step: two independent MFMA chains, the second tile's
        // chain in flight while the first tile's values are tested
#pragma nounroll
        for (int tau = 0; tau < KNN_CHUNK / 32; tau += 2) {
            h8 ah0[KSTEPS], al0[KSTEPS], ah1[KSTEPS], al1[KSTEPS];
            KNN_LOAD_A(ah0, al0, tau * 32 + col);
            KNN_LOAD_A(ah1, al1, tau * 32 + 32 + col);
            f32x16 acc0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            f32x16 acc1 = acc0;
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0[s], qh[s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1[s], qh[s], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0[s], ql[s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1[s], ql[s], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al0[s], qh[s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al1[s], qh[s], acc1, 0, 0, 0);
            }
            KNN_TILE_POST(acc0, c * KNN_CHUNK + tau * 32);
            KNN_TILE_POST(acc1, c * KNN_CHUNK + tau * 32 + 32);
        }
#else
#pragma nounroll  // unrolling the tiles multiplies live registers
        for (int tau = 0; tau < KNN_CHUNK / 32; ++tau) {
            h8 ah[KSTEPS], al[KSTEPS];
            KNN_LOAD_A(ah, al, tau * 32 + col);
            f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], qh[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], ql[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], qh[s], acc, 0, 0, 0);
            }
            KNN_TILE_POST(acc, c * KNN_CHUNK + tau * 32);
        }
#endif
#undef KNN_LOAD_A
#undef KNN_TILE_POST
#undef KNN_TILE_TEST
    }
    KNN_FLUSH();
    T = fmaxf(T0, union_kth<KP, R>(lv));
#undef KNN_FLUSH
#undef KNN_STAGE_GLDS
#undef chunk_at
#undef lds
    if (q < qhi) {
        int* out = cand_idx + ((int64_t)q * 2 + h) * KP;
#pragma unroll
        for (int t = 0; t < KP; ++t) out[t] = li[t];
        // Certification threshold: every ref this half excluded is at or below
        // it.  Rejected refs were <= the T in force then (T only ever held the
        // union value or this half's own lv[KP-1], both monotone); evicted refs
        // are <= this half's final lv[KP-1], which can sit ABOVE the union T
        // when this half owns most of the union's top ranks.
        cand_thr[(int64_t)q * 2 + h] = fmaxf(T, lv[KP - 1]);
    }
}

// -------------------------------------------------------------- certify --
// segment s of global row q: seg_off[s] <= q < seg_off[s+1] (binary search)
__device__ __forceinline__ int knn_seg_of(const int64_t* __restrict__ seg_off, int nseg, int64_t q) {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (seg_off[mid] <= q) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ bool key_less(double a, int ia, double b, int ib) {
    return (a < b) || (a == b && ia < ib);
}

// Bitonic sort of 64 (key, idx) pairs held one per lane, ascending.
__device__ __forceinline__ void wave_bitonic64(double& key, int& id) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            double ok = __shfl_xor(key, j, 64);
            int oi = __shfl_xor(id, j, 64);
            bool up = ((lane & k) == 0);
            bool lower = ((lane & j) == 0);
            bool other_less = key_less(ok, oi, key, id);
            // lower lane keeps min when ascending block, max otherwise
            bool take = (lower == up) ? other_less : !other_less;
            // never swap equal elements (ids are distinct except padding)
            if (take && !(ok == key && oi == id)) {
                key = ok;
                id = oi;
            }
        }
    }
}

template <int KP, int DMAX>
__global__ __launch_bounds__(256) void knn_certify_kernel(
    const double* __restrict__ rows, int n, int d, int kmax,
    const int* __restrict__ cand_idx, const float* __restrict__ cand_thr,
    const double* __restrict__ inv_scale2, double err_ulps, const int* __restrict__ perm,
    int32_t* __restrict__ out_idx, double* __restrict__ out_dist, int* __restrict__ fail_list,
    int* __restrict__ fail_count, int npos, const int64_t* __restrict__ seg_off, int nseg, bool dist_sq,
    double* __restrict__ fail_tau) {
    const int lane = threadIdx.x & 63;
    const int qs = blockIdx.x * 4 + (threadIdx.x >> 6);  // screening position
    if (qs >= npos) return;
    const int q = perm ? perm[qs] : qs;                   // bootstrap row
    if (q < 0) return;                                    // segment padding
    const int base = seg_off ? (int)seg_off[knn_seg_of(seg_off, nseg, q)] : 0;  // output ids are segment-local
    const double* x = rows + (int64_t)q * d;
    int j = (lane < 2 * KP) ? cand_idx[(int64_t)qs * 2 * KP + lane] : -1;
    if (j >= 0 && perm) j = perm[j];
    // unrolled over DMAX so all of a row's loads are in flight together
    double xq[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) xq[k] = k < d ? x[k] : 0.0;
    double key = INFINITY;
    int id = 0x7fffffff - 64 + lane;  // distinct padding ids sort after real ones
    if (j >= 0) {
        const double* y = rows + (int64_t)j * d;
        double yv[DMAX];
        if ((d & 1) == 0) {  // rows are 16-B aligned: half the load instructions
            const double2* y2 = reinterpret_cast<const double2*>(y);
#pragma unroll
            for (int k2 = 0; k2 < DMAX / 2; ++k2) {
                const double2 v = 2 * k2 < d ? y2[k2] : make_double2(0.0, 0.0);
                yv[2 * k2] = v.x;
                yv[2 * k2 + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < DMAX; ++k) yv[k] = k < d ? y[k] : 0.0;
        }
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k)
            if (k < d) {
                const double t = __dsub_rn(xq[k], yv[k]);
                s = __dadd_rn(s, __dmul_rn(t, t));
            }
        key = s;
        id = j;
    }
    wave_bitonic64(key, id);

    // certification (wave-uniform values)
    double nq = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) nq += xq[k] * xq[k];
    const float t0 = cand_thr[(int64_t)qs * 2 + 0];
    const float t1 = cand_thr[(int64_t)qs * 2 + 1];
    const float tmax = fmaxf(t0, t1);
    const double dK = __shfl(key, kmax - 1, 64);
    const int idK = __shfl(id, kmax - 1, 64);
    bool ok = (idK < n);  // at least kmax real candidates
    if (tmax != -INFINITY) {
        // An excluded ref y has approx d2 >= excl (tmax: each half's
        // certification threshold, at or above every value it rejected or
        // evicted).  If y were as close as the k-th candidate (|x-y|^2 <= dK)
        // then |y| <= |x| + sqrt(dK), so with s = 2|x| + sqrt(dK) >= |x| + |y|
        // its screening error is at most
        //   E = c*2^-24*s^2                      (fp16 split + fp32 accumulation)
        //     + 2^-12*sqrt(d)*s/sigma + 2^-26*d/sigma^2   (flushed parts < 2^-14)
        //     + 8/sigma^2      (the norm dimension: 2^15 x a flushed part < 2^-14)
        // and its approx d2 at most dK + E.  excl > dK + E therefore proves it
        // is farther (DESIGN.md "kNN certification bound").
        const double s = 2.0 * sqrt(nq) + sqrt(dK);
        const double isc = sqrt(*inv_scale2);  // 1/sigma, a power of two
        const double E = err_ulps * 0x1p-24 * s * s + 0x1p-12 * sqrt((double)d) * s * isc +
                         (0x1p-26 * (double)d + 8.0) * isc * isc + 1e-300;
        const double excl = nq - 2.0 * (double)tmax * (*inv_scale2);  // thresholds are in scaled units
        ok = ok && (excl - E > dK);
    }
    if (ok) {
        if (lane < kmax) {
            out_idx[(int64_t)q * kmax + lane] = id - base;
            if (out_dist) out_dist[(int64_t)q * kmax + lane] = dist_sq ? key : sqrt(key);
        }
    } else if (lane == 0) {
        int p = atomicAdd(fail_count, 1);
        fail_list[p] = q;
        // the radius search's bound: kmax candidates (a subset of the references) lie within dK
        if (fail_tau) fail_tau[p] = idK < n ? dK : INFINITY;
    }
}

// ------------------------------------------------------------- fallback --
// Exact fp64 search for the rows certification could not prove.  Each failed
// row is split over S reference ranges (S chosen on the device so that
// nfail * S lists fit the scratch); one 256-thread block per (row, range)
// scans its range with the query in registers (unfused, dimension order),
// each thread keeping a sorted list, then merges 64 lists per wave by wave
// arg-min and the 4 wave lists into one sorted top-kmax list in scratch.
// knn_fallback_merge_kernel merges the S lists of each row.
__device__ __forceinline__ int knn_fb_splits(int nfail, int slots) {
    if (nfail <= 0) return 1;
    int S = slots / nfail;
    // about KNN_FB_UNITS (row, range) blocks in all: more ranges only add merge
    // rounds once the failed rows' scans fill the GPU (16 ranges x ~22 rows: 102 us
    // at cfg3; 64 ranges: 139 us; 8 ranges: 132 us)
    const int T = KNN_FB_UNITS / nfail;
    S = T < S ? T : S;
    return S < 1 ? 1 : (S > KNN_FB_S ? KNN_FB_S : S);
}

template <int DMAX, int FBK>
__global__ __launch_bounds__(256) void knn_fallback_kernel(
    const double* __restrict__ rows, int n, int d, int kmax,
    const int* __restrict__ fail_list, const int* __restrict__ fail_count, int slots,
    double* __restrict__ lst_d, int* __restrict__ lst_i, const int64_t* __restrict__ seg_off, int nseg) {
    // (with seg_off: each row searches only its own segment's references)
    __shared__ double sd[4][KNN_FB_K];
    __shared__ int si[4][KNN_FB_K];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nfail = *fail_count;
    const int S = knn_fb_splits(nfail, slots);
    for (int64_t w = blockIdx.x; w < (int64_t)nfail * S; w += gridDim.x) {
        const int f = (int)(w / S), sp = (int)(w - (int64_t)f * S);
        const int q = fail_list[f];
        int s0 = 0, s1 = n;  // the row's reference range (its segment)
        if (seg_off) {
            const int sg = knn_seg_of(seg_off, nseg, q);
            s0 = (int)seg_off[sg];
            s1 = (int)seg_off[sg + 1];
        }
        const int span = (s1 - s0 + S - 1) / S;
        const int j0 = s0 + sp * span, j1 = min(s1, j0 + span);
        double xq[DMAX];
#pragma unroll
        for (int k = 0; k < DMAX; ++k) xq[k] = k < d ? rows[(int64_t)q * d + k] : 0.0;
        double lv[FBK];
        int li[FBK];
#pragma unroll
        for (int t = 0; t < FBK; ++t) {
            lv[t] = INFINITY;
            li[t] = 0x7fffffff;
        }
        for (int j = j0 + threadIdx.x; j < j1; j += 256) {
            const double* y = rows + (int64_t)j * d;
            double yv[DMAX];
            if ((d & 1) == 0) {  // 16-B aligned rows: half the load instructions
                const double2* y2 = reinterpret_cast<const double2*>(y);
#pragma unroll
                for (int k2 = 0; k2 < DMAX / 2; ++k2) {
                    const double2 v = 2 * k2 < d ? y2[k2] : make_double2(0.0, 0.0);
                    yv[2 * k2] = v.x;
                    yv[2 * k2 + 1] = v.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < DMAX; ++k) yv[k] = k < d ? y[k] : 0.0;
            }
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < DMAX; ++k)
                if (k < d) {
                    const double t = __dsub_rn(xq[k], yv[k]);
                    s = __dadd_rn(s, __dmul_rn(t, t));
                }
            if (j == q || !(s < lv[FBK - 1])) continue;  // j ascending per thread
            double cv = s;
            int ci = j;
#pragma unroll
            for (int t = 0; t < FBK; ++t) {
                bool sw = key_less(cv, ci, lv[t], li[t]);
                double tv = lv[t];
                int ti = li[t];
                lv[t] = sw ? cv : tv;
                li[t] = sw ? ci : ti;
                cv = sw ? tv : cv;
                ci = sw ? ti : ci;
            }
        }
        // per-wave merge of 64 sorted lists -> sd[wv][0..kmax)
        for (int r = 0; r < kmax; ++r) {
            double bk = lv[0];
            int bi = li[0];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                double ok = __shfl_xor(bk, o, 64);
                int oi = __shfl_xor(bi, o, 64);
                if (key_less(ok, oi, bk, bi)) {
                    bk = ok;
                    bi = oi;
                }
            }
            if (lane == 0) {
                sd[wv][r] = bk;
                si[wv][r] = bi;
            }
            if (bi != 0x7fffffff && li[0] == bi) {  // the winning thread pops its head (ids are unique)
#pragma unroll
                for (int t = 0; t < FBK - 1; ++t) {
                    lv[t] = lv[t + 1];
                    li[t] = li[t + 1];
                }
                lv[FBK - 1] = INFINITY;
                li[FBK - 1] = 0x7fffffff;
            }
        }
        __syncthreads();
        if (wv == 0) {
            // lanes 0..3 walk the 4 wave lists; k rounds of arg-min over heads
            int pos = 0;
            double* od = lst_d + w * KNN_FB_K;
            int* oi_ = lst_i + w * KNN_FB_K;
            for (int r = 0; r < kmax; ++r) {
                double bk = INFINITY;
                int bi = 0x7fffffff;
                if (lane < 4 && pos < kmax) {
                    bk = sd[lane][pos];
                    bi = si[lane][pos];
                }
                const double mk = bk;
                const int mi = bi;
#pragma unroll
                for (int o = 2; o > 0; o >>= 1) {
                    double ok = __shfl_xor(bk, o, 64);
                    int oi = __shfl_xor(bi, o, 64);
                    if (key_less(ok, oi, bk, bi)) {
                        bk = ok;
                        bi = oi;
                    }
                }
                if (lane == 0) {
                    od[r] = bk;
                    oi_[r] = bi;
                }
                if (lane < 4 && mi == bi && mk == bk) ++pos;
            }
        }
        __syncthreads();
    }
}

// One wave per failed row: lane s walks the sorted list of range s.
__global__ __launch_bounds__(64) void knn_fallback_merge_kernel(
    int kmax, const int* __restrict__ fail_list, const int* __restrict__ fail_count, int slots,
    const double* __restrict__ lst_d, const int* __restrict__ lst_i,
    int32_t* __restrict__ out_idx, double* __restrict__ out_dist, const int64_t* __restrict__ seg_off, int nseg,
    bool dist_sq, bool seg_local = true) {
    const int lane = threadIdx.x;
    const int nfail = *fail_count;
    const int S = knn_fb_splits(nfail, slots);
    for (int f = blockIdx.x; f < nfail; f += gridDim.x) {
        const int q = fail_list[f];
        const int base = (seg_off && seg_local) ? (int)seg_off[knn_seg_of(seg_off, nseg, q)] : 0;
        const double* ld = lst_d + (int64_t)f * S * KNN_FB_K + (int64_t)lane * KNN_FB_K;
        const int* li = lst_i + (int64_t)f * S * KNN_FB_K + (int64_t)lane * KNN_FB_K;
        int pos = 0;
        for (int r = 0; r < kmax; ++r) {
            double bk = INFINITY;
            int bi = 0x7fffffff;
            if (lane < S && pos < kmax) {
                bk = ld[pos];
                bi = li[pos];
            }
            const double mk = bk;
            const int mi = bi;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                double ok = __shfl_xor(bk, o, 64);
                int oi = __shfl_xor(bi, o, 64);
                if (key_less(ok, oi, bk, bi)) {
                    bk = ok;
                    bi = oi;
                }
            }
            if (lane == 0) {
                out_idx[(int64_t)q * kmax + r] = bi - base;
                if (out_dist) out_dist[(int64_t)q * kmax + r] = dist_sq ? bk : sqrt(bk);
            }
            if (lane < S && mi == bi && mk == bk) ++pos;
        }
    }
}

// --------------------------------------------------------------- driver --
extern "C" int ccg_gather_rows_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                                   const int32_t* idx, int64_t n, double* rows, void* stream) {
    CCG_REQUIRE(ctx && pcs && idx && rows, "ccg_gather_rows_dev: NULL argument");
    CCG_REQUIRE(N > 0 && n > 0 && d > 0, "ccg_gather_rows_dev: bad sizes");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    if (d <= 16) gather_rows_kernel<16><<<(unsigned)ccg_cdiv(n, 16), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    else if (d <= 32) gather_rows_kernel<32><<<(unsigned)ccg_cdiv(n, 8), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    else gather_rows_kernel<64><<<(unsigned)ccg_cdiv(n, 4), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// row-major source: GR_LPR lanes per output row (a power of two >= the
// row's 16-byte pieces, d <= 2 GR_LPR), 256 / GR_LPR rows per block: no
// per-element division (round 4 divided a 64-bit thread index by d / 2:
// ~19 us per 90k-row bootstrap at d = 30).  Odd d: one value per lane.
template <int LPR>
__global__ __launch_bounds__(256) void gather_rows_rm_kernel(const double* __restrict__ pcs, int64_t N, int d,
                                                             const int32_t* __restrict__ idx, int64_t n,
                                                             double* __restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    const int k = threadIdx.x & (LPR - 1);
    if (i >= n) return;
    const int c = idx[i];
    const bool ok = c >= 0 && c < N;
    if ((d & 1) == 0) {
        const int h = d >> 1;
        if (k < h)
            reinterpret_cast<double2*>(rows)[i * h + k] =
                ok ? reinterpret_cast<const double2*>(pcs)[(int64_t)c * h + k] : make_double2(0.0, 0.0);
    } else {
        for (int kk = k; kk < d; kk += LPR) rows[i * d + kk] = ok ? pcs[(int64_t)c * d + kk] : 0.0;
    }
}

// lanes per row: the row's 16-byte pieces (or values, odd d) rounded up to a power of two, <= 64
static void knn_gather_rm(const double* pcs, int64_t N, int d, const int32_t* idx, int64_t n, double* rows,
                          hipStream_t st) {
    const int pieces = (d & 1) == 0 ? d / 2 : d;
    if (pieces <= 8) gather_rows_rm_kernel<8><<<(unsigned)ccg_cdiv(n, 32), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    else if (pieces <= 16) gather_rows_rm_kernel<16><<<(unsigned)ccg_cdiv(n, 16), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    else if (pieces <= 32) gather_rows_rm_kernel<32><<<(unsigned)ccg_cdiv(n, 8), 256, 0, st>>>(pcs, N, d, idx, n, rows);
    else gather_rows_rm_kernel<64><<<(unsigned)ccg_cdiv(n, 4), 256, 0, st>>>(pcs, N, d, idx, n, rows);
}

extern "C" int ccg_gather_rows_rm_dev(ccg_ctx* ctx, const double* pcs_rm, int64_t N, int d, const int32_t* idx,
                                      int64_t n, double* rows, void* stream) {
    CCG_REQUIRE(ctx && pcs_rm && idx && rows, "ccg_gather_rows_rm_dev: NULL argument");
    CCG_REQUIRE(N > 0 && n > 0 && d > 0, "ccg_gather_rows_rm_dev: bad sizes");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    knn_gather_rm(pcs_rm, N, d, idx, n, rows, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// Batched-segment description (ccg_knn_segments_dev): screening positions
// are the segments laid end to end, each padded to a multiple of KNN_QPB.
struct KnnSegs {
    int nseg;
    const int64_t* seg_off;  // device, nseg + 1 row offsets
    int64_t npos;            // padded positions
    int* perm;               // device, position -> row (-1: padding); knn_run writes each segment's Morton order
    const int4* blk;         // device, per query block: chunk range [x, y), query limit z
    const int64_t* pos_off;  // device, nseg + 1 position offsets (multiples of KNN_QPB)
};

// (segment << 15 | Morton code, row) pairs: rows grouped by segment, each
// segment in the spatial order of its leading coordinates
__global__ void knn_seg_morton_keys_kernel(const double* __restrict__ rows, int64_t n, int d,
                                           const unsigned* __restrict__ bnd, const int64_t* __restrict__ seg_off,
                                           int nseg, int32_t* __restrict__ keys, int32_t* __restrict__ ids) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const unsigned sg = (unsigned)knn_seg_of(seg_off, nseg, r);
    keys[r] = (int32_t)((sg << (KNN_MD * KNN_MORTON_BITS)) | morton_key(rows + r * d, d, bnd));
    ids[r] = (int32_t)r;
}

// sorted rank t (rows grouped by segment) -> the segment's padded position
__global__ void knn_seg_perm_kernel(int64_t n, const int32_t* __restrict__ sorted_ids,
                                    const int64_t* __restrict__ seg_off, const int64_t* __restrict__ pos_off, int nseg,
                                    int* __restrict__ perm) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int s = knn_seg_of(seg_off, nseg, t);
    perm[pos_off[s] + (t - seg_off[s])] = sorted_ids[t];
}

// Host plan of a segmented run: segment s occupies positions [po_s, po_s +
// n_s), po_s a multiple of KNN_QPB; each query block scans its segment's
// chunks.  Uploads seg_off, the position offsets, the blocks and an identity
// permutation (-1 padding; knn_run reorders each segment spatially) into
// WS_SEGS on st.  The host vectors must outlive the uploads: the caller
// synchronises st before they go out of scope.
static int knn_seg_plan(ccg_ctx* ctx, const int64_t* seg_off, int nseg, int d, int kmax, hipStream_t st,
                        std::vector<int64_t>& po, std::vector<int>& hperm, std::vector<int4>& hblk, KnnSegs* out) {
    po.assign(nseg + 1, 0);
    for (int s = 0; s < nseg; ++s) {
        const int64_t ns = seg_off[s + 1] - seg_off[s];
        CCG_REQUIRE(ns >= kmax + 1, "kNN segments: segment %d has %lld rows, needs >= kmax+1 = %d", s,
                    (long long)ns, kmax + 1);
        po[s + 1] = po[s] + ccg_cdiv(ns, KNN_QPB) * KNN_QPB;
    }
    const int64_t npos = po[nseg];
    CCG_REQUIRE(npos < (1LL << 30), "kNN segments: too many positions");
    const int64_t nblk = npos / KNN_QPB;
    const int KNN_CHUNK = knn_chunk(knn_ksteps(d));
    hperm.assign(npos, -1);
    hblk.resize(nblk);
    for (int s = 0; s < nseg; ++s) {
        const int64_t ns = seg_off[s + 1] - seg_off[s];
        for (int64_t i = 0; i < ns; ++i) hperm[po[s] + i] = (int)(seg_off[s] + i);
        const int cl = (int)(po[s] / KNN_CHUNK), ch = (int)((po[s] + ns + KNN_CHUNK - 1) / KNN_CHUNK);
        for (int64_t b = po[s] / KNN_QPB; b < po[s + 1] / KNN_QPB; ++b)
            hblk[b] = make_int4(cl, ch, (int)(po[s] + ns), 0);
    }
    const size_t offb = ccg_cdiv(sizeof(int64_t) * (nseg + 1), 16) * 16;
    char* tab = (char*)ccg_ws(ctx, WS_SEGS, 2 * offb + sizeof(int4) * nblk + sizeof(int) * npos + 64);
    if (!tab) return CCG_ENOMEM;
    int64_t* d_off = (int64_t*)tab;
    int64_t* d_po = (int64_t*)(tab + offb);
    int4* d_blk = (int4*)(tab + 2 * offb);
    int* d_perm = (int*)(d_blk + nblk);
    // (host tables through the context's pinned ring: they are freed when the call returns)
    int rc = ccg_h2d_staged(ctx, d_off, seg_off, sizeof(int64_t) * (nseg + 1), st);
    if (!rc) rc = ccg_h2d_staged(ctx, d_po, po.data(), sizeof(int64_t) * (nseg + 1), st);
    if (!rc) rc = ccg_h2d_staged(ctx, d_blk, hblk.data(), sizeof(int4) * nblk, st);
    if (!rc) rc = ccg_h2d_staged(ctx, d_perm, hperm.data(), sizeof(int) * npos, st);
    if (rc) return rc;
    *out = KnnSegs{nseg, d_off, npos, d_perm, d_blk, d_po};
    return CCG_OK;
}

// ------------------------------------------ exact search by a radius --
// The exact search of the rows certification (or a cell table) could not
// settle, when the caller knows for each such row a radius tau that at least
// kmax references lie within (certify: the kmax-th exact candidate distance;
// a candidate set is a subset of the references, so its kmax-th distance
// bounds the true kmax-th from above):
//   prep   : each failed row's fp16 hi/lo image at its own power-of-two
//            scale, its part of the test and its id;
//   scan   : 128 references per block on the fp16 matrix core against the
//            failed rows staged in groups of 128 (below); every reference
//            that passes the pre-test (a superset of those within tau) is
//            appended to the row's candidate buffer (rare: tau is tight);
//   select : one wave per row takes the candidates' exact fp64 d2 (the
//            contract's unfused dimension-order arithmetic), keeps those
//            within tau, sorts them by (d2, row) and writes the first kmax.
// Rows with tau = +inf, past KNN_FX_ROWS, or with more than KNN_FX_CAP
// candidates (massive ties at the radius) go to the per-thread-list kernels
// below.
#define KNN_FX_CAP 1024
#define KNN_FX_ROWS 16384
#define KNN_FX_CHUNK 64
#define KNN_FX_PREP_GRID 16  // failed-row prep: grid-stride over <= KNN_FX_ROWS rows

template <int DMAX>
__device__ __forceinline__ double knn_exact_d2(const double (&xq)[DMAX], const double* y, int d) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k)
        if (k < d) {
            const double t = __dsub_rn(xq[k], y[k]);
            s = __dadd_rn(s, __dmul_rn(t, t));
        }
    return s;
}

// In-LDS bitonic sort of m (a power of two) (key, id) pairs, ascending.
__device__ void knn_lds_bitonic(double* kd, int* ki, int m) {
    for (int k = 2; k <= m; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                const int p = i ^ j;
                if (p > i) {
                    const bool up = (i & k) == 0;
                    const double a = kd[i], b = kd[p];
                    const int ia = ki[i], ib = ki[p];
                    if (key_less(b, ib, a, ia) == up) {
                        kd[i] = b;
                        kd[p] = a;
                        ki[i] = ib;
                        ki[p] = ia;
                    }
                }
            }
        }
    __syncthreads();
}

// The scan on the fp16 matrix core (round 5).  Every row is scaled by its
// own power of two 2^e (max_k |x_k| 2^e < 2^12) and split into fp16 hi + lo
// (knn_split16); x'.y' ~ hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_f16
// with A = 32 failed rows (LDS) and B = 32 references (registers), so lane
// (h, j) gets 16 failed rows against reference j, and x.y = x'.y' 2^-(ex+ey)
// (a product of powers of two: one fp32 multiply, exact).  The error of the
// product is below 2^-17.2 |x||y| (split residuals 2^-22 relative per
// factor, fp32 accumulation of 48 KSTEPS exact products) plus the parts
// flushed below 2^-14 of each scaled row (< 2^-25 max|x| per component),
// inside the margin the test takes: a pair within the radius,
// nx + ny - 2 x.y <= tau, passes
//   2 x.y (fp32, from the matrix core) >= A_x + B_y,
//   A_x = (1 - 2^-14) nx - tau - 2^-60 - 2^-21 (nx + tau),
//   B_y = (1 - 2^-14 - 2^-21) ny
// (both rounded down to fp32: 2^-14 (nx + ny) covers the product's error
// and the fp32 sums), so the candidates are a superset of the pairs within
// the radius, and knn_fx_select_kernel keeps exactly those whose fp64 d2
// is.  Per pair 3 MACs of 16 KSTEPS dims on the matrix core and ~4 VALU,
// against the round-4 scan's 16 KSTEPS packed fp32 FMAs and 8 LDS reads.
// (A first matrix-core version, round 5, scaled by the rows' global max|x|:
// its same-address atomicMax in the distinct-row gather cost 80 us per
// bootstrap; per-row scales need no reduction.)
// Failed rows: KNN_FXQ per staged group; prep writes each row's image
// (chunks (s, hi/lo, h) of 8 fp16, chunk q of row c at q ^ (c & (NCH - 1))),
// A_x, its scale 2^-e and its id.
#define KNN_FXQ 128

// Segmented exact search (a batch of bootstraps, ccg_knn_boots_table_dev):
// the references of segment s are [soff[s], soff[s+1]) and its failed
// entries sit at list[soff[s] .. soff[s] + fcnt[s]) (each segment appends to
// its own region).  The prep compacts them, segment by segment, into
// cf_list / cf_tau (cf_count entries; segment s from cf_off[s]) and writes
// each compact entry's segment (qsg); the scan walks, per block of
// references, only the failed rows of the segments its references belong to
// (a pair of different segments never becomes a candidate); the select runs
// on the compact list.  nseg <= KNN_SEG_MAX.
#define KNN_SEG_MAX 64
struct FxSeg {
    const int* fcnt;
    const int64_t* soff;
    int nseg;
    int* cf_list;
    double* cf_tau;
    int* cf_count;
    int* cf_off;
    int* qsg;
};

__device__ __forceinline__ int knn_row_exp(double mx) {
    return mx > 0.0 ? 11 - ilogb(mx) : 0;  // mx 2^e < 2^12
}

template <int KSTEPS, bool SEG>
__global__ __launch_bounds__(256) void knn_fx_prep16_kernel(const double* __restrict__ rows, int d,
                                                            const int* __restrict__ fail_list,
                                                            const int* __restrict__ fail_count,
                                                            const double* __restrict__ fail_tau,
                                                            uint4* __restrict__ qimg, float* __restrict__ qa,
                                                            float* __restrict__ qs, int* __restrict__ qid,
                                                            int* __restrict__ ovf_count, FxSeg sg) {
    constexpr int NCH = 4 * KSTEPS;
    __shared__ int sfo[KNN_SEG_MAX + 1];  // (SEG) compact offsets of the segments' failed entries
    if (blockIdx.x == 0 && threadIdx.x == 0) *ovf_count = 0;
    int F;
    if (SEG) {
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            int incl = lane < sg.nseg ? sg.fcnt[lane] : 0;
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            sfo[lane + 1] = incl;
            if (lane == 0) sfo[0] = 0;
        }
        __syncthreads();
        F = sfo[sg.nseg];
        if (blockIdx.x == 0) {
            for (int t = threadIdx.x; t <= sg.nseg; t += blockDim.x) sg.cf_off[t] = sfo[t];
            if (threadIdx.x == 0) *sg.cf_count = F;
        }
    } else {
        F = *fail_count;
    }
    const int nf = min(F, KNN_FX_ROWS);
    const int nfp = (nf + KNN_FXQ - 1) / KNN_FXQ * KNN_FXQ;
    const int fend = SEG ? max(nfp, F) : nfp;  // (SEG: entries past KNN_FX_ROWS are compacted too)
    for (int f = blockIdx.x * blockDim.x + threadIdx.x; f < fend; f += gridDim.x * blockDim.x) {
        const bool valid = f < nf;
        int q;
        double t;
        if (SEG) {
            q = -1;
            t = -1.0;
            if (f < F) {
                int lo = 0, hi = sg.nseg;  // the segment: the last s with sfo[s] <= f
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (sfo[mid] <= f) lo = mid; else hi = mid;
                }
                const int64_t p = sg.soff[lo] + (f - sfo[lo]);
                q = fail_list[p];
                t = fail_tau[p];
                sg.cf_list[f] = q;
                sg.cf_tau[f] = t;
                if (valid) sg.qsg[f] = lo;
            }
            if (f >= nfp) continue;
            if (!valid) t = -1.0;
        } else {
            q = valid ? fail_list[f] : -1;
            t = valid ? fail_tau[f] : -1.0;
        }
        if (!(t < INFINITY)) t = -1.0;  // no radius: the per-thread-list kernels
        double x[KSTEPS * 16];
        double mx = 0.0, nx = 0.0;
#pragma unroll
        for (int k = 0; k < KSTEPS * 16; ++k) {
            x[k] = (valid && k < d) ? rows[(int64_t)q * d + k] : 0.0;
            mx = fmax(mx, fabs(x[k]));
            nx = fma(x[k], x[k], nx);
        }
        const int e = knn_row_exp(mx);
        _Float16 hv[NCH * 8];
#pragma unroll
        for (int k = 0; k < KSTEPS * 16; ++k) {
            _Float16 hi, lo;
            knn_split16(ldexp(x[k], e), hi, lo);
            const int s = k >> 4, h = (k >> 3) & 1, i = k & 7;
            hv[(s * 4 + h) * 8 + i] = hi;
            hv[(s * 4 + 2 + h) * 8 + i] = lo;
        }
        const int c = f & (NCH - 1);  // the swizzle key (the scan stages rows g0 .. g0 + KNN_FXQ, any g0)
        uint4* out = qimg + (int64_t)f * NCH;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) out[ch ^ c] = *reinterpret_cast<const uint4*>(&hv[ch * 8]);
        qa[f] = t < 0.0 ? INFINITY : __double2float_rd((1.0 - 0x1p-14) * nx - t - 0x1p-60 - 0x1p-21 * (nx + t));
        qs[f] = ldexpf(1.0f, -e);
        qid[f] = q;
    }
}

// Grid: 128 references per block (4 waves x 32); every block walks the
// failed rows in staged groups of KNN_FXQ.  An empty failed list exits at
// once.
template <int KSTEPS, bool SEG>
__global__ __launch_bounds__(256) void knn_fx_scan16_kernel(const double* __restrict__ rows, int n, int d,
                                                            const int* __restrict__ fail_count,
                                                            const uint4* __restrict__ qimg,
                                                            const float* __restrict__ qa,
                                                            const float* __restrict__ qs,
                                                            const int* __restrict__ qid, int* __restrict__ cnt,
                                                            int* __restrict__ bi, FxSeg sg) {
    constexpr int NCH = 4 * KSTEPS;
    __shared__ uint4 sq[KNN_FXQ * NCH];
    __shared__ __attribute__((aligned(16))) float sa[KNN_FXQ];
    __shared__ __attribute__((aligned(16))) float ss[KNN_FXQ];
    __shared__ int sid[KNN_FXQ];
    __shared__ int ssg[SEG ? KNN_FXQ : 1];
    const int nf = min(*fail_count, KNN_FX_ROWS);
    if (nf == 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, j = lane & 31;
    // the wave's 32 references: B fragments (dims 16 s + 8 h ..), the
    // reference's scale and its part of the test
    const int jr = blockIdx.x * 128 + wave * 32 + j;
    const bool inr = jr < n;
    int gb = 0, ge = nf, sj = 0;
    if (SEG) {  // the failed rows of the segments of the block's references (block-uniform range)
        const int sa0 = knn_seg_of(sg.soff, sg.nseg, (int64_t)blockIdx.x * 128);
        const int sb0 = knn_seg_of(sg.soff, sg.nseg, min((int64_t)blockIdx.x * 128 + 127, (int64_t)n - 1));
        gb = sg.cf_off[sa0];
        ge = min(sg.cf_off[sb0 + 1], nf);
        if (gb >= ge) return;
        sj = inr ? knn_seg_of(sg.soff, sg.nseg, jr) : -1;
    }
    double y[KSTEPS * 8];
    double my = 0.0, ny = 0.0;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int k = 16 * s + 8 * h + i;
            y[8 * s + i] = (inr && k < d) ? rows[(int64_t)jr * d + k] : 0.0;
            my = fmax(my, fabs(y[8 * s + i]));
            ny = fma(y[8 * s + i], y[8 * s + i], ny);
        }
    my = fmax(my, __shfl_xor(my, 32, 64));
    ny += __shfl_xor(ny, 32, 64);
    const int ey = knn_row_exp(my);
    h8 bh[KSTEPS], bl[KSTEPS];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            _Float16 hi, lo;
            knn_split16(ldexp(y[8 * s + i], ey), hi, lo);
            bh[s][i] = hi;
            bl[s][i] = lo;
        }
    const float sy = 2.0f * ldexpf(1.0f, -ey);  // (the test's factor 2 folded in)
    const float bj = inr ? __double2float_rd((1.0 - 0x1p-14 - 0x1p-21) * ny) : INFINITY;
    for (int g0 = gb; g0 < ge; g0 += KNN_FXQ) {
        const int nq = min(KNN_FXQ, ge - g0);
        __syncthreads();  // the previous group's reads of the stage are done
        // (SEG: g0 need not be a multiple of KNN_FXQ; the buffers hold
        // KNN_FX_ROWS + KNN_FXQ rows, and rows past nq are masked below)
        for (int t = threadIdx.x; t < KNN_FXQ * NCH; t += 256) sq[t] = qimg[(int64_t)g0 * NCH + t];
        if (threadIdx.x < KNN_FXQ) {
            sa[threadIdx.x] = qa[g0 + threadIdx.x];  // (the prep writes whole groups: INFINITY past nf)
            ss[threadIdx.x] = qs[g0 + threadIdx.x];
            sid[threadIdx.x] = qid[g0 + threadIdx.x];
            if (SEG) ssg[threadIdx.x] = sg.qsg[g0 + threadIdx.x];
        }
        __syncthreads();
        for (int t = 0; t < (nq + 31) >> 5; ++t) {  // block-uniform
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
            const int c = t * 32 + j;
            const uint4* ar = sq + c * NCH;
            const int cx = (g0 + c) & (NCH - 1);  // the prep's swizzle key of failed row g0 + c
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                const uint4 ahv = ar[(s * 4 + h) ^ cx];
                const uint4 alv = ar[(s * 4 + 2 + h) ^ cx];
                const h8 ah = *reinterpret_cast<const h8*>(&ahv);
                const h8 al = *reinterpret_cast<const h8*>(&alv);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc, 0, 0, 0);
            }
            // register r holds failed row t*32 + (r & 3) + 8 (r >> 2) + 4h against reference jr
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 a4 = *reinterpret_cast<const float4*>(&sa[t * 32 + 8 * g + 4 * h]);
                const float4 s4 = *reinterpret_cast<const float4*>(&ss[t * 32 + 8 * g + 4 * h]);
                const float av[4] = {a4.x, a4.y, a4.z, a4.w};
                const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (acc[4 * g + q] * (sv[q] * sy) >= av[q] + bj) {  // rare: the candidates
                        const int i = t * 32 + 8 * g + 4 * h + q;
                        if (i < nq && jr != sid[i] && (!SEG || ssg[i] == sj)) {
                            const int slot = atomicAdd(&cnt[g0 + i], 1);
                            if (slot < KNN_FX_CAP) bi[(int64_t)(g0 + i) * KNN_FX_CAP + slot] = jr;
                        }
                    }
                }
            }
        }
    }
}

#ifndef WAVE_LDS_SYNC
// a wave's LDS writes are visible to its other lanes' later LDS reads (the
// LDS pipeline is in order per wave); the clobber stops compiler reordering
#define WAVE_LDS_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)
#endif

// One wave per failed row: the exact fp64 d2 (the contract's arithmetic)
// of every candidate, those within the radius sorted by (d2, row) -- a wave
// bitonic sort in registers for <= 64 candidates (the usual ~26), a wave
// bitonic sort in the wave's LDS slice beyond -- and the first kmax written.
// (Round 3's block per row ran its LDS sort with two block barriers per
// stage and took two rounds of the grid for ~270 rows.)
template <int DMAX>
__global__ __launch_bounds__(256) void knn_fx_select_kernel(const double* __restrict__ rows, int d, int kmax,
                                                            const int* __restrict__ fail_list,
                                                            const int* __restrict__ fail_count,
                                                            const double* __restrict__ fail_tau,
                                                            int* __restrict__ cnt, const int* __restrict__ bi,
                                                            int32_t* __restrict__ out_idx,
                                                            double* __restrict__ out_dist, bool dist_sq,
                                                            int* __restrict__ ovf_list, int* __restrict__ ovf_count) {
    __shared__ double kd_all[4][KNN_FX_CAP];
    __shared__ int ki_all[4][KNN_FX_CAP];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* kd = kd_all[wv];
    int* ki = ki_all[wv];
    const int nf = *fail_count;
    for (int f = blockIdx.x * 4 + wv; f < nf; f += gridDim.x * 4) {
        const int q = fail_list[f];
        int c = KNN_FX_CAP + 1;
        double t = INFINITY;
        if (f < KNN_FX_ROWS) {
            c = cnt[f];
            t = fail_tau[f];
            if (!(t < INFINITY)) c = KNN_FX_CAP + 1;
        }
        const bool ovf = c > KNN_FX_CAP || c < kmax;  // (c is in a register before the counter is cleared)
        if (f < KNN_FX_ROWS && lane == 0) cnt[f] = 0;    // zero for the next call
        if (ovf) {  // the per-thread-list kernels take it
            if (lane == 0) ovf_list[atomicAdd(ovf_count, 1)] = q;
            continue;
        }
        double xq[DMAX];
#pragma unroll
        for (int k = 0; k < DMAX; ++k) xq[k] = k < d ? rows[(int64_t)q * d + k] : 0.0;
        if (c <= 64) {
            double v = INFINITY;
            int jx = 0x7fffffff;
            if (lane < c) {
                const int jj = bi[(int64_t)f * KNN_FX_CAP + lane];
                const double e = knn_exact_d2<DMAX>(xq, rows + (int64_t)jj * d, d);
                if (e <= t) {
                    v = e;
                    jx = jj;
                }
            }
            if (__popcll(__ballot(jx != 0x7fffffff)) < kmax) {  // (cannot happen: tau bounds kmax exact distances)
                if (lane == 0) ovf_list[atomicAdd(ovf_count, 1)] = q;
                continue;
            }
            for (int k = 2; k <= 64; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const double ov = __shfl_xor(v, j, 64);
                    const int oj = __shfl_xor(jx, j, 64);
                    const bool up = (lane & k) == 0, lo = (lane & j) == 0;
                    const bool take = (lo == up) ? key_less(ov, oj, v, jx) : key_less(v, jx, ov, oj);
                    if (take) {
                        v = ov;
                        jx = oj;
                    }
                }
            if (lane < kmax) {
                out_idx[(int64_t)q * kmax + lane] = jx;
                if (out_dist) out_dist[(int64_t)q * kmax + lane] = dist_sq ? v : sqrt(v);
            }
            continue;
        }
        int m = 128;
        while (m < c) m <<= 1;
        int nin = 0;
        for (int s0 = 0; s0 < m; s0 += 64) {
            const int s = s0 + lane;
            double v = INFINITY;
            int jx = 0x7fffffff;
            if (s < c) {
                const int jj = bi[(int64_t)f * KNN_FX_CAP + s];
                const double e = knn_exact_d2<DMAX>(xq, rows + (int64_t)jj * d, d);
                if (e <= t) {
                    v = e;
                    jx = jj;
                }
            }
            nin += __popcll(__ballot(jx != 0x7fffffff));
            kd[s] = v;
            ki[s] = jx;
        }
        if (nin < kmax) {
            if (lane == 0) ovf_list[atomicAdd(ovf_count, 1)] = q;
            continue;
        }
        for (int k = 2; k <= m; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                WAVE_LDS_SYNC();
                for (int i = lane; i < m; i += 64) {
                    const int p = i ^ j;
                    if (p > i) {
                        const bool up = (i & k) == 0;
                        const double x0 = kd[i], x1 = kd[p];
                        const int i0 = ki[i], i1 = ki[p];
                        if (key_less(x1, i1, x0, i0) == up) {
                            kd[i] = x1;
                            kd[p] = x0;
                            ki[i] = i1;
                            ki[p] = i0;
                        }
                    }
                }
            }
        WAVE_LDS_SYNC();
        for (int r = lane; r < kmax; r += 64) {
            out_idx[(int64_t)q * kmax + r] = ki[r];
            if (out_dist) out_dist[(int64_t)q * kmax + r] = dist_sq ? kd[r] : sqrt(kd[r]);
        }
        WAVE_LDS_SYNC();  // the slice is rewritten by the wave's next row
    }
}

// The failed-row list of n rows and the radii beside it (one workspace).
static int* knn_fail_ws(ccg_ctx* ctx, int64_t n, double** tau) {
    const size_t li = (size_t)ccg_cdiv(n, 2) * 2;
    int* p = (int*)ccg_ws(ctx, WS_FAIL_LIST, sizeof(int) * li + sizeof(double) * (size_t)n + 16);
    if (p && tau) *tau = (double*)(p + li);
    return p;
}

// Workspace bytes of the exact search of n rows (knn_fallback_launch): the
// radius search's WS_FX_A / WS_FX_C, the per-thread-list search's WS_FB_D /
// WS_FB_I.  knn_fx_reserve sizes them up front (a batch runs the search on
// its distinct cells, then on its rows: no growth -- a device
// synchronisation -- between the two, nor inside a graph capture).
static size_t knn_fx_ints(int64_t n) { return (size_t)KNN_FX_ROWS + 64 + (size_t)n + 4 * ((size_t)KNN_FX_ROWS + KNN_FXQ) + 4; }
static size_t knn_fxa_bytes(int64_t n, int d) {
    const int nch = d <= 16 ? 4 : (d <= 32 ? 8 : 16);
    return sizeof(int) * knn_fx_ints(n) + 16 + sizeof(uint4) * ((size_t)KNN_FX_ROWS + KNN_FXQ) * nch;
}
static size_t knn_fxc_bytes(int64_t n) { return (sizeof(double) + sizeof(int)) * (size_t)n + sizeof(int) * (KNN_SEG_MAX + 8); }
static int knn_fb_slots(int64_t n) { return (int)std::max<int64_t>(n, KNN_FB_SLOTS); }
static int knn_fx_reserve(ccg_ctx* ctx, int64_t n, int d) {
    const size_t fb = (size_t)knn_fb_slots(n) * KNN_FB_K;
    if (!ccg_ws(ctx, WS_FX_A, knn_fxa_bytes(n, d)) || !ccg_ws(ctx, WS_FX_C, knn_fxc_bytes(n)) ||
        !ccg_ws(ctx, WS_FX_B, sizeof(int) * (size_t)KNN_FX_ROWS * KNN_FX_CAP) ||
        !ccg_ws(ctx, WS_FB_D, sizeof(double) * fb) || !ccg_ws(ctx, WS_FB_I, sizeof(int) * fb))
        return CCG_ENOMEM;
    return CCG_OK;
}

// Exact fp64 search (fallback + merge kernels) for the rows in fail_list.
// seg_fcnt (segmented batch, ccg_knn_boots_table_dev): segment s's failed
// rows are fail_list[seg_off[s] .. + seg_fcnt[s]) with radii in fail_tau,
// its references [seg_off[s], seg_off[s+1]); outputs are ids of the
// concatenation (not segment-local).
static int knn_fallback_launch(ccg_ctx* ctx, const double* rows, int64_t n, int d, int kmax, const int* fail_list,
                               const int* fail_count, int32_t* out_idx, double* out_dist, const int64_t* seg_off,
                               int nseg, hipStream_t st, bool dist_sq = false, const double* fail_tau = nullptr,
                               const int* seg_fcnt = nullptr, const int** cf_out = nullptr,
                               const int** cf_count_out = nullptr) {
    bool seg_local = true;
    if (fail_tau && (!seg_off || seg_fcnt)) {
        // the radius search; its leftovers (overflow) continue below
        // WS_FX_A: counters [KNN_FX_ROWS], overflow count + list [64 + n], the
        // failed rows' A_x, scales, ids, segments [4 x (KNN_FX_ROWS + KNN_FXQ)]
        // and images [KNN_FX_ROWS + KNN_FXQ] (the segmented scan stages
        // groups from any row); WS_FX_C (segmented): the compact list and
        // radii [n], its count and segment offsets
        const size_t fxr = (size_t)KNN_FX_ROWS + KNN_FXQ;
        const size_t fx_ints = knn_fx_ints(n);
        char* fxa = (char*)ccg_ws(ctx, WS_FX_A, knn_fxa_bytes(n, d));
        int* cnt = (int*)fxa;
        int* bi = (int*)ccg_ws(ctx, WS_FX_B, sizeof(int) * (size_t)KNN_FX_ROWS * KNN_FX_CAP);
        if (!fxa || !bi) return CCG_ENOMEM;
        if (ctx->fx_zeroed != (void*)cnt) {  // fresh buffer: the select kernel keeps the counters zero afterwards
            CCG_HIP(hipMemsetAsync(cnt, 0, sizeof(int) * KNN_FX_ROWS, st));
            ctx->fx_zeroed = (void*)cnt;
        }
        int* ovf_count = cnt + KNN_FX_ROWS;
        int* ovf_list = ovf_count + 64;
        float* qa = (float*)(ovf_list + n);
        float* qs = qa + fxr;
        int* qid = (int*)(qs + fxr);
        int* qsg = qid + fxr;
        uint4* qimg = (uint4*)(fxa + ccg_cdiv(sizeof(int) * fx_ints, 16) * 16);
        const unsigned gs = (unsigned)ccg_cdiv(n, 128);
        FxSeg sg = {seg_fcnt, seg_off, nseg, nullptr, nullptr, nullptr, nullptr, qsg};
        const int* sl_list = fail_list;  // what the select walks
        const int* sl_count = fail_count;
        const double* sl_tau = fail_tau;
        if (seg_fcnt) {
            CCG_REQUIRE(nseg <= KNN_SEG_MAX, "knn: %d segments (max %d)", nseg, KNN_SEG_MAX);
            double* fxc = (double*)ccg_ws(ctx, WS_FX_C, knn_fxc_bytes(n));
            if (!fxc) return CCG_ENOMEM;
            sg.cf_tau = fxc;
            sg.cf_list = (int*)(fxc + n);
            sg.cf_count = sg.cf_list + n;
            sg.cf_off = sg.cf_count + 4;
            sl_list = sg.cf_list;
            sl_count = sg.cf_count;
            sl_tau = sg.cf_tau;
            if (cf_out) *cf_out = sg.cf_list;  // the compacted list (ccg_knn_last_fallback)
            if (cf_count_out) *cf_count_out = sg.cf_count;
        }
#define CCG_FX(DM_, KS_, SEG_)                                                                                    \
    do {                                                                                                         \
        knn_fx_prep16_kernel<KS_, SEG_><<<KNN_FX_PREP_GRID, 256, 0, st>>>(rows, d, fail_list, fail_count, fail_tau, \
                                                                          qimg, qa, qs, qid, ovf_count, sg);     \
        knn_fx_scan16_kernel<KS_, SEG_><<<gs, 256, 0, st>>>(rows, (int)n, d, sl_count, qimg, qa, qs, qid, cnt, bi, \
                                                            sg);                                                 \
        knn_fx_select_kernel<DM_><<<256, 256, 0, st>>>(rows, d, kmax, sl_list, sl_count, sl_tau, cnt, bi,         \
                                                       out_idx, out_dist, dist_sq, ovf_list, ovf_count);          \
    } while (0)
        if (seg_fcnt) {
            if (d <= 16) CCG_FX(16, 1, true);
            else if (d <= 32) CCG_FX(32, 2, true);
            else CCG_FX(64, 4, true);
        } else {
            if (d <= 16) CCG_FX(16, 1, false);
            else if (d <= 32) CCG_FX(32, 2, false);
            else CCG_FX(64, 4, false);
        }
#undef CCG_FX
        fail_list = ovf_list;
        fail_count = ovf_count;
        seg_local = !seg_fcnt;
    }
    const int fb_slots = knn_fb_slots(n);
    double* fb_d = (double*)ccg_ws(ctx, WS_FB_D, sizeof(double) * (size_t)fb_slots * KNN_FB_K);
    int* fb_i = (int*)ccg_ws(ctx, WS_FB_I, sizeof(int) * (size_t)fb_slots * KNN_FB_K);
    if (!fb_d || !fb_i) return CCG_ENOMEM;
#define CCG_FALLBACK(DM_, FK_)                                                                            \
    knn_fallback_kernel<DM_, FK_><<<KNN_FB_GRID, 256, 0, st>>>(rows, (int)n, d, kmax, fail_list, fail_count,      \
                                                               fb_slots,                                          \
                                                               fb_d, fb_i, seg_off, nseg)
    if (kmax <= KNN_KP) {  // per-thread lists of kmax <= 20 entries
        if (d <= 16) CCG_FALLBACK(16, KNN_KP);
        else if (d <= 32) CCG_FALLBACK(32, KNN_KP);
        else CCG_FALLBACK(64, KNN_KP);
    } else if (kmax <= KNN_KP_BIG) {
        if (d <= 16) CCG_FALLBACK(16, KNN_KP_BIG);
        else if (d <= 32) CCG_FALLBACK(32, KNN_KP_BIG);
        else CCG_FALLBACK(64, KNN_KP_BIG);
    } else {  // cell tables (kmax <= KNN_TAB_K): long lists, a rare path
        if (d <= 16) CCG_FALLBACK(16, KNN_FB_K);
        else if (d <= 32) CCG_FALLBACK(32, KNN_FB_K);
        else CCG_FALLBACK(64, KNN_FB_K);
    }
#undef CCG_FALLBACK
    knn_fallback_merge_kernel<<<KNN_FB_GRID, 64, 0, st>>>(kmax, fail_list, fail_count, fb_slots, fb_d, fb_i, out_idx,
                                                   out_dist, seg_off, nseg, dist_sq, seg_local);
    return CCG_OK;
}

// dist_sq: out_dist receives the squared distances (the certified fp64 sums)
static int knn_run(ccg_ctx* ctx, const double* rows, int64_t n, int d, int kmax, int32_t* out_idx,
                   double* out_dist, ccg_knn_stats* stats, hipStream_t st, const KnnSegs* sg, bool dist_sq = false,
                   const float* row_hint = nullptr) {
    const int KP = kmax <= KNN_KP ? KNN_KP : KNN_KP_BIG;
    const int64_t npos = sg ? sg->npos : n;  // screening positions
    int* cand_idx = (int*)ccg_ws(ctx, WS_CAND_IDX, sizeof(int) * npos * 2 * KP);
    float* cand_thr = (float*)ccg_ws(ctx, WS_CAND_THR, sizeof(float) * npos * 2);
    double* fail_tau = nullptr;
    int* fail_list = knn_fail_ws(ctx, n, &fail_tau);
    unsigned int* misc = (unsigned int*)ccg_ws(ctx, WS_MISC, 256);
    if (!cand_idx || !cand_thr || !fail_list || !misc) return CCG_ENOMEM;
    // misc: [0] max-norm / max|x| bits, [1] fail count, [2..3] double 1/sigma^2
    unsigned int* mbits = misc;
    int* fail_count = (int*)(misc + 1);
    double* inv_scale2 = (double*)(misc + 2);
    const int t_all = ccg_timer_start(ctx, CCG_KT_KNN_TOTAL, st);
    int rc = CCG_OK;
    const double err_ulps = KNN_ERR_ULPS_F16;
    const int* order_perm = nullptr;  // screening position -> bootstrap row
    {
        const int KSTEPS = knn_ksteps(d);
        const int KNN_CHUNK = knn_chunk(KSTEPS);
        const int64_t npad = ccg_cdiv(npos, KNN_CHUNK) * KNN_CHUNK;
        uint4* img = (uint4*)ccg_ws(ctx, WS_REFS32, (size_t)npad * 64 * KSTEPS + sizeof(float) * npad + 256);
        if (!img) return CCG_ENOMEM;
        float* pos_t0 = row_hint ? (float*)((char*)img + (size_t)npad * 64 * KSTEPS) : nullptr;
        unsigned* bnd = misc + 8;  // [2 KNN_MD]: minima then maxima of the leading coordinates
        const bool buckets = !sg && !KNN_NO_MORTON && KNN_MORTON_DIMS * KNN_MORTON_BITS <= 15;
        const int64_t NB = 1LL << (KNN_MORTON_DIMS * KNN_MORTON_BITS);
        int64_t* hist = nullptr;
        if (buckets) {
            hist = (int64_t*)ccg_ws(ctx, WS_ORDER, sizeof(int64_t) * (2 * (NB + 1)) + sizeof(int) * n + 64);
            if (!hist) return CCG_ENOMEM;
        }
        knn_init_kernel<<<buckets ? 64 : 1, 256, 0, st>>>(misc, bnd, hist, NB + 1);
        knn_rowstats_kernel<<<(unsigned)std::min<int64_t>(ccg_cdiv(n * d, 1024), 256), 256, 0, st>>>(rows, n, d,
                                                                                                    mbits, bnd);
        if (sg) {
            // each segment in the Morton order of its rows (radix sort on segment << 15 | code)
            int sbits = 0;
            while ((1 << sbits) < sg->nseg) ++sbits;
            if (!KNN_NO_MORTON && sbits + KNN_MORTON_DIMS * KNN_MORTON_BITS <= 31) {
                int32_t* kk = (int32_t*)ccg_ws(ctx, WS_ORDER, sizeof(int32_t) * 4 * n + 64);
                if (!kk) return CCG_ENOMEM;
                int32_t* ids = kk + n;
                int32_t* skeys = ids + n;
                int32_t* sids = skeys + n;
                const unsigned gn = (unsigned)ccg_cdiv(n, 256);
                knn_seg_morton_keys_kernel<<<gn, 256, 0, st>>>(rows, n, d, bnd, sg->seg_off, sg->nseg, kk, ids);
                rc = ccg_sort_pairs_i32(ctx, kk, skeys, ids, sids, n, sbits + KNN_MORTON_DIMS * KNN_MORTON_BITS, st);
                if (rc) return rc;
                knn_seg_perm_kernel<<<gn, 256, 0, st>>>(n, sids, sg->seg_off, sg->pos_off, sg->nseg, sg->perm);
            }
            order_perm = sg->perm;
        } else if (KNN_NO_MORTON) {
            order_perm = nullptr;  // tools only: input order
        } else if (buckets) {
            // spatial order: Morton buckets of the leading coordinates (counting sort)
            int64_t* cursor = hist + (NB + 1);
            int* perm = (int*)(cursor + (NB + 1));
            knn_bucket_count_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(rows, n, d, bnd, hist);
            rc = ccg_scan_i64(ctx, hist, cursor, NB, st);  // the bucket starts, advanced by the scatter
            if (rc) return rc;
            knn_bucket_scatter_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(rows, n, d, bnd, cursor, perm);
            order_perm = perm;
        } else {
            // spatial order: radix-sorted Morton codes of the leading coordinates
            int32_t* kk = (int32_t*)ccg_ws(ctx, WS_ORDER, sizeof(int32_t) * 4 * n + 64);
            if (!kk) return CCG_ENOMEM;
            int32_t* ids = kk + n;
            int32_t* skeys = ids + n;
            int32_t* perm = skeys + n;
            knn_morton_keys_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(rows, n, d, bnd, kk, ids);
            rc = ccg_sort_pairs_i32(ctx, kk, skeys, ids, perm, n, KNN_MORTON_DIMS * KNN_MORTON_BITS, st);
            if (rc) return rc;
            order_perm = perm;
        }
        const unsigned pg = (unsigned)ccg_cdiv(npad, 256);
        if (KSTEPS == 1)
            knn_prep16_kernel<1><<<pg, 256, 0, st>>>(rows, npos, npad, d, mbits, order_perm, img, inv_scale2,
                                                      row_hint, pos_t0);
        else if (KSTEPS == 2)
            knn_prep16_kernel<2><<<pg, 256, 0, st>>>(rows, npos, npad, d, mbits, order_perm, img, inv_scale2,
                                                      row_hint, pos_t0);
        else
            knn_prep16_kernel<4><<<pg, 256, 0, st>>>(rows, npos, npad, d, mbits, order_perm, img, inv_scale2,
                                                      row_hint, pos_t0);
        const int nch = (int)(npad / KNN_CHUNK);
        const unsigned grid = (unsigned)ccg_cdiv(npos, KNN_QPB);
        const int4* blk = sg ? sg->blk : nullptr;
        const int t_scr = ccg_timer_start(ctx, CCG_KT_KNN_SCREEN, st);
#define CCG_SCREEN16(KS_, KP_, R_, ...)                                                                      \
    knn_screen16_kernel<KS_, KP_, R_, ##__VA_ARGS__><<<grid, 256, 0, st>>>(img, (int)npos, nch, d, cand_idx, cand_thr, \
                                                                           blk, pos_t0)
        if (KP == KNN_KP) {
            if (KSTEPS == 1) CCG_SCREEN16(1, KNN_KP, KNN_KP + KNN_TMARGIN);
            else if (KSTEPS == 2) CCG_SCREEN16(2, KNN_KP, KNN_KP + KNN_TMARGIN);
            else CCG_SCREEN16(4, KNN_KP, KNN_KP + KNN_TMARGIN);
        } else if (kmax <= KNN_KP_BIG) {
            if (KSTEPS == 1) CCG_SCREEN16(1, KNN_KP_BIG, KNN_KP_BIG + KNN_TMARGIN);
            else if (KSTEPS == 2) CCG_SCREEN16(2, KNN_KP_BIG, KNN_KP_BIG + KNN_TMARGIN);
            else CCG_SCREEN16(4, KNN_KP_BIG, KNN_KP_BIG + KNN_TMARGIN);
        } else {  // cell tables: the union threshold KNN_TMARGIN ranks past kmax <= KNN_TAB_K (2 waves per
                  // SIMD: the 32-entry lists do not fit the 3-wave register budget)
            if (KSTEPS == 1) CCG_SCREEN16(1, KNN_KP_BIG, KNN_TAB_K + KNN_TMARGIN, 2);
            else if (KSTEPS == 2) CCG_SCREEN16(2, KNN_KP_BIG, KNN_TAB_K + KNN_TMARGIN, 2);
            else CCG_SCREEN16(4, KNN_KP_BIG, KNN_TAB_K + KNN_TMARGIN, 2);
        }
#undef CCG_SCREEN16
        ccg_timer_stop(ctx, t_scr, st);
    }
    const int64_t* seg_off = sg ? sg->seg_off : nullptr;
    const int nseg = sg ? sg->nseg : 1;
#define CCG_CERTIFY(KP_, DM_)                                                                             \
    knn_certify_kernel<KP_, DM_><<<(unsigned)ccg_cdiv(npos, 4), 256, 0, st>>>(                              \
        rows, (int)n, d, kmax, cand_idx, cand_thr, inv_scale2, err_ulps, order_perm, out_idx, out_dist, \
        fail_list, fail_count, (int)npos, seg_off, nseg, dist_sq, fail_tau)
    if (KP == KNN_KP) {
        if (d <= 16) CCG_CERTIFY(KNN_KP, 16);
        else if (d <= 32) CCG_CERTIFY(KNN_KP, 32);
        else CCG_CERTIFY(KNN_KP, 64);
    } else {
        if (d <= 16) CCG_CERTIFY(KNN_KP_BIG, 16);
        else if (d <= 32) CCG_CERTIFY(KNN_KP_BIG, 32);
        else CCG_CERTIFY(KNN_KP_BIG, 64);
    }
#undef CCG_CERTIFY
    rc = knn_fallback_launch(ctx, rows, n, d, kmax, fail_list, fail_count, out_idx, out_dist, seg_off, nseg, st,
                             dist_sq, fail_tau);
    if (rc) return rc;
    ctx->last_fail_list = fail_list;
    ctx->last_fail_count = fail_count;
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    if (stats) {
        int nf = 0;
        CCG_HIP(hipMemcpyAsync(&nf, fail_count, sizeof(int), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        stats->queries = n;
        stats->fallback = nf;
        ctx->last_stats = *stats;
    }
    return CCG_OK;
}

extern "C" int ccg_knn_rows_dev(ccg_ctx* ctx, const double* rows, int64_t n, int d, int kmax,
                                int32_t* out_idx, double* out_dist, ccg_knn_stats* stats,
                                void* stream) {
    CCG_REQUIRE(ctx && rows && out_idx, "ccg_knn_rows_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_rows_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(n >= 2 && n < (1LL << 30), "ccg_knn_rows_dev: n=%lld out of range", (long long)n);
    CCG_REQUIRE(kmax >= 1 && kmax <= KNN_KP_BIG && kmax <= n - 1,
                "ccg_knn_rows_dev: kmax=%d must be in [1, min(%d, n-1)]", kmax, KNN_KP_BIG);
    return knn_run(ctx, rows, n, d, kmax, out_idx, out_dist, stats, ccg_pick_stream(ctx, stream), nullptr);
}

extern "C" int ccg_knn_segments_dev(ccg_ctx* ctx, const double* rows, int64_t n, int d, const int64_t* seg_off,
                                    int nseg, int kmax, int32_t* out_idx, double* out_dist, ccg_knn_stats* stats,
                                    void* stream) {
    CCG_REQUIRE(ctx && rows && seg_off && out_idx, "ccg_knn_segments_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_segments_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(nseg >= 1 && n >= 2 && n < (1LL << 30), "ccg_knn_segments_dev: bad sizes");
    CCG_REQUIRE(kmax >= 1 && kmax <= KNN_KP_BIG, "ccg_knn_segments_dev: kmax=%d must be in [1, %d]", kmax,
                KNN_KP_BIG);
    CCG_REQUIRE(seg_off[0] == 0 && seg_off[nseg] == n, "ccg_knn_segments_dev: seg_off must run from 0 to n");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    std::vector<int64_t> po;
    std::vector<int> hperm;
    std::vector<int4> hblk;
    KnnSegs sg;
    int rc0 = knn_seg_plan(ctx, seg_off, nseg, d, kmax, st, po, hperm, hblk, &sg);
    if (rc0) return rc0;
    // (the plan's tables went through the pinned ring, ccg_h2d_staged: the
    // host vectors may go now, and the call stays asynchronous)
    return knn_run(ctx, rows, n, d, kmax, out_idx, out_dist, stats, st, &sg);
}

// ---------------------------------------------------- distinct cells --
// A bootstrap draws cells with replacement (R/consensusClust.R:394), so at
// cfg3 only about 1 - e^-0.9 = 59% of its rows are distinct cells; the rest
// are copies at distance 0.  Under the contract (d2 of the rows, ties by row
// index) the neighbours of row i (cell c) are, in (d2, row) order, the other
// copies of c and the copies of c's nearest distinct cells.  So the screen /
// certify / fallback pipeline runs on the u distinct cells only (about 0.35 of
// the n^2 work), and an expansion pass turns each cell's kq = min(kmax, u-1)
// nearest distinct cells back into row lists: groups of equal d2 (exact fp64,
// unfused, dimension order -- the oracle's arithmetic) are merged by row
// index.  A row whose kmax-th entry falls in a group that reaches the last
// computed distinct neighbour (a tie that may continue past the list) is
// re-searched exactly over all rows by the fallback kernels.

// Rows grouped by cell with a counting sort over the N cells (ccg_knn_boot
// and its table flavour; the segments keep the radix sort): per-cell counts
// with a presence bit, pk[c] = present << 32 | count, so ONE exclusive scan
// gives every present cell its distinct id (high word) and its first sorted
// position (low word).  pk and the cursors are zero between calls (each call
// clears what it used).  The cells' rows are then scattered by per-cell
// atomic cursors and each cell's few rows sorted ascending, so the result is
// exactly the stable sort's.
// (also zeroes the ucap + 1 words of ustart, so a wrong caller u leaves no
// garbage offsets behind)
// (zc: three counters zeroed by the first threads -- the table path's fail
// counts -- in place of a memset launch; may be NULL)
// (segn > 0: a batch of bootstraps of segn rows each -- row t belongs to
// bootstrap t / segn, whose cell c is the virtual cell (t / segn) N + c, so
// the bootstraps' distinct cells get disjoint, bootstrap-major ids)
__global__ void kb_count_kernel(const int32_t* __restrict__ idx, int64_t n, int64_t N,
                                unsigned long long* __restrict__ pk, int* __restrict__ err,
                                int32_t* __restrict__ ztab, int64_t nz, unsigned* __restrict__ zc, int nzc = 3,
                                int64_t segn = 0) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = t; i < nz; i += (int64_t)gridDim.x * blockDim.x) ztab[i] = 0;
    if (zc && t < nzc) zc[t] = 0u;
    if (t >= n) return;
    int c = idx[t];
    if (c < 0 || c >= N) {
        atomicOr(err, CCG_DERR_KNN_UNIQUE);
        c = 0;
    }
    const int64_t vc = segn ? (t / segn) * N + c : c;
    const unsigned long long old = atomicAdd(&pk[vc], 1ull);
    if ((old & 0xffffffffull) == 0ull) atomicAdd(&pk[vc], 1ull << 32);  // the first row: the presence bit
}

// Per cell c (and c = N): cell2u[c] (-1: absent), ustart[uid]; pk[c] back to
// 0 and the scatter cursor zeroed (for every cell, whatever the caller's u).
// A caller's u that differs from the count sets the sticky error; ids are
// clamped into [0, ucap) so every later access stays in bounds.
// (a batch, nseg > 0: N = nseg Nc virtual cells; the bootstraps' first
// distinct ids go to useg, their first rows to dso, and a bootstrap with
// fewer than kmin distinct cells sets the sticky error)
__global__ void kb_cells_kernel(unsigned long long* __restrict__ pk, const int64_t* __restrict__ pko, int64_t N,
                                int64_t n, int ucap, int u_given, int* __restrict__ cell2u,
                                int* __restrict__ ustart, int* __restrict__ cursor, int* __restrict__ nbig,
                                int* __restrict__ err, int nseg = 0, int64_t Nc = 0, int kmin = 0,
                                int64_t* __restrict__ useg = nullptr, int64_t* __restrict__ dso = nullptr,
                                int64_t segn = 0) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < N) {
        const unsigned long long a = (unsigned long long)pko[c], b = (unsigned long long)pko[c + 1];
        const bool present = (b >> 32) > (a >> 32);
        const int uid = min((int)(a >> 32), ucap - 1);
        cell2u[c] = present ? uid : -1;
        if (present) ustart[uid] = (int)(a & 0xffffffffull);
        pk[c] = 0ull;
        cursor[c] = 0;
        if (nseg > 0 && c % Nc == 0) {
            const int sg = (int)(c / Nc);
            const int64_t us = (int64_t)((unsigned long long)pko[c + Nc] >> 32) - (int64_t)(a >> 32);
            if (us < kmin) atomicOr(err, CCG_DERR_KNN_UNIQUE);
            useg[sg] = (int64_t)(a >> 32);
            dso[sg] = sg * segn;
        }
    } else if (c == N) {
        const int u = (int)((unsigned long long)pko[N] >> 32);
        if (u_given >= 0 && u != u_given) atomicOr(err, CCG_DERR_KNN_UNIQUE);
        ustart[min(u, ucap)] = (int)n;
        *nbig = 0;
        if (nseg > 0) {
            useg[nseg] = min(u, ucap);
            dso[nseg] = nseg * segn;
        }
    }
}

__global__ void kb_scatter_kernel(const int32_t* __restrict__ idx, int64_t n, int64_t N,
                                  const int* __restrict__ cell2u, const int* __restrict__ ustart,
                                  int* __restrict__ cursor, int32_t* __restrict__ srow, int32_t* __restrict__ scell,
                                  int64_t segn = 0) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int c = idx[t];
    if (c < 0 || c >= N) c = 0;  // (flagged by the count kernel)
    if (segn) c = (int)((t / segn) * N + c);  // the virtual cell (a batch)
    const int64_t pos = min((int64_t)ustart[max(cell2u[c], 0)] + atomicAdd(&cursor[c], 1), n - 1);
    srow[pos] = (int32_t)t;
    scell[pos] = c;
}

// One thread per distinct cell: its rows sorted ascending (an insertion sort
// in place: a cell has ~1.5 rows), row2u.  A cell drawn more than 32 times
// (tiny N) goes to kb_fixup_big_kernel's list.
#define KB_FIX_SMALL 32
__global__ __launch_bounds__(256) void kb_fixup_kernel(int u, int64_t n, const int* __restrict__ ustart,
                                                       int32_t* __restrict__ srow, int* __restrict__ row2u,
                                                       int* __restrict__ big, int* __restrict__ nbig) {
    const int uid = blockIdx.x * blockDim.x + threadIdx.x;
    if (uid >= u) return;
    const int s = min(max(ustart[uid], 0), (int)n), e = min(max(ustart[uid + 1], s), (int)n);
    const int k = e - s;
    if (k <= 0) return;
    if (k > KB_FIX_SMALL) {
        big[atomicAdd(nbig, 1)] = uid;
        return;
    }
    for (int i = 1; i < k; ++i) {
        const int v = srow[s + i];
        int q = i - 1;
        while (q >= 0 && srow[s + q] > v) {
            srow[s + q + 1] = srow[s + q];
            --q;
        }
        srow[s + q + 1] = v;
    }
    for (int p = s; p < e; ++p) row2u[srow[p]] = uid;
}

// The listed cells, one wave each: a wave bitonic sort up to 64 rows, ranks
// by counting beyond (through tmp).
__global__ __launch_bounds__(256) void kb_fixup_big_kernel(int64_t n, const int* __restrict__ ustart,
                                                           int32_t* __restrict__ srow, int* __restrict__ row2u,
                                                           const int* __restrict__ big, const int* __restrict__ nbig,
                                                           int32_t* __restrict__ tmp) {
    const int lane = threadIdx.x & 63;
    const int nb = *nbig;
    for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < nb; w += gridDim.x * 4) {
        const int uid = big[w];
        const int s = min(max(ustart[uid], 0), (int)n), e = min(max(ustart[uid + 1], s), (int)n);
        const int k = e - s;
        if (k <= 64) {
            int v = lane < k ? srow[s + lane] : 0x7fffffff;
            for (int kk = 2; kk <= 64; kk <<= 1)
                for (int j = kk >> 1; j > 0; j >>= 1) {
                    const int o = __shfl_xor(v, j, 64);
                    const bool up = (lane & kk) == 0, lo = (lane & j) == 0;
                    v = (lo == up) ? min(v, o) : max(v, o);
                }
            if (lane < k) {
                srow[s + lane] = v;
                row2u[v] = uid;
            }
            continue;
        }
        for (int i = lane; i < k; i += 64) {
            const int v = srow[s + i];
            int r = 0;
            for (int j = 0; j < k; ++j) r += srow[s + j] < v ? 1 : 0;
            tmp[s + r] = v;
        }
        __builtin_amdgcn_wave_barrier();
        __threadfence_block();
        for (int i = lane; i < k; i += 64) {
            const int v = tmp[s + i];
            srow[s + i] = v;
            row2u[v] = uid;
        }
    }
}

// (cell, row) pairs sorted by cell (stable: each cell's rows ascending)
// (also zeroes the u + 1 words of ustart when u is known: ztab / nz)
__global__ void kb_heads_kernel(const int32_t* __restrict__ scell, int64_t n, int64_t* __restrict__ head,
                                int32_t* __restrict__ ztab, int64_t nz) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) head[t] = (t == 0 || scell[t] != scell[t - 1]) ? 1 : 0;
    if (ztab)
        for (int64_t i = t; i < nz; i += (int64_t)gridDim.x * blockDim.x) ztab[i] = 0;
}

// hs: exclusive scan of the heads (hs[n] = the number of distinct cells).
// Distinct cell uid owns the sorted positions [ustart[uid], ustart[uid + 1]);
// row2u maps a row to its uid.  If the caller's u is wrong the sticky error is
// set and uids are clamped into [0, u) (ustart zeroed beforehand), so every
// later access stays in bounds; the outputs are then undefined.
__global__ void kb_tables_kernel(const int32_t* __restrict__ scell, const int32_t* __restrict__ srow, int64_t n,
                                 const int64_t* __restrict__ hs, int u, int* __restrict__ ustart,
                                 int* __restrict__ row2u, int* __restrict__ err) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (t == 0 && hs[n] != u) atomicOr(err, CCG_DERR_KNN_UNIQUE);
    const bool head = t == 0 || scell[t] != scell[t - 1];
    const int uid = min((int)hs[t] - (head ? 0 : 1), u - 1);
    if (head) ustart[uid] = (int)t;
    row2u[srow[t]] = uid;
    if (t == 0) ustart[u] = (int)n;
}

// the distinct cells' rows, copied from the gathered (row-major) bootstrap
// rows of each cell's first copy: coalesced, unlike a gather from the
// column-major PCs
// (LPR lanes per distinct cell, a lane per dimension: no per-element 64-bit
// division)
template <int LPR>
__global__ __launch_bounds__(256) void kb_urows_kernel(const double* __restrict__ rows, int d, int u,
                                                       const int* __restrict__ ustart, const int* __restrict__ srow,
                                                       double* __restrict__ urows, const int32_t* __restrict__ idx,
                                                       const float* __restrict__ cell_hint,
                                                       float* __restrict__ urow_hint) {
    const int64_t uid = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    const int k = threadIdx.x & (LPR - 1);
    if (uid >= u) return;
    const int r0 = srow[ustart[uid]];
    if (k < d) urows[uid * d + k] = rows[(int64_t)r0 * d + k];
    if (k == 0 && urow_hint) urow_hint[uid] = cell_hint[idx[r0]];
}

// The hint for the next bootstrap: each distinct cell's certified squared
// distance to its kq-th nearest distinct cell (rows that went to the exact
// fallback keep their previous hint).
__global__ void kb_hint_kernel(int u, int kq, const int* __restrict__ ustart, const int* __restrict__ srow,
                               const int32_t* __restrict__ idx, const double* __restrict__ ud2,
                               float* __restrict__ cell_hint) {
    const int64_t uid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (uid >= u || kq < 1) return;
    const double v = ud2[uid * kq + kq - 1];
    if (v > 0.0 && v < 3.0e38) cell_hint[idx[srow[ustart[uid]]]] = (float)v;
}

#define KB_GMAX 33  // cells of one merge group (the own cell + kq <= 32 neighbours)
__device__ void kb_expand_row(int64_t i, int u, int kq, const int* __restrict__ uidx, const double* __restrict__ ud2,
                              const int* __restrict__ ustart, const int* __restrict__ srow,
                              const int* __restrict__ row2u, int kmax, int32_t* __restrict__ out_idx,
                              double* __restrict__ out_dist, int* __restrict__ fail_list, int* __restrict__ fail_count,
                              double* __restrict__ fail_tau, const int64_t* __restrict__ useg = nullptr,
                              int nseg = 1, const int64_t* __restrict__ fbase = nullptr,
                              int* __restrict__ fcnt = nullptr) {
    const int uc = row2u[i];
    int sg = 0;
    if (useg) {  // segmented run: the distinct cells of the row's own segment
        sg = knn_seg_of(useg, nseg, uc);
        u = (int)(useg[sg + 1] - useg[sg]);
    }
    // the distinct cell's kq nearest distinct cells with their certified d2
    // (fp64, unfused, dimension order: the oracle's sums; copies share them)
    const int* nbl = uidx + (int64_t)uc * kq;
    const double* d2l = ud2 + (int64_t)uc * kq;
    int o = 0;     // rows written
    int t = 0;     // next distinct neighbour
    double dn = kq > 0 ? d2l[0] : INFINITY;
    double gd = 0.0;  // the group's d2 (group 0: the own cell, d2 = 0)
    bool first = true, fail = false;
    double ftau = INFINITY;  // no radius (n - 1 < kmax): the per-thread-list search
    int lo[KB_GMAX], hi[KB_GMAX];  // ranges of a multi-cell group (exact ties between distinct cells: rare)
    while (o < kmax) {
        // the group: the own cell first (group 0), then the distinct neighbours at d2 == gd
        int g = 0, lo0 = 0, hi0 = 0;
        if (first) {
            lo0 = ustart[uc];
            hi0 = ustart[uc + 1];
            g = 1;
        }
        const int t0 = t;
        while (t < kq && dn == gd) {
            const int v = nbl[t];
            const int a = ustart[v], b = ustart[v + 1];
            if (g == 0) {
                lo0 = a;
                hi0 = b;
            } else {
                if (g == 1) {
                    lo[0] = lo0;
                    hi[0] = hi0;
                }
                lo[g] = a;
                hi[g] = b;
            }
            ++g;
            ++t;
            dn = t < kq ? d2l[t] : INFINITY;
        }
        if (t == kq && t > t0 && kq < u - 1) {  // the group may continue past the computed list
            fail = true;
            ftau = gd;  // the radius search's bound: the rows so far and the cut group lie within gd
            break;
        }
        const double dist = out_dist ? sqrt(gd) : 0.0;
        if (g == 1) {  // one cell: its rows are already ascending
            for (int q = lo0; q < hi0 && o < kmax; ++q) {
                const int r = srow[q];
                if (r == (int)i) continue;
                out_idx[i * kmax + o] = r;
                if (out_dist) out_dist[i * kmax + o] = dist;
                ++o;
            }
        } else {
            // merge the group's row lists (each ascending) by row index, skipping row i
            while (o < kmax) {
                int best = 0x7fffffff, bg = -1;
                for (int q = 0; q < g; ++q)
                    if (lo[q] < hi[q]) {
                        const int r = srow[lo[q]];
                        if (r < best) {
                            best = r;
                            bg = q;
                        }
                    }
                if (bg < 0) break;
                ++lo[bg];
                if (best == (int)i) continue;
                out_idx[i * kmax + o] = best;
                if (out_dist) out_dist[i * kmax + o] = dist;
                ++o;
            }
        }
        if (o >= kmax) break;
        if (t >= kq) {  // every distinct cell is listed (kq = u - 1) yet fewer than kmax rows: n - 1 < kmax
            fail = true;
            break;
        }
        gd = dn;
        first = false;
    }
    if (fail) {
        // (fbase: a batch -- each segment appends to its own region)
        const int64_t p = fbase ? fbase[sg] + atomicAdd(&fcnt[sg], 1) : atomicAdd(fail_count, 1);
        fail_list[p] = (int)i;
        if (fail_tau) fail_tau[p] = ftau;
    }
}

__global__ __launch_bounds__(256) void kb_expand_kernel(int64_t n, int u, int kq, const int* __restrict__ uidx,
                                                        const double* __restrict__ ud2,
                                                        const int* __restrict__ ustart, const int* __restrict__ srow,
                                                        const int* __restrict__ row2u, int kmax,
                                                        int32_t* __restrict__ out_idx, double* __restrict__ out_dist,
                                                        int* __restrict__ fail_list, int* __restrict__ fail_count,
                                                        double* __restrict__ fail_tau) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        kb_expand_row(i, u, kq, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist, fail_list, fail_count,
                      fail_tau);
}

// The rows of the cells kb_expand_cells_kernel left to the per-row merge.
__global__ __launch_bounds__(256) void kb_expand_ties_kernel(int u, int kq, const int* __restrict__ uidx,
                                                             const double* __restrict__ ud2,
                                                             const int* __restrict__ ustart,
                                                             const int* __restrict__ srow,
                                                             const int* __restrict__ row2u, int kmax,
                                                             int32_t* __restrict__ out_idx,
                                                             double* __restrict__ out_dist, int* __restrict__ fail_list,
                                                             int* __restrict__ fail_count, double* __restrict__ fail_tau,
                                                             const int* __restrict__ tie_list,
                                                             const int* __restrict__ tie_count,
                                                             const int64_t* __restrict__ useg = nullptr,
                                                             int nseg = 1, const int64_t* __restrict__ fbase = nullptr,
                                                             int* __restrict__ fcnt = nullptr) {
    const int nt = *tie_count;
    for (int f = blockIdx.x * blockDim.x + threadIdx.x; f < nt; f += gridDim.x * blockDim.x) {
        const int uc = tie_list[f];
        for (int z = ustart[uc]; z < ustart[uc + 1]; ++z)
            kb_expand_row(srow[z], u, kq, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist, fail_list,
                          fail_count, fail_tau, useg, nseg, fbase, fcnt);
    }
}

// The same expansion, one wave per DISTINCT cell (copies of a cell share
// everything but the row they exclude): lanes load the cell's kq neighbour
// cells and their row ranges at once, a wave scan places each neighbour's
// rows, and every copy writes its list.  Valid when no two listed cells tie in
// d2 (nor a listed cell with the own cell at d2 = 0): every group is one cell
// whose rows are already ascending.  A cell with such a tie takes the
// per-row merge (kb_expand_kernel's loop) for its rows.  kq <= 64.
__global__ __launch_bounds__(256) void kb_expand_cells_kernel(int64_t n, int u, int kq, const int* __restrict__ uidx,
                                                              const double* __restrict__ ud2,
                                                              const int* __restrict__ ustart,
                                                              const int* __restrict__ srow, const int* __restrict__ row2u,
                                                              int kmax, int32_t* __restrict__ out_idx,
                                                              double* __restrict__ out_dist, int* __restrict__ fail_list,
                                                              int* __restrict__ fail_count,
                                                              double* __restrict__ fail_tau,
                                                              int* __restrict__ tie_list, int* __restrict__ tie_count,
                                                              const int64_t* __restrict__ useg = nullptr,
                                                              int nseg = 1, const int64_t* __restrict__ fbase = nullptr,
                                                              int* __restrict__ fcnt = nullptr) {
    // two distinct cells per wave, one per 32-lane half (kq <= kmax <= 32):
    // a cell's list takes at most 32 lanes
    const int lane = threadIdx.x & 31;
    const int half = (threadIdx.x >> 5) & 1;
    const int uc = blockIdx.x * 8 + (threadIdx.x >> 5);
    const bool live = uc < u;
    if (__ballot(live) == 0ull) return;
    int uu = u, sg = 0;
    if (useg && live) {  // segmented run: the cut test counts the distinct cells of the cell's own segment
        sg = knn_seg_of(useg, nseg, uc);
        uu = (int)(useg[sg + 1] - useg[sg]);
    }
    const int oa = live ? ustart[uc] : 0, ob = live ? ustart[uc + 1] : 0, oc = ob - oa;  // the own cell's rows
    const bool has = live && lane < kq;
    const int v = has ? uidx[(int64_t)uc * kq + lane] : 0;
    const double dd = has ? ud2[(int64_t)uc * kq + lane] : INFINITY;
    const int a = has ? ustart[v] : 0, cn = has ? ustart[v + 1] - a : 0;
    const double dprev = __shfl_up(dd, 1, 32);
    const bool tie = has && (lane == 0 ? dd == 0.0 : dd == dprev);
    const unsigned long long bt = __ballot(tie);
    const bool htie = ((half ? bt >> 32 : bt) & 0xffffffffull) != 0ull;
    if (htie && lane == 0) tie_list[atomicAdd(tie_count, 1)] = uc;  // equal-d2 groups of several cells: the per-row merge
    int incl = cn;  // exclusive prefix of the neighbours' row counts
    for (int o = 1; o < 32; o <<= 1) {
        const int y = __shfl_up(incl, o, 32);
        if (lane >= o) incl += y;
    }
    const int pre = incl - cn;
    const int own = oc - 1;                    // own rows in every copy's list
    const int need = kmax - own;               // neighbour rows a list takes (<= 0: own rows only)
    const int total = __shfl(incl, 31, 32);    // all listed neighbours' rows
    // the last listed cell reached while the list is short: a tie may continue past it
    const int plast = __shfl(pre, kq - 1, 32);
    const bool cut = need > 0 && kq >= 1 && plast < need && kq < uu - 1;
    const bool shortl = need > 0 && total < need;  // (kq = u - 1 and fewer than kmax rows: n - 1 < kmax)
    const double glast = __shfl(dd, kq - 1, 32);
    if (!live || htie) return;
    for (int z = oa; z < ob; ++z) {
        const int i = srow[z];  // a copy (uniform in the half)
        if (cut || shortl) {
            if (lane == 0) {
                const int64_t p = fbase ? fbase[sg] + atomicAdd(&fcnt[sg], 1) : atomicAdd(fail_count, 1);
                fail_list[p] = i;
                if (fail_tau) fail_tau[p] = cut ? glast : INFINITY;
            }
            continue;
        }
        int32_t* oi = out_idx + (int64_t)i * kmax;
        double* od = out_dist ? out_dist + (int64_t)i * kmax : nullptr;
        // own copies except i, ascending
        for (int q = lane; q < oc && q - (q > z - oa ? 1 : 0) < kmax; q += 32) {
            if (oa + q == z) continue;
            const int pos = q - (q > z - oa ? 1 : 0);
            oi[pos] = srow[oa + q];
            if (od) od[pos] = 0.0;
        }
        // neighbour cells' rows
        if (has && pre < need) {
            const double dist = od ? sqrt(dd) : 0.0;
            for (int q = 0; q < cn && pre + q < need; ++q) {
                oi[own + pre + q] = srow[a + q];
                if (od) od[own + pre + q] = dist;
            }
        }
    }
}

extern "C" int ccg_knn_boot_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d, const int32_t* idx, int64_t n,
                                int n_unique, const double* rows, int kmax, int32_t* out_idx, double* out_dist,
                                ccg_knn_stats* stats, void* stream) {
    return ccg_knn_boot_hint_dev(ctx, pcs, N, d, idx, n, n_unique, rows, kmax, out_idx, out_dist, nullptr, stats,
                                 stream);
}

// ------------------------------------------------------- cell tables --
// Every bootstrap of one consensusClust call draws from the same N cells
// (R/consensusClust.R:394), so a cell's nearest distinct cells in a bootstrap
// are the first kq PRESENT entries of its list of nearest cells among all N,
// in that list's (d2, cell) order -- the distinct-cell order, since distinct
// ids follow the cell order.  ccg_knn_table_dev computes the K nearest other
// cells of every cell once (screen / certify / fallback over the N cells,
// certified squared distances); ccg_knn_boot_table_dev then replaces the
// per-bootstrap screen by a filter of the table rows (one wave per distinct
// cell: presence ballot, prefix count).  A cell with fewer than kq present
// entries in its K (about 0.6% of the distinct cells at a 59% presence rate
// and K = 48, kq = 20) is searched exactly among the bootstrap's distinct
// cells; the expansion to rows is shared with the screen path.  Results are
// bit-identical to the screen path.
__global__ void kt_transpose_kernel(const double* __restrict__ pcs, int64_t N, int d, double* __restrict__ rows) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // column-major position
    if (t >= N * d) return;
    const int64_t k = t / N, i = t - k * N;
    rows[i * d + k] = pcs[t];
}

// Radius for a cell short of kq present table entries (one wave per cell):
// the kq-th smallest exact d2 over distinct present cells near it -- its
// present table entries, and for every table entry the first present cell of
// that entry's own row outside the cell's row.  Any kq distinct present
// cells bound the kq-th neighbour distance from above; +inf (the
// per-thread-list search) when fewer than kq are found.  Lane t holds the
// cell's table entry v (-1 past K), present as distinct cell u1 (-1: absent).
#define KT_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)
#define KT_TB 8  // table entries tested per round in kt_tau_wave
struct KtTauLds {
    int hset[128];  // the cell's own table row as an open-addressing set (K <= 48 of 128 slots)
    double val[128];
};
__device__ __forceinline__ double kt_tau_wave(KtTauLds& S, int lane, int kq, int K, int d, int uid, int64_t c, int v,
                                              int u1, double val1, const int* __restrict__ cell2u,
                                              const int32_t* __restrict__ tab_idx, const double* __restrict__ urows) {
    auto hslot = [](int x) { return (int)(((unsigned)x * 2654435761u) >> 25); };
    S.hset[lane] = -1;
    S.hset[64 + lane] = -1;
    KT_SYNC();
    if (v >= 0)
        for (int h = hslot(v);; h = (h + 1) & 127) {
            const int prev = atomicCAS(&S.hset[h], -1, v);
            if (prev == -1 || prev == v) break;
        }
    KT_SYNC();
    // the first entry of v's row that is present and outside the cell's row:
    // KT_TB entries per round (independent loads; one entry per round was a
    // chain of dependent loads tens of entries long, and this wave the
    // filter kernel's critical path)
    int w = -1;
    if (v >= 0) {
        for (int s0 = 0; s0 < K && w < 0; s0 += KT_TB) {
            int x[KT_TB], pr[KT_TB];
#pragma unroll
            for (int j = 0; j < KT_TB; ++j) x[j] = s0 + j < K ? tab_idx[(int64_t)v * K + s0 + j] : -1;
#pragma unroll
            for (int j = 0; j < KT_TB; ++j) pr[j] = (x[j] >= 0 && x[j] != (int)c) ? cell2u[x[j]] : -1;
#pragma unroll
            for (int j = 0; j < KT_TB; ++j) {
                if (w >= 0 || pr[j] < 0) continue;
                bool in_row = false;
                for (int h = hslot(x[j]);; h = (h + 1) & 127) {
                    const int y = S.hset[h];
                    if (y == x[j]) {
                        in_row = true;
                        break;
                    }
                    if (y == -1) break;
                }
                if (!in_row) w = x[j];
            }
        }
    }
    // a pick already made by a lower lane is a duplicate (the lanes' picks by
    // v_readlane: no LDS round trips)
    bool dup = false;
#pragma unroll 16
    for (int t = 0; t < 64; ++t) dup |= t < lane && w >= 0 && __builtin_amdgcn_readlane(w, t) == w;
    double val2 = INFINITY;
    if (w >= 0 && !dup) {
        const double* xr = urows + (int64_t)uid * d;
        const double* yr = urows + (int64_t)cell2u[w] * d;
        // (the dimension-order sum; loads issued 8 dimensions at a time --
        // one dependent load pair per dimension made this the filter
        // kernel's critical path)
        double s2 = 0.0;
        for (int k0 = 0; k0 < d; k0 += 8) {
            double a[8], b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[j] = k0 + j < d ? xr[k0 + j] : 0.0;
                b[j] = k0 + j < d ? yr[k0 + j] : 0.0;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (k0 + j < d) {
                    const double t = __dsub_rn(a[j], b[j]);
                    s2 = __dadd_rn(s2, __dmul_rn(t, t));
                }
        }
        val2 = s2;
    }
    if (u1 < 0) val1 = INFINITY;
    S.val[lane] = val1;
    S.val[64 + lane] = val2;
    KT_SYNC();
    int c1 = 0, c2 = 0;
    for (int t = 0; t < 128; ++t) {
        const double b = S.val[t];
        c1 += b <= val1 ? 1 : 0;
        c2 += b <= val2 ? 1 : 0;
    }
    double best = INFINITY;
    if (val1 < INFINITY && c1 >= kq) best = val1;
    if (val2 < INFINITY && c2 >= kq) best = fmin(best, val2);
    for (int o = 32; o > 0; o >>= 1) best = fmin(best, __shfl_xor(best, o, 64));
    KT_SYNC();
    return best;
}

// KT_CPW distinct cells per wave: the first kq present entries of each one's
// table row; a cell short of kq of them joins the exact search with its
// radius (round 5: taken here, in the same wave, instead of a separate
// kt_tau pass over the failed list).  The kernel is a chain of dependent
// gathers (distinct id -> cell -> table row -> presence); the cells of a wave
// issue each level's loads together.
// SEG (a batch, ccg_knn_boots_table_dev): scell holds virtual cells
// s Nc + c; bootstrap s's presence map is cell2u + s Nc, and a short cell
// appends to its bootstrap's region of the failed list (useg[s] + fcnt[s]).
#define KT_CPW 2
template <bool SEG>
__global__ __launch_bounds__(256) void kt_filter_kernel(int u, int kq, int K, int d, const int* __restrict__ ustart,
                                                        const int32_t* __restrict__ scell,
                                                        const int* __restrict__ cell2u,
                                                        const int32_t* __restrict__ tab_idx,
                                                        const double* __restrict__ tab_d2,
                                                        const double* __restrict__ urows, int32_t* __restrict__ uidx,
                                                        double* __restrict__ ud2, int* __restrict__ fail_list,
                                                        int* __restrict__ fail_count, double* __restrict__ tau,
                                                        int64_t Nc = 0, const int64_t* __restrict__ useg = nullptr,
                                                        int* __restrict__ fcnt = nullptr) {
    __shared__ KtTauLds tl[4];
    const int u0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * KT_CPW;
    if (u0 >= u) return;
    const int lane = threadIdx.x & 63;
    int64_t c[KT_CPW];
    int v[KT_CPW], w[KT_CPW], sg[KT_CPW];
    const int* c2u[KT_CPW];
    double dv[KT_CPW];
#pragma unroll
    for (int i = 0; i < KT_CPW; ++i) c[i] = u0 + i < u ? ustart[u0 + i] : -1;
#pragma unroll
    for (int i = 0; i < KT_CPW; ++i) {
        c[i] = c[i] >= 0 ? scell[c[i]] : -1;
        sg[i] = 0;
        c2u[i] = cell2u;
        if (SEG && c[i] >= 0) {  // virtual cell -> (bootstrap, cell)
            sg[i] = (int)(c[i] / Nc);
            c[i] -= (int64_t)sg[i] * Nc;
            c2u[i] = cell2u + (int64_t)sg[i] * Nc;
        }
    }
#pragma unroll
    for (int i = 0; i < KT_CPW; ++i) {
        const bool e = c[i] >= 0 && lane < K;
        v[i] = e ? tab_idx[c[i] * K + lane] : -1;
        dv[i] = e ? tab_d2[c[i] * K + lane] : INFINITY;
    }
#pragma unroll
    for (int i = 0; i < KT_CPW; ++i) w[i] = v[i] >= 0 ? c2u[i][v[i]] : -1;
    for (int i = 0; i < KT_CPW; ++i) {
        const int uid = u0 + i;
        if (uid >= u) break;  // (wave-uniform)
        const double di = w[i] >= 0 ? dv[i] : INFINITY;
        const unsigned long long m = __ballot(w[i] >= 0);
        const int rank = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
        if (w[i] >= 0 && rank < kq) {
            uidx[(int64_t)uid * kq + rank] = w[i];
            ud2[(int64_t)uid * kq + rank] = di;
        }
        if (__popcll(m) < kq) {  // (wave-uniform)
            const double best = kt_tau_wave(tl[threadIdx.x >> 6], lane, kq, K, d, uid, c[i], v[i], w[i], di, c2u[i],
                                            tab_idx, urows);
            if (lane == 0) {
                const int64_t f = SEG ? useg[sg[i]] + atomicAdd(&fcnt[sg[i]], 1) : atomicAdd(fail_count, 1);
                fail_list[f] = uid;
                tau[f] = best;
            }
        }
    }
}

// Cell-major form of kt_filter_kernel<true> for a batch (round 6): one wave
// per CELL c of the N, over the nb bootstraps: c's table row is read once and
// filtered against each bootstrap's presence map in turn, instead of once per
// (bootstrap, distinct cell) -- the same cell's row was read by ~0.6 nb waves
// scattered over the grid and the XCDs (2.7x10^8 B of table rows per launch
// set of 8 at cfg3).  Outputs per distinct cell exactly as kt_filter_kernel.
__global__ __launch_bounds__(256) void kt_filter_cells_kernel(int nb, int64_t Nc, int kq, int K, int d,
                                                              const int* __restrict__ cell2u,
                                                              const int32_t* __restrict__ tab_idx,
                                                              const double* __restrict__ tab_d2,
                                                              const double* __restrict__ urows,
                                                              int32_t* __restrict__ uidx, double* __restrict__ ud2,
                                                              int* __restrict__ fail_list, double* __restrict__ tau,
                                                              const int64_t* __restrict__ useg,
                                                              int* __restrict__ fcnt, int u) {
    __shared__ KtTauLds tl[4];
    const int64_t cb = ccg_cdiv(Nc, 4);  // blocks of cells; the rest fill phantom ids
    if ((int64_t)blockIdx.x >= cb) {
        // a caller's u above the distinct count (the sticky error is set):
        // ids [count, u) belong to no cell; give them in-bounds lists (the
        // outputs are undefined then, as in kt_filter_kernel)
        const int64_t p0 = useg[nb];
        for (int64_t t = (int64_t)(blockIdx.x - cb) * blockDim.x + threadIdx.x; t < ((int64_t)u - p0) * kq;
             t += (int64_t)(gridDim.x - cb) * blockDim.x) {
            uidx[p0 * kq + t] = 0;
            ud2[p0 * kq + t] = INFINITY;
        }
        return;
    }
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= Nc) return;
    const int lane = threadIdx.x & 63;
    // the bootstraps holding c (lane s < nb <= 64: one ballot)
    const int us = lane < nb ? cell2u[(int64_t)lane * Nc + c] : -1;
    unsigned long long pres = __ballot(us >= 0);
    if (!pres) return;
    const bool e = lane < K;
    const int v = e ? tab_idx[c * K + lane] : -1;
    const double dv = e ? tab_d2[c * K + lane] : INFINITY;
    // KT_BR bootstraps per round: their presence lookups issued together (one
    // round at nb <= 8: the lookups are the kernel's dependent-load chain)
    constexpr int KT_BR = 8;
    while (pres) {
        int sb[KT_BR], wb[KT_BR];
#pragma unroll
        for (int r = 0; r < KT_BR; ++r) {
            sb[r] = -1;
            if (pres) {
                sb[r] = __ffsll((long long)pres) - 1;
                pres &= pres - 1;
            }
        }
#pragma unroll
        for (int r = 0; r < KT_BR; ++r) wb[r] = (sb[r] >= 0 && v >= 0) ? cell2u[(int64_t)sb[r] * Nc + v] : -1;
#pragma unroll
        for (int r = 0; r < KT_BR; ++r) {
            if (sb[r] < 0) break;  // (wave-uniform)
            const int uid = __shfl(us, sb[r], 64), w = wb[r];
            const double di = w >= 0 ? dv : INFINITY;
            const unsigned long long m = __ballot(w >= 0);
            const int rank = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
            if (w >= 0 && rank < kq) {
                uidx[(int64_t)uid * kq + rank] = w;
                ud2[(int64_t)uid * kq + rank] = di;
            }
            if (__popcll(m) < kq) {  // (wave-uniform)
                const int* c2u = cell2u + (int64_t)sb[r] * Nc;
                const double best = kt_tau_wave(tl[threadIdx.x >> 6], lane, kq, K, d, uid, c, v, w, di, c2u, tab_idx,
                                                urows);
                if (lane == 0) {
                    const int64_t f = useg[sb[r]] + atomicAdd(&fcnt[sb[r]], 1);
                    fail_list[f] = uid;
                    tau[f] = best;
                }
            }
        }
    }
}

extern "C" int ccg_knn_table_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d, int K, int32_t* tab_idx,
                                 double* tab_d2, ccg_knn_stats* stats, void* stream) {
    CCG_REQUIRE(ctx && pcs && tab_idx && tab_d2, "ccg_knn_table_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_table_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(N >= 2 && N < (1LL << 30), "ccg_knn_table_dev: N=%lld out of range", (long long)N);
    CCG_REQUIRE(K >= 1 && K <= KNN_TAB_K && K <= N - 1, "ccg_knn_table_dev: K=%d must be in [1, min(%d, N-1)]", K,
                KNN_TAB_K);
    hipStream_t st = ccg_pick_stream(ctx, stream);
    double* rows = (double*)ccg_ws(ctx, WS_TAB_ROWS, sizeof(double) * (size_t)N * d);
    if (!rows) return CCG_ENOMEM;
    kt_transpose_kernel<<<(unsigned)ccg_cdiv(N * d, 256), 256, 0, st>>>(pcs, N, d, rows);
    return knn_run(ctx, rows, N, d, K, tab_idx, tab_d2, stats, st, nullptr, true);
}

static int knn_boot_impl(ccg_ctx* ctx, const double* pcs, int64_t N, int d, const int32_t* idx, int64_t n,
                         int n_unique, const double* rows, int kmax, int32_t* out_idx, double* out_dist,
                         float* cell_hint, const int32_t* tab_idx, const double* tab_d2, int K,
                         ccg_knn_stats* stats, hipStream_t st);

extern "C" int ccg_knn_boot_table_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d, const int32_t* idx,
                                      int64_t n, int n_unique, const double* rows, int kmax, const int32_t* tab_idx,
                                      const double* tab_d2, int K, int32_t* out_idx, double* out_dist,
                                      ccg_knn_stats* stats, void* stream) {
    CCG_REQUIRE(tab_idx && tab_d2, "ccg_knn_boot_table_dev: NULL table");
    CCG_REQUIRE(K >= 1 && K <= KNN_TAB_K && K <= N - 1, "ccg_knn_boot_table_dev: K=%d must be in [1, min(%d, N-1)]",
                K, KNN_TAB_K);
    return knn_boot_impl(ctx, pcs, N, d, idx, n, n_unique, rows, kmax, out_idx, out_dist, nullptr, tab_idx, tab_d2, K,
                         stats, ccg_pick_stream(ctx, stream));
}

extern "C" int ccg_knn_boot_hint_dev(ccg_ctx* ctx, const double* pcs, int64_t N, int d, const int32_t* idx,
                                     int64_t n, int n_unique, const double* rows, int kmax, int32_t* out_idx,
                                     double* out_dist, float* cell_hint, ccg_knn_stats* stats, void* stream) {
    return knn_boot_impl(ctx, pcs, N, d, idx, n, n_unique, rows, kmax, out_idx, out_dist, cell_hint, nullptr, nullptr,
                         0, stats, ccg_pick_stream(ctx, stream));
}

static int knn_boot_impl(ccg_ctx* ctx, const double* pcs, int64_t N, int d, const int32_t* idx, int64_t n,
                         int n_unique, const double* rows, int kmax, int32_t* out_idx, double* out_dist,
                         float* cell_hint, const int32_t* tab_idx, const double* tab_d2, int K,
                         ccg_knn_stats* stats, hipStream_t st) {
    CCG_REQUIRE(ctx && pcs && idx && rows && out_idx, "ccg_knn_boot_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_boot_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(N >= 1 && N < (1LL << 31) && n >= 2 && n < (1LL << 30), "ccg_knn_boot_dev: bad sizes");
    CCG_REQUIRE(n_unique == -1 || (n_unique >= 1 && n_unique <= n && n_unique <= N),
                "ccg_knn_boot_dev: n_unique=%d out of range", n_unique);
    CCG_REQUIRE(kmax >= 1 && kmax <= KNN_KP_BIG && kmax <= n - 1,
                "ccg_knn_boot_dev: kmax=%d must be in [1, min(%d, n-1)]", kmax, KNN_KP_BIG);
    // n_unique = -1: counted on the device (one stream synchronisation); the
    // workspaces are then sized for u <= min(n, N)
    const int ucap = n_unique >= 0 ? n_unique : (int)std::min<int64_t>(n, N);
    // workspaces (the full-size fail list first, so the distinct-cell run never grows it)
    double* ftau = nullptr;
    int* fail_list = knn_fail_ws(ctx, n, &ftau);
    char* ta = (char*)ccg_ws(ctx, WS_KB_A, sizeof(int64_t) * (n + 1) + sizeof(int32_t) * (4 * n + (size_t)ucap + 1));
    double* urows = (double*)ccg_ws(ctx, WS_KB_B, sizeof(double) * (size_t)ucap * (d + kmax) +
                                                      sizeof(int32_t) * (size_t)ucap * kmax +
                                                      sizeof(float) * (size_t)ucap + 64);
    unsigned int* misc = (unsigned int*)ccg_ws(ctx, WS_MISC, 256);
    if (!fail_list || !ta || !urows || !misc) return CCG_ENOMEM;
    int64_t* head = (int64_t*)ta;                // [n + 1] heads, then their exclusive scan in place
    int32_t* cells = (int32_t*)(head + n + 1);   // [n] sort keys (the cells), later row2u
    int32_t* scell = cells + n;                  // [n] sorted keys
    int32_t* rid = scell + n;                    // [n] sort values (the rows)
    int32_t* srow = rid + n;                     // [n] rows sorted by cell
    int32_t* row2u = cells;
    int* fail_count = (int*)(misc + 4);  // zeroed by knn_run's init kernel (or below when u == 1)
    const int t_all = ccg_timer_start(ctx, CCG_KT_KNN_TOTAL, st);
    // 1-2. rows grouped by cell: a counting sort over the N cells (one scan
    // gives the distinct ids and the cells' first positions)
    const unsigned ng = (unsigned)ccg_cdiv(n, 256);
    char* tc = (char*)ccg_ws(ctx, WS_KB_C, 2 * sizeof(int64_t) * (size_t)(N + 1) +
                                               sizeof(int) * (2 * (size_t)N + (size_t)ucap + 8));
    if (!tc) return CCG_ENOMEM;
    unsigned long long* pk = (unsigned long long*)tc;    // [N + 1] counts | presence (zero between calls)
    int64_t* pko = (int64_t*)(pk + N + 1);               // [N + 1] their exclusive scan
    int* cursor = (int*)(pko + N + 1);                   // [N] scatter cursors (zeroed by kb_cells_kernel)
    int* cell2u = cursor + N;                            // [N] cell -> distinct id (-1: absent)
    int* nbig = cell2u + N;                              // [1] cells with more than KB_FIX_SMALL rows
    int* big = nbig + 4;                                 // [ucap] their ids
    if (ctx->kb_zeroed != (void*)tc || ctx->kb_zero_n != N) {
        CCG_HIP(hipMemsetAsync(pk, 0, sizeof(int64_t) * (size_t)(N + 1), st));
        ctx->kb_zeroed = (void*)tc;
        ctx->kb_zero_n = N;
    }
    // (the table path: its fail counts and the expansion tie count, misc[4..6], zeroed here)
    kb_count_kernel<<<ng, 256, 0, st>>>(idx, n, N, pk, ctx->d_err, srow + n, (int64_t)ucap + 1,
                                        tab_idx ? misc + 4 : nullptr);
    int rc = ccg_scan_i64(ctx, (const int64_t*)pk, pko, N, st);
    if (rc) {
        ctx->kb_zeroed = nullptr;  // the counts were not cleared: the next call zeroes them
        return rc;
    }
    int u = n_unique;
    if (u < 0) {
        int64_t hu = 0;
        CCG_HIP(hipMemcpyAsync(&hu, pko + N, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        u = (int)((uint64_t)hu >> 32);
    }
    const int kq = std::min(kmax, u - 1);
    int32_t* ustart = srow + n;                  // [u + 1]
    double* ud2 = urows + (size_t)u * d;         // [u][kq] certified squared distances
    int32_t* uidx = (int32_t*)(ud2 + (size_t)u * kq);
    kb_cells_kernel<<<(unsigned)ccg_cdiv(N + 1, 256), 256, 0, st>>>(pk, pko, N, n, u, n_unique, cell2u, ustart,
                                                                    cursor, nbig, ctx->d_err);
    kb_scatter_kernel<<<ng, 256, 0, st>>>(idx, n, N, cell2u, ustart, cursor, srow, scell);
    kb_fixup_kernel<<<(unsigned)ccg_cdiv(u, 256), 256, 0, st>>>(u, n, ustart, srow, row2u, big, nbig);
    kb_fixup_big_kernel<<<16, 256, 0, st>>>(n, ustart, srow, row2u, big, nbig, rid);
    // 3. the distinct cells' rows and their kq nearest distinct cells
    float* urow_hint = cell_hint ? (float*)(uidx + (size_t)u * kq) : nullptr;
    // (the table path's fail counts and tie count, misc[4..6]: zeroed by kb_count_kernel)
    if (d <= 32)
        kb_urows_kernel<32><<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(rows, d, u, ustart, srow, urows, idx, cell_hint,
                                                                      urow_hint);
    else
        kb_urows_kernel<64><<<(unsigned)ccg_cdiv(u, 4), 256, 0, st>>>(rows, d, u, ustart, srow, urows, idx, cell_hint,
                                                                      urow_hint);
    ccg_knn_stats us = {0, 0};
    if (kq >= 1 && tab_idx) {
        // the table's present entries; cells short of kq of them: exact search among the distinct cells
        int* ufail = (int*)(misc + 5);
        kt_filter_kernel<false><<<(unsigned)ccg_cdiv(u, 4 * KT_CPW), 256, 0, st>>>(
            u, kq, K, d, ustart, scell, cell2u, tab_idx, tab_d2, urows, uidx, ud2, fail_list, ufail, ftau);
        rc = knn_fallback_launch(ctx, urows, u, d, kq, fail_list, ufail, uidx, ud2, nullptr, 1, st, true, ftau);
        if (rc) return rc;
        if (stats) {
            int nf = 0;
            CCG_HIP(hipMemcpyAsync(&nf, ufail, sizeof(int), hipMemcpyDeviceToHost, st));
            CCG_HIP(hipStreamSynchronize(st));
            us.fallback = nf;
        }
    } else if (kq >= 1) {
        rc = knn_run(ctx, urows, u, d, kq, uidx, ud2, stats ? &us : nullptr, st, nullptr, true, urow_hint);
        if (rc) return rc;
        if (cell_hint)
            kb_hint_kernel<<<(unsigned)ccg_cdiv(u, 256), 256, 0, st>>>(u, kq, ustart, srow, idx, ud2, cell_hint);
    }
    // 4. expansion to rows; ties cut by the list go to the exact search over all rows
    if (kq < 1) CCG_HIP(hipMemsetAsync(fail_count, 0, 3 * sizeof(int), st));  // (the table path zeroed it above)
    // one wave per distinct cell; cells whose list holds an equal-d2 tie
    // between cells take the per-row merge.  Cut ties: a radius search over
    // all rows (fewer than kmax rows within the radius, or more than the
    // candidate cap: the per-thread-list search)
    if (KNN_EXPAND_CELLS) {
        int* tie_count = (int*)(misc + 6);  // zeroed with the fail counts
        int* tie_list = (int*)head;         // the heads' scan is consumed (kb_tables_kernel)
        kb_expand_cells_kernel<<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(n, u, kq, uidx, ud2, ustart, srow, row2u,
                                                                         kmax, out_idx, out_dist, fail_list, fail_count,
                                                                         ftau, tie_list, tie_count);
        kb_expand_ties_kernel<<<64, 256, 0, st>>>(u, kq, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist,
                                                  fail_list, fail_count, ftau, tie_list, tie_count);
    } else {
        kb_expand_kernel<<<ng, 256, 0, st>>>(n, u, kq, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist,
                                             fail_list, fail_count, ftau);
    }
    rc = knn_fallback_launch(ctx, rows, n, d, kmax, fail_list, fail_count, out_idx, out_dist, nullptr, 1, st, false,
                             KNN_EXPAND_RADIUS ? ftau : nullptr);
    if (rc) return rc;
    ctx->last_fail_list = fail_list;
    ctx->last_fail_count = fail_count;
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    if (stats) {
        int nf = 0;
        CCG_HIP(hipMemcpyAsync(&nf, fail_count, sizeof(int), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        stats->queries = n;
        stats->fallback = us.fallback + nf;
        ctx->last_stats = *stats;
    }
    return CCG_OK;
}

// ------------------------------------------------- bootstrap batches --
// ccg_knn_boots_table_dev: nb bootstraps of the same PCs (n rows each, the
// rows of bootstrap s at s n .. (s + 1) n) through ONE set of launches of the
// table path above.  Bootstrap s's cell c is the virtual cell s N + c, so one
// counting sort over nb N virtual cells groups every bootstrap's rows by
// cell and numbers the distinct cells bootstrap by bootstrap (useg: the first
// distinct id of each bootstrap); the filter reads the cell's table row
// against its own bootstrap's presence map (cell2u + s N); cells short of kq
// present entries and rows with a cut tie go to the segmented radius search
// (each bootstrap's failed entries in their own region of the list, each
// searched among its own bootstrap's distinct cells or rows).  The result is
// every bootstrap's ccg_knn_boot_table_dev result, bit for bit, with row ids
// of the concatenation (local_ids = 0: the disjoint union of the nb graphs,
// ready for one SNN pass) or of the bootstrap (local_ids = 1).  Per batch the
// launches are those of one bootstrap (about 20), so a step of 125
// bootstraps in batches of 16 issues ~170 kNN launches instead of ~2000.
__global__ void kbs_rebase_kernel(int64_t n, int kmax, const int64_t* __restrict__ seg_off, int nseg, int sign,
                                  int32_t* __restrict__ out_idx);

extern "C" int ccg_knn_boots_table_dev(ccg_ctx* ctx, int64_t N, int d, const int32_t* idx, int64_t n, int nb,
                                       const int* n_unique, const double* rows, int kmax, const int32_t* tab_idx,
                                       const double* tab_d2, int K, int local_ids, int32_t* out_idx,
                                       double* out_dist, ccg_knn_stats* stats, void* stream) {
    CCG_REQUIRE(ctx && idx && n_unique && rows && tab_idx && tab_d2 && out_idx,
                "ccg_knn_boots_table_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_boots_table_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(nb >= 1 && nb <= KNN_SEG_MAX, "ccg_knn_boots_table_dev: nb=%d must be in [1, %d]", nb, KNN_SEG_MAX);
    CCG_REQUIRE(N >= 2 && n >= 2 && (int64_t)nb * n < (1LL << 30) && (int64_t)nb * N < (1LL << 31) - 1,
                "ccg_knn_boots_table_dev: bad sizes (N=%lld, n=%lld, nb=%d: nb n < 2^30, nb N < 2^31 - 1)",
                (long long)N, (long long)n, nb);
    CCG_REQUIRE(K >= 1 && K <= KNN_TAB_K && K <= N - 1,
                "ccg_knn_boots_table_dev: K=%d must be in [1, min(%d, N-1)]", K, KNN_TAB_K);
    CCG_REQUIRE(kmax >= 1 && kmax <= KNN_KP_BIG && kmax <= n - 1,
                "ccg_knn_boots_table_dev: kmax=%d must be in [1, min(%d, n-1)]", kmax, KNN_KP_BIG);
    int64_t ut = 0;
    for (int s = 0; s < nb; ++s) {
        CCG_REQUIRE(n_unique[s] >= kmax + 1 && n_unique[s] <= n && n_unique[s] <= N,
                    "ccg_knn_boots_table_dev: bootstrap %d has n_unique=%d (needs kmax + 1 = %d .. min(n, N))", s,
                    n_unique[s], kmax + 1);
        ut += n_unique[s];
    }
    const int u = (int)ut;
    const int64_t nt = (int64_t)nb * n, V = (int64_t)nb * N;
    hipStream_t st = ccg_pick_stream(ctx, stream);
    // workspaces (the exact search's for the larger of its two runs first)
    double* ftau = nullptr;
    int* fail_list = knn_fail_ws(ctx, nt, &ftau);  // per-bootstrap regions: distinct cells, then rows
    if (knn_fx_reserve(ctx, nt, d)) return CCG_ENOMEM;
    char* ta = (char*)ccg_ws(ctx, WS_KB_A, sizeof(int64_t) * (nt + 1) + sizeof(int32_t) * (4 * nt + (size_t)u + 1));
    double* urows = (double*)ccg_ws(ctx, WS_KB_B, sizeof(double) * (size_t)u * (d + kmax) +
                                                      sizeof(int32_t) * (size_t)u * kmax + 64);
    char* tc = (char*)ccg_ws(ctx, WS_KB_C, 2 * sizeof(int64_t) * (size_t)(V + 1) +
                                               sizeof(int) * (2 * (size_t)V + (size_t)u + 8));
    int64_t* useg = (int64_t*)ccg_ws(ctx, WS_KBT, sizeof(int64_t) * 2 * (KNN_SEG_MAX + 1) +
                                                      sizeof(int) * (2 * KNN_SEG_MAX + 8));
    if (!fail_list || !ta || !urows || !tc || !useg) return CCG_ENOMEM;
    int64_t* dso = useg + KNN_SEG_MAX + 1;              // [nb + 1] first row of every bootstrap
    int* fcnt_u = (int*)(dso + KNN_SEG_MAX + 1);        // [nb] failed distinct cells per bootstrap
    int* fcnt_r = fcnt_u + nb;                          // [nb] failed rows per bootstrap
    int* tie_count = fcnt_r + nb;                       // [1]
    int64_t* head = (int64_t*)ta;
    int32_t* cells = (int32_t*)(head + nt + 1);
    int32_t* scell = cells + nt;
    int32_t* rid = scell + nt;
    int32_t* srow = rid + nt;
    int32_t* ustart = srow + nt;                        // [u + 1]
    int32_t* row2u = cells;
    int32_t* tie_list = (int32_t*)head;
    unsigned long long* pk = (unsigned long long*)tc;   // [V + 1] counts | presence (zero between calls)
    int64_t* pko = (int64_t*)(pk + V + 1);
    int* cursor = (int*)(pko + V + 1);
    int* cell2u = cursor + V;
    int* nbig = cell2u + V;
    int* big = nbig + 4;
    double* ud2 = urows + (size_t)u * d;
    int32_t* uidx = (int32_t*)(ud2 + (size_t)u * kmax);
    const int t_all = ccg_timer_start(ctx, CCG_KT_KNN_TOTAL, st);
    if (ctx->kb_zeroed != (void*)tc || ctx->kb_zero_n != V) {
        CCG_HIP(hipMemsetAsync(pk, 0, sizeof(int64_t) * (size_t)(V + 1), st));
        ctx->kb_zeroed = (void*)tc;
        ctx->kb_zero_n = V;
    }
    // 1. every bootstrap's rows grouped by cell (one counting sort over the
    // virtual cells); the per-bootstrap fail counts and the tie count zeroed
    const unsigned ng = (unsigned)ccg_cdiv(nt, 256);
    kb_count_kernel<<<ng, 256, 0, st>>>(idx, nt, N, pk, ctx->d_err, ustart, (int64_t)u + 1, (unsigned*)fcnt_u,
                                        2 * nb + 1, n);
    int rc = ccg_scan_i64(ctx, (const int64_t*)pk, pko, V, st);
    if (rc) {
        ctx->kb_zeroed = nullptr;
        return rc;
    }
    kb_cells_kernel<<<(unsigned)ccg_cdiv(V + 1, 256), 256, 0, st>>>(pk, pko, V, nt, u, u, cell2u, ustart, cursor,
                                                                    nbig, ctx->d_err, nb, N, kmax + 1, useg, dso, n);
    kb_scatter_kernel<<<ng, 256, 0, st>>>(idx, nt, N, cell2u, ustart, cursor, srow, scell, n);
    kb_fixup_kernel<<<(unsigned)ccg_cdiv(u, 256), 256, 0, st>>>(u, nt, ustart, srow, row2u, big, nbig);
    kb_fixup_big_kernel<<<16, 256, 0, st>>>(nt, ustart, srow, row2u, big, nbig, rid);
    // 2. the distinct cells' rows; their kmax nearest distinct cells of the
    // same bootstrap from the table; short cells: the radius search among
    // their bootstrap's distinct cells
    if (d <= 32)
        kb_urows_kernel<32><<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(rows, d, u, ustart, srow, urows, idx, nullptr,
                                                                      nullptr);
    else
        kb_urows_kernel<64><<<(unsigned)ccg_cdiv(u, 4), 256, 0, st>>>(rows, d, u, ustart, srow, urows, idx, nullptr,
                                                                      nullptr);
#ifdef CCG_KT_UID_MAJOR
    kt_filter_kernel<true><<<(unsigned)ccg_cdiv(u, 4 * KT_CPW), 256, 0, st>>>(
        u, kmax, K, d, ustart, scell, cell2u, tab_idx, tab_d2, urows, uidx, ud2, fail_list, nullptr, ftau, N, useg,
        fcnt_u);
#else
    kt_filter_cells_kernel<<<(unsigned)(ccg_cdiv(N, 4) + 16), 256, 0, st>>>(
        nb, N, kmax, K, d, cell2u, tab_idx, tab_d2, urows, uidx, ud2, fail_list, ftau, useg, fcnt_u, u);
#endif
    rc = knn_fallback_launch(ctx, urows, u, d, kmax, fail_list, fcnt_u, uidx, ud2, useg, nb, st, true, ftau, fcnt_u);
    if (rc) return rc;
    // 3. expansion to rows (ids of the concatenation); cut ties: the radius
    // search among the bootstrap's rows
    kb_expand_cells_kernel<<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(nt, u, kmax, uidx, ud2, ustart, srow, row2u,
                                                                     kmax, out_idx, out_dist, fail_list, nullptr, ftau,
                                                                     tie_list, tie_count, useg, nb, dso, fcnt_r);
    kb_expand_ties_kernel<<<64, 256, 0, st>>>(u, kmax, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist,
                                              fail_list, nullptr, ftau, tie_list, tie_count, useg, nb, dso, fcnt_r);
    const int* cf = nullptr;
    const int* cfc = nullptr;
    rc = knn_fallback_launch(ctx, rows, nt, d, kmax, fail_list, fcnt_r, out_idx, out_dist, dso, nb, st, false, ftau,
                             fcnt_r, &cf, &cfc);
    if (rc) return rc;
    if (local_ids)
        kbs_rebase_kernel<<<(unsigned)ccg_cdiv(nt * kmax, 256), 256, 0, st>>>(nt, kmax, dso, nb, -1, out_idx);
    ctx->last_fail_list = cf;
    ctx->last_fail_count = cfc;
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    if (stats) {
        int h[2 * KNN_SEG_MAX];
        CCG_HIP(hipMemcpyAsync(h, fcnt_u, sizeof(int) * 2 * nb, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        int64_t f = 0;
        for (int s = 0; s < 2 * nb; ++s) f += h[s];
        stats->queries = nt;
        stats->fallback = f;
        ctx->last_stats = *stats;
    }
    return CCG_OK;
}

// --------------------------------------------- batched bootstrap segments --
// iterate=TRUE (R/consensusClust.R:541-567) re-runs the bootstrap loop
// (:391-400) on every subcluster: many small bootstraps of many small PC
// matrices.  ccg_knn_boot_segments_dev runs all of them -- one segment per
// (subcluster, bootstrap) -- through ONE distinct-cell pipeline: rows grouped
// by (segment, cell) with one radix sort, one segmented screen / certify /
// fallback over every segment's distinct cells (each segment in its own
// Morton order), one expansion back to rows, one exact search for cut ties.
__global__ void kbs_keys_kernel(const int32_t* __restrict__ idx, int64_t n, int64_t Ntot,
                                const int64_t* __restrict__ seg_off, int nseg, int32_t* __restrict__ keys,
                                int32_t* __restrict__ rid, int* __restrict__ err) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int c = idx[t];
    if (c < 0 || c >= Ntot) {
        atomicOr(err, CCG_DERR_KNN_UNIQUE);
        c = 0;
    }
    keys[t] = (int32_t)((int64_t)knn_seg_of(seg_off, nseg, t) * Ntot + c);
    rid[t] = (int32_t)t;
}

// the distinct-cell search returns segment-local distinct ids: back to global ids
__global__ void kbs_uglobal_kernel(int64_t u, int kq, const int64_t* __restrict__ useg, int nseg,
                                   int32_t* __restrict__ uidx) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= u * kq) return;
    uidx[t] += (int32_t)useg[knn_seg_of(useg, nseg, t / kq)];
}

// neighbour rows: subtract (sign -1) or add (+1) the row's segment start
__global__ void kbs_rebase_kernel(int64_t n, int kmax, const int64_t* __restrict__ seg_off, int nseg, int sign,
                                  int32_t* __restrict__ out_idx) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kmax) return;
    out_idx[t] += sign * (int32_t)seg_off[knn_seg_of(seg_off, nseg, t / kmax)];
}

extern "C" int ccg_knn_boot_segments_dev(ccg_ctx* ctx, const double* cells, int64_t Ntot, int d, const int32_t* idx,
                                         int64_t n, const int64_t* seg_off, const int* seg_unique, int nseg, int kmax,
                                         int local_ids, int32_t* out_idx, double* out_dist, ccg_knn_stats* stats,
                                         void* stream) {
    CCG_REQUIRE(ctx && cells && idx && seg_off && seg_unique && out_idx, "ccg_knn_boot_segments_dev: NULL argument");
    CCG_REQUIRE(d >= 1 && d <= 63, "ccg_knn_boot_segments_dev: d=%d must be in [1, 63]", d);
    CCG_REQUIRE(nseg >= 1 && n >= 2 && n < (1LL << 30) && Ntot >= 1 && Ntot < (1LL << 30),
                "ccg_knn_boot_segments_dev: bad sizes");
    CCG_REQUIRE(kmax >= 1 && kmax <= KNN_KP_BIG, "ccg_knn_boot_segments_dev: kmax=%d must be in [1, %d]", kmax,
                KNN_KP_BIG);
    CCG_REQUIRE(seg_off[0] == 0 && seg_off[nseg] == n, "ccg_knn_boot_segments_dev: seg_off must run from 0 to n");
    CCG_REQUIRE((int64_t)nseg * Ntot < (1LL << 31),
                "ccg_knn_boot_segments_dev: nseg x Ntot = %lld must be below 2^31 (split the batch)",
                (long long)nseg * Ntot);
    std::vector<int64_t> uoff(nseg + 1, 0);
    for (int s = 0; s < nseg; ++s) {
        const int64_t ns = seg_off[s + 1] - seg_off[s];
        CCG_REQUIRE(ns >= 2 && seg_unique[s] >= kmax + 1 && seg_unique[s] <= ns,
                    "ccg_knn_boot_segments_dev: segment %d has %d distinct cells in %lld rows (needs >= kmax+1 = %d)",
                    s, seg_unique[s], (long long)ns, kmax + 1);
        uoff[s + 1] = uoff[s] + seg_unique[s];
    }
    const int64_t u = uoff[nseg];
    hipStream_t st = ccg_pick_stream(ctx, stream);
    double* ftau = nullptr;
    int* fail_list = knn_fail_ws(ctx, n, &ftau);
    char* ta = (char*)ccg_ws(ctx, WS_KB_A, sizeof(int64_t) * (n + 1) + sizeof(int32_t) * (4 * n + (size_t)u + 1));
    double* urows = (double*)ccg_ws(ctx, WS_KB_B, sizeof(double) * (size_t)u * (d + kmax) +
                                                      sizeof(int32_t) * (size_t)u * kmax + 64);
    double* rows = (double*)ccg_ws(ctx, WS_SEG_ROWS, sizeof(double) * (size_t)n * d);
    int64_t* dso = (int64_t*)ccg_ws(ctx, WS_SEG_TAB, sizeof(int64_t) * 2 * (size_t)(nseg + 1));
    unsigned int* misc = (unsigned int*)ccg_ws(ctx, WS_MISC, 256);
    if (!fail_list || !ta || !urows || !rows || !dso || !misc) return CCG_ENOMEM;
    int64_t* duo = dso + nseg + 1;
    int64_t* head = (int64_t*)ta;
    int32_t* keys = (int32_t*)(head + n + 1);
    int32_t* skeys = keys + n;
    int32_t* rid = skeys + n;
    int32_t* srow = rid + n;
    int32_t* ustart = srow + n;
    int32_t* row2u = keys;
    double* ud2 = urows + (size_t)u * d;
    int32_t* uidx = (int32_t*)(ud2 + (size_t)u * kmax);
    int* fail_count = (int*)(misc + 4);
    {
        int rs = ccg_h2d_staged(ctx, dso, seg_off, sizeof(int64_t) * (nseg + 1), st);
        if (!rs) rs = ccg_h2d_staged(ctx, duo, uoff.data(), sizeof(int64_t) * (nseg + 1), st);
        if (rs) return rs;
    }
    const int t_all = ccg_timer_start(ctx, CCG_KT_KNN_TOTAL, st);
    const unsigned ng = (unsigned)ccg_cdiv(n, 256);
    // 1. the rows, and (segment, cell) keys sorted stably: each segment's cells, each cell's rows ascending
    knn_gather_rm(cells, Ntot, d, idx, n, rows, st);
    kbs_keys_kernel<<<ng, 256, 0, st>>>(idx, n, Ntot, dso, nseg, keys, rid, ctx->d_err);
    int bits = 1;
    while (bits < 31 && (1LL << bits) < (int64_t)nseg * Ntot) ++bits;
    int rc = ccg_sort_pairs_i32(ctx, keys, skeys, rid, srow, n, bits, st);
    if (rc) return rc;
    // 2. distinct (segment, cell) ids: ids of a segment are contiguous, in cell order
    kb_heads_kernel<<<ng, 256, 0, st>>>(skeys, n, head, ustart, u + 1);
    rc = ccg_scan_i64(ctx, head, head, n, st);
    if (rc) return rc;
    kb_tables_kernel<<<ng, 256, 0, st>>>(skeys, srow, n, head, (int)u, ustart, row2u, ctx->d_err);
    if (d <= 32)
        kb_urows_kernel<32><<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(rows, d, (int)u, ustart, srow, urows, idx, nullptr,
                                                                      nullptr);
    else
        kb_urows_kernel<64><<<(unsigned)ccg_cdiv(u, 4), 256, 0, st>>>(rows, d, (int)u, ustart, srow, urows, idx, nullptr,
                                                                      nullptr);
    // 3. every segment's distinct cells among themselves (kq = kmax: each has >= kmax + 1)
    std::vector<int64_t> po;
    std::vector<int> hperm;
    std::vector<int4> hblk;
    KnnSegs sg;
    rc = knn_seg_plan(ctx, uoff.data(), nseg, d, kmax, st, po, hperm, hblk, &sg);
    if (rc) return rc;
    ccg_knn_stats us = {0, 0};
    rc = knn_run(ctx, urows, u, d, kmax, uidx, ud2, stats ? &us : nullptr, st, &sg, true);
    if (rc) return rc;
    kbs_uglobal_kernel<<<(unsigned)ccg_cdiv(u * kmax, 256), 256, 0, st>>>(u, kmax, duo, nseg, uidx);
    // 4. expansion to rows (global row ids), then segment-local ids; cut ties: the exact search in the segment
    CCG_HIP(hipMemsetAsync(misc + 4, 0, 3 * sizeof(unsigned), st));
    int* tie_count = (int*)(misc + 6);
    int* tie_list = (int*)head;  // the heads' scan is consumed (kb_tables_kernel)
    kb_expand_cells_kernel<<<(unsigned)ccg_cdiv(u, 8), 256, 0, st>>>(n, (int)u, kmax, uidx, ud2, ustart, srow, row2u,
                                                                     kmax, out_idx, out_dist, fail_list, fail_count,
                                                                     ftau, tie_list, tie_count, duo, nseg);
    kb_expand_ties_kernel<<<64, 256, 0, st>>>((int)u, kmax, uidx, ud2, ustart, srow, row2u, kmax, out_idx, out_dist,
                                              fail_list, fail_count, ftau, tie_list, tie_count, duo, nseg);
    const unsigned gk = (unsigned)ccg_cdiv(n * kmax, 256);
    kbs_rebase_kernel<<<gk, 256, 0, st>>>(n, kmax, dso, nseg, -1, out_idx);
    rc = knn_fallback_launch(ctx, rows, n, d, kmax, fail_list, fail_count, out_idx, out_dist, dso, nseg, st, false,
                             nullptr);
    if (rc) return rc;
    if (!local_ids) kbs_rebase_kernel<<<gk, 256, 0, st>>>(n, kmax, dso, nseg, 1, out_idx);
    ctx->last_fail_list = fail_list;
    ctx->last_fail_count = fail_count;
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    // (the plan's tables went through the pinned ring: no synchronisation
    // unless statistics are asked for -- round 5 synchronised every call,
    // which left the GPU idle between the launch sets of cfg5)
    if (stats) {
        int nf = 0;
        CCG_HIP(hipMemcpyAsync(&nf, fail_count, sizeof(int), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        stats->queries = n;
        stats->fallback = us.fallback + nf;
        ctx->last_stats = *stats;
    }
    return CCG_OK;
}

extern "C" int ccg_knn_boot_segments(ccg_ctx* ctx, const double* cells, int64_t Ntot, int d, const int32_t* idx,
                                     int64_t n, const int64_t* seg_off, const int* seg_unique, int nseg, int kmax,
                                     int32_t* out_idx, double* out_dist, ccg_knn_stats* stats) {
    CCG_REQUIRE(ctx && cells && idx && seg_off && out_idx, "ccg_knn_boot_segments: NULL argument");
    CCG_REQUIRE(Ntot >= 1 && n >= 2 && d >= 1 && nseg >= 1 && seg_off[0] == 0 && seg_off[nseg] == n,
                "ccg_knn_boot_segments: bad sizes");
    for (int64_t t = 0; t < n; ++t)
        CCG_REQUIRE(idx[t] >= 0 && idx[t] < Ntot, "ccg_knn_boot_segments: idx[%lld] out of range", (long long)t);
    std::vector<int> su(nseg);
    if (seg_unique) {
        std::copy(seg_unique, seg_unique + nseg, su.begin());
    } else {  // length(unique(...)) of every segment
        std::vector<int> stamp(Ntot, -1);
        for (int s = 0; s < nseg; ++s) {
            int c = 0;
            for (int64_t t = seg_off[s]; t < seg_off[s + 1]; ++t)
                if (stamp[idx[t]] != s) {
                    stamp[idx[t]] = s;
                    ++c;
                }
            su[s] = c;
        }
    }
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* dcells = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * Ntot * d);
    int32_t* didx = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * n);
    int32_t* dout = (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * n * kmax);
    double* ddist = out_dist ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * n * kmax) : nullptr;
    if (!dcells || !didx || !dout || (out_dist && !ddist)) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dcells, cells, sizeof(double) * Ntot * d, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(didx, idx, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
    int rc = ccg_knn_boot_segments_dev(ctx, dcells, Ntot, d, didx, n, seg_off, su.data(), nseg, kmax, 1, dout, ddist,
                                       stats, st);
    if (rc) return rc;
    rc = ccg_take_device_error(ctx);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(out_idx, dout, sizeof(int32_t) * n * kmax, hipMemcpyDeviceToHost, st));
    if (out_dist) CCG_HIP(hipMemcpyAsync(out_dist, ddist, sizeof(double) * n * kmax, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}

extern "C" int ccg_knn_last_fallback(ccg_ctx* ctx, int32_t* rows, int64_t cap, int64_t* count) {
    CCG_REQUIRE(ctx && count && (rows || cap == 0), "ccg_knn_last_fallback: NULL argument");
    *count = 0;
    if (!ctx->last_fail_list) return CCG_OK;
    CCG_HIP(hipSetDevice(ctx->device));
    CCG_HIP(hipDeviceSynchronize());
    int nf = 0;
    CCG_HIP(hipMemcpy(&nf, ctx->last_fail_count, sizeof(int), hipMemcpyDeviceToHost));
    *count = nf;
    const int64_t m = std::min<int64_t>(nf, cap);
    if (m > 0) CCG_HIP(hipMemcpy(rows, ctx->last_fail_list, sizeof(int32_t) * m, hipMemcpyDeviceToHost));
    return CCG_OK;
}

extern "C" int ccg_knn_boot(ccg_ctx* ctx, const double* pcs, int64_t N, int d,
                            const int32_t* boot_idx, int64_t n, int nb, int kmax,
                            int32_t* out_idx, double* out_dist, ccg_knn_stats* stats) {
    CCG_REQUIRE(ctx && pcs && boot_idx && out_idx, "ccg_knn_boot: NULL argument");
    CCG_REQUIRE(N > 0 && n >= 2 && nb >= 1 && d >= 1, "ccg_knn_boot: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* dpcs = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * N * d);
    int32_t* didx = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * n * nb);
    int32_t* dout = (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * n * kmax);
    double* ddist = out_dist ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * n * kmax) : nullptr;
    double* rows = (double*)ccg_ws(ctx, WS_ROWS64, sizeof(double) * n * d);
    if (!dpcs || !didx || !dout || !rows || (out_dist && !ddist)) return CCG_ENOMEM;
    for (int64_t t = 0; t < n * nb; ++t)
        CCG_REQUIRE(boot_idx[t] >= 0 && boot_idx[t] < N, "ccg_knn_boot: boot_idx out of range");
    CCG_HIP(hipMemcpyAsync(dpcs, pcs, sizeof(double) * N * d, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(didx, boot_idx, sizeof(int32_t) * n * nb, hipMemcpyHostToDevice, st));
    ccg_knn_stats acc = {0, 0};
    // Many bootstraps: one cell table for the call (ccg_knn_table_dev), each
    // bootstrap filters it.  Few: per-bootstrap screens sharing a hint array
    // (each bootstrap's certified k-th distances warm-start the next one's
    // screen).  Results are identical either way.
    const int K = (int)std::min<int64_t>(KNN_TAB_K, N - 1);
    const bool table = nb >= KNN_TABLE_MIN_BOOTS && N >= 2;
    float* hint = nullptr;
    int32_t* tab_idx = nullptr;
    double* tab_d2 = nullptr;
    if (table) {
        char* tb = (char*)ccg_ws(ctx, WS_TAB, (sizeof(int32_t) + sizeof(double)) * (size_t)N * K + 256);
        if (!tb) return CCG_ENOMEM;
        tab_d2 = (double*)tb;
        tab_idx = (int32_t*)(tab_d2 + (size_t)N * K);
        int rc = ccg_knn_table_dev(ctx, dpcs, N, d, K, tab_idx, tab_d2, nullptr, st);
        if (rc) return rc;
    } else {
        hint = (float*)ccg_ws(ctx, WS_HINT, sizeof(float) * N);
        if (!hint) return CCG_ENOMEM;
        CCG_HIP(hipMemsetAsync(hint, 0, sizeof(float) * N, st));
    }
    std::vector<unsigned char> seen(N);
    for (int b = 0; b < nb; ++b) {
        // the bootstrap's distinct cells (R: length(unique(idx)))
        std::fill(seen.begin(), seen.end(), 0);
        int u = 0;
        for (int64_t t = 0; t < n; ++t) {
            const int32_t c = boot_idx[(int64_t)b * n + t];
            u += seen[c] ? 0 : 1;
            seen[c] = 1;
        }
        int rc = ccg_gather_rows_dev(ctx, dpcs, N, d, didx + (int64_t)b * n, n, rows, st);
        if (rc) return rc;
        ccg_knn_stats s;
        rc = table ? ccg_knn_boot_table_dev(ctx, dpcs, N, d, didx + (int64_t)b * n, n, u, rows, kmax, tab_idx, tab_d2,
                                            K, dout, ddist, &s, st)
                   : ccg_knn_boot_hint_dev(ctx, dpcs, N, d, didx + (int64_t)b * n, n, u, rows, kmax, dout, ddist, hint,
                                           &s, st);
        if (rc) return rc;
        acc.queries += s.queries;
        acc.fallback += s.fallback;
        CCG_HIP(hipMemcpyAsync(out_idx + (int64_t)b * n * kmax, dout, sizeof(int32_t) * n * kmax,
                               hipMemcpyDeviceToHost, st));
        if (out_dist)
            CCG_HIP(hipMemcpyAsync(out_dist + (int64_t)b * n * kmax, ddist,
                                   sizeof(double) * n * kmax, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
    }
    if (stats) *stats = acc;
    ctx->last_stats = acc;
    return CCG_OK;
}

extern "C" int ccg_knn_segments(ccg_ctx* ctx, const double* rows, int64_t n, int d, const int64_t* seg_off,
                                int nseg, int kmax, int32_t* out_idx, double* out_dist, ccg_knn_stats* stats) {
    CCG_REQUIRE(ctx && rows && seg_off && out_idx, "ccg_knn_segments: NULL argument");
    CCG_REQUIRE(n >= 2 && d >= 1 && nseg >= 1, "ccg_knn_segments: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* drows = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * n * d);
    int32_t* dout = (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * n * kmax);
    double* ddist = out_dist ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * n * kmax) : nullptr;
    if (!drows || !dout || (out_dist && !ddist)) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(drows, rows, sizeof(double) * n * d, hipMemcpyHostToDevice, st));
    ccg_knn_stats s;
    const int rc = ccg_knn_segments_dev(ctx, drows, n, d, seg_off, nseg, kmax, dout, ddist, &s, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(out_idx, dout, sizeof(int32_t) * n * kmax, hipMemcpyDeviceToHost, st));
    if (out_dist) CCG_HIP(hipMemcpyAsync(out_dist, ddist, sizeof(double) * n * kmax, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (stats) *stats = s;
    return CCG_OK;
}
