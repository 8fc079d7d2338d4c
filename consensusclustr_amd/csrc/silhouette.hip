// Batched approximate silhouette on gfx950.
//
// Reference: mean(bluster::approxSilhouette(x, clusters)[,3], na.rm=TRUE)
// (R/consensusClust.R:447, :518, :664).  For each of L label vectors over
// the same m x d matrix:
//   mu_c  = colMeans(x[c, ])                 v_c = mean_i in c |x_i - mu_c|^2
//   D_i(c) = sqrt(|x_i - mu_c|^2 + v_c)      self = D_i(own), other = min_{c!=own}
//   width_i = (other - self) / max(other, self)   (0 for every row if C == 1)
// and the mean over non-NaN widths.
//
// Every cross-row reduction (cluster sums, variances, the mean) is done in
// 64-bit fixed point with integer atomics, so the result is bitwise
// reproducible regardless of scheduling; the scale is chosen on the device
// from max|x| so no partial sum can overflow.  Quantisation error is below
// 2^-36 relative for the sizes we support, far inside the 1e-5 tolerance.
// The widths' squared distances are |x|^2 + |mu|^2 + v - 2 x.mu with x.mu on
// the fp64 matrix core (a fixed-order MFMA chain, so also reproducible).
// Grid: (row tiles) x (groups of SIL_LG labelings); x rows are held in
// registers and reused across the group.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "ccg_internal.h"

#define SIL_T 256
// centroid granularity of the width tiles (v_mfma_f64_4x4x4f64: C padded to
// a multiple of 4; the 16x16x4 tiles of round 3 padded to 16, 1.37x at C =
// 2..40: silhouette 0.454 -> 0.435 ms per bootstrap at cfg3)
#define SIL_CGRP 4
#ifndef SIL_LG
#define SIL_LG 5
#endif

__device__ __forceinline__ int scale_exp(double bound) {
    // largest e with bound * 2^e <= 2^61
    if (!(bound > 0.0)) return 52;
    int e = 61 - (ilogb(bound) + 1);
    return e > 52 ? 52 : e;
}

// one atomic per block on one word: a small grid (a 1024-block grid spent
// ~10 us serialising its atomics at the L2)
#define SIL_MAXABS_GRID 256
__global__ __launch_bounds__(256) void sil_maxabs(const double* __restrict__ x, int64_t tot,
                                                  unsigned* __restrict__ bits) {
    __shared__ unsigned red[4];
    double mx = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0;  // four loads in flight per step
    const int64_t stp = (int64_t)gridDim.x * blockDim.x;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; t + 3 * stp < tot; t += 4 * stp) {
        mx = fmax(mx, fabs(x[t]));
        m1 = fmax(m1, fabs(x[t + stp]));
        m2 = fmax(m2, fabs(x[t + 2 * stp]));
        m3 = fmax(m3, fabs(x[t + 3 * stp]));
    }
    for (; t < tot; t += stp) mx = fmax(mx, fabs(x[t]));
    mx = fmax(fmax(mx, m1), fmax(m2, m3));
    // a float at or above max|x| (rounded up)
    unsigned local = __float_as_uint(nextafterf((float)mx, INFINITY));
    for (int o = 32; o > 0; o >>= 1) local = max(local, (unsigned)__shfl_xor((int)local, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = local;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(bits, max(max(red[0], red[1]), max(red[2], red[3])));  // one atomic per block
}

template <int DMAX>
__device__ __forceinline__ void load_row(const double* __restrict__ x, int64_t r, int d,
                                         double (&xr)[DMAX]) {
#pragma unroll
    for (int k = 0; k < DMAX; ++k) xr[k] = (k < d) ? x[r * d + k] : 0.0;
}

// K1 (fallback for large cmax, whose sorted-segment LDS would not fit):
// fixed-point cluster sums and counts, one atomic per (row, dimension),
// staged in LDS when (cmax + 1) x d accumulators fit (SIL_LDS_CAP), else added
// straight to the global sums.  v_c then comes from sil_var.
#define SIL_LDS_CAP 65536
template <int DMAX, bool LDS>
__global__ __launch_bounds__(SIL_T) void sil_centroid(const double* __restrict__ x, int64_t m,
                                                      int d, const int32_t* __restrict__ labels,
                                                      int L, int cmax,
                                                      const unsigned* __restrict__ maxabs_bits,
                                                      unsigned long long* __restrict__ gsum,
                                                      unsigned long long* __restrict__ gcnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* acc = (unsigned long long*)smem;          // [cmax+1][d]
    unsigned* cnt = (unsigned*)(acc + (int64_t)(cmax + 1) * d);   // [cmax+1]
    const int64_t r = (int64_t)blockIdx.x * SIL_T + threadIdx.x;
    const bool in = r < m;
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double sc = ldexp(1.0, scale_exp(maxabs * (double)m));
    long long q[DMAX];  // the row, quantised once for all of the block's labelings
#pragma unroll
    for (int k = 0; k < DMAX; ++k) q[k] = (in && k < d) ? __double2ll_rn(x[r * d + k] * sc) : 0ll;
    const int nacc = (cmax + 1) * d;
    const int l1 = min(L, (int)(blockIdx.y + 1) * SIL_LG);
    for (int l = blockIdx.y * SIL_LG; l < l1; ++l) {
        unsigned long long* gs = gsum + (int64_t)l * nacc;
        unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
        if (LDS) {
            for (int t = threadIdx.x; t < nacc; t += SIL_T) acc[t] = 0ull;
            for (int t = threadIdx.x; t <= cmax; t += SIL_T) cnt[t] = 0u;
            __syncthreads();
        }
        if (in) {
            const int lab = labels[(int64_t)l * m + r];
            if (lab >= 1 && lab <= cmax) {
#pragma unroll
                for (int k = 0; k < DMAX; ++k)
                    if (k < d) {
                        if (LDS) atomicAdd(&acc[lab * d + k], (unsigned long long)q[k]);
                        else atomicAdd(&gs[(int64_t)lab * d + k], (unsigned long long)q[k]);
                    }
                if (LDS) atomicAdd(&cnt[lab], 1u);
                else atomicAdd(&gc[lab], 1ull);
            }
        }
        if (LDS) {
            __syncthreads();
            for (int t = threadIdx.x; t < nacc; t += SIL_T)
                if (acc[t]) atomicAdd(&gs[t], acc[t]);
            for (int t = threadIdx.x; t <= cmax; t += SIL_T)
                if (cnt[t]) atomicAdd(&gc[t], (unsigned long long)cnt[t]);
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int sil_block_excl_scan(int v, int* sh, int* total) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    int woff = 0, tot = 0;
    for (int w = 0; w < SIL_T / 64; ++w) {
        if (w < wv) woff += sh[w];
        tot += sh[w];
    }
    __syncthreads();
    *total = tot;
    return woff + x - v;
}

// K1': fixed-point rows, once per call: q1 = round(x * sc) [m][DMAX] int64
// (zero past d) and q2 = round(|x|^2 * sc2) [m] (v_c needs only the
// cluster's total sum of squares: v_c = S2 / n - |mu_c|^2).
__host__ __device__ inline double sil_s2_bound(double maxabs, int d, int64_t m) {
    return maxabs * maxabs * (double)d * (double)m;
}
template <int DMAX>
__global__ void sil_quant(const double* __restrict__ x, int64_t m, int d, const unsigned* __restrict__ maxabs_bits,
                          long long* __restrict__ q1, long long* __restrict__ q2) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = t / DMAX;  // m * DMAX is a multiple of DMAX: a row's threads are all in or all out
    if (r >= m) return;
    const int k = (int)(t - r * DMAX);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double sc = ldexp(1.0, scale_exp(maxabs * (double)m));
    const double v = k < d ? x[r * d + k] : 0.0;
    q1[t] = __double2ll_rn(v * sc);
    // |x|^2 of the row: its DMAX threads are DMAX-aligned lanes of one wave
    // (fixed xor tree: deterministic)
    double s2 = v * v;
#pragma unroll
    for (int o = DMAX / 2; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    if (k == 0) q2[r] = __double2ll_rn(s2 * ldexp(1.0, scale_exp(sil_s2_bound(maxabs, d, m))));
}

// K1 (sorted segments): cluster sums S1 = sum x, S2 = sum |x|^2 and counts of
// a SIL_SORT_ROWS-row tile for one labeling (grid y), without a per-row
// atomic.  The tile's rows are counting-sorted by label in LDS; each wave
// then walks a quarter of the sorted rows with lanes along the dimensions
// (64 / DMAX rows per step) and keeps running sums in registers while the
// label repeats, so a lane issues one LDS atomic per label segment instead of
// one per row.  Large tiles keep the flush of the LDS sums to the global sums
// (atomics from every block on the same words) rare.  Integer sums: any
// order gives the same bits.  LDS: acc1 [cmax+1][DMAX] and acc2 [cmax+1]
// int64, counts/offsets [cmax+1], sorted rows, labels and weights
// [SIL_SORT_ROWS].
#ifndef SIL_SORT_ROWS
#define SIL_SORT_ROWS 1024
#endif
#ifndef SIL_SUMS_UNROLL
#define SIL_SUMS_UNROLL 8  // walk steps whose loads are in flight together per wave
#endif
#ifndef SIL_SUMS_ROWS
#define SIL_SUMS_ROWS 0  // tools only: 1 = cluster sums over every row, not the representatives (A/B)
#endif
template <int DMAX>
__host__ __device__ constexpr size_t sil_sorted_lds(int cmax) {
    return (size_t)(cmax + 1) * DMAX * 8 + (size_t)(cmax + 1) * 16 + 3 * SIL_SORT_ROWS * 4;
}

// Distinct-cell form (rep != nullptr): tile position p is the representative
// row rep[p] of a cell, weighted by the cnt[p] rows of the cell less the
// mult[l][p] of them labelled apart in labeling l (those rows are added by
// sil_sums_exc); the integer sums are those of the rows.  (Grid order: tiles
// fastest.  Dealing a tile's labelings to one XCD instead, so its rows are
// read into one L2, measured slower: 335 against 223 us at cfg3.)

template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_sums_sorted(int64_t m, int d, const int32_t* __restrict__ labels,
                                                         int cmax, const long long* __restrict__ q1,
                                                         const long long* __restrict__ q2,
                                                         unsigned long long* __restrict__ gsum,
                                                         unsigned long long* __restrict__ gsum2,
                                                         unsigned long long* __restrict__ gcnt,
                                                         const int* __restrict__ rep, const int* __restrict__ mult,
                                                         const int* __restrict__ cnt, int64_t mw,
                                                         const int64_t* __restrict__ nrep) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RPT = SIL_SORT_ROWS / SIL_T;  // rows per thread in the sort
    constexpr int RPW = 64 / DMAX;              // rows per wave step
    constexpr int STEPS = SIL_SORT_ROWS / 4 / RPW;
    unsigned long long* acc1 = (unsigned long long*)smem;                 // [cmax+1][DMAX]
    unsigned long long* acc2 = acc1 + (int64_t)(cmax + 1) * DMAX;         // [cmax+1]
    int* hcnt = (int*)(acc2 + (cmax + 1));                                // [cmax+1]
    int* hoff = hcnt + (cmax + 1);                                        // [cmax+1]
    int* srow = hoff + (cmax + 1);                                        // [SIL_SORT_ROWS]
    int* slab = srow + SIL_SORT_ROWS;                                     // [SIL_SORT_ROWS]
    int* swgt = slab + SIL_SORT_ROWS;                                     // [SIL_SORT_ROWS]
    __shared__ int sh[SIL_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k = lane % DMAX, sub = lane / DMAX;
    const int l = blockIdx.y;
    const int64_t rb = (int64_t)blockIdx.x * SIL_SORT_ROWS;
    const int64_t npos = rep ? *nrep : m;  // positions: rows, or the representatives (counted on the device)
    if (rb >= npos) return;
    const int nacc = (cmax + 1) * DMAX;
    for (int t = tid; t < nacc + cmax + 1; t += SIL_T) acc1[t] = 0ull;
    for (int t = tid; t <= cmax; t += SIL_T) hcnt[t] = 0;
    __syncthreads();
    // label 0 collects rows past m and codes outside [1, cmax]
    int lab[RPT], rank[RPT], wgt[RPT], row[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int64_t p = rb + i * SIL_T + tid;
        int lb = 0, w = 0, r = 0;
        if (p < npos) {
            r = rep ? rep[p] : (int)p;
            lb = labels[(int64_t)l * m + r];
            w = rep ? cnt[p] - mult[(int64_t)l * mw + p] : 1;
            if (lb < 1 || lb > cmax || w <= 0) lb = 0;
        }
        lab[i] = lb;
        wgt[i] = w;
        row[i] = r;
        rank[i] = atomicAdd(&hcnt[lb], 1);
    }
    __syncthreads();
    int carry = 0;
    for (int c0 = 0; c0 <= cmax; c0 += SIL_T) {
        const int c = c0 + tid;
        const int v = c <= cmax ? hcnt[c] : 0;
        int tot;
        const int ex = carry + sil_block_excl_scan(v, sh, &tot);
        if (c <= cmax) hoff[c] = ex;
        carry += tot;
    }
    __syncthreads();
    // the sorted positions carry (position in the tile, weight); hcnt becomes
    // the weighted row count of each label
    __syncthreads();
    for (int t = tid; t <= cmax; t += SIL_T) hcnt[t] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        srow[hoff[lab[i]] + rank[i]] = row[i];  // the row itself: no dependent load in the walk
        slab[hoff[lab[i]] + rank[i]] = lab[i];
        swgt[hoff[lab[i]] + rank[i]] = wgt[i];
        if (lab[i]) atomicAdd(&hcnt[lab[i]], wgt[i]);
    }
    __syncthreads();
    long long a1 = 0, a2 = 0;
    int cur = 0;
    const int p0 = wave * (SIL_SORT_ROWS / 4) + sub;
    // batches of U steps: the batch's LDS reads, then its gathered global
    // loads (all in flight together), then the segment logic and its LDS
    // atomics (an atomic between them would keep the compiler from hoisting
    // the next step's reads: the walk waited on one load at a time)
    constexpr int U = SIL_SUMS_UNROLL;
    static_assert(STEPS % U == 0, "walk batches");
    for (int st0 = 0; st0 < STEPS; st0 += U) {
        int lbv[U];
        int64_t rv[U];
        long long wv[U], v1[U], v2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int pos = p0 + (st0 + u) * RPW;
            lbv[u] = slab[pos];
            rv[u] = srow[pos];
            wv[u] = swgt[pos];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v1[u] = lbv[u] ? q1[rv[u] * DMAX + k] : 0ll;
            v2[u] = (lbv[u] && k == 0) ? q2[rv[u]] : 0ll;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int lb = lbv[u];
            if (lb != cur) {
                if (cur && k < d) {
                    atomicAdd(&acc1[cur * DMAX + k], (unsigned long long)a1);
                    if (k == 0) atomicAdd(&acc2[cur], (unsigned long long)a2);
                }
                cur = lb;
                a1 = 0;
                a2 = 0;
            }
            a1 += wv[u] * v1[u];
            a2 += wv[u] * v2[u];
        }
    }
    if (cur && k < d) {
        atomicAdd(&acc1[cur * DMAX + k], (unsigned long long)a1);
        if (k == 0) atomicAdd(&acc2[cur], (unsigned long long)a2);
    }
    __syncthreads();
    unsigned long long* gs = gsum + (int64_t)l * (cmax + 1) * d;
    for (int t = tid; t < nacc; t += SIL_T) {
        const int c = t / DMAX, kk = t - c * DMAX;
        if (kk < d && c >= 1 && acc1[t]) atomicAdd(&gs[(int64_t)c * d + kk], acc1[t]);
    }
    for (int c = 1 + tid; c <= cmax; c += SIL_T) {
        if (hcnt[c]) atomicAdd(&gcnt[(int64_t)l * (cmax + 1) + c], (unsigned long long)hcnt[c]);
        if (acc2[c]) atomicAdd(&gsum2[(int64_t)l * (cmax + 1) + c], acc2[c]);
    }
}

// Rows labelled apart from their cell's representative (the exception list
// of sil_mult_kernel, l << 32 | row): their fixed-point rows added alone.
template <int DMAX>
__global__ void sil_sums_exc(int64_t m, int d, const int32_t* __restrict__ labels, int cmax,
                             const long long* __restrict__ q1, const long long* __restrict__ q2,
                             const unsigned long long* __restrict__ exc, const int* __restrict__ nexc,
                             unsigned long long* __restrict__ gsum, unsigned long long* __restrict__ gsum2,
                             unsigned long long* __restrict__ gcnt) {
    const int ne = *nexc;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x) {
        const int l = (int)(exc[e] >> 32);
        const int64_t r = (int64_t)(exc[e] & 0xffffffffull);
        const int lab = labels[(int64_t)l * m + r];
        if (lab < 1 || lab > cmax) continue;
        unsigned long long* gs = gsum + ((int64_t)l * (cmax + 1) + lab) * d;
        for (int k = 0; k < d; ++k) atomicAdd(&gs[k], (unsigned long long)q1[r * DMAX + k]);
        atomicAdd(&gsum2[(int64_t)l * (cmax + 1) + lab], (unsigned long long)q2[r]);
        atomicAdd(&gcnt[(int64_t)l * (cmax + 1) + lab], 1ull);
    }
}

// Dimension order of a centroid row in muc: position p holds dimension
// (p % KS) * 4 + p / KS (KS = DMAX / 4), so the KS values a lane feeds to the
// K steps of v_mfma_f64_16x16x4f64 (dims 4s + (lane >> 4)) are contiguous.
template <int DMAX>
__host__ __device__ __forceinline__ int sil_mfma_pos(int k) {
    constexpr int KS = DMAX / 4;
    return (k & 3) * KS + (k >> 2);
}

// K2: per labeling, the present codes (ascending = sort(unique(clusters)))
// and the centroids mu[l][c][0..DMAX) (zero padded; muc: present clusters
// only, in MFMA dimension order) plus |mu_c|^2, from the fixed-point sums.
// With the sums of squares (gsum2, the sorted-segment path) also
// v_c = mean |x - mu_c|^2 = sum_k (S2 / n - mu_k^2).  One block per labeling.
template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_mu(int64_t m, int d, int cmax,
                                                const unsigned* __restrict__ maxabs_bits,
                                                const unsigned long long* __restrict__ gsum,
                                                const unsigned long long* __restrict__ gsum2,
                                                const unsigned long long* __restrict__ gcnt,
                                                int* __restrict__ npres, int* __restrict__ codes,
                                                int* __restrict__ pos, double* __restrict__ mu,
                                                double* __restrict__ muc, double* __restrict__ auxc) {
    __shared__ int sh[SIL_T / 64];
    const int l = blockIdx.x;
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double inv_sc = ldexp(1.0, -scale_exp(maxabs * (double)m));
    const unsigned long long* gs = gsum + (int64_t)l * (cmax + 1) * d;
    const unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
    int* pl = pos + (int64_t)l * (cmax + 1);
    int carry = 0;
    for (int c0 = 0; c0 <= cmax; c0 += SIL_T) {
        const int c = c0 + threadIdx.x;
        const bool present = c >= 1 && c <= cmax && gc[c] != 0ull;
        int tot;
        const int ex = carry + sil_block_excl_scan(present ? 1 : 0, sh, &tot);
        if (c <= cmax) pl[c] = present ? ex : -1;
        if (present) codes[(int64_t)l * cmax + ex] = c;
        carry += tot;
    }
    if (threadIdx.x == 0) npres[l] = carry;
    __syncthreads();
    double* ml = mu + (int64_t)l * (cmax + 1) * DMAX;
    double* mcl = muc + (int64_t)l * cmax * DMAX;
    for (int64_t t = threadIdx.x; t < (int64_t)(cmax + 1) * DMAX; t += SIL_T) {
        const int c = (int)(t / DMAX), k = (int)(t - (int64_t)c * DMAX);
        const unsigned long long n = gc[c];
        const double v = (n && k < d) ? ((double)(long long)gs[(int64_t)c * d + k] * inv_sc) / (double)n : 0.0;
        ml[t] = v;
        const int pc = pl[c];
        if (pc >= 0) mcl[(int64_t)pc * DMAX + sil_mfma_pos<DMAX>(k)] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c <= cmax; c += SIL_T) {
        const int pc = pl[c];
        if (pc < 0) continue;
        double s = 0.0;
        for (int k = 0; k < d; ++k) s = fma(ml[(int64_t)c * DMAX + k], ml[(int64_t)c * DMAX + k], s);
        auxc[((int64_t)l * cmax + pc) * 2] = s;
        if (gsum2) {  // v_c = S2 / n - |mu_c|^2
            const double inv_sc2 = ldexp(1.0, -scale_exp(sil_s2_bound(maxabs, d, m)));
            const double n = (double)gc[c];
            const double v = ((double)(long long)gsum2[(int64_t)l * (cmax + 1) + c] * inv_sc2) / n - s;
            auxc[((int64_t)l * cmax + pc) * 2 + 1] = fmax(v, 0.0);  // clamp the cancellation noise of equal points
        }
    }
}

// K3: fixed-point within-cluster sum of squared distances to the centroid
// (the exact difference form, as colMeans(sweep(x, 2, centroid)^2)).
template <int DMAX, bool LDS>
__global__ __launch_bounds__(SIL_T) void sil_var(const double* __restrict__ x, int64_t m, int d,
                                                 const int32_t* __restrict__ labels, int L, int cmax,
                                                 const unsigned* __restrict__ maxabs_bits,
                                                 const double* __restrict__ mu,
                                                 unsigned long long* __restrict__ gvar) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* mus = (double*)smem;                                              // [cmax+1][DMAX]
    unsigned long long* vacc = (unsigned long long*)(mus + (int64_t)(cmax + 1) * DMAX);  // [cmax+1]
    const int64_t r = (int64_t)blockIdx.x * SIL_T + threadIdx.x;
    const bool in = r < m;
    double xr[DMAX];
    load_row<DMAX>(x, in ? r : 0, d, xr);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double vb = 4.0 * maxabs * maxabs * (double)d * (double)m;
    const double vsc = ldexp(1.0, scale_exp(vb));
    const int l1 = min(L, (int)(blockIdx.y + 1) * SIL_LG);
    for (int l = blockIdx.y * SIL_LG; l < l1; ++l) {
        const double* ml = mu + (int64_t)l * (cmax + 1) * DMAX;
        unsigned long long* gv = gvar + (int64_t)l * (cmax + 1);
        if (LDS) {
            for (int t = threadIdx.x; t < (cmax + 1) * DMAX; t += SIL_T) mus[t] = ml[t];
            for (int t = threadIdx.x; t <= cmax; t += SIL_T) vacc[t] = 0ull;
            __syncthreads();
        }
        if (in) {
            const int lab = labels[(int64_t)l * m + r];
            if (lab >= 1 && lab <= cmax) {
                const double* mc = LDS ? mus + lab * DMAX : ml + (int64_t)lab * DMAX;
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < DMAX; ++k)
                    if (k < d) {
                        const double t = xr[k] - mc[k];
                        s += t * t;
                    }
                const unsigned long long q = (unsigned long long)__double2ll_rn(s * vsc);
                if (LDS) atomicAdd(&vacc[lab], q);
                else atomicAdd(&gv[lab], q);
            }
        }
        if (LDS) {
            __syncthreads();
            for (int t = threadIdx.x; t <= cmax; t += SIL_T)
                if (vacc[t]) atomicAdd(&gv[t], vacc[t]);
            __syncthreads();
        }
    }
}

// K4: v_c = (sum of squared distances) / n_c next to |mu_c|^2 in auxc.
__global__ void sil_vfin(int64_t m, int d, int L, int cmax, const unsigned* __restrict__ maxabs_bits,
                         const unsigned long long* __restrict__ gcnt,
                         const unsigned long long* __restrict__ gvar, const int* __restrict__ pos,
                         double* __restrict__ auxc) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)L * (cmax + 1)) return;
    const int p = pos[t];
    if (p < 0) return;
    const int64_t l = t / (cmax + 1);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double vb = 4.0 * maxabs * maxabs * (double)d * (double)m;
    const double inv_vsc = ldexp(1.0, -scale_exp(vb));
    auxc[(l * cmax + p) * 2 + 1] = ((double)gvar[t] * inv_vsc) / (double)gcnt[t];
}

// K5: widths and their fixed-point sum over non-NaN rows.
//   D^2(i, c) = |x_i|^2 + (|mu_c|^2 + v_c) - 2 x_i.mu_c
// with x.mu on the fp64 matrix core: v_mfma_f64_4x4x4f64 with A = 4
// centroids x 4 dims (LDS) and B = 4 dims x 16 rows (registers, loaded once
// per block), so lane (g, j) receives centroid c0 + g of the group against
// row j of the lane's row tile.  The epilogue is branch-free and
// per value costs one fma, one compare, three selects and one min: each lane
// keeps, per row, min over the other clusters of (|mu|^2 + v - 2 x.mu) and the
// own cluster's value; |x|^2 is added once per row, then clamped at 0 (the
// identity's cancellation noise is ~1e-16 |x|^2, far inside the 1e-5
// tolerance).  D is monotone in the square: one sqrt per row.  The four lane
// groups are merged at the end.  Rows per block: 4 waves x RT tiles x 16.
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int DMAX>
constexpr int sil_rt() {
    return DMAX <= 32 ? 4 : 2;  // row tiles per wave (B fragments: RT x DMAX/4 doubles per lane)
}

__device__ __forceinline__ void sil_row_width(double selfsq, double oth2, bool in, int np, double wsc,
                                              double* out_w, long long& wq, unsigned& wn, int wt = 1) {
    if (!in) return;
    const double selfd = sqrt(selfsq), othd = sqrt(oth2);
    double w;
    if (np > 1) {
        double mx = fmax(othd, selfd);
        if (isnan(othd) || isnan(selfd)) mx = NAN;
        w = (othd - selfd) / mx;
    } else {
        w = 0.0;
    }
    if (out_w) *out_w = w;
    if (!isnan(w)) {
        wq += (long long)wt * __double2ll_rn(w * wsc);
        wn += (unsigned)wt;
    }
}

// LDS stage of sil_width: ch centroids ([ch][DMAX + 2] f64: the 16-byte row
// pad spreads the 16 lanes of a fragment read over distinct banks), [ch] f64
// |mu|^2 + v and [ch] codes; ch = min(sil_chunk, SIL_LG x cmax rounded up to
// 16): a group of SIL_LG labelings with up to ~50 clusters each is staged at
// once, and the stage (<= 73 KB) leaves room for two blocks per CU.
template <int DMAX>
constexpr int sil_chunk() {
    return DMAX <= 16 ? 384 : (DMAX <= 32 ? 256 : 112);
}
template <int DMAX>
constexpr int sil_sp() {
    return DMAX + 2;
}

template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_width(const double* __restrict__ x, int64_t m, int d,
                                                   const int32_t* __restrict__ labels, int L, int cmax,
                                                   const int* __restrict__ npres,
                                                   const int* __restrict__ codes,
                                                   const double* __restrict__ muc,
                                                   const double* __restrict__ auxc,
                                                   unsigned long long* __restrict__ wsum,
                                                   unsigned long long* __restrict__ wcnt,
                                                   double* __restrict__ out_width, int CH,
                                                   const int* __restrict__ rep, const int* __restrict__ mult,
                                                   const int* __restrict__ cnt, int64_t mw, int nbw,
                                                   const int64_t* __restrict__ nrep) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // CH: centroids staged per pass (a multiple of 16)
    constexpr int KS = DMAX / 4;  // K steps of 4 dims
    constexpr int RT = sil_rt<DMAX>();
    constexpr int SP = sil_sp<DMAX>();
    double* smu = (double*)smem;              // [CH][SP], MFMA dimension order
    double* smv = smu + (int64_t)CH * SP;     // [CH] |mu|^2 + v (+inf: padding)
    int* scode = (int*)(smv + CH);            // [CH]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, j = lane & 15;
    // tile position p = r0 + 16 t + j is row p, or (distinct-cell widths)
    // the representative row rep[p] of a cell, weighted by its cnt[p] rows
    // less the mult[l][p] of them labelled apart in labeling l
    const int64_t r0 = (int64_t)blockIdx.x * (4 * RT * 16) + wave * (RT * 16);
    const int64_t npos = rep ? *nrep : m;  // representatives: counted on the device
    if ((int64_t)blockIdx.x * (4 * RT * 16) >= npos) return;  // the partials of idle blocks stay 0
    double xb[RT][KS];
    double xx[RT];
    bool in[RT];
    int64_t rowof[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int64_t pp = r0 + t * 16 + j;
        in[t] = pp < npos;
        const int64_t r = in[t] ? (rep ? (int64_t)rep[pp] : pp) : 0;
        rowof[t] = r;
        double p = 0.0;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + g;
            xb[t][s] = (in[t] && k < d) ? x[r * d + k] : 0.0;
            p = fma(xb[t][s], xb[t][s], p);
        }
        p += __shfl_xor(p, 16, 64);
        p += __shfl_xor(p, 32, 64);
        xx[t] = p;
    }
    const double wsc = ldexp(1.0, scale_exp((double)m));
    const int lg0 = blockIdx.y * SIL_LG, l1 = min(L, lg0 + SIL_LG);
    // x.mu of one staged 4-centroid group against the RT row tiles, folded into
    // the rows' running own / other minima
    auto tile = [&](int c0, const int (&lab)[RT], double (&oth)[RT], double (&self)[RT]) {
        // 4 centroids x 16 rows per v_mfma_f64_4x4x4f64: its 4 blocks are the
        // row tile's 4-row groups against the same 4 centroids.  Lane (g, j)
        // feeds A = dim 4s + g of centroid c0 + (lane & 3), B = dim 4s + g of
        // row j (the 16x16x4 form's B), and receives x_j . mu_{c0 + g}
        // (measured on gfx950: 18 clocks per 4x4x4 against 64 per 16x16x4,
        // 0.89 of its rate per flop, for C padded to 4 instead of 16)
        double a[KS];
        const double* ap = smu + (c0 + (lane & 3)) * SP + g * KS;
#pragma unroll
        for (int s = 0; s < KS; s += 2) {
            const double2 v = *reinterpret_cast<const double2*>(ap + s);
            a[s] = v.x;
            a[s + 1] = v.y;
        }
        const double mv = smv[c0 + g];
        const int code = scode[c0 + g];
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            double acc = 0.0;
#pragma unroll
            for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a[s], xb[t][s], acc, 0, 0, 0);
            const double tv = fma(-2.0, acc, mv);
            const bool own = code == lab[t];
            self[t] = own ? tv : self[t];
            // the own cluster leaves the minimum by a high word of +DBL_MAX
            const double cand = __hiloint2double(own ? 0x7fefffff : __double2hiint(tv), __double2loint(tv));
            oth[t] = __builtin_fmin(oth[t], cand);
        }
    };
    // stage centroids [p0, p0 + nc) of labeling l at LDS position off (whole
    // 4-centroid groups; padding: zero centroid, +inf offset)
    auto stage = [&](int l, int p0, int nc, int off) {
        const int nct = (nc + SIL_CGRP - 1) & ~(SIL_CGRP - 1);
        const double* ml = muc + ((int64_t)l * cmax + p0) * DMAX;
        const double* al = auxc + ((int64_t)l * cmax + p0) * 2;
        for (int t = threadIdx.x; t < nct * DMAX; t += SIL_T) {
            const int c = t / DMAX, p = t - c * DMAX;
            smu[(off + c) * SP + p] = t < nc * DMAX ? ml[t] : 0.0;
        }
        for (int t = threadIdx.x; t < nct; t += SIL_T) {
            smv[off + t] = t < nc ? al[2 * t] + al[2 * t + 1] : INFINITY;
            scode[off + t] = t < nc ? codes[(int64_t)l * cmax + p0 + t] : -1;
        }
    };
    // one labeling's widths from the rows' minima: the four lane groups
    // (each saw every fourth centroid of a tile) merged; lane group g then
    // finishes row tile t = g, so every lane takes one row's square roots and
    // division.  The wave's integer sums go to its own partial (no block
    // barrier): wsum[l][4 block + wave].
    auto finish = [&](int l, int np, double (&oth)[RT], double (&self)[RT]) {
        double ow = 0.0, sw = 0.0;
        bool iw = false;
        int64_t pw = 0;
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            double o = oth[t], sf = self[t];
            o = fmin(o, __shfl_xor(o, 16, 64));
            o = fmin(o, __shfl_xor(o, 32, 64));
            sf = fmin(sf, __shfl_xor(sf, 16, 64));
            sf = fmin(sf, __shfl_xor(sf, 32, 64));
            ow = t == g ? fmax(xx[t] + o, 0.0) : ow;
            sw = t == g ? fmax(xx[t] + sf, 0.0) : sw;
            iw = t == g ? in[t] : iw;
            pw = t == g ? r0 + t * 16 + j : pw;
        }
        const int wt = (rep && iw) ? cnt[pw] - mult[(int64_t)l * mw + pw] : 1;
        long long wq = 0;
        unsigned wn = 0;
        sil_row_width(sw, ow, iw, np, wsc,
                      (out_width && !rep) ? out_width + (int64_t)l * m + r0 + g * 16 + j : nullptr, wq, wn, wt);
        for (int o = 32; o > 0; o >>= 1) {
            wq += __shfl_xor(wq, o, 64);
            wn += __shfl_xor(wn, o, 64);
        }
        if (lane == 0) {
            wsum[(int64_t)l * nbw + 4 * blockIdx.x + wave] = (unsigned long long)wq;
            wcnt[(int64_t)l * nbw + 4 * blockIdx.x + wave] = (unsigned long long)wn;
        }
    };
    int tot = 0;  // staged centroids of the whole group (uniform)
    for (int l = lg0; l < l1; ++l) tot += (npres[l] + SIL_CGRP - 1) & ~(SIL_CGRP - 1);
    if (tot <= CH) {
        // the group's centroids in one stage, one barrier; the labels of all its
        // labelings loaded up front
        int labg[SIL_LG][RT], npg[SIL_LG];
#pragma unroll
        for (int li = 0; li < SIL_LG; ++li) {
            const int l = lg0 + li;
            npg[li] = l < l1 ? npres[l] : 0;
#pragma unroll
            for (int t = 0; t < RT; ++t) labg[li][t] = (l < l1 && in[t]) ? labels[(int64_t)l * m + rowof[t]] : 0;
        }
        int off = 0;
#pragma unroll
        for (int li = 0; li < SIL_LG; ++li) {
            if (lg0 + li < l1) stage(lg0 + li, 0, npg[li], off);
            off += (npg[li] + SIL_CGRP - 1) & ~(SIL_CGRP - 1);
        }
        __syncthreads();
        off = 0;
#pragma unroll
        for (int li = 0; li < SIL_LG; ++li) {
            if (lg0 + li >= l1) break;
            double oth[RT], self[RT];
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                oth[t] = INFINITY;
                self[t] = INFINITY;
            }
            const int nct = (npg[li] + SIL_CGRP - 1) & ~(SIL_CGRP - 1);
            for (int c0 = 0; c0 < nct; c0 += SIL_CGRP) tile(off + c0, labg[li], oth, self);
            off += nct;
            finish(lg0 + li, npg[li], oth, self);
        }
        return;
    }
    // a group larger than the stage: each labeling in chunks of CH centroids
    for (int l = lg0; l < l1; ++l) {
        const int np = npres[l];
        int lab[RT];
        double oth[RT], self[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            lab[t] = in[t] ? labels[(int64_t)l * m + rowof[t]] : 0;
            oth[t] = INFINITY;
            self[t] = INFINITY;
        }
        for (int p0 = 0; p0 < np; p0 += CH) {
            const int nc = min(CH, np - p0);
            __syncthreads();  // the previous chunk's reads are done
            stage(l, p0, nc, 0);
            __syncthreads();
            for (int c0 = 0; c0 < nc; c0 += SIL_CGRP) tile(c0, lab, oth, self);
        }
        finish(l, np, oth, self);
    }
}

// One block per labeling: the cluster count and smallest size from the
// counts, and the mean width from the per-block fixed-point partials.
__global__ __launch_bounds__(256) void sil_final(int64_t m, int L, int cmax, int nbw,
                                                 const unsigned long long* __restrict__ gcnt,
                                                 const unsigned long long* __restrict__ wsum,
                                                 const unsigned long long* __restrict__ wcnt,
                                                 double* __restrict__ out_mean, int32_t* __restrict__ out_nclust,
                                                 int32_t* __restrict__ out_minsize) {
    __shared__ unsigned long long rq[4], rn[4];
    __shared__ int rc[4];
    __shared__ long long rmin[4];
    const int l = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
    int np = 0;
    long long mn = LLONG_MAX;
    for (int c = 1 + threadIdx.x; c <= cmax; c += 256)
        if (gc[c]) {
            ++np;
            mn = min(mn, (long long)gc[c]);
        }
    unsigned long long q = 0, n = 0;
    for (int b = threadIdx.x; b < nbw; b += 256) {
        q += wsum[(int64_t)l * nbw + b];
        n += wcnt[(int64_t)l * nbw + b];
    }
    for (int o = 32; o > 0; o >>= 1) {
        q += __shfl_xor(q, o, 64);
        n += __shfl_xor(n, o, 64);
        np += __shfl_xor(np, o, 64);
        mn = min(mn, __shfl_xor(mn, o, 64));
    }
    if (lane == 0) {
        rq[wv] = q;
        rn[wv] = n;
        rc[wv] = np;
        rmin[wv] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        q = rq[0] + rq[1] + rq[2] + rq[3];
        n = rn[0] + rn[1] + rn[2] + rn[3];
        np = rc[0] + rc[1] + rc[2] + rc[3];
        mn = min(min(rmin[0], rmin[1]), min(rmin[2], rmin[3]));
        const double inv_wsc = ldexp(1.0, -scale_exp((double)m));
        if (out_mean) out_mean[l] = n ? ((double)(long long)q * inv_wsc) / (double)n : NAN;
        if (out_nclust) out_nclust[l] = np;
        if (out_minsize) out_minsize[l] = (int32_t)(mn == LLONG_MAX ? 0 : mn);
    }
}

// rows per sil_width block, and the width partials per labeling (one per
// wave of every block)
template <int DMAX>
constexpr int sil_width_rows() {
    return 4 * sil_rt<DMAX>() * 16;
}
static int sil_width_blocks(int64_t m, int d) {
    const int rb = d <= 16 ? sil_width_rows<16>() : (d <= 32 ? sil_width_rows<32>() : sil_width_rows<64>());
    return 4 * (int)ccg_cdiv(m, rb);
}

// ---------------------------------------------- distinct-cell widths --
// Bootstrap rows repeat cells (R/consensusClust.R:394): copies of a cell are
// the same point, and with the same label they have the same width.  So the
// widths run over one representative row per cell (its first row), weighted
// by the number of the cell's rows that share the representative's label in
// that labeling; rows whose label differs (rare) are exceptions, each
// computed alone (sil_width_exc).  Cluster sums still run over every row.
__global__ void sil_first_kernel(const int32_t* __restrict__ cell, int64_t m, int* __restrict__ first) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < m) atomicMin(&first[cell[r]], (int)r);
}

__global__ void sil_init_kernel(int* __restrict__ first, int64_t ncell, int* __restrict__ zero, int64_t nzero) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ncell || t < nzero;
         t += (int64_t)gridDim.x * blockDim.x) {
        if (t < ncell) first[t] = 0x7fffffff;
        if (t < nzero) zero[t] = 0;
    }
}

__global__ void sil_isrep_kernel(const int32_t* __restrict__ cell, int64_t m, const int* __restrict__ first,
                                 int64_t* __restrict__ flag) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < m) flag[r] = first[cell[r]] == (int)r ? 1 : 0;
}

// rep[pos] = the representative rows in row order (pos = exclusive scan);
// cnt[pos] = the cell's rows; the other rows listed in row order (r - scan[r]
// of them come before r) as (row, its representative, the representative's
// position): sil_mult_kernel reads them per labeling without a dependent
// chain of gathers
__global__ void sil_rep_kernel(const int32_t* __restrict__ cell, int64_t m, const int* __restrict__ first,
                               const int64_t* __restrict__ scan, int* __restrict__ rep, int* __restrict__ cnt,
                               int3* __restrict__ nonrep) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int rp = first[cell[r]];
    const int pp = (int)scan[rp];
    atomicAdd(&cnt[pp], 1);
    if (rp == (int)r) rep[pp] = (int)r;
    else nonrep[r - scan[r]] = make_int3((int)r, rp, pp);
}

// Per labeling (blockIdx.y strides), every non-representative row whose
// label differs from its representative's: dis[l][pos] += 1 (the weight is
// cnt - dis) and the row joins the exception list (l << 32 | row).
__global__ void sil_mult_kernel(int64_t m, int L, const int32_t* __restrict__ labels,
                                const int64_t* __restrict__ scan, const int3* __restrict__ nonrep, int64_t mw,
                                int* __restrict__ dis, unsigned long long* __restrict__ exc, int* __restrict__ nexc) {
    const int64_t nn = m - scan[m];
    for (int l = blockIdx.y; l < L; l += gridDim.y) {
        const int32_t* lab = labels + (int64_t)l * m;
        for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nn; j += (int64_t)gridDim.x * blockDim.x) {
            const int3 e = nonrep[j];
            const int r = e.x, rp = e.y;
            if (lab[r] != lab[rp]) {
                atomicAdd(&dis[(int64_t)l * mw + e.z], 1);
                const int e = atomicAdd(nexc, 1);
                exc[e] = ((unsigned long long)l << 32) | (unsigned long long)r;
            }
        }
    }
}

// One thread per exception row: its width against labeling l's centroids
// (fp64, the same D^2 = |x|^2 + (|mu|^2 + v) - 2 x.mu), added to the
// labeling's first width partial (integer atomics: order-independent).
template <int DMAX>
__global__ void sil_width_exc(const double* __restrict__ x, int64_t m, int d, const int32_t* __restrict__ labels,
                              int cmax, const int* __restrict__ npres, const int* __restrict__ codes,
                              const double* __restrict__ muc, const double* __restrict__ auxc,
                              const unsigned long long* __restrict__ exc, const int* __restrict__ nexc, int nbw,
                              unsigned long long* __restrict__ wsum, unsigned long long* __restrict__ wcnt) {
    const int ne = *nexc;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x) {
    const int l = (int)(exc[e] >> 32);
    const int64_t r = (int64_t)(exc[e] & 0xffffffffull);
    const int lab = labels[(int64_t)l * m + r];
    double xr[DMAX];
    double xx = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
        xr[k] = k < d ? x[r * d + k] : 0.0;
        xx = fma(xr[k], xr[k], xx);
    }
    const int np = npres[l];
    double self = INFINITY, oth = INFINITY;
    for (int p = 0; p < np; ++p) {
        const double* mp = muc + ((int64_t)l * cmax + p) * DMAX;
        double dot = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) dot = fma(xr[k], mp[sil_mfma_pos<DMAX>(k)], dot);
        const double tv = fma(-2.0, dot, auxc[2 * ((int64_t)l * cmax + p)] + auxc[2 * ((int64_t)l * cmax + p) + 1]);
        if (codes[(int64_t)l * cmax + p] == lab) self = tv;
        else oth = fmin(oth, tv);
    }
    long long wq = 0;
    unsigned wn = 0;
    sil_row_width(fmax(xx + self, 0.0), fmax(xx + oth, 0.0), true, np, ldexp(1.0, scale_exp((double)m)), nullptr,
                  wq, wn);
    if (wn) {
        atomicAdd(&wsum[(int64_t)l * nbw], (unsigned long long)wq);  // the first partial of the labeling
        atomicAdd(&wcnt[(int64_t)l * nbw], 1ull);
    }
    }
}

template <int DMAX>
static void sil_launch(const double* x, int64_t m, int d, const int32_t* labels, int L, int cmax,
                       unsigned* maxabs, unsigned long long* gsum, unsigned long long* gsum2, unsigned long long* gcnt,
                       unsigned long long* gvar, unsigned long long* wsum, unsigned long long* wcnt,
                       int* npres, int* codes, int* pos, double* mu, double* muc, double* auxc, long long* q,
                       double* out_width, hipStream_t st, const int* rep = nullptr, const int* mult = nullptr,
                       const int* cnt = nullptr, int64_t mw = 0, const unsigned long long* exc = nullptr,
                       const int* nexc = nullptr, const int64_t* nrep = nullptr) {
    if (q) {
        // sorted segments: S1, S2 and counts in one pass, v_c in sil_mu
        sil_quant<DMAX><<<(unsigned)ccg_cdiv(m * DMAX, 256), 256, 0, st>>>(x, m, d, maxabs, q, q + m * DMAX);
        dim3 grid((unsigned)ccg_cdiv(m, SIL_SORT_ROWS), (unsigned)L);
        const bool reps = rep && !SIL_SUMS_ROWS;
        sil_sums_sorted<DMAX><<<grid, SIL_T, sil_sorted_lds<DMAX>(cmax), st>>>(
            m, d, labels, cmax, q, q + m * DMAX, gsum, gsum2, gcnt, reps ? rep : nullptr, mult, cnt, mw, nrep);
        if (reps)
            sil_sums_exc<DMAX><<<64, 256, 0, st>>>(m, d, labels, cmax, q, q + m * DMAX, exc, nexc, gsum, gsum2, gcnt);
        sil_mu<DMAX><<<L, SIL_T, 0, st>>>(m, d, cmax, maxabs, gsum, gsum2, gcnt, npres, codes, pos, mu, muc, auxc);
    } else {
        dim3 grid((unsigned)ccg_cdiv(m, SIL_T), (unsigned)ccg_cdiv(L, SIL_LG));
        const size_t lds1 = (size_t)(cmax + 1) * d * 8 + (size_t)(cmax + 1) * 4;
        const size_t lds2 = (size_t)(cmax + 1) * DMAX * 8 + (size_t)(cmax + 1) * 8;
        if (lds1 <= SIL_LDS_CAP)
            sil_centroid<DMAX, true><<<grid, SIL_T, lds1, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt);
        else
            sil_centroid<DMAX, false><<<grid, SIL_T, 0, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt);
        sil_mu<DMAX><<<L, SIL_T, 0, st>>>(m, d, cmax, maxabs, gsum, nullptr, gcnt, npres, codes, pos, mu, muc, auxc);
        if (lds2 <= SIL_LDS_CAP)
            sil_var<DMAX, true><<<grid, SIL_T, lds2, st>>>(x, m, d, labels, L, cmax, maxabs, mu, gvar);
        else
            sil_var<DMAX, false><<<grid, SIL_T, 0, st>>>(x, m, d, labels, L, cmax, maxabs, mu, gvar);
        sil_vfin<<<(unsigned)ccg_cdiv((int64_t)L * (cmax + 1), 256), 256, 0, st>>>(m, d, L, cmax, maxabs, gcnt,
                                                                                    gvar, pos, auxc);
    }
    // the width partials are laid out for m rows (nbw blocks per labeling);
    // the representative grid uses its first blocks
    const int64_t nrows = rep ? mw : m;
    dim3 grid2((unsigned)ccg_cdiv(nrows, sil_width_rows<DMAX>()), (unsigned)ccg_cdiv(L, SIL_LG));
    // the stage holds a whole group of SIL_LG labelings when it can
    const int CH = (int)std::min<int64_t>(sil_chunk<DMAX>(), (int64_t)SIL_LG * (((int64_t)cmax + 15) / 16 * 16));
    const size_t lds5 = (size_t)CH * sil_sp<DMAX>() * 8 + (size_t)CH * 8 + (size_t)CH * 4;
    const int nbw = 4 * (int)ccg_cdiv(m, sil_width_rows<DMAX>());
    if (rep) {
        // partials of blocks past the representative grid stay 0 (zeroed with the buffer)
        sil_width<DMAX><<<grid2, SIL_T, lds5, st>>>(x, m, d, labels, L, cmax, npres, codes, muc, auxc, wsum, wcnt,
                                                nullptr, CH, rep, mult, cnt, mw, nbw, nrep);
        sil_width_exc<DMAX><<<64, 256, 0, st>>>(
            x, m, d, labels, cmax, npres, codes, muc, auxc, exc, nexc, nbw, wsum, wcnt);
    } else {
        sil_width<DMAX><<<grid2, SIL_T, lds5, st>>>(x, m, d, labels, L, cmax, npres, codes, muc, auxc, wsum, wcnt,
                                                out_width, CH, nullptr, nullptr, nullptr, 0, nbw, nullptr);
    }
}

extern "C" int ccg_silhouette_dev(ccg_ctx* ctx, const double* x, int64_t m, int d,
                                  const int32_t* labels, int L, int cmax, double* out_mean,
                                  int32_t* out_nclust, int32_t* out_minsize, double* out_width,
                                  void* stream) {
    CCG_REQUIRE(ctx && x && labels, "ccg_silhouette_dev: NULL argument");
    CCG_REQUIRE(m >= 1 && m < (1LL << 31) && d >= 1 && d <= 64 && L >= 1,
                "ccg_silhouette_dev: bad sizes m=%lld d=%d L=%d", (long long)m, d, L);
    CCG_REQUIRE(cmax >= 1 && cmax <= (1 << 24), "ccg_silhouette_dev: cmax=%d must be in [1, 2^24]", cmax);
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int64_t nacc = (int64_t)(cmax + 1) * d;
    const int nbw = sil_width_blocks(m, d);
    const int64_t words = 2 * (int64_t)L * nacc + 2 * (int64_t)L * (cmax + 1) + 2 * (int64_t)L * nbw + 8;
    unsigned long long* buf = (unsigned long long*)ccg_ws(ctx, WS_SIL_A, sizeof(unsigned long long) * words);
    if (!buf) return CCG_ENOMEM;
    unsigned long long* gsum = buf;
    unsigned long long* gsum2 = gsum + (int64_t)L * nacc;
    unsigned long long* gcnt = gsum2 + (int64_t)L * nacc;
    unsigned long long* gvar = gcnt + (int64_t)L * (cmax + 1);
    unsigned long long* wsum = gvar + (int64_t)L * (cmax + 1);
    unsigned long long* wcnt = wsum + (int64_t)L * nbw;
    unsigned* maxabs = (unsigned*)(wcnt + (int64_t)L * nbw);
    const int dmax = d <= 16 ? 16 : (d <= 32 ? 32 : 64);
    const size_t mu_words = (size_t)L * (cmax + 1) * dmax + (size_t)L * cmax * dmax + 2 * (size_t)L * cmax;
    const size_t tab_ints = (size_t)L * cmax + (size_t)L * (cmax + 1) + L + 8;
    double* mu = (double*)ccg_ws(ctx, WS_SIL_B, sizeof(double) * mu_words + sizeof(int) * tab_ints);
    if (!mu) return CCG_ENOMEM;
    double* muc = mu + (size_t)L * (cmax + 1) * dmax;
    double* auxc = muc + (size_t)L * cmax * dmax;
    int* npres = (int*)(auxc + 2 * (size_t)L * cmax);
    int* codes = npres + L;
    int* pos = codes + (size_t)L * cmax;
    const size_t lds_sorted = dmax == 16 ? sil_sorted_lds<16>(cmax)
                                         : (dmax == 32 ? sil_sorted_lds<32>(cmax) : sil_sorted_lds<64>(cmax));
    long long* q = nullptr;  // fixed-point rows of the sorted-segment path (cmax small enough for its LDS)
    if (lds_sorted <= SIL_LDS_CAP) {
        q = (long long*)ccg_ws(ctx, WS_SIL_Q, 2 * sizeof(long long) * (size_t)m * dmax);
        if (!q) return CCG_ENOMEM;
    }
    const int t_all = ccg_timer_start(ctx, CCG_KT_SILHOUETTE, st);
    CCG_HIP(hipMemsetAsync(buf, 0, sizeof(unsigned long long) * words, st));
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 4096), SIL_MAXABS_GRID), 256, 0, st>>>(x, m * d, maxabs);
    if (d <= 16)
        sil_launch<16>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        out_width, st);
    else if (d <= 32)
        sil_launch<32>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        out_width, st);
    else
        sil_launch<64>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        out_width, st);
    sil_final<<<L, 256, 0, st>>>(m, L, cmax, nbw, gcnt, wsum, wcnt, out_mean,
                                                       out_nclust, out_minsize);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_silhouette_cells_dev(ccg_ctx* ctx, const double* x, int64_t m, int d, const int32_t* labels,
                                        int L, int cmax, const int32_t* cell, int64_t ncell, double* out_mean,
                                        int32_t* out_nclust, int32_t* out_minsize, void* stream) {
    CCG_REQUIRE(ctx && x && labels && cell, "ccg_silhouette_cells_dev: NULL argument");
    CCG_REQUIRE(m >= 1 && m < (1LL << 31) && d >= 1 && d <= 64 && L >= 1 && (int64_t)L * m < (1LL << 31),
                "ccg_silhouette_cells_dev: bad sizes m=%lld d=%d L=%d", (long long)m, d, L);
    CCG_REQUIRE(cmax >= 1 && cmax <= (1 << 24), "ccg_silhouette_cells_dev: cmax=%d must be in [1, 2^24]", cmax);
    CCG_REQUIRE(ncell >= 1 && ncell < (1LL << 31), "ccg_silhouette_cells_dev: bad ncell");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int64_t nacc = (int64_t)(cmax + 1) * d;
    const int nbw = sil_width_blocks(m, d);
    const int64_t words = 2 * (int64_t)L * nacc + 2 * (int64_t)L * (cmax + 1) + 2 * (int64_t)L * nbw + 8;
    unsigned long long* buf = (unsigned long long*)ccg_ws(ctx, WS_SIL_A, sizeof(unsigned long long) * words);
    if (!buf) return CCG_ENOMEM;
    unsigned long long* gsum = buf;
    unsigned long long* gsum2 = gsum + (int64_t)L * nacc;
    unsigned long long* gcnt = gsum2 + (int64_t)L * nacc;
    unsigned long long* gvar = gcnt + (int64_t)L * (cmax + 1);
    unsigned long long* wsum = gvar + (int64_t)L * (cmax + 1);
    unsigned long long* wcnt = wsum + (int64_t)L * nbw;
    unsigned* maxabs = (unsigned*)(wcnt + (int64_t)L * nbw);
    const int dmax = d <= 16 ? 16 : (d <= 32 ? 32 : 64);
    const size_t mu_words = (size_t)L * (cmax + 1) * dmax + (size_t)L * cmax * dmax + 2 * (size_t)L * cmax;
    const size_t tab_ints = (size_t)L * cmax + (size_t)L * (cmax + 1) + L + 8;
    double* mu = (double*)ccg_ws(ctx, WS_SIL_B, sizeof(double) * mu_words + sizeof(int) * tab_ints);
    if (!mu) return CCG_ENOMEM;
    double* muc = mu + (size_t)L * (cmax + 1) * dmax;
    double* auxc = muc + (size_t)L * cmax * dmax;
    int* npres = (int*)(auxc + 2 * (size_t)L * cmax);
    int* codes = npres + L;
    int* pos = codes + (size_t)L * cmax;
    const size_t lds_sorted = dmax == 16 ? sil_sorted_lds<16>(cmax)
                                         : (dmax == 32 ? sil_sorted_lds<32>(cmax) : sil_sorted_lds<64>(cmax));
    long long* q = nullptr;
    if (lds_sorted <= SIL_LDS_CAP) {
        q = (long long*)ccg_ws(ctx, WS_SIL_Q, 2 * sizeof(long long) * (size_t)m * dmax);
        if (!q) return CCG_ENOMEM;
    }
    // distinct-cell tables: first row per cell, representative list, rows per
    // cell, the other rows, per-labeling disagreements, exceptions
    char* tb = (char*)ccg_ws(ctx, WS_SIL_C, sizeof(int) * (size_t)ncell + sizeof(int64_t) * (size_t)(m + 1) +
                                                5 * sizeof(int) * (size_t)m + sizeof(int) * (size_t)L * m +
                                                sizeof(unsigned long long) * (size_t)L * m + 512);
    if (!tb) return CCG_ENOMEM;
    int* first = (int*)tb;
    int64_t* scan = (int64_t*)(tb + ccg_cdiv(sizeof(int) * ncell, 16) * 16);
    int* rep = (int*)(scan + m + 1);
    int3* nonrep = (int3*)(rep + m);    // [m] (row, representative, its position)
    int* nexc = (int*)(nonrep + m);     // [0] exception count; then cnt and the disagreements (zeroed together)
    int* cnt = nexc + 4;                // [m] (first mw used)
    int* mult = cnt + m;                // [L][m] (first mw columns used)
    // the u64 exceptions start on an 8-byte boundary whatever the parity of m
    unsigned long long* exc =
        (unsigned long long*)(tb + ccg_cdiv((int64_t)((char*)(mult + (int64_t)L * m) - tb), 16) * 16);
    const int t_all = ccg_timer_start(ctx, CCG_KT_SILHOUETTE, st);
    CCG_HIP(hipMemsetAsync(buf, 0, sizeof(unsigned long long) * words, st));
    const unsigned gm = (unsigned)ccg_cdiv(m, 256);
    sil_init_kernel<<<(unsigned)std::min<int64_t>(ccg_cdiv(std::max(ncell, (int64_t)(L + 1) * m + 4), 256), 4096), 256,
                      0, st>>>(first, ncell, nexc, (int64_t)(L + 1) * m + 4);
    sil_first_kernel<<<gm, 256, 0, st>>>(cell, m, first);
    sil_isrep_kernel<<<gm, 256, 0, st>>>(cell, m, first, scan);
    int rc = ccg_scan_i64(ctx, scan, scan, m, st);
    if (rc) return rc;
    sil_rep_kernel<<<gm, 256, 0, st>>>(cell, m, first, scan, rep, cnt, nonrep);
    // mw = the number of representatives (the distinct cells): device-side
    // only, so the width grid covers m positions and the weights' stride is m
    dim3 gx((unsigned)std::min<int64_t>(ccg_cdiv(m, 256), 32), (unsigned)std::min(L, 65535));
    sil_mult_kernel<<<gx, 256, 0, st>>>(m, L, labels, scan, nonrep, m, mult, exc, nexc);
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 4096), SIL_MAXABS_GRID), 256, 0, st>>>(x, m * d, maxabs);
#define SIL_CELLS(DM_)                                                                                              \
    sil_launch<DM_>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, \
                    auxc, q, nullptr, st, rep, mult, cnt, m, exc, nexc, scan + m)
    if (d <= 16) SIL_CELLS(16);
    else if (d <= 32) SIL_CELLS(32);
    else SIL_CELLS(64);
#undef SIL_CELLS
    sil_final<<<L, 256, 0, st>>>(m, L, cmax, nbw, gcnt, wsum, wcnt, out_mean, out_nclust, out_minsize);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_silhouette(ccg_ctx* ctx, const double* x, int64_t m, int d, const int32_t* labels,
                              int L, int cmax, double* out_mean, int32_t* out_nclust,
                              int32_t* out_minsize, double* out_width) {
    CCG_REQUIRE(ctx && x && labels && out_mean, "ccg_silhouette: NULL argument");
    CCG_REQUIRE(m >= 1 && d >= 1 && L >= 1, "ccg_silhouette: bad sizes");
    for (int64_t t = 0; t < (int64_t)L * m; ++t)
        if (labels[t] < 1 || labels[t] > cmax) {
            ccg_set_error("ccg_silhouette: label %d at %lld outside [1, %d]", labels[t], (long long)t, cmax);
            return CCG_ERANGE;
        }
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* dx = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * m * d);
    int32_t* dl = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * m * L);
    double* dmean = (double*)ccg_ws(ctx, WS_HOST_C, sizeof(double) * L + 2 * sizeof(int32_t) * L + 64);
    double* dw = out_width ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * m * L) : nullptr;
    if (!dx || !dl || !dmean || (out_width && !dw)) return CCG_ENOMEM;
    int32_t* dnc = (int32_t*)(dmean + L);
    int32_t* dms = dnc + L;
    CCG_HIP(hipMemcpyAsync(dx, x, sizeof(double) * m * d, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dl, labels, sizeof(int32_t) * m * L, hipMemcpyHostToDevice, st));
    int rc = ccg_silhouette_dev(ctx, dx, m, d, dl, L, cmax, dmean, dnc, dms, dw, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(out_mean, dmean, sizeof(double) * L, hipMemcpyDeviceToHost, st));
    if (out_nclust) CCG_HIP(hipMemcpyAsync(out_nclust, dnc, sizeof(int32_t) * L, hipMemcpyDeviceToHost, st));
    if (out_minsize) CCG_HIP(hipMemcpyAsync(out_minsize, dms, sizeof(int32_t) * L, hipMemcpyDeviceToHost, st));
    if (out_width) CCG_HIP(hipMemcpyAsync(out_width, dw, sizeof(double) * m * L, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}

extern "C" int ccg_silhouette_cells(ccg_ctx* ctx, const double* x, int64_t m, int d, const int32_t* labels, int L,
                                    int cmax, const int32_t* cell, int64_t ncell, double* out_mean,
                                    int32_t* out_nclust, int32_t* out_minsize) {
    CCG_REQUIRE(ctx && x && labels && cell && out_mean, "ccg_silhouette_cells: NULL argument");
    CCG_REQUIRE(m >= 1 && d >= 1 && L >= 1 && ncell >= 1, "ccg_silhouette_cells: bad sizes");
    for (int64_t t = 0; t < (int64_t)L * m; ++t)
        if (labels[t] < 1 || labels[t] > cmax) {
            ccg_set_error("ccg_silhouette_cells: label %d at %lld outside [1, %d]", labels[t], (long long)t, cmax);
            return CCG_ERANGE;
        }
    for (int64_t r = 0; r < m; ++r)
        CCG_REQUIRE(cell[r] >= 0 && cell[r] < ncell, "ccg_silhouette_cells: cell[%lld] out of range", (long long)r);
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* dx = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * m * d);
    int32_t* dl = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * m * L);
    double* dmean = (double*)ccg_ws(ctx, WS_HOST_C, sizeof(double) * L + 2 * sizeof(int32_t) * L + 64);
    int32_t* dc = (int32_t*)ccg_ws(ctx, WS_HOST_D, sizeof(int32_t) * m);
    if (!dx || !dl || !dmean || !dc) return CCG_ENOMEM;
    int32_t* dnc = (int32_t*)(dmean + L);
    int32_t* dms = dnc + L;
    CCG_HIP(hipMemcpyAsync(dx, x, sizeof(double) * m * d, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dl, labels, sizeof(int32_t) * m * L, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dc, cell, sizeof(int32_t) * m, hipMemcpyHostToDevice, st));
    int rc = ccg_silhouette_cells_dev(ctx, dx, m, d, dl, L, cmax, dc, ncell, dmean, dnc, dms, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(out_mean, dmean, sizeof(double) * L, hipMemcpyDeviceToHost, st));
    if (out_nclust) CCG_HIP(hipMemcpyAsync(out_nclust, dnc, sizeof(int32_t) * L, hipMemcpyDeviceToHost, st));
    if (out_minsize) CCG_HIP(hipMemcpyAsync(out_minsize, dms, sizeof(int32_t) * L, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}
