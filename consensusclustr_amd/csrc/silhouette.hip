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
// fixed point with integer atomics, so the result is bitwise reproducible
// regardless of scheduling; the scales are chosen on the device from max|x|
// so no partial sum can overflow.  The cluster sums take int64 rows at scale
// 2^e with m max|x| 2^e <= 2^61;
// the squared norms and the widths' sum 64-bit values.  (An int32 row scale,
// 2^-30 max|x|, was tried in round 5: v_c = S2/n - |mu_c|^2 then mixes the
// unquantised S2 with quantised centroids, and a singleton cluster's v_c came
// out ~1e-8 instead of 0 -- its rows' own distance ~1e-4, widths off by
// ~1e-4, means by up to 1.6e-4 relative on the pipeline tests.)
// The widths' squared distances are |x|^2 + |mu|^2 + v - 2 x.mu with x.mu on
// the fp64 matrix core (a fixed-order MFMA chain, so also reproducible).
// Grid: (row tiles) x (groups of SIL_LG labelings); x rows are held in
// registers and reused across the group.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "ccg_internal.h"

#define SIL_T 256
// centroid granularity of the width tiles (v_mfma_f64_4x4x4f64: C padded to
// a multiple of 4; the 16x16x4 tiles of round 3 padded to 16, 1.37x at C =
// 2..40: silhouette 0.454 -> 0.435 ms per bootstrap at cfg3)
#define SIL_CGRP 4
#ifndef SIL_LG
#define SIL_LG 5
#endif

__host__ __device__ __forceinline__ int scale_exp(double bound) {
    // largest e with bound * 2^e <= 2^61
    if (!(bound > 0.0)) return 52;
    int e = 61 - (ilogb(bound) + 1);
    return e > 52 ? 52 : e;
}

// A batch of segments (ccg_silhouette_segments_dev): segment q holds rows
// [off[q], off[q+1]) of the concatenation and labels lab[q] ([L][m_q]); its
// tiles of the sums / width grids start at ts[q] / tw[q]; the means,
// cluster counts and smallest sizes of its L labelings go to mean[q],
// ncl[q], mns[q] (each may be NULL).  Labeling l of segment q is the
// "virtual labeling" q L + l of every per-labeling table.  nseg = 0: one
// matrix (the single-call entry points).
struct SilSegs {
    int nseg;
    const int64_t* off;
    const int32_t* const* lab;
    const int* ts;
    const int* tw;
    double* const* mean;
    int32_t* const* ncl;
    int32_t* const* mns;
};
// the segment of tile b: the largest q with pre[q] <= b
__device__ __forceinline__ int sil_seg_tile(const int* __restrict__ pre, int nseg, int b) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// the segment of row r
__device__ __forceinline__ int sil_seg_row(const int64_t* __restrict__ off, int nseg, int64_t r) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// label of row r in labeling l (segments: of r's segment q)
__device__ __forceinline__ int sil_label(const int32_t* __restrict__ labels, int64_t m, const SilSegs& sg, int q,
                                         int l, int64_t r) {
    if (sg.nseg) {
        const int64_t o = sg.off[q];
        return sg.lab[q][(int64_t)l * (sg.off[q + 1] - o) + (r - o)];
    }
    return labels[(int64_t)l * m + r];
}

// one atomic per block on one word: a small grid (a 1024-block grid spent
// ~10 us serialising its atomics at the L2) of 1024-thread blocks (16 waves
// per CU in flight: 256-thread blocks read at ~2.3 TB/s)
#define SIL_MAXABS_GRID 256
#define SIL_MAXABS_T 1024
__global__ __launch_bounds__(SIL_MAXABS_T) void sil_maxabs(const double* __restrict__ x, int64_t tot,
                                                           unsigned* __restrict__ bits) {
    __shared__ unsigned red[SIL_MAXABS_T / 64];
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
    if (threadIdx.x == 0) {
        unsigned b = red[0];
#pragma unroll
        for (int w = 1; w < SIL_MAXABS_T / 64; ++w) b = max(b, red[w]);
        atomicMax(bits, b);  // one atomic per block
    }
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
// (zero past d; sc = 2^scale_exp(m max|x|)) and q2 = round(|x|^2 * sc2) [m]
// (v_c needs only the cluster's total sum of squares: v_c = S2 / n - |mu_c|^2).
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
    const long long qv = __double2ll_rn(v * sc);
    q1[t] = qv;
    // |x_q|^2 of the QUANTISED row (exact in fp64: qv is an integer-valued
    // double), so that v_c = S2/n - |mu_c|^2 is the spread of the same points
    // the centroid averages: copies of one point give v_c = 0 up to fp64
    // rounding (with |x|^2 of the raw row, a singleton's v_c was the
    // quantisation residue 2 |x| 2^-e).  Its DMAX threads are DMAX-aligned
    // lanes of one wave (fixed xor tree: deterministic).
    const double vq = (double)qv / sc;
    double s2 = vq * vq;
#pragma unroll
    for (int o = DMAX / 2; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    if (k == 0) q2[r] = __double2ll_rn(s2 * ldexp(1.0, scale_exp(sil_s2_bound(maxabs, d, m))));
}

// K1 (round 5): cluster sums S1 = sum x, S2 = sum |x|^2 and counts, one
// block of 1024 threads per (tile of SIL_SP positions, group of G <=
// SIL_SGMAX labelings).  A position is a row, or a representative row
// weighted by its cell's copies.  The block first writes its positions'
// rows, and their labels and weights in each labeling of the group, to LDS
// (coalesced), then walks them: lanes along the dimensions, 64 / DMAX
// positions per wave instruction, the fixed-point row read from the L2 ONCE
// for the group and one int64 LDS atomic per (position, dimension,
// labeling) into the block's [G][cmax+1][d] sums; a barrier; one global
// atomic per present (labeling, cluster, dimension).  The rows are re-read
// per group (60 / G x 59k x 256 B at cfg3), and the grid is XCD-aware: the
// blocks of a tile, over all groups, run on one XCD (block b on XCD b mod
// 8), whose 4 MB L2 then holds its eighth of the rows (23 MB of int64 rows
// at cfg3 would not fit one L2).  Measured at cfg3: one labeling per block
// 137 us per bootstrap; an earlier round-5 form that staged a tile's rows in
// LDS once for many labelings paid two barriers per labeling, each waiting
// on the previous flush's global atomics (170 us).  Integer sums: any order
// gives the same bits.  LDS (dynamic): rows [SIL_SP], labels and weights
// [G][SIL_SP] int, acc [G]{[cmax+1][d] sums, [cmax+1] S2, [cmax+1] counts}
// int64.
#define SIL_SB 1024   // threads of the sums kernel
#define SIL_SP 1024   // positions per sums block
#ifndef SIL_SGMAX
#define SIL_SGMAX 4   // labelings per sums block
#endif
#define SIL_LDS_CU 163840
#ifndef SIL_LDS_SUMS
#define SIL_LDS_SUMS 81920  // two blocks per CU
#endif
__host__ __device__ inline size_t sil_tile_lds(int d, int cmax, int G) {
    return (size_t)SIL_SP * 4 + (size_t)G * SIL_SP * 8 + (size_t)G * (cmax + 1) * (d + 2) * 8;
}
// labelings per sums block: the most whose LDS keeps two blocks per CU (one
// if even G = 1 needs more), 0 if G = 1 does not fit the CU
static inline int sil_sums_G(int d, int cmax) {
    for (int G = SIL_SGMAX; G >= 1; G >>= 1)
        if (sil_tile_lds(d, cmax, G) <= SIL_LDS_SUMS) return G;
    return sil_tile_lds(d, cmax, 1) <= SIL_LDS_CU ? 1 : 0;
}

// Distinct-cell form (rep != nullptr): position p is the representative
// row rep[p] of a cell, weighted by the cnt[p] rows of the cell less the
// mult[l][p] of them labelled apart in labeling l (those rows are added by
// sil_sums_exc); the integer sums are those of the rows.  Grid: 8 tpx
// cdiv(L, G) blocks; block b takes group (b / 8) / tpx and tile ((b / 8)
// mod tpx) 8 + b mod 8 of the ntile tiles.
template <int DMAX, bool SEG>
__global__ __launch_bounds__(SIL_SB) void sil_sums_blk(int64_t m, int d, int ntile, int tpx, int G,
                                                       const int32_t* __restrict__ labels, int L, int cmax,
                                                       const long long* __restrict__ q1,
                                                       const long long* __restrict__ q2,
                                                       unsigned long long* __restrict__ gsum,
                                                       unsigned long long* __restrict__ gsum2,
                                                       unsigned long long* __restrict__ gcnt,
                                                       const int* __restrict__ rep, const int* __restrict__ mult,
                                                       const int* __restrict__ cnt, int64_t mw,
                                                       const int64_t* __restrict__ nrep,
                                                       const int64_t* __restrict__ scan, SilSegs sgs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int* srow = (int*)smem;                                      // [SIL_SP]
    int* slab = srow + SIL_SP;                                   // [G][SIL_SP]
    int* swgt = slab + G * SIL_SP;                               // [G][SIL_SP]
    unsigned long long* acc = (unsigned long long*)(swgt + G * SIL_SP);  // [G][(cmax+1)(d+2)]
    const int na = (cmax + 1) * (d + 2);                         // per labeling: sums, then S2, then counts
    constexpr int NW = SIL_SB / 64;
    constexpr int RPW = 64 / DMAX;      // positions per wave instruction
    constexpr int PPW = SIL_SP / NW;    // positions per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k = lane % DMAX, sub = lane / DMAX;
    const int loc = blockIdx.x >> 3;
    const int grp = loc / tpx;
    const int tile = (loc - grp * tpx) * 8 + (blockIdx.x & 7);
    const int l0 = grp * G;
    if (l0 >= L || tile >= ntile) return;
    const int ng = min(G, L - l0);
    int64_t rb, npos;  // the tile's first position, the end of its positions
    int q = 0;
    if constexpr (SEG) {  // a tile of segment q: its representatives are positions [scan[off_q], scan[off_q+1])
        q = sil_seg_tile(sgs.ts, sgs.nseg, tile);
        rb = scan[sgs.off[q]] + (int64_t)(tile - sgs.ts[q]) * SIL_SP;
        npos = scan[sgs.off[q + 1]];
    } else {
        rb = (int64_t)tile * SIL_SP;
        npos = rep ? *nrep : m;  // positions: rows, or the representatives (counted on the device)
    }
    if (rb >= npos) return;
    for (int t = tid; t < ng * na; t += SIL_SB) acc[t] = 0ull;
    // label 0: positions past npos, codes outside [1, cmax] and weight 0
    for (int p = tid; p < SIL_SP; p += SIL_SB) {
        const int64_t ps = rb + p;
        const bool in = ps < npos;
        const int row = in ? (rep ? rep[ps] : (int)ps) : 0;
        srow[p] = row;
        const int c0 = (in && rep) ? cnt[ps] : 1;
        for (int g = 0; g < G; ++g) {
            int lb = 0, wg = 0;
            if (in && g < ng) {
                const int l = l0 + g;
                if constexpr (SEG) lb = sil_label(labels, m, sgs, q, l, row);
                else lb = labels[(int64_t)l * m + row];
                wg = rep ? c0 - mult[(int64_t)l * mw + ps] : 1;
            }
            const bool ok = lb >= 1 && lb <= cmax && wg > 0;
            slab[g * SIL_SP + p] = ok ? lb : 0;
            swgt[g * SIL_SP + p] = ok ? wg : 0;
        }
    }
    __syncthreads();
    // SU positions per lane in flight: rows from LDS, then the row loads
    // (unconditional: q1 is zero past d, row 0 stands in for an empty
    // position), then per labeling of the group the atomics
    constexpr int SU = 8;
    static_assert((PPW / RPW) % SU == 0, "walk unroll");
    for (int i0 = 0; i0 < PPW / RPW; i0 += SU) {
        int rr[SU];
        long long v[SU], v2[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) rr[u] = srow[wave * PPW + (i0 + u) * RPW + sub];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            v[u] = q1[(int64_t)rr[u] * DMAX + k];
            v2[u] = q2[rr[u]];
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) asm volatile("" : "+v"(v[u]), "+v"(v2[u]));  // (keeps every load ahead of the atomics)
        for (int g = 0; g < ng; ++g) {
            unsigned long long* ag = acc + g * na;
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                const int pl = g * SIL_SP + wave * PPW + (i0 + u) * RPW + sub;
                const int lb = slab[pl];
                if (lb) {
                    const long long w = swgt[pl];
                    if (k < d) atomicAdd(&ag[lb * d + k], (unsigned long long)(w * v[u]));
                    if (k == 0) {
                        atomicAdd(&ag[(cmax + 1) * d + lb], (unsigned long long)(w * v2[u]));
                        atomicAdd(&ag[(cmax + 1) * (d + 1) + lb], (unsigned long long)w);
                    }
                }
            }
        }
    }
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
        const int lv = q * L + l0 + g;  // (the virtual labeling)
        const unsigned long long* ag = acc + g * na;
        unsigned long long* gs = gsum + (int64_t)lv * (cmax + 1) * d;
        for (int t = tid; t < (cmax + 1) * d; t += SIL_SB) {
            const unsigned long long v = ag[t];
            if (v) atomicAdd(&gs[t], v);
        }
        for (int c = tid; c <= cmax; c += SIL_SB) {
            const unsigned long long n = ag[(cmax + 1) * (d + 1) + c];
            if (n) {
                atomicAdd(&gcnt[(int64_t)lv * (cmax + 1) + c], n);
                atomicAdd(&gsum2[(int64_t)lv * (cmax + 1) + c], ag[(cmax + 1) * d + c]);
            }
        }
    }
}

// Rows labelled apart from their cell's representative (the exception list
// of sil_mult_kernel, l << 32 | row): their fixed-point rows added alone.
template <int DMAX>
__global__ void sil_sums_exc(int64_t m, int d, const int32_t* __restrict__ labels, int L, int cmax,
                             const long long* __restrict__ q1, const long long* __restrict__ q2,
                             const unsigned long long* __restrict__ exc, const int* __restrict__ nexc,
                             unsigned long long* __restrict__ gsum, unsigned long long* __restrict__ gsum2,
                             unsigned long long* __restrict__ gcnt, SilSegs sgs) {
    const int ne = *nexc;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x) {
        const int l = (int)(exc[e] >> 32);
        const int64_t r = (int64_t)(exc[e] & 0xffffffffull);
        const int q = sgs.nseg ? sil_seg_row(sgs.off, sgs.nseg, r) : 0;
        const int lab = sil_label(labels, m, sgs, q, l, r);
        if (lab < 1 || lab > cmax) continue;
        const int64_t lv = (int64_t)q * L + l;
        unsigned long long* gs = gsum + (lv * (cmax + 1) + lab) * d;
        for (int k = 0; k < d; ++k) atomicAdd(&gs[k], (unsigned long long)q1[r * DMAX + k]);
        atomicAdd(&gsum2[lv * (cmax + 1) + lab], (unsigned long long)q2[r]);
        atomicAdd(&gcnt[lv * (cmax + 1) + lab], 1ull);
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
    // the sums' scale (the tiled sums' rows and sil_centroid's alike)
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
            // equal points (a singleton, a cell's copies) have v_c = 0; the
            // formula leaves the rounding of the rows' |x|^2 (<= 2^-s2 / 2
            // each) and of |mu|^2: below that floor v_c is taken as 0, so the
            // result does not depend on the batch's scale (m)
            const double floor_v = inv_sc2 + 0x1p-50 * s;
            auxc[((int64_t)l * cmax + pc) * 2 + 1] = v > floor_v ? v : 0.0;
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

// K5' (round 5, d <= 32): the nearest other cluster screened on the fp16
// matrix core, the two distances a width needs taken exactly in fp64.
//
// Screen: rows and centroids scaled by 2^e (max|x| 2^e < 2^12) and split
// into fp16 hi + lo (flushed below 2^-14); x.mu ~ hi.hi + hi.lo + lo.hi on
// v_mfma_f32_32x32x16_f16 with A = 32 centroids (LDS) and B = 32
// representatives (registers, built once per block), so lane (h, j) gets 16
// centroids of the tile against representative j.  Per value
// a = (|mu|^2 + v) 2^2e - 2 x.mu (= D^2 - |x|^2, scaled) with the value's
// register and tile packed into its 7 low mantissa bits, the own cluster
// masked, and the two smallest kept (two med3): 6 VALU per value.  The
// error of a is taken as
//   E = 2^-14 (|x'| + max|mu'|)^2 + 2^-11 sqrt(d) (|x'| + max|mu'|)
//       + 2^-14 max A' + 8
// (the kNN screen's certification budget, 1024 fp32 ulps of s^2, for the
// split residuals and the fp32 accumulation of 3 DMAX products; the flushed
// parts below 2^-14; the fp32 A' and the 7-bit packing), so
// when the second smallest exceeds the smallest by more than 2E the
// smallest is the true nearest other cluster; otherwise (rare) every
// centroid is taken exactly.  Exact: D^2 = sum_k (x_k - mu_k)^2 + v_c in
// fp64 (fixed order: reproducible), lane h = 0 for the own cluster, h = 1
// for the nearest other one.  The matrix work per (representative,
// centroid) is 3 x 16 DMAX/16 fp16 MACs against round 4's DMAX fp64 MACs
// on the fp64 matrix core (78.6 vs 2500 dense TFLOP/s).
//
// Each labeling's LDS image (fp16 fragments, fp64 centroids, v, A', the
// screen's bounds, code -> ordinal) is built once by sil_w16_prep; the
// width kernel double-buffers the images and copies the next one with
// global_load_lds while it screens the current one (one barrier per
// labeling, no dependent loads in the stage).
// Grid: 128 representatives per block (4 waves x 32) x groups of SIL_WLG
// labelings.
typedef _Float16 sil_h8 __attribute__((ext_vector_type(8)));
typedef float sil_f16x __attribute__((ext_vector_type(16)));
#define SIL_WT 256      // threads of sil_width16 (4 waves x 32 representatives)
#define SIL_WLG 15      // labelings per sil_width16 block
#define SIL_WCMAX 256   // 8 tiles of 32: the tile fits the packed minimum's 3 bits
#define SIL_BIG 1.0e38f
#define SIL_NCAND 4  // exact candidates listed per lane for a near tie
#define SIL_W16_LDS 81920  // two image buffers (40 KB each) per block: cmax <= 96 at d <= 32

// image of a labeling with cpl = 32 x tiles centroid slots: fragments
// [cpl][64] f16 (8 chunks (s, hi/lo, h) of 8, chunk q at q ^ (c & 7)),
// centroid rows [cpl][DMAX + 2] f64 (mu, then v_c, then a pad: the odd
// 16-byte stride puts the lanes' reads of different centroids in different
// bank groups, and a lane's 16 reads of one row take immediate offsets --
// round 5 first XOR-swizzled the chunks, two VALU per read), A' [cpl] f32
// (SIL_BIG: padding), bounds 2 f64, code -> ordinal [cmax+1] int
__host__ __device__ inline size_t sil_img_bytes(int cpl, int dmax, int cmax) {
    return (size_t)cpl * (128 + 8 * ((size_t)dmax + 2) + 4) + 16 + 4 * (size_t)(cmax + 1);
}
__host__ __device__ inline size_t sil_img_stride(int cmax, int dmax) {
    return (sil_img_bytes((cmax + 31) & ~31, dmax, cmax) + 1023) & ~(size_t)1023;
}
__host__ __device__ inline int sil_e16(double maxabs) {
    return maxabs > 0.0 ? 11 - ilogb(maxabs) : 0;
}

__device__ __forceinline__ void sil_split16(double v, _Float16& hi, _Float16& lo) {
    // (fp32 pinned in registers: see knn_split16)
    float f = (float)v;
    asm volatile("" : "+v"(f));
    hi = fabsf(f) < 0x1p-14f ? (_Float16)0.0f : (_Float16)f;
    float r = (float)(v - (double)(float)hi);
    asm volatile("" : "+v"(r));
    lo = fabsf(r) < 0x1p-14f ? (_Float16)0.0f : (_Float16)r;
}

// One block per labeling: its image (layout above).
template <int DMAX>
__global__ __launch_bounds__(256) void sil_w16_prep(int cmax, const unsigned* __restrict__ maxabs_bits,
                                                    const int* __restrict__ npres, const int* __restrict__ codes,
                                                    const int* __restrict__ pos, const double* __restrict__ mu,
                                                    const double* __restrict__ auxc, unsigned char* __restrict__ img,
                                                    size_t imgs) {
    __shared__ double red[2][4];
    const int l = blockIdx.x, tid = threadIdx.x;
    const int C = npres[l], cpl = ((C + 31) >> 5) << 5;
    unsigned char* base = img + (size_t)l * imgs;
    _Float16* fr = (_Float16*)base;
    double* m64 = (double*)(base + (size_t)cpl * 128);
    float* sa = (float*)(m64 + (size_t)cpl * (DMAX + 2));
    double* bnd = (double*)(sa + cpl);
    int* sp = (int*)(bnd + 2);
    const int e16 = sil_e16((double)__uint_as_float(*maxabs_bits));
    const double* ml = mu + (int64_t)l * (cmax + 1) * DMAX;
    const int* cl = codes + (int64_t)l * cmax;
    for (int t = tid; t < cpl * DMAX; t += 256) {
        const int c = t / DMAX, k = t - c * DMAX;
        const double v = c < C ? ml[(int64_t)cl[c] * DMAX + k] : 0.0;
        m64[c * (DMAX + 2) + k] = v;
        _Float16 hi, lo;
        sil_split16(ldexp(v, e16), hi, lo);
        const int s = k >> 4, hh = (k >> 3) & 1, i = k & 7;
        fr[c * 64 + (((s * 4 + hh) ^ (c & 7)) << 3) + i] = hi;
        fr[c * 64 + (((s * 4 + 2 + hh) ^ (c & 7)) << 3) + i] = lo;
    }
    const double* al = auxc + (int64_t)l * cmax * 2;
    double mb = 0.0, ab = 0.0;
    for (int c = tid; c < cpl; c += 256) {
        const bool pr = c < C;
        const double a0 = pr ? al[2 * c] : 0.0, a1 = pr ? al[2 * c + 1] : 0.0;
        m64[c * (DMAX + 2) + DMAX] = a1;
        m64[c * (DMAX + 2) + DMAX + 1] = 0.0;
        sa[c] = pr ? (float)ldexp(a0 + a1, 2 * e16) : SIL_BIG;
        mb = fmax(mb, a0);
        ab = fmax(ab, a0 + a1);
    }
    for (int c = tid; c <= cmax; c += 256) sp[c] = pos[(int64_t)l * (cmax + 1) + c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mb = fmax(mb, __shfl_xor(mb, o, 64));
        ab = fmax(ab, __shfl_xor(ab, o, 64));
    }
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = mb;
        red[1][tid >> 6] = ab;
    }
    __syncthreads();
    if (tid == 0) {
        bnd[0] = sqrt(fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3])));
        bnd[1] = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
    }
}

typedef float sil_f2 __attribute__((ext_vector_type(2)));
// the value of lane (lane mod 32) + 32 hb of the wave (v_permlane32_swap:
// no LDS permute); hb = 0 the low half, 1 the high half
__device__ __forceinline__ unsigned sil_half(unsigned v, int hb) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // {low half twice, high half twice}
    return hb ? r[1] : r[0];
}
__device__ __forceinline__ int sil_half(int v, int hb) { return (int)sil_half((unsigned)v, hb); }
__device__ __forceinline__ float sil_half(float v, int hb) { return __uint_as_float(sil_half(__float_as_uint(v), hb)); }
__device__ __forceinline__ double sil_half(double v, int hb) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = sil_half((unsigned)b, hb), hi = sil_half((unsigned)(b >> 32), hb);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// the sum over the wave of a 64-bit integer (uniform result): DPP within
// each row of 16 (quad xor 1, xor 2, row rotate 4, 8), then the four rows'
// sums read from lanes 15, 31, 47, 63 -- no LDS permutes
template <int CTRL>
__device__ __forceinline__ unsigned long long sil_dpp64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)v, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(v >> 32), CTRL, 0xf, 0xf, false);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned sil_wave_sum_u32(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 15) + (unsigned)__builtin_amdgcn_readlane((int)v, 31) +
           (unsigned)__builtin_amdgcn_readlane((int)v, 47) + (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ unsigned long long sil_wave_sum_u64(unsigned long long v) {
    v += sil_dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += sil_dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += sil_dpp64<0x124>(v);  // row_ror:4
    v += sil_dpp64<0x128>(v);  // row_ror:8
    unsigned long long t = 0;
#pragma unroll
    for (int r = 15; r < 64; r += 16)
        t += ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), r) << 32) |
             (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, r);
    return t;
}

template <int DMAX, int IMGB, bool SEG>
__global__ __launch_bounds__(SIL_WT, 3) void sil_width16(
    const double* __restrict__ x, int64_t m, int d, const int32_t* __restrict__ labels, int L, int cmax,
    const unsigned* __restrict__ maxabs_bits, const int* __restrict__ npres, const unsigned char* __restrict__ img,
    size_t imgs, unsigned long long* __restrict__ wsum, unsigned long long* __restrict__ wcnt,
    double* __restrict__ out_width, const int* __restrict__ rep, const int* __restrict__ mult,
    const int* __restrict__ cnt, int64_t mw, int nbw, const int64_t* __restrict__ nrep, double wsc, double sqd,
    const int64_t* __restrict__ scan, SilSegs sgs) {
    constexpr int KS = DMAX / 16;  // K steps of 16 dimensions
    // two image buffers as two objects, and the labeling loop unrolled by two,
    // so the compiler sees that the copy into one does not alias the reads of
    // the other (with one array it waits for the copy before every LDS read)
    __shared__ __attribute__((aligned(1024))) unsigned char buf0[IMGB];
    __shared__ __attribute__((aligned(1024))) unsigned char buf1[IMGB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    // 32 representatives per wave; tile tb of the (segment's) positions
    int64_t pb, npos;
    int q = 0, tb = blockIdx.x;
    if constexpr (SEG) {  // segment q's representatives are positions [scan[off_q], scan[off_q+1])
        q = sil_seg_tile(sgs.tw, sgs.nseg, blockIdx.x);
        tb = blockIdx.x - sgs.tw[q];
        pb = scan[sgs.off[q]] + (int64_t)tb * (SIL_WT / 2);
        npos = scan[sgs.off[q + 1]];
    } else {
        pb = (int64_t)blockIdx.x * (SIL_WT / 2);
        npos = rep ? *nrep : m;  // representatives: counted on the device
    }
    if (pb >= npos) return;  // the partials of idle blocks stay 0
    const int l0 = blockIdx.y * SIL_WLG, l1 = min(L, l0 + SIL_WLG);
    const int lq = q * L;  // virtual labeling of (q, 0)
    // copy labeling l's image into buffer b: 1 KB per wave instruction
    auto stage = [&](int l, unsigned char* dst) {
        const int cpl = ((npres[lq + l] + 31) >> 5) << 5;
        const int nch = (int)((sil_img_bytes(cpl, DMAX, cmax) + 1023) >> 10);
        const unsigned char* src = img + (size_t)(lq + l) * imgs;
        for (int ch = wave; ch < nch; ch += SIL_WT / 64)
            __builtin_amdgcn_global_load_lds(
                (const void __attribute__((address_space(1)))*)(src + (size_t)ch * 1024 + lane * 16),
                (void __attribute__((address_space(3)))*)(dst + (size_t)ch * 1024), 16, 0, 0);
    };
    stage(l0, buf0);
    // representative j of the wave (both lane halves hold it)
    const int64_t p = pb + wave * 32 + j;
    const bool in = p < npos;
    const int64_t row = in ? (rep ? (int64_t)rep[p] : p) : 0;
    const int e16 = sil_e16((double)__uint_as_float(*maxabs_bits));
    double xr[DMAX];
    double xx = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
        xr[k] = (in && k < d) ? x[row * d + k] : 0.0;
        xx = fma(xr[k], xr[k], xx);
    }
    const double xn = ldexp(sqrt(xx), e16);
    sil_h8 bh[KS], bl[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            _Float16 hi, lo;
            // a bit select, not a lane-dependent register index (which spills to scratch)
            const long long hm = -(long long)h;
            const double v = __longlong_as_double((__double_as_longlong(xr[16 * s + i]) & ~hm) |
                                                  (__double_as_longlong(xr[16 * s + 8 + i]) & hm));
            sil_split16(ldexp(v, e16), hi, lo);
            bh[s][i] = hi;
            bl[s][i] = lo;
        }
    const int cw = rep && in ? cnt[p] : 1;
    // 32-bit offsets from wave-uniform bases (no 64-bit address pairs held across the loop)
    const int pi = (int)p;
    const int32_t* lbase = labels;  // labels of row rowl in labeling l: lbase[l * lstride + rowl]
    int64_t lstride = m;
    int rowl = (int)row;
    if constexpr (SEG) {
        lbase = sgs.lab[q];
        lstride = sgs.off[q + 1] - sgs.off[q];
        rowl = (int)(row - sgs.off[q]);
    }
    int lab = in ? (lbase + (int64_t)l0 * lstride)[rowl] : 0;
    int mlt = (rep && in) ? (mult + (int64_t)l0 * mw)[pi] : 0;
    // (wsc = 2^scale_exp(m) and sqd = sqrt(d) come as kernel arguments: SGPRs)
    auto labeling = [&](int l, const unsigned char* __restrict__ bs, unsigned char* __restrict__ nxt) {
        const int C = npres[lq + l];
        const int nt = (C + 31) >> 5, cpl = nt << 5;
        __syncthreads();  // image l has landed; the other buffer is free
        const _Float16* sA = (const _Float16*)bs;
        const double* smu = (const double*)(bs + (size_t)cpl * 128);
        const float* sAf = (const float*)(smu + (size_t)cpl * (DMAX + 2));
        const double* sbnd = (const double*)(sAf + cpl);
        const int* spos = (const int*)(sbnd + 2);
        // lab and mlt are consumed before the next image's copy is issued: a
        // use of an ordinary load after it would wait for the copy too
        const int po = (lab >= 1 && lab <= cmax) ? spos[lab] : -1;  // own ordinal
        const int wt = cw - mlt;
        int labn = 0, mltn = 0;
        if (l + 1 < l1) {
            labn = in ? (lbase + (int64_t)(l + 1) * lstride)[rowl] : 0;
            mltn = (rep && in) ? (mult + (int64_t)(l + 1) * mw)[pi] : 0;
            stage(l + 1, nxt);
        }
        // the own cluster's (register, tile) in this lane's values, or -1
        int ownkey = -1;
        if (po >= 0) {
            const int i = po & 31;
            if (((i >> 2) & 1) == h) ownkey = (i & 3) + 4 * (i >> 3) + 16 * (po >> 5);
        }
        // the three smallest packed values (the own cluster is dropped after
        // the loop: three med3 per value instead of a compare, a select and
        // two med3)
        float m1 = SIL_BIG, m2 = SIL_BIG, m3 = SIL_BIG;
        // the packing mask in a VGPR (one v_and_or per value: VOP3 takes no literal here)
        unsigned msk = ~127u;
        asm volatile("" : "+v"(msk));
        for (int t = 0; t < nt; ++t) {
            sil_f16x acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
            const int c = t * 32 + j;
            const _Float16* ar = sA + c * 64;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const sil_h8 ah = *reinterpret_cast<const sil_h8*>(ar + (((s * 4 + h) ^ (c & 7)) << 3));
                const sil_h8 alo = *reinterpret_cast<const sil_h8*>(ar + (((s * 4 + 2 + h) ^ (c & 7)) << 3));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bh[s], acc, 0, 0, 0);
            }
            // register r holds centroid t*32 + (r & 3) + 8 (r >> 2) + 4h
            const float4* af = reinterpret_cast<const float4*>(sAf + t * 32 + 4 * h);
            const int key0 = 16 * t;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 a4 = af[2 * g];
                // a = A' - 2 x.mu, two values per packed fma
                const sil_f2 lo2 = __builtin_elementwise_fma((sil_f2){acc[4 * g], acc[4 * g + 1]}, (sil_f2){-2.0f, -2.0f},
                                                             (sil_f2){a4.x, a4.y});
                const sil_f2 hi2 = __builtin_elementwise_fma((sil_f2){acc[4 * g + 2], acc[4 * g + 3]},
                                                             (sil_f2){-2.0f, -2.0f}, (sil_f2){a4.z, a4.w});
                const float av[4] = {lo2.x, lo2.y, hi2.x, hi2.y};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = 4 * g + q;
                    unsigned kr = (unsigned)(key0 + r);
                    asm volatile("" : "+s"(kr));  // (the key in an SGPR: one v_and_or, not and + or3)
                    const float pk = __uint_as_float((__float_as_uint(av[q]) & msk) | kr);
                    // (med3 throughout: fminf would add a canonicalising max per value)
                    m3 = __builtin_amdgcn_fmed3f(m2, pk, m3);
                    m2 = __builtin_amdgcn_fmed3f(m1, pk, m2);
                    m1 = __builtin_amdgcn_fmed3f(-SIL_BIG, m1, pk);
                }
            }
        }
        if (ownkey >= 0) {  // (keys are distinct: at most one of the three is the own cluster)
            if ((int)(__float_as_uint(m1) & 127u) == ownkey) {
                m1 = m2;
                m2 = m3;
            } else if ((int)(__float_as_uint(m2) & 127u) == ownkey) {
                m2 = m3;
            }
        }
        // merge the lane halves (v_permlane32_swap: each half gets the other's
        // value): the smallest, its centroid, the second smallest
        const unsigned kb = __float_as_uint(m1) & 127u;
        const int myarg = (int)((kb & 3) + 8 * ((kb >> 2) & 3) + 4 * h + 32 * (kb >> 4));
        const float m1l = sil_half(m1, 0), m1h = sil_half(m1, 1);
        const float m2l = sil_half(m2, 0), m2h = sil_half(m2, 1);
        const int al = sil_half(myarg, 0), ahh = sil_half(myarg, 1);
        const int arg1 = m1l <= m1h ? al : ahh;
        const float n1 = fminf(m1l, m1h), n2 = fminf(fmaxf(m1l, m1h), fminf(m2l, m2h));
        const bool none = !(n1 < 1.0e37f);  // no other cluster
        // E bounds the error of one screened value a (scaled units; see the
        // header): 2 x (3 2^-22 + 95 2^-24) xn mbs for the split and the fp32
        // accumulation of 3 DMAX products, 2^-13 sqrt(d) (xn + mbs) for the
        // parts flushed below 2^-14, (2^-16 + 2^-23) |a| for the 7-bit
        // packing and the fma, |a| <= abs2 + 2 xn mbs: within 2^-14 xn mbs +
        // 2^-13 sqrt(d) (xn + mbs) + 2^-15 abs2 (+8 for what is left)
        const double mbs = ldexp(sbnd[0], e16), abs2 = ldexp(sbnd[1], 2 * e16);
        const double E = 0x1p-14 * xn * mbs + 0x1p-13 * sqd * (xn + mbs) + 0x1p-15 * abs2 + 8.0;
        const bool amb = !none && (double)n2 - (double)n1 <= 2.0 * E;
        auto dsq = [&](int c) {
            const double* mr = smu + c * (DMAX + 2);
            double s = mr[DMAX];  // v_c
#pragma unroll
            for (int q = 0; q < DMAX / 2; ++q) {
                const double2 v = *reinterpret_cast<const double2*>(mr + 2 * q);
                const double t0 = xr[2 * q] - v.x, t1 = xr[2 * q + 1] - v.y;
                s = fma(t0, t0, s);
                s = fma(t1, t1, s);
            }
            return s;
        };
        // one exact distance per lane: h = 0 the own cluster, h = 1 the nearest other
        const int cx = h == 0 ? (po >= 0 ? po : 0) : ((none || amb) ? 0 : arg1);
        const double dx = dsq(cx);
        const double S = po >= 0 ? dx : INFINITY;  // (read on h = 0)
        double O = (h == 1 && !none && !amb) ? dx : INFINITY;
        if (__any(amb)) {
            // a near tie in the screen: the tiles again, listing (per lane) the
            // other centroids whose screen value is within 2E of the smallest --
            // every centroid that can be the nearest -- and each taken exactly.
            // (Round 5 first took every centroid of an ambiguous lane: 60% of
            // the waves paid C exact distances.)
            const float thr = amb ? (float)((double)n1 + 2.0 * E) * (1.0f + 0x1p-20f) : -SIL_BIG;
            int cand[SIL_NCAND];
            int nc = 0;
#pragma unroll
            for (int u = 0; u < SIL_NCAND; ++u) cand[u] = 0;
            for (int t = 0; t < nt; ++t) {
                sil_f16x acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
                const int c = t * 32 + j;
                const _Float16* ar = sA + c * 64;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const sil_h8 ah = *reinterpret_cast<const sil_h8*>(ar + (((s * 4 + h) ^ (c & 7)) << 3));
                    const sil_h8 alo = *reinterpret_cast<const sil_h8*>(ar + (((s * 4 + 2 + h) ^ (c & 7)) << 3));
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bh[s], acc, 0, 0, 0);
                }
                const float4* af = reinterpret_cast<const float4*>(sAf + t * 32 + 4 * h);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 a4 = af[2 * g];
                    const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = 4 * g + q;
                        const int ci = t * 32 + q + 8 * g + 4 * h;
                        const float a = fmaf(-2.0f, acc[r], av[q]);
                        if (a <= thr && ci != po && ci < C) {
#pragma unroll
                            for (int u = 0; u < SIL_NCAND; ++u) cand[u] = nc == u ? ci : cand[u];
                            ++nc;
                        }
                    }
                }
            }
            // a lane with more candidates than its list takes every centroid of its half
            const bool full = nc > SIL_NCAND;
            int ncw = full ? 0 : nc;
            for (int o = 32; o > 0; o >>= 1) ncw = max(ncw, __shfl_xor(ncw, o, 64));
            for (int u = 0; u < SIL_NCAND; ++u) {
                if (u >= ncw) break;  // (wave-uniform)
                if (!full && u < nc) O = fmin(O, dsq(cand[u]));
            }
            if (__any(full))
                for (int c = h; c < C; c += 2)
                    if (full && c != po) O = fmin(O, dsq(c));
        }
        O = fmin(O, sil_half(O, 0));
        O = fmin(O, sil_half(O, 1));  // (both halves: the minimum over the wave's pair of lanes)
        // one square root per lane (h = 0 the own distance, h = 1 the other),
        // exchanged between the halves
        const double rt = sqrt(h == 0 ? S : O);
        const double rt1 = sil_half(rt, 1);  // (every lane takes part in the swap)
        const double ort = h == 0 ? rt1 : rt;
        long long wq = 0;
        unsigned wn = 0;
        if (in && h == 0) {
            double w = 0.0;
            if (C > 1) {
                double mx = fmax(ort, rt);
                if (isnan(ort) || isnan(rt)) mx = NAN;
                w = (ort - rt) / mx;
            }
            if (out_width && !rep) out_width[(int64_t)l * m + p] = w;
            if (!isnan(w)) {
                wq = (long long)wt * __double2ll_rn(w * wsc);
                wn = (unsigned)wt;
            }
        }
        const unsigned long long tq = sil_wave_sum_u64((unsigned long long)wq);
        const unsigned long long tn = sil_wave_sum_u32(wn);  // (a wave's weights: < 2^32)
        if (lane == 0) {
            wsum[(int64_t)(lq + l) * nbw + 4 * tb + wave] = tq;
            wcnt[(int64_t)(lq + l) * nbw + 4 * tb + wave] = tn;
        }
        lab = labn;
        mlt = mltn;
    };
    for (int l = l0; l < l1; l += 2) {
        labeling(l, buf0, buf1);
        if (l + 1 < l1) labeling(l + 1, buf1, buf0);
    }
}

// One block per labeling: the cluster count and smallest size from the
// counts, and the mean width from the per-block fixed-point partials.
__global__ __launch_bounds__(256) void sil_final(int64_t m, int L, int cmax, int nbw,
                                                 const unsigned long long* __restrict__ gcnt,
                                                 const unsigned long long* __restrict__ wsum,
                                                 const unsigned long long* __restrict__ wcnt,
                                                 double* __restrict__ out_mean, int32_t* __restrict__ out_nclust,
                                                 int32_t* __restrict__ out_minsize, SilSegs sgs) {
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
        int lo = l;  // (blockIdx.x: the virtual labeling q L + lo of segment q)
        if (sgs.nseg) {
            const int qs = l / L;
            lo = l - qs * L;
            out_mean = sgs.mean[qs];
            out_nclust = sgs.ncl[qs];
            out_minsize = sgs.mns[qs];
        }
        if (out_mean) out_mean[lo] = n ? ((double)(long long)q * inv_wsc) / (double)n : NAN;
        if (out_nclust) out_nclust[lo] = np;
        if (out_minsize) out_minsize[lo] = (int32_t)(mn == LLONG_MAX ? 0 : mn);
    }
}

// rows per sil_width block, and the width partials per labeling (one per
// wave of every block)
template <int DMAX>
constexpr int sil_width_rows() {
    return 4 * sil_rt<DMAX>() * 16;
}
// (d <= 32: sil_width16's 4 waves x 32 representatives per block; the round-4
// kernel, kept for d > 32 and cmax past sil_width16's stage, takes 256 rows
// per block, so it uses the first half of the partials)
static int sil_width_blocks(int64_t m, int d) {
    if (d <= 32) return 4 * (int)ccg_cdiv(m, SIL_WT / 2);
    return 4 * (int)ccg_cdiv(m, sil_width_rows<64>());
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

// (also zeroes the call's sums and width partials, zw words: one launch
// instead of a memset and this kernel)
__global__ void sil_init_kernel(int* __restrict__ first, int64_t ncell, int* __restrict__ zero, int64_t nzero,
                                unsigned long long* __restrict__ zw, int64_t nzw) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ncell || t < nzero || t < nzw;
         t += (int64_t)gridDim.x * blockDim.x) {
        if (t < ncell) first[t] = 0x7fffffff;
        if (t < nzero) zero[t] = 0;
        if (t < nzw) zw[t] = 0ull;
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

// Every non-representative row whose label differs from its
// representative's: dis[l][pos] += 1 (the weight is cnt - dis) and the row
// joins the exception list (l << 32 | row).  A thread takes one row and
// SIL_MULT_LG labelings (blockIdx.y: the group): one (row, representative)
// load and the group's label pairs in flight together (one labeling per
// thread and a grid-stride row loop chained two dependent loads per row).
#define SIL_MULT_LG 8
__global__ __launch_bounds__(256) void sil_mult_kernel(int64_t m, int L, const int32_t* __restrict__ labels,
                                                       const int64_t* __restrict__ scan,
                                                       const int3* __restrict__ nonrep, int64_t mw,
                                                       int* __restrict__ dis, unsigned long long* __restrict__ exc,
                                                       int* __restrict__ nexc, SilSegs sgs) {
    const int64_t nn = m - scan[m];
    for (int l0 = blockIdx.y * SIL_MULT_LG; l0 < L; l0 += gridDim.y * SIL_MULT_LG)
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nn; j += (int64_t)gridDim.x * blockDim.x) {
        const int3 e = nonrep[j];
        const int r = e.x, rp = e.y;
        // (a row and its representative are in one segment: the cell ids are per segment)
        const int q = sgs.nseg ? sil_seg_row(sgs.off, sgs.nseg, r) : 0;
        int a[SIL_MULT_LG], b[SIL_MULT_LG];
#pragma unroll
        for (int t = 0; t < SIL_MULT_LG; ++t) {
            a[t] = b[t] = 0;
            if (l0 + t < L) {
                a[t] = sil_label(labels, m, sgs, q, l0 + t, r);
                b[t] = sil_label(labels, m, sgs, q, l0 + t, rp);
            }
        }
#pragma unroll
        for (int t = 0; t < SIL_MULT_LG; ++t) {
            if (a[t] != b[t]) {
                const int l = l0 + t;
                atomicAdd(&dis[(int64_t)l * mw + e.z], 1);
                const int x = atomicAdd(nexc, 1);
                exc[x] = ((unsigned long long)l << 32) | (unsigned long long)r;
            }
        }
    }
}

// One thread per exception row: its width against labeling l's centroids
// (fp64, D^2 = sum_k (x_k - mu_k)^2 + v_c as sil_width16 takes it), added
// to the labeling's first width partial (integer atomics: order-independent).
template <int DMAX>
__global__ void sil_width_exc(const double* __restrict__ x, int64_t m, int d, const int32_t* __restrict__ labels,
                              int L, int cmax, const int* __restrict__ npres, const int* __restrict__ codes,
                              const double* __restrict__ muc, const double* __restrict__ auxc,
                              const unsigned long long* __restrict__ exc, const int* __restrict__ nexc, int nbw,
                              unsigned long long* __restrict__ wsum, unsigned long long* __restrict__ wcnt,
                              SilSegs sgs) {
    const int ne = *nexc;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x) {
    const int l = (int)(exc[e] >> 32);
    const int64_t r = (int64_t)(exc[e] & 0xffffffffull);
    const int q = sgs.nseg ? sil_seg_row(sgs.off, sgs.nseg, r) : 0;
    const int lab = sil_label(labels, m, sgs, q, l, r);
    const int64_t lv = (int64_t)q * L + l;
    double xr[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) xr[k] = k < d ? x[r * d + k] : 0.0;
    const int np = npres[lv];
    double self = INFINITY, oth = INFINITY;
    for (int p = 0; p < np; ++p) {
        const double* mp = muc + (lv * cmax + p) * DMAX;
        double s2 = fmax(auxc[2 * (lv * cmax + p) + 1], 0.0);
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
            const double t = xr[k] - mp[sil_mfma_pos<DMAX>(k)];
            s2 = fma(t, t, s2);
        }
        if (codes[lv * cmax + p] == lab) self = s2;
        else oth = fmin(oth, s2);
    }
    long long wq = 0;
    unsigned wn = 0;
    sil_row_width(self, oth, true, np, ldexp(1.0, scale_exp((double)m)), nullptr, wq, wn);
    if (wn) {
        atomicAdd(&wsum[lv * nbw], (unsigned long long)wq);  // the first partial of the labeling
        atomicAdd(&wcnt[lv * nbw], 1ull);
    }
    }
}

// Positions per sums block (SIL_SP when the block's sums fit the CU's
// LDS), or 0: the unsorted sil_centroid path.
static int sil_tile_T(int d, int cmax) {
    return sil_sums_G(d, cmax) ? SIL_SP : 0;
}

// The launch set after max|x| (and, for the distinct-cell forms, the
// representative tables).  Segments (sgs.nseg > 0, cells form only) run the
// tiled sums and sil_width16 over every segment at once: the sums' tiles and
// the width tiles are laid out per segment (ts_tiles, tw_tiles blocks), the
// per-labeling tables over Lv = nseg L virtual labelings.
template <int DMAX>
static void sil_launch(const double* x, int64_t m, int d, const int32_t* labels, int L, int cmax,
                       unsigned* maxabs, unsigned long long* gsum, unsigned long long* gsum2, unsigned long long* gcnt,
                       unsigned long long* gvar, unsigned long long* wsum, unsigned long long* wcnt,
                       int* npres, int* codes, int* pos, double* mu, double* muc, double* auxc, void* q,
                       unsigned char* img, double* out_width, int nbw, hipStream_t st, const int* rep = nullptr,
                       const int* mult = nullptr, const int* cnt = nullptr, int64_t mw = 0,
                       const unsigned long long* exc = nullptr, const int* nexc = nullptr,
                       const int64_t* nrep = nullptr, const int64_t* scan = nullptr, SilSegs sgs = SilSegs{},
                       int ts_tiles = 0, int tw_tiles = 0) {
    const bool seg = sgs.nseg > 0;
    const int Lv = seg ? sgs.nseg * L : L;  // virtual labelings
    const int T = q ? sil_tile_T(d, cmax) : 0;
    if (T) {
        // tiled sums: S1, S2 and counts in one pass, v_c in sil_mu
        long long* q1 = (long long*)q;
        long long* q2 = q1 + m * DMAX;
        sil_quant<DMAX><<<(unsigned)ccg_cdiv(m * DMAX, 256), 256, 0, st>>>(x, m, d, maxabs, q1, q2);
        const int ntile = (int)(seg ? ts_tiles : ccg_cdiv(m, T));
        const int tpx = (int)ccg_cdiv(ntile, 8);
        const int G = sil_sums_G(d, cmax);
        const unsigned gb = (unsigned)(8 * (int64_t)tpx * ccg_cdiv(L, G));
        const size_t lds = sil_tile_lds(d, cmax, G);
        if (seg)
            sil_sums_blk<DMAX, true><<<gb, SIL_SB, lds, st>>>(m, d, ntile, tpx, G, labels, L, cmax, q1, q2, gsum, gsum2,
                                                              gcnt, rep, mult, cnt, mw, nrep, scan, sgs);
        else
            sil_sums_blk<DMAX, false><<<gb, SIL_SB, lds, st>>>(m, d, ntile, tpx, G, labels, L, cmax, q1, q2, gsum, gsum2,
                                                               gcnt, rep, mult, cnt, mw, nrep, scan, sgs);
        if (rep)
            sil_sums_exc<DMAX><<<64, 256, 0, st>>>(m, d, labels, L, cmax, q1, q2, exc, nexc, gsum, gsum2, gcnt, sgs);
        sil_mu<DMAX><<<Lv, SIL_T, 0, st>>>(m, d, cmax, maxabs, gsum, gsum2, gcnt, npres, codes, pos, mu, muc, auxc);
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
    bool w16 = false;
    if constexpr (DMAX <= 32) w16 = cmax <= SIL_WCMAX && 2 * sil_img_stride(cmax, DMAX) <= SIL_W16_LDS && img;
    if (w16) {
        if constexpr (DMAX <= 32) {
        const size_t imgs = sil_img_stride(cmax, DMAX);
        sil_w16_prep<DMAX><<<Lv, 256, 0, st>>>(cmax, maxabs, npres, codes, pos, mu, auxc, img, imgs);
        dim3 g16((unsigned)(seg ? tw_tiles : ccg_cdiv(nrows, SIL_WT / 2)), (unsigned)ccg_cdiv(L, SIL_WLG));
        const double wsc = ldexp(1.0, scale_exp((double)m)), sqd = sqrt((double)d);
        double* ow = rep ? nullptr : out_width;
#define SIL_W16(B_)                                                                                                  \
        if (seg)                                                                                                     \
            sil_width16<DMAX, B_, true><<<g16, SIL_WT, 0, st>>>(x, m, d, labels, L, cmax, maxabs, npres, img, imgs,  \
                                                                wsum, wcnt, ow, rep, mult, cnt, mw, nbw, nrep, wsc,  \
                                                                sqd, scan, sgs);                                     \
        else                                                                                                         \
            sil_width16<DMAX, B_, false><<<g16, SIL_WT, 0, st>>>(x, m, d, labels, L, cmax, maxabs, npres, img, imgs, \
                                                                 wsum, wcnt, ow, rep, mult, cnt, mw, nbw, nrep, wsc, \
                                                                 sqd, scan, sgs)
        if (imgs <= 14336) { SIL_W16(14336); }
        else if (imgs <= 26624) { SIL_W16(26624); }
        else { SIL_W16(40960); }
#undef SIL_W16
        if (rep)
            sil_width_exc<DMAX><<<64, 256, 0, st>>>(x, m, d, labels, L, cmax, npres, codes, muc, auxc, exc, nexc, nbw,
                                                    wsum, wcnt, sgs);
        }
        return;
    }
    dim3 grid2((unsigned)ccg_cdiv(nrows, sil_width_rows<DMAX>()), (unsigned)ccg_cdiv(L, SIL_LG));
    // the stage holds a whole group of SIL_LG labelings when it can
    const int CH = (int)std::min<int64_t>(sil_chunk<DMAX>(), (int64_t)SIL_LG * (((int64_t)cmax + 15) / 16 * 16));
    const size_t lds5 = (size_t)CH * sil_sp<DMAX>() * 8 + (size_t)CH * 8 + (size_t)CH * 4;
    if (rep) {
        // partials of blocks past the representative grid stay 0 (zeroed with the buffer)
        sil_width<DMAX><<<grid2, SIL_T, lds5, st>>>(x, m, d, labels, L, cmax, npres, codes, muc, auxc, wsum, wcnt,
                                                nullptr, CH, rep, mult, cnt, mw, nbw, nrep);
        sil_width_exc<DMAX><<<64, 256, 0, st>>>(x, m, d, labels, L, cmax, npres, codes, muc, auxc, exc, nexc, nbw,
                                                wsum, wcnt, sgs);
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
    void* q = nullptr;  // fixed-point rows of the tiled sorted-segment path (cmax small enough for its LDS)
    if (sil_tile_T(d, cmax)) {
        q = ccg_ws(ctx, WS_SIL_Q, sizeof(long long) * (size_t)m * dmax + sizeof(long long) * (size_t)m + 64);
        if (!q) return CCG_ENOMEM;
    }
    unsigned char* img = nullptr;  // LDS images of the fp16-screen widths (d <= 32, cmax small enough)
    if (dmax <= 32 && cmax <= SIL_WCMAX && 2 * sil_img_stride(cmax, dmax) <= SIL_W16_LDS) {
        img = (unsigned char*)ccg_ws(ctx, WS_SIL_IMG, (size_t)L * sil_img_stride(cmax, dmax));
        if (!img) return CCG_ENOMEM;
    }
    const int t_all = ccg_timer_start(ctx, CCG_KT_SILHOUETTE, st);
    CCG_HIP(hipMemsetAsync(buf, 0, sizeof(unsigned long long) * words, st));
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 4 * SIL_MAXABS_T), SIL_MAXABS_GRID), SIL_MAXABS_T, 0,
                 st>>>(x, m * d, maxabs);
    if (d <= 16)
        sil_launch<16>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        img, out_width, nbw, st);
    else if (d <= 32)
        sil_launch<32>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        img, out_width, nbw, st);
    else
        sil_launch<64>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc, q,
                        img, out_width, nbw, st);
    sil_final<<<L, 256, 0, st>>>(m, L, cmax, nbw, gcnt, wsum, wcnt, out_mean, out_nclust, out_minsize, SilSegs{});
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// The distinct-cell launch set over m rows (one matrix, or a batch of
// segments: sgs.nseg > 0, per-labeling tables over nseg L virtual
// labelings, nbw width partials per virtual labeling).
static int sil_cells_run(ccg_ctx* ctx, const double* x, int64_t m, int d, const int32_t* labels, int L, int cmax,
                         const int32_t* cell, int64_t ncell, double* out_mean, int32_t* out_nclust,
                         int32_t* out_minsize, hipStream_t st, SilSegs sgs, int ts_tiles, int tw_tiles, int nbw) {
    const int64_t Lv = sgs.nseg ? (int64_t)sgs.nseg * L : L;
    const int64_t nacc = (int64_t)(cmax + 1) * d;
    const int64_t words = 2 * Lv * nacc + 2 * Lv * (cmax + 1) + 2 * Lv * nbw + 8;
    unsigned long long* buf = (unsigned long long*)ccg_ws(ctx, WS_SIL_A, sizeof(unsigned long long) * words);
    if (!buf) return CCG_ENOMEM;
    unsigned long long* gsum = buf;
    unsigned long long* gsum2 = gsum + Lv * nacc;
    unsigned long long* gcnt = gsum2 + Lv * nacc;
    unsigned long long* gvar = gcnt + Lv * (cmax + 1);
    unsigned long long* wsum = gvar + Lv * (cmax + 1);
    unsigned long long* wcnt = wsum + Lv * nbw;
    unsigned* maxabs = (unsigned*)(wcnt + Lv * nbw);
    const int dmax = d <= 16 ? 16 : (d <= 32 ? 32 : 64);
    const size_t mu_words = (size_t)Lv * (cmax + 1) * dmax + (size_t)Lv * cmax * dmax + 2 * (size_t)Lv * cmax;
    const size_t tab_ints = (size_t)Lv * cmax + (size_t)Lv * (cmax + 1) + Lv + 8;
    double* mu = (double*)ccg_ws(ctx, WS_SIL_B, sizeof(double) * mu_words + sizeof(int) * tab_ints);
    if (!mu) return CCG_ENOMEM;
    double* muc = mu + (size_t)Lv * (cmax + 1) * dmax;
    double* auxc = muc + (size_t)Lv * cmax * dmax;
    int* npres = (int*)(auxc + 2 * (size_t)Lv * cmax);
    int* codes = npres + Lv;
    int* pos = codes + (size_t)Lv * cmax;
    void* q = nullptr;  // fixed-point rows of the tiled sums (cmax small enough for its LDS)
    if (sil_tile_T(d, cmax)) {
        q = ccg_ws(ctx, WS_SIL_Q, sizeof(long long) * (size_t)m * dmax + sizeof(long long) * (size_t)m + 64);
        if (!q) return CCG_ENOMEM;
    }
    unsigned char* img = nullptr;  // LDS images of the fp16-screen widths (d <= 32, cmax small enough)
    if (dmax <= 32 && cmax <= SIL_WCMAX && 2 * sil_img_stride(cmax, dmax) <= SIL_W16_LDS) {
        img = (unsigned char*)ccg_ws(ctx, WS_SIL_IMG, (size_t)Lv * sil_img_stride(cmax, dmax));
        if (!img) return CCG_ENOMEM;
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
    const unsigned gm = (unsigned)ccg_cdiv(m, 256);
    sil_init_kernel<<<(unsigned)std::min<int64_t>(
                          ccg_cdiv(std::max(std::max(ncell, (int64_t)(L + 1) * m + 4), words), 256), 4096),
                      256, 0, st>>>(first, ncell, nexc, (int64_t)(L + 1) * m + 4, buf, words);
    sil_first_kernel<<<gm, 256, 0, st>>>(cell, m, first);
    sil_isrep_kernel<<<gm, 256, 0, st>>>(cell, m, first, scan);
    int rc = ccg_scan_i64(ctx, scan, scan, m, st);
    if (rc) return rc;
    sil_rep_kernel<<<gm, 256, 0, st>>>(cell, m, first, scan, rep, cnt, nonrep);
    // mw = the number of representatives (the distinct cells): device-side
    // only, so the width grid covers m positions and the weights' stride is m
    // rows: the non-representatives are typically about a third of m (grid-stride past half)
    dim3 gx((unsigned)ccg_cdiv(m, 512), (unsigned)std::min<int64_t>(ccg_cdiv(L, SIL_MULT_LG), 65535));
    sil_mult_kernel<<<gx, 256, 0, st>>>(m, L, labels, scan, nonrep, m, mult, exc, nexc, sgs);
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 4 * SIL_MAXABS_T), SIL_MAXABS_GRID), SIL_MAXABS_T, 0,
                 st>>>(x, m * d, maxabs);
#define SIL_CELLS(DM_)                                                                                              \
    sil_launch<DM_>(x, m, d, labels, L, cmax, maxabs, gsum, gsum2, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, \
                    auxc, q, img, nullptr, nbw, st, rep, mult, cnt, m, exc, nexc, scan + m, scan, sgs, ts_tiles,     \
                    tw_tiles)
    if (d <= 16) SIL_CELLS(16);
    else if (d <= 32) SIL_CELLS(32);
    else SIL_CELLS(64);
#undef SIL_CELLS
    sil_final<<<(unsigned)Lv, 256, 0, st>>>(m, L, cmax, nbw, gcnt, wsum, wcnt, out_mean, out_nclust, out_minsize, sgs);
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
    return sil_cells_run(ctx, x, m, d, labels, L, cmax, cell, ncell, out_mean, out_nclust, out_minsize, st, SilSegs{},
                         0, 0, sil_width_blocks(m, d));
}

// Segments (R/consensusClust.R:562-566, :664: every subcluster of an
// iterate=TRUE level scores its bootstraps' clusterings): one launch set for
// a batch of segments whose rows are concatenated in x.  The sums and width
// kernels tile each segment's representatives separately; the per-labeling
// tables hold nseg x L virtual labelings.  Outside the tiled sums /
// sil_width16 envelope (d > 32 or a large cmax) the segments run one call
// each.
extern "C" int ccg_silhouette_segments_dev(ccg_ctx* ctx, const double* x, int d, int nseg, const int64_t* seg_off,
                                           const int32_t* const* labels, int L, int cmax, const int32_t* cell,
                                           int64_t ncell, double* const* out_mean, int32_t* const* out_nclust,
                                           int32_t* const* out_minsize, void* stream) {
    CCG_REQUIRE(ctx && x && seg_off && labels && cell, "ccg_silhouette_segments_dev: NULL argument");
    CCG_REQUIRE(nseg >= 1 && d >= 1 && d <= 64 && L >= 1, "ccg_silhouette_segments_dev: bad sizes nseg=%d d=%d L=%d",
                nseg, d, L);
    CCG_REQUIRE(cmax >= 1 && cmax <= (1 << 24), "ccg_silhouette_segments_dev: cmax=%d must be in [1, 2^24]", cmax);
    CCG_REQUIRE(ncell >= 1 && ncell < (1LL << 31), "ccg_silhouette_segments_dev: bad ncell");
    CCG_REQUIRE(seg_off[0] == 0, "ccg_silhouette_segments_dev: seg_off[0] must be 0");
    int64_t mq_max = 0;
    for (int s = 0; s < nseg; ++s) {
        CCG_REQUIRE(seg_off[s + 1] > seg_off[s], "ccg_silhouette_segments_dev: segment %d is empty", s);
        CCG_REQUIRE(labels[s], "ccg_silhouette_segments_dev: labels of segment %d are NULL", s);
        mq_max = std::max(mq_max, seg_off[s + 1] - seg_off[s]);
    }
    const int64_t m = seg_off[nseg];
    CCG_REQUIRE(m < (1LL << 31) && (int64_t)L * m < (1LL << 31) && (int64_t)nseg * L < (1LL << 31),
                "ccg_silhouette_segments_dev: %lld rows x %d labelings too many", (long long)m, L);
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int dmax = d <= 16 ? 16 : (d <= 32 ? 32 : 64);
    const int T = sil_tile_T(d, cmax);
    const bool one_set = dmax <= 32 && T && cmax <= SIL_WCMAX && 2 * sil_img_stride(cmax, dmax) <= SIL_W16_LDS;
    if (!one_set) {
        for (int s = 0; s < nseg; ++s) {
            const int64_t o = seg_off[s];
            const int rc = ccg_silhouette_cells_dev(ctx, x + o * d, seg_off[s + 1] - o, d, labels[s], L, cmax, cell + o,
                                                    ncell, out_mean ? out_mean[s] : nullptr,
                                                    out_nclust ? out_nclust[s] : nullptr,
                                                    out_minsize ? out_minsize[s] : nullptr, st);
            if (rc) return rc;
        }
        return CCG_OK;
    }
    // the segment table: offsets, tile starts, label and output pointers
    const size_t n1 = (size_t)nseg + 1;
    const size_t bytes = 8 * n1 + 8 * n1 + 8 * (size_t)nseg * 4;
    std::vector<unsigned char> hb(bytes);
    int64_t* hoff = (int64_t*)hb.data();
    int* hts = (int*)(hoff + n1);
    int* htw = hts + n1;
    const void** hptr = (const void**)(hts + 2 * n1 + ((2 * n1) & 1));
    int64_t ts = 0, tw = 0;
    for (size_t s = 0; s < n1; ++s) {
        hoff[s] = seg_off[s];
        hts[s] = (int)ts;
        htw[s] = (int)tw;
        if (s < (size_t)nseg) {
            const int64_t mq = seg_off[s + 1] - seg_off[s];
            ts += ccg_cdiv(mq, T);
            tw += ccg_cdiv(mq, SIL_WT / 2);
        }
    }
    CCG_REQUIRE(ts < (1LL << 31) && tw < (1LL << 31), "ccg_silhouette_segments_dev: too many tiles");
    for (int s = 0; s < nseg; ++s) {
        hptr[s] = labels[s];
        hptr[nseg + s] = out_mean ? out_mean[s] : nullptr;
        hptr[2 * nseg + s] = out_nclust ? out_nclust[s] : nullptr;
        hptr[3 * nseg + s] = out_minsize ? out_minsize[s] : nullptr;
    }
    unsigned char* db = (unsigned char*)ccg_ws(ctx, WS_SIL_SEG, bytes);
    if (!db) return CCG_ENOMEM;
    {
        const int rs = ccg_h2d_staged(ctx, db, hb.data(), bytes, st);  // (hb is freed when this call returns)
        if (rs) return rs;
    }
    const size_t po = (const unsigned char*)hptr - hb.data();
    SilSegs sgs;
    sgs.nseg = nseg;
    sgs.off = (const int64_t*)db;
    sgs.ts = (const int*)(db + 8 * n1);
    sgs.tw = sgs.ts + n1;
    sgs.lab = (const int32_t* const*)(db + po);
    sgs.mean = (double* const*)(db + po + 8 * (size_t)nseg);
    sgs.ncl = (int32_t* const*)(db + po + 16 * (size_t)nseg);
    sgs.mns = (int32_t* const*)(db + po + 24 * (size_t)nseg);
    // width partials per virtual labeling: 4 per 128-position tile of the largest segment
    const int nbw = 4 * (int)ccg_cdiv(mq_max, SIL_WT / 2);
    return sil_cells_run(ctx, x, m, d, nullptr, L, cmax, cell, ncell, nullptr, nullptr, nullptr, st, sgs, (int)ts,
                         (int)tw, nbw);
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
