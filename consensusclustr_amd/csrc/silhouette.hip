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
// Grid: (row tiles of 256) x (groups of SIL_LG labelings); x rows are held in
// registers and reused across the group.
#include <math.h>

#include "ccg_internal.h"

#define SIL_T 256
#ifndef SIL_LG
#define SIL_LG 10
#endif

__device__ __forceinline__ int scale_exp(double bound) {
    // largest e with bound * 2^e <= 2^61
    if (!(bound > 0.0)) return 52;
    int e = 61 - (ilogb(bound) + 1);
    return e > 52 ? 52 : e;
}

__global__ __launch_bounds__(256) void sil_maxabs(const double* __restrict__ x, int64_t tot,
                                                  unsigned* __restrict__ bits) {
    __shared__ unsigned red[4];
    unsigned local = 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot;
         t += (int64_t)gridDim.x * blockDim.x) {
        float f = (float)fabs(x[t]);
        f = nextafterf(f, INFINITY);
        local = max(local, __float_as_uint(f));
    }
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

// K1: fixed-point cluster sums and counts, staged in LDS when (cmax + 1) x d
// accumulators fit (SIL_LDS_CAP), else added straight to the global sums.
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
    double xr[DMAX];
    load_row<DMAX>(x, in ? r : 0, d, xr);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double sc = ldexp(1.0, scale_exp(maxabs * (double)m));
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
                        const unsigned long long q = (unsigned long long)__double2ll_rn(xr[k] * sc);
                        if (LDS) atomicAdd(&acc[lab * d + k], q);
                        else atomicAdd(&gs[(int64_t)lab * d + k], q);
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

// K2: per labeling, the present codes (ascending = sort(unique(clusters)))
// and the centroids mu[l][c][0..DMAX) (zero padded) plus |mu_c|^2, from the
// fixed-point sums.  One block per labeling.
template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_mu(int64_t m, int d, int cmax,
                                                const unsigned* __restrict__ maxabs_bits,
                                                const unsigned long long* __restrict__ gsum,
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
        if (pc >= 0) mcl[(int64_t)pc * DMAX + k] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c <= cmax; c += SIL_T) {
        const int pc = pl[c];
        if (pc < 0) continue;
        double s = 0.0;
        for (int k = 0; k < d; ++k) s = fma(ml[(int64_t)c * DMAX + k], ml[(int64_t)c * DMAX + k], s);
        auxc[((int64_t)l * cmax + pc) * 2] = s;
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

// K5: widths and their fixed-point sum over non-NaN rows.  Each thread
// owns two rows (r and r + SIL_T of a 2*SIL_T-row tile) so that every
// centroid value read from LDS (a broadcast ds_read_b128 = 2 dims) feeds 4
// FMAs.  Squared distances to the other clusters use |x|^2 + |mu|^2 - 2 x.mu
// (one FMA per dimension), clamped at 0 (|error| ~ 1e-16 |x|^2, far inside
// the 1e-5 tolerance); the own-cluster distance, the one that can be ~0, is
// taken in the difference form.  D is monotone in s + v_c, so the minimum is
// taken on the squares and one sqrt applied at the end.
template <int DMAX>
__device__ __forceinline__ void sil_row_width(const double (&xr)[DMAX], double selfsq, double oth2, bool in,
                                              int np, double wsc, double* out_w, long long& wq, unsigned& wn) {
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
        wq += __double2ll_rn(w * wsc);
        wn += 1;
    }
}

// centroids per LDS stage of sil_width: [CH][DMAX] f64 + [CH][2] f64 + [CH] int within 64 KB
template <int DMAX>
constexpr int sil_chunk() {
    return DMAX <= 16 ? 256 : (DMAX <= 32 ? 224 : 112);
}

template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_width(const double* __restrict__ x, int64_t m, int d,
                                                   const int32_t* __restrict__ labels, int L, int cmax,
                                                   const int* __restrict__ npres,
                                                   const int* __restrict__ codes,
                                                   const int* __restrict__ pos,
                                                   const double* __restrict__ muc,
                                                   const double* __restrict__ auxc,
                                                   unsigned long long* __restrict__ wsum,
                                                   unsigned long long* __restrict__ wcnt,
                                                   double* __restrict__ out_width) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int CH = sil_chunk<DMAX>();          // centroids staged per pass
    double* smu = (double*)smem;                  // [CH][DMAX]
    double* sau = smu + (int64_t)CH * DMAX;       // [CH][2]
    int* scode = (int*)(sau + 2 * (int64_t)CH);   // [CH]
    const int64_t ra = (int64_t)blockIdx.x * (2 * SIL_T) + threadIdx.x, rb = ra + SIL_T;
    const bool ina = ra < m, inb = rb < m;
    double xa[DMAX], xb[DMAX];
    load_row<DMAX>(x, ina ? ra : 0, d, xa);
    load_row<DMAX>(x, inb ? rb : 0, d, xb);
    double xxa = 0.0, xxb = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
        xxa = fma(xa[k], xa[k], xxa);
        xxb = fma(xb[k], xb[k], xxb);
    }
    const double wsc = ldexp(1.0, scale_exp((double)m));
    const int l1 = min(L, (int)(blockIdx.y + 1) * SIL_LG);
    for (int l = blockIdx.y * SIL_LG; l < l1; ++l) {
        const int np = npres[l];
        const int laba = ina ? labels[(int64_t)l * m + ra] : 0;
        const int labb = inb ? labels[(int64_t)l * m + rb] : 0;
        const double* ml = muc + (int64_t)l * cmax * DMAX;
        const double* al = auxc + (int64_t)l * cmax * 2;
        double otha = INFINITY, othb = INFINITY;
        for (int p0 = 0; p0 < np; p0 += CH) {
            const int nc = min(CH, np - p0);
            for (int t = threadIdx.x; t < nc * DMAX; t += SIL_T) smu[t] = ml[(int64_t)p0 * DMAX + t];
            for (int t = threadIdx.x; t < 2 * nc; t += SIL_T) sau[t] = al[2 * (int64_t)p0 + t];
            for (int t = threadIdx.x; t < nc; t += SIL_T) scode[t] = codes[(int64_t)l * cmax + p0 + t];
            __syncthreads();
            for (int pi = 0; pi < nc; ++pi) {
                const double2* mc = reinterpret_cast<const double2*>(smu + pi * DMAX);
                double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
#pragma unroll
                for (int k2 = 0; k2 < DMAX / 2; ++k2) {
                    const double2 mv = mc[k2];
                    a0 = fma(xa[2 * k2], mv.x, a0);
                    a1 = fma(xa[2 * k2 + 1], mv.y, a1);
                    b0 = fma(xb[2 * k2], mv.x, b0);
                    b1 = fma(xb[2 * k2 + 1], mv.y, b1);
                }
                const double mm = sau[2 * pi], vc = sau[2 * pi + 1];
                const int c = scode[pi];
                const double sa = fmax(fma(-2.0, a0 + a1, xxa + mm), 0.0) + vc;
                const double sb = fmax(fma(-2.0, b0 + b1, xxb + mm), 0.0) + vc;
                if (c != laba && sa < otha) otha = sa;
                if (c != labb && sb < othb) othb = sb;
            }
            __syncthreads();  // before the next chunk (or labeling) overwrites the stage
        }
        // own cluster in the difference form: exact 0 for a singleton, as in R
        double selfa = INFINITY, selfb = INFINITY;
        if (ina && laba >= 1 && laba <= cmax) {
            const int p = pos[(int64_t)l * (cmax + 1) + laba];
            const double* mcp = ml + (int64_t)p * DMAX;
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < DMAX; ++k) {
                const double t = xa[k] - mcp[k];
                s = fma(t, t, s);
            }
            selfa = s + al[2 * (int64_t)p + 1];
        }
        if (inb && labb >= 1 && labb <= cmax) {
            const int p = pos[(int64_t)l * (cmax + 1) + labb];
            const double* mcp = ml + (int64_t)p * DMAX;
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < DMAX; ++k) {
                const double t = xb[k] - mcp[k];
                s = fma(t, t, s);
            }
            selfb = s + al[2 * (int64_t)p + 1];
        }
        long long wq = 0;
        unsigned wn = 0;
        sil_row_width<DMAX>(xa, selfa, otha, ina, np, wsc, out_width ? out_width + (int64_t)l * m + ra : nullptr,
                            wq, wn);
        sil_row_width<DMAX>(xb, selfb, othb, inb, np, wsc, out_width ? out_width + (int64_t)l * m + rb : nullptr,
                            wq, wn);
        // integer wave reduction (order-independent), one atomic per wave
        for (int o = 32; o > 0; o >>= 1) {
            wq += __shfl_xor(wq, o, 64);
            wn += __shfl_xor(wn, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (wq) atomicAdd(&wsum[l], (unsigned long long)wq);
            if (wn) atomicAdd(&wcnt[l], (unsigned long long)wn);
        }
    }
}

__global__ void sil_final(int64_t m, int L, int cmax, const unsigned long long* __restrict__ gcnt,
                          const unsigned long long* __restrict__ wsum,
                          const unsigned long long* __restrict__ wcnt, double* __restrict__ out_mean,
                          int32_t* __restrict__ out_nclust, int32_t* __restrict__ out_minsize) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= L) return;
    const unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
    int np = 0;
    long long mn = -1;
    for (int c = 1; c <= cmax; ++c)
        if (gc[c]) {
            ++np;
            if (mn < 0 || (long long)gc[c] < mn) mn = (long long)gc[c];
        }
    const double inv_wsc = ldexp(1.0, -scale_exp((double)m));
    const unsigned long long n = wcnt[l];
    if (out_mean) out_mean[l] = n ? ((double)(long long)wsum[l] * inv_wsc) / (double)n : NAN;
    if (out_nclust) out_nclust[l] = np;
    if (out_minsize) out_minsize[l] = (int32_t)(mn < 0 ? 0 : mn);
}

template <int DMAX>
static void sil_launch(const double* x, int64_t m, int d, const int32_t* labels, int L, int cmax,
                       unsigned* maxabs, unsigned long long* gsum, unsigned long long* gcnt,
                       unsigned long long* gvar, unsigned long long* wsum, unsigned long long* wcnt,
                       int* npres, int* codes, int* pos, double* mu, double* muc, double* auxc,
                       double* out_width, hipStream_t st) {
    dim3 grid((unsigned)ccg_cdiv(m, SIL_T), (unsigned)ccg_cdiv(L, SIL_LG));
    const size_t lds1 = (size_t)(cmax + 1) * d * 8 + (size_t)(cmax + 1) * 4;
    const size_t lds2 = (size_t)(cmax + 1) * DMAX * 8 + (size_t)(cmax + 1) * 8;
    if (lds1 <= SIL_LDS_CAP)
        sil_centroid<DMAX, true><<<grid, SIL_T, lds1, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt);
    else
        sil_centroid<DMAX, false><<<grid, SIL_T, 0, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt);
    sil_mu<DMAX><<<L, SIL_T, 0, st>>>(m, d, cmax, maxabs, gsum, gcnt, npres, codes, pos, mu, muc, auxc);
    if (lds2 <= SIL_LDS_CAP)
        sil_var<DMAX, true><<<grid, SIL_T, lds2, st>>>(x, m, d, labels, L, cmax, maxabs, mu, gvar);
    else
        sil_var<DMAX, false><<<grid, SIL_T, 0, st>>>(x, m, d, labels, L, cmax, maxabs, mu, gvar);
    sil_vfin<<<(unsigned)ccg_cdiv((int64_t)L * (cmax + 1), 256), 256, 0, st>>>(m, d, L, cmax, maxabs, gcnt,
                                                                                gvar, pos, auxc);
    dim3 grid2((unsigned)ccg_cdiv(m, 2 * SIL_T), (unsigned)ccg_cdiv(L, SIL_LG));
    constexpr int CH = sil_chunk<DMAX>();
    const size_t lds5 = (size_t)CH * DMAX * 8 + (size_t)CH * 16 + (size_t)CH * 4;
    sil_width<DMAX><<<grid2, SIL_T, lds5, st>>>(x, m, d, labels, L, cmax, npres, codes, pos, muc, auxc, wsum,
                                            wcnt, out_width);
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
    const int64_t words = (int64_t)L * nacc + 2 * (int64_t)L * (cmax + 1) + 2 * (int64_t)L + 8;
    unsigned long long* buf = (unsigned long long*)ccg_ws(ctx, WS_SIL_A, sizeof(unsigned long long) * words);
    if (!buf) return CCG_ENOMEM;
    unsigned long long* gsum = buf;
    unsigned long long* gcnt = gsum + (int64_t)L * nacc;
    unsigned long long* gvar = gcnt + (int64_t)L * (cmax + 1);
    unsigned long long* wsum = gvar + (int64_t)L * (cmax + 1);
    unsigned long long* wcnt = wsum + L;
    unsigned* maxabs = (unsigned*)(wcnt + L);
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
    const int t_all = ccg_timer_start(ctx, CCG_KT_SILHOUETTE, st);
    CCG_HIP(hipMemsetAsync(buf, 0, sizeof(unsigned long long) * words, st));
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 1024), 256), 256, 0, st>>>(x, m * d, maxabs);
    if (d <= 16)
        sil_launch<16>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc,
                        out_width, st);
    else if (d <= 32)
        sil_launch<32>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc,
                        out_width, st);
    else
        sil_launch<64>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, npres, codes, pos, mu, muc, auxc,
                        out_width, st);
    sil_final<<<(unsigned)ccg_cdiv(L, 64), 64, 0, st>>>(m, L, cmax, gcnt, wsum, wcnt, out_mean,
                                                       out_nclust, out_minsize);
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
