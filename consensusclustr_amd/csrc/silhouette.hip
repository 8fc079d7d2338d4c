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
#define SIL_LG 10

__device__ __forceinline__ int scale_exp(double bound) {
    // largest e with bound * 2^e <= 2^61
    if (!(bound > 0.0)) return 52;
    int e = 61 - (ilogb(bound) + 1);
    return e > 52 ? 52 : e;
}

__global__ void sil_maxabs(const double* __restrict__ x, int64_t tot, unsigned* __restrict__ bits) {
    unsigned local = 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot;
         t += (int64_t)gridDim.x * blockDim.x) {
        float f = (float)fabs(x[t]);
        f = nextafterf(f, INFINITY);
        local = max(local, __float_as_uint(f));
    }
    for (int o = 32; o > 0; o >>= 1) local = max(local, (unsigned)__shfl_xor((int)local, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(bits, local);
}

template <int DMAX>
__device__ __forceinline__ void load_row(const double* __restrict__ x, int64_t r, int d,
                                         double (&xr)[DMAX]) {
#pragma unroll
    for (int k = 0; k < DMAX; ++k) xr[k] = (k < d) ? x[r * d + k] : 0.0;
}

// K1: fixed-point cluster sums and counts.
template <int DMAX>
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
        for (int t = threadIdx.x; t < nacc; t += SIL_T) acc[t] = 0ull;
        for (int t = threadIdx.x; t <= cmax; t += SIL_T) cnt[t] = 0u;
        __syncthreads();
        if (in) {
            const int lab = labels[(int64_t)l * m + r];
            if (lab >= 1 && lab <= cmax) {
#pragma unroll
                for (int k = 0; k < DMAX; ++k)
                    if (k < d) atomicAdd(&acc[lab * d + k], (unsigned long long)__double2ll_rn(xr[k] * sc));
                atomicAdd(&cnt[lab], 1u);
            }
        }
        __syncthreads();
        unsigned long long* gs = gsum + (int64_t)l * nacc;
        unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
        for (int t = threadIdx.x; t < nacc; t += SIL_T)
            if (acc[t]) atomicAdd(&gs[t], acc[t]);
        for (int t = threadIdx.x; t <= cmax; t += SIL_T)
            if (cnt[t]) atomicAdd(&gc[t], (unsigned long long)cnt[t]);
        __syncthreads();
    }
}

// Centroids of labeling l into LDS (all codes 0..cmax).
__device__ __forceinline__ void load_centroids(double* mu, const unsigned long long* __restrict__ gsum,
                                               const unsigned long long* __restrict__ gcnt, int l,
                                               int cmax, int d, double inv_sc) {
    const int nacc = (cmax + 1) * d;
    const unsigned long long* gs = gsum + (int64_t)l * nacc;
    const unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
    for (int t = threadIdx.x; t < nacc; t += SIL_T) {
        const int c = t / d;
        const unsigned long long n = gc[c];
        mu[t] = n ? ((double)(long long)gs[t] * inv_sc) / (double)n : 0.0;
    }
}

// K2: fixed-point within-cluster sum of squared distances to the centroid.
template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_var(const double* __restrict__ x, int64_t m, int d,
                                                 const int32_t* __restrict__ labels, int L, int cmax,
                                                 const unsigned* __restrict__ maxabs_bits,
                                                 const unsigned long long* __restrict__ gsum,
                                                 const unsigned long long* __restrict__ gcnt,
                                                 unsigned long long* __restrict__ gvar) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* mu = (double*)smem;                                          // [cmax+1][d]
    unsigned long long* vacc = (unsigned long long*)(mu + (int64_t)(cmax + 1) * d);  // [cmax+1]
    const int64_t r = (int64_t)blockIdx.x * SIL_T + threadIdx.x;
    const bool in = r < m;
    double xr[DMAX];
    load_row<DMAX>(x, in ? r : 0, d, xr);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double inv_sc = ldexp(1.0, -scale_exp(maxabs * (double)m));
    const double vb = 4.0 * maxabs * maxabs * (double)d * (double)m;
    const double vsc = ldexp(1.0, scale_exp(vb));
    const int l1 = min(L, (int)(blockIdx.y + 1) * SIL_LG);
    for (int l = blockIdx.y * SIL_LG; l < l1; ++l) {
        load_centroids(mu, gsum, gcnt, l, cmax, d, inv_sc);
        for (int t = threadIdx.x; t <= cmax; t += SIL_T) vacc[t] = 0ull;
        __syncthreads();
        if (in) {
            const int lab = labels[(int64_t)l * m + r];
            if (lab >= 1 && lab <= cmax) {
                const double* mc = mu + lab * d;
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < DMAX; ++k)
                    if (k < d) {
                        const double t = xr[k] - mc[k];
                        s += t * t;
                    }
                atomicAdd(&vacc[lab], (unsigned long long)__double2ll_rn(s * vsc));
            }
        }
        __syncthreads();
        unsigned long long* gv = gvar + (int64_t)l * (cmax + 1);
        for (int t = threadIdx.x; t <= cmax; t += SIL_T)
            if (vacc[t]) atomicAdd(&gv[t], vacc[t]);
        __syncthreads();
    }
}

// K3: widths and their fixed-point sum over non-NaN rows.
template <int DMAX>
__global__ __launch_bounds__(SIL_T) void sil_width(const double* __restrict__ x, int64_t m, int d,
                                                   const int32_t* __restrict__ labels, int L, int cmax,
                                                   const unsigned* __restrict__ maxabs_bits,
                                                   const unsigned long long* __restrict__ gsum,
                                                   const unsigned long long* __restrict__ gcnt,
                                                   const unsigned long long* __restrict__ gvar,
                                                   unsigned long long* __restrict__ wsum,
                                                   unsigned long long* __restrict__ wcnt,
                                                   double* __restrict__ out_width) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* mu = (double*)smem;                                  // [npres][d]
    double* vv = mu + (int64_t)(cmax + 1) * d;                   // [npres]
    int* code = (int*)(vv + (cmax + 1));                         // [npres]
    int* npres_s = code + (cmax + 1);
    const int64_t r = (int64_t)blockIdx.x * SIL_T + threadIdx.x;
    const bool in = r < m;
    double xr[DMAX];
    load_row<DMAX>(x, in ? r : 0, d, xr);
    const double maxabs = (double)__uint_as_float(*maxabs_bits);
    const double inv_sc = ldexp(1.0, -scale_exp(maxabs * (double)m));
    const double vb = 4.0 * maxabs * maxabs * (double)d * (double)m;
    const double inv_vsc = ldexp(1.0, -scale_exp(vb));
    const double wsc = ldexp(1.0, scale_exp((double)m));
    const int l1 = min(L, (int)(blockIdx.y + 1) * SIL_LG);
    for (int l = blockIdx.y * SIL_LG; l < l1; ++l) {
        const unsigned long long* gs = gsum + (int64_t)l * (cmax + 1) * d;
        const unsigned long long* gc = gcnt + (int64_t)l * (cmax + 1);
        const unsigned long long* gv = gvar + (int64_t)l * (cmax + 1);
        if (threadIdx.x == 0) {
            int np = 0;
            for (int c = 1; c <= cmax; ++c)
                if (gc[c]) code[np++] = c;  // ascending = sort(unique(clusters))
            *npres_s = np;
        }
        __syncthreads();
        const int np = *npres_s;
        for (int t = threadIdx.x; t < np * d; t += SIL_T) {
            const int pi = t / d, k = t - pi * d;
            const int c = code[pi];
            mu[t] = ((double)(long long)gs[c * d + k] * inv_sc) / (double)gc[c];
        }
        for (int t = threadIdx.x; t < np; t += SIL_T) {
            const int c = code[t];
            vv[t] = ((double)gv[c] * inv_vsc) / (double)gc[c];
        }
        __syncthreads();
        long long wq = 0;
        unsigned wn = 0;
        if (in) {
            const int lab = labels[(int64_t)l * m + r];
            double selfd = INFINITY, othd = INFINITY;
            for (int pi = 0; pi < np; ++pi) {
                const double* mc = mu + pi * d;
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < DMAX; ++k)
                    if (k < d) {
                        const double t = xr[k] - mc[k];
                        s += t * t;
                    }
                const double Dc = sqrt(s + vv[pi]);
                if (code[pi] == lab) selfd = Dc;
                else if (Dc < othd) othd = Dc;
            }
            double w;
            if (np > 1) {
                double mx = fmax(othd, selfd);
                if (isnan(othd) || isnan(selfd)) mx = NAN;
                w = (othd - selfd) / mx;
            } else {
                w = 0.0;
            }
            if (out_width) out_width[(int64_t)l * m + r] = w;
            if (!isnan(w)) {
                wq = __double2ll_rn(w * wsc);
                wn = 1;
            }
        }
        // integer wave reduction (order-independent), one atomic per wave
        for (int o = 32; o > 0; o >>= 1) {
            wq += __shfl_xor(wq, o, 64);
            wn += __shfl_xor(wn, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (wq) atomicAdd(&wsum[l], (unsigned long long)wq);
            if (wn) atomicAdd(&wcnt[l], (unsigned long long)wn);
        }
        __syncthreads();
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
                       double* out_width, hipStream_t st) {
    dim3 grid((unsigned)ccg_cdiv(m, SIL_T), (unsigned)ccg_cdiv(L, SIL_LG));
    size_t lds1 = (size_t)(cmax + 1) * d * 8 + (size_t)(cmax + 1) * 4;
    size_t lds2 = (size_t)(cmax + 1) * d * 8 + (size_t)(cmax + 1) * 8;
    size_t lds3 = (size_t)(cmax + 1) * d * 8 + (size_t)(cmax + 1) * 8 + (size_t)(cmax + 2) * 4;
    sil_centroid<DMAX><<<grid, SIL_T, lds1, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt);
    sil_var<DMAX><<<grid, SIL_T, lds2, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar);
    sil_width<DMAX><<<grid, SIL_T, lds3, st>>>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar,
                                               wsum, wcnt, out_width);
}

extern "C" int ccg_silhouette_dev(ccg_ctx* ctx, const double* x, int64_t m, int d,
                                  const int32_t* labels, int L, int cmax, double* out_mean,
                                  int32_t* out_nclust, int32_t* out_minsize, double* out_width,
                                  void* stream) {
    CCG_REQUIRE(ctx && x && labels, "ccg_silhouette_dev: NULL argument");
    CCG_REQUIRE(m >= 1 && m < (1LL << 31) && d >= 1 && d <= 64 && L >= 1,
                "ccg_silhouette_dev: bad sizes m=%lld d=%d L=%d", (long long)m, d, L);
    CCG_REQUIRE(cmax >= 1 && cmax <= 256, "ccg_silhouette_dev: cmax=%d must be in [1, 256]", cmax);
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
    const int t_all = ccg_timer_start(ctx, CCG_KT_SILHOUETTE, st);
    CCG_HIP(hipMemsetAsync(buf, 0, sizeof(unsigned long long) * words, st));
    sil_maxabs<<<(unsigned)std::min<int64_t>(ccg_cdiv(m * d, 256), 1024), 256, 0, st>>>(x, m * d, maxabs);
    if (d <= 16)
        sil_launch<16>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, out_width, st);
    else if (d <= 32)
        sil_launch<32>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, out_width, st);
    else
        sil_launch<64>(x, m, d, labels, L, cmax, maxabs, gsum, gcnt, gvar, wsum, wcnt, out_width, st);
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
