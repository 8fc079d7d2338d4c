// Consumers of the co-clustering distance after the consensus clustering
// (SURVEY 8(f) row 2), computed from the assignment matrix without ever
// storing the N x N distance (the reference builds as.matrix(jaccardDist),
// 80 GB at 100k cells):
//   * determineHierachy(as.matrix(jaccardDist), f, return="distance")
//     (R/consensusClust.R:463, :585, :621, :699-721): the mean distance
//     between every pair of clusters = block means of D over the cluster
//     one-hot.  Accumulated EXACTLY: D = 1 - sim with sim = (float)co /
//     (float)both, and every such fp32 ratio is an integer multiple of 2^-39
//     (both <= 65535 puts a nonzero sim above 2^-16, so its ulp is >= 2^-39),
//     so sum(sim) is an integer sum of sim * 2^39 in 128-bit words --
//     associative, hence deterministic in any launch order.
//   * bluster::pairwiseRand(f[mask], A[, b][mask]) per bootstrap column
//     (:470-474): the contingency table of each column against f (the
//     O(N B) counting); the ratio formula on top is host arithmetic
//     (ccg_pairwise_rand_ratio).
#include <algorithm>
#include <cmath>

#include "ccg_internal.h"

#define HB_FIX_BITS 39
#define HB_KLDS 256                 // clusters held in LDS per wave
#define HB_SCRATCH_PAIRS (1LL << 30)  // co + both sub-slab: 4 GB

static inline int64_t hb_tri_off(int64_t N, int64_t i) { return i * N - i * (i + 1) / 2; }

__device__ __forceinline__ void hb_add_u128(unsigned long long* p, unsigned long long v) {
    const unsigned long long old = atomicAdd(p, v);
    if (old + v < old) atomicAdd(p + 1, 1ull);  // carry into the high word
}

// One wave per row i of the packed slab [a, b): pairs (i, j > i).  Per-wave
// LDS accumulators over the partner's cluster q, flushed once per row to the
// global [f_i][q] entries.
__global__ __launch_bounds__(256) void hb_rows_kernel(const uint16_t* __restrict__ co,
                                                      const uint16_t* __restrict__ both, int64_t N, int64_t a,
                                                      int64_t b, const int32_t* __restrict__ f, int K,
                                                      unsigned long long* __restrict__ simsum,
                                                      unsigned long long* __restrict__ npairs, int* __restrict__ err) {
    __shared__ unsigned long long ls[4][HB_KLDS];
    __shared__ unsigned int lc[4][HB_KLDS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t i = a + (int64_t)blockIdx.x * 4 + w;
    const bool lds = K <= HB_KLDS;
    if (lds)
        for (int c = lane; c < K; c += 64) {
            ls[w][c] = 0ull;
            lc[w][c] = 0u;
        }
    __syncthreads();
    int fi = -1;
    if (i < b) {
        fi = f[i];
        if (fi < 0 || fi >= K) {
            if (lane == 0) atomicOr(err, CCG_DERR_CLUSTER_INDEX);
            fi = -1;
        }
    }
    if (fi >= 0) {
        // element (i, j) of the slab lives at base + j
        const int64_t base = i * N - i * (i + 1) / 2 - (a * N - a * (a + 1) / 2) - i - 1;
        for (int64_t j = i + 1 + lane; j < N; j += 64) {
            const unsigned u = both[base + j];
            if (!u) continue;  // never co-sampled: NaN, dropped by na.rm
            const int q = f[j];
            if (q < 0 || q >= K) {
                atomicOr(err, CCG_DERR_CLUSTER_INDEX);
                continue;
            }
            const float s = (float)co[base + j] / (float)u;  // customDist's float division
            const unsigned long long fx = (unsigned long long)(s * 0x1p39f);  // exact
            if (lds) {
                atomicAdd(&ls[w][q], fx);
                atomicAdd(&lc[w][q], 1u);
            } else {
                hb_add_u128(&simsum[2 * ((int64_t)fi * K + q)], fx);
                atomicAdd(&npairs[(int64_t)fi * K + q], 1ull);
            }
        }
    }
    __syncthreads();
    if (fi >= 0 && lds)
        for (int c = lane; c < K; c += 64)
            if (lc[w][c]) {
                hb_add_u128(&simsum[2 * ((int64_t)fi * K + c)], ls[w][c]);
                atomicAdd(&npairs[(int64_t)fi * K + c], (unsigned long long)lc[w][c]);
            }
}

extern "C" int ccg_cluster_block_sums_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                                          const int32_t* f, int K, uint64_t* simsum, int64_t* npairs,
                                          void* stream) {
    CCG_REQUIRE(ctx && A && f && simsum && npairs, "ccg_cluster_block_sums_dev: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_cluster_block_sums_dev: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && N < (1LL << 24), "ccg_cluster_block_sums_dev: need 2 <= N < 2^24");
    CCG_REQUIRE(B >= 1 && B <= 65535, "ccg_cluster_block_sums_dev: B must be in [1, 65535]");
    CCG_REQUIRE(K >= 1 && K <= 65536, "ccg_cluster_block_sums_dev: need 1 <= K <= 65536");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    CCG_HIP(hipMemsetAsync(simsum, 0, sizeof(uint64_t) * 2 * K * K, st));
    CCG_HIP(hipMemsetAsync(npairs, 0, sizeof(int64_t) * K * K, st));
    // rows in sub-slabs of <= HB_SCRATCH_PAIRS packed pairs (row cuts on the
    // co-cluster tile grid)
    const int64_t RA = CCG_COCLUSTER_ROW_ALIGN;
    int64_t cap = 0;
    {
        int64_t a = 0;
        while (a < N) {
            int64_t b = std::min(N, a + RA);
            while (b < N && hb_tri_off(N, std::min(N, b + RA)) - hb_tri_off(N, a) <= HB_SCRATCH_PAIRS)
                b = std::min(N, b + RA);
            cap = std::max(cap, hb_tri_off(N, b) - hb_tri_off(N, a));
            a = b;
        }
    }
    uint16_t* scr = (uint16_t*)ccg_ws(ctx, WS_HIER, sizeof(uint16_t) * 2 * cap + 64);
    if (!scr) return CCG_ENOMEM;
    uint16_t *co = scr, *both = scr + cap;
    int64_t a = 0;
    while (a < N) {
        int64_t b = std::min(N, a + RA);
        while (b < N && hb_tri_off(N, std::min(N, b + RA)) - hb_tri_off(N, a) <= HB_SCRATCH_PAIRS)
            b = std::min(N, b + RA);
        int rc = ccg_cocluster_dev(ctx, A, label_bits, N, B, a, b, co, both, nullptr, st);
        if (rc) return rc;
        hb_rows_kernel<<<(unsigned)ccg_cdiv(b - a, 4), 256, 0, st>>>(co, both, N, a, b, f, K,
                                                                     (unsigned long long*)simsum,
                                                                     (unsigned long long*)npairs, ctx->d_err);
        CCG_HIP(hipGetLastError());
        a = b;
    }
    return CCG_OK;
}

// ------------------------------------------------------- contingency --
// tab[(b*K + p)*(C+1) + a] = #{i : f_i = p, A_bi = a}.  Grid (cell chunks,
// columns); per-block LDS table when K (C+1) fits, else global atomics.
#define HB_CT_LDS 12288
template <typename T>
__global__ __launch_bounds__(256) void hb_contingency_kernel(const T* __restrict__ A, int64_t N,
                                                             const int32_t* __restrict__ f, int K, int C,
                                                             int32_t* __restrict__ tab, int* __restrict__ err) {
    __shared__ int h[HB_CT_LDS];
    const int64_t b = blockIdx.y;
    const int W = K * (C + 1);
    const bool lds = W <= HB_CT_LDS;
    int32_t* out = tab + b * (int64_t)W;
    if (lds)
        for (int e = threadIdx.x; e < W; e += 256) h[e] = 0;
    __syncthreads();
    const T* col = A + b * N;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
        const int av = (int)col[i];
        const int p = f[i];
        if (av > C || p < 0 || p >= K) {
            atomicOr(err, av > C ? CCG_DERR_LABEL_RANGE : CCG_DERR_CLUSTER_INDEX);
            continue;
        }
        if (lds) atomicAdd(&h[p * (C + 1) + av], 1);
        else atomicAdd(&out[p * (C + 1) + av], 1);
    }
    if (!lds) return;
    __syncthreads();
    for (int e = threadIdx.x; e < W; e += 256)
        if (h[e]) atomicAdd(&out[e], h[e]);
}

extern "C" int ccg_contingency_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                                   const int32_t* f, int K, int C, int32_t* tab, void* stream) {
    CCG_REQUIRE(ctx && A && f && tab, "ccg_contingency_dev: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_contingency_dev: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 1 && N < (1LL << 31) && B >= 1 && B < 65536, "ccg_contingency_dev: bad sizes");
    CCG_REQUIRE(K >= 1 && C >= 0 && (int64_t)K * (C + 1) < (1LL << 31), "ccg_contingency_dev: bad K/C");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    CCG_HIP(hipMemsetAsync(tab, 0, sizeof(int32_t) * B * K * (C + 1), st));
    const dim3 g((unsigned)std::min<int64_t>(ccg_cdiv(N, 256 * 16), 128), (unsigned)B);
    if (label_bits == 8)
        hb_contingency_kernel<uint8_t><<<g, 256, 0, st>>>((const uint8_t*)A, N, f, K, C, tab, ctx->d_err);
    else
        hb_contingency_kernel<uint16_t><<<g, 256, 0, st>>>((const uint16_t*)A, N, f, K, C, tab, ctx->d_err);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------- host flavours --
extern "C" int ccg_cluster_block_sums(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                                      const int32_t* f, int K, uint64_t* simsum, int64_t* npairs) {
    CCG_REQUIRE(ctx && A && f && simsum && npairs, "ccg_cluster_block_sums: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_cluster_block_sums: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && B >= 1 && K >= 1, "ccg_cluster_block_sums: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t abytes = (size_t)(B * N) * (label_bits / 8);
    void* dA = ccg_ws(ctx, WS_HOST_A, abytes);
    int32_t* df = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * N);
    uint64_t* ds = (uint64_t*)ccg_ws(ctx, WS_HOST_C, sizeof(uint64_t) * 3 * K * K);
    if (!dA || !df || !ds) return CCG_ENOMEM;
    int64_t* dn = (int64_t*)(ds + 2 * K * K);
    CCG_HIP(hipMemcpyAsync(dA, A, abytes, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(df, f, sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    int rc = ccg_cluster_block_sums_dev(ctx, dA, label_bits, N, B, df, K, ds, dn, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(simsum, ds, sizeof(uint64_t) * 2 * K * K, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipMemcpyAsync(npairs, dn, sizeof(int64_t) * K * K, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return ccg_take_device_error(ctx);
}

extern "C" int ccg_contingency(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                               const int32_t* f, int K, int C, int32_t* tab) {
    CCG_REQUIRE(ctx && A && f && tab, "ccg_contingency: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_contingency: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 1 && B >= 1 && K >= 1 && C >= 0, "ccg_contingency: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t abytes = (size_t)(B * N) * (label_bits / 8);
    const size_t tbytes = sizeof(int32_t) * (size_t)(B * K * (C + 1));
    void* dA = ccg_ws(ctx, WS_HOST_A, abytes);
    int32_t* df = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * N);
    int32_t* dt = (int32_t*)ccg_ws(ctx, WS_HOST_C, tbytes);
    if (!dA || !df || !dt) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dA, A, abytes, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(df, f, sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    int rc = ccg_contingency_dev(ctx, dA, label_bits, N, B, df, K, C, dt, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(tab, dt, tbytes, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return ccg_take_device_error(ctx);
}

// ------------------------------------------------ host-only arithmetic --
extern "C" int ccg_cluster_block_means(int K, const uint64_t* simsum, const int64_t* npairs, double* out) {
    CCG_REQUIRE(K >= 1 && simsum && npairs && out, "ccg_cluster_block_means: bad arguments");
    for (int p = 0; p < K; ++p)
        for (int q = 0; q < K; ++q) {
            if (p == q) {
                out[(int64_t)p * K + q] = 0.0;  // never written by determineHierachy (:702-717)
                continue;
            }
            const int64_t pq = (int64_t)p * K + q, qp = (int64_t)q * K + p;
            unsigned __int128 s = ((unsigned __int128)simsum[2 * pq + 1] << 64) + simsum[2 * pq];
            s += ((unsigned __int128)simsum[2 * qp + 1] << 64) + simsum[2 * qp];
            const unsigned __int128 cnt = (unsigned __int128)(npairs[pq] + npairs[qp]);
            if (cnt == 0) {
                out[pq] = NAN;  // mean of an empty (all-NA) block
                continue;
            }
            // mean(D) = 1 - S / (cnt 2^39) = (cnt 2^39 - S) / (cnt 2^39)
            const unsigned __int128 den = cnt << HB_FIX_BITS;
            const unsigned __int128 num = den - s;
            out[pq] = (double)((long double)num / (long double)den);
        }
    return CCG_OK;
}

extern "C" int ccg_pairwise_rand_ratio(int K, int C, const int32_t* tab, int adjusted, double* out) {
    CCG_REQUIRE(K >= 1 && C >= 0 && tab && out, "ccg_pairwise_rand_ratio: bad arguments");
    // table(ref, alt) over the sampled cells: column 0 (unsampled) is masked
    // out as the reference subsets both vectors by clustAssignments != -1
    const int W = C + 1;
    auto c2 = [](double x) { return x * (x - 1.0) / 2.0; };
    double n = 0.0, same_alt = 0.0;
    for (int a = 1; a <= C; ++a) {
        double na = 0.0;
        for (int p = 0; p < K; ++p) na += tab[(int64_t)p * W + a];
        n += na;
        same_alt += c2(na);
    }
    const double p_same = n > 1.0 ? same_alt / c2(n) : NAN;
    for (int p = 0; p < K; ++p)
        for (int q = 0; q < K; ++q) {
            double np_ = 0.0, nq = 0.0, shared = 0.0;
            for (int a = 1; a <= C; ++a) {
                const double tp = tab[(int64_t)p * W + a], tq = tab[(int64_t)q * W + a];
                np_ += tp;
                nq += tq;
                shared += p == q ? c2(tp) : tp * tq;
            }
            double obs, tot, exp;
            if (p == q) {
                tot = c2(np_);
                obs = shared;
                exp = tot * p_same;
            } else {
                tot = np_ * nq;
                obs = tot - shared;
                exp = tot * (1.0 - p_same);
            }
            out[(int64_t)p * K + q] = adjusted ? (obs - exp) / (tot - exp) : obs / tot;
        }
    return CCG_OK;
}
