// Shared-nearest-neighbour graphs on gfx950.
//
// Reference path: bluster::neighborsToSNNGraph(index, type="number") inside
// SNNGraphParam (R/consensusClust.R:656-658) and type="rank" on the
// consensus kNN (:426); bluster's C++ build_snn_number / build_snn_rank.
//
// For node j, every shared member s of N+(j) = {j} u knn(j) contributes to
// the partners p with s in N+(p), i.e. p in {s} u hosts(s) where hosts(s)
// lists the nodes that have s as a neighbour (with s's 1-based rank there).
// NUMBER counts the shared members; RANK keeps min(rank_j(s) + rank_p(s)).
// Each undirected edge is emitted by its smaller endpoint, so node j keeps
// partners p > j only.  One wave per node gathers (p, value) keys into LDS,
// bitonic-sorts them and reduces runs.  Two passes (count, emit) give a
// deterministic, (i, j)-sorted edge list without scratch memory; nodes whose
// gathered list exceeds the LDS capacity take an exact O(n) dense path.
#include <algorithm>

#include "ccg_internal.h"

// Compiler-only barrier: LDS operations of one wave execute in order.
#define WAVE_LDS_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)

#define SNN_CAP 1024        // LDS keys per wave
#define SNN_WAVES 4
#define SNN_DENSE_BLOCKS 64 // concurrent overflow nodes

__global__ void snn_count_hosts(const int32_t* __restrict__ knn, int64_t n, int kstride, int k,
                                unsigned long long* __restrict__ hcnt, int* __restrict__ err) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * k) return;
    int64_t h = t / k;
    int r = (int)(t - h * k);
    int32_t x = knn[h * kstride + r];
    if (x < 0 || x >= n || x == h) {
        atomicOr(err, 1);
        return;
    }
    atomicAdd(&hcnt[x], 1ull);
}

__global__ void snn_fill_hosts(const int32_t* __restrict__ knn, int64_t n, int kstride, int k,
                               unsigned long long* __restrict__ cursor, int2* __restrict__ hosts) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * k) return;
    int64_t h = t / k;
    int r = (int)(t - h * k);
    int32_t x = knn[h * kstride + r];
    if (x < 0 || x >= n || x == h) return;
    unsigned long long p = atomicAdd(&cursor[x], 1ull);
    hosts[p] = make_int2((int)h, r + 1);
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Gather node j's partner keys (p << 32 | value), p > j, into lds.
// Returns the (wave-uniform) number of keys; > SNN_CAP means overflow.
__device__ int snn_gather(int64_t j, const int32_t* __restrict__ knn, int kstride, int k,
                          const int64_t* __restrict__ hoff, const int2* __restrict__ hosts,
                          unsigned long long* lds) {
    const int lane = threadIdx.x & 63;
    int pos = 0;
    for (int i = 0; i <= k; ++i) {
        const int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
        const int64_t h0 = hoff[cur];
        const int64_t len = hoff[cur + 1] - h0 + 1;  // hosts + cur itself
        for (int64_t o0 = 0; o0 < len; o0 += 64) {
            const int64_t o = o0 + lane;
            bool keep = false;
            unsigned long long key = 0;
            if (o < len) {
                int p, val;
                if (o == len - 1) {
                    p = cur;
                    val = i;
                } else {
                    int2 hr = hosts[h0 + o];
                    p = hr.x;
                    val = hr.y + i;
                }
                keep = p > j;
                key = ((unsigned long long)(unsigned)p << 32) | (unsigned)val;
            }
            const unsigned long long m = __ballot(keep);
            const int pre = __popcll(m & lanemask_lt());
            if (keep && pos + pre < SNN_CAP) lds[pos + pre] = key;
            pos += __popcll(m);
        }
    }
    return pos;
}

__device__ void wave_sort_lds(unsigned long long* lds, int cnt) {
    const int lane = threadIdx.x & 63;
    int P = 64;
    while (P < cnt) P <<= 1;
    for (int i = cnt + lane; i < P; i += 64) lds[i] = ~0ull;
    WAVE_LDS_SYNC();
    for (int kk = 2; kk <= P; kk <<= 1) {
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            for (int i = lane; i < P; i += 64) {
                int l = i ^ jj;
                if (l > i) {
                    unsigned long long a = lds[i], b = lds[l];
                    bool up = (i & kk) == 0;
                    if ((a > b) == up) {
                        lds[i] = b;
                        lds[l] = a;
                    }
                }
            }
            WAVE_LDS_SYNC();
        }
    }
}

// Reduce sorted runs.  emit == false: returns the number of runs.
// emit == true: writes edges (j, p, w) starting at out index `base`.
__device__ int64_t snn_reduce_runs(const unsigned long long* lds, int cnt, int64_t j, int k,
                                   int type, bool emit, int64_t base, int64_t cap,
                                   int32_t* __restrict__ oi, int32_t* __restrict__ oj,
                                   double* __restrict__ ow) {
    const int lane = threadIdx.x & 63;
    int64_t runs = 0;
    int carry_start = 0;
    for (int c0 = 0; c0 < cnt; c0 += 64) {
        const int i = c0 + lane;
        const bool in = i < cnt;
        unsigned long long key = in ? lds[i] : ~0ull;
        const unsigned p = (unsigned)(key >> 32);
        const bool start = in && (i == 0 || (unsigned)(lds[i - 1] >> 32) != p);
        const bool last = in && (i == cnt - 1 || (unsigned)(lds[i + 1] >> 32) != p);
        const unsigned long long sm = __ballot(start);
        if (emit) {
            // run start for this position: inclusive prefix max over lanes
            int rs = start ? i : -1;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                int y = __shfl_up(rs, o, 64);
                if (lane >= o) rs = max(rs, y);
            }
            if (rs < 0) rs = carry_start;
            const int64_t rid = runs + __popcll(sm & (lanemask_lt() | (1ull << lane))) - 1;
            if (last) {
                const int64_t e = base + rid;
                if (e < cap) {
                    double w;
                    if (type == CCG_SNN_NUMBER) {
                        w = (double)(i - rs + 1);
                    } else {
                        const unsigned mn = (unsigned)(lds[rs] & 0xffffffffu);
                        w = (double)k - 0.5 * (double)mn;
                        w = w < 1e-6 ? 1e-6 : w;
                    }
                    oi[e] = (int32_t)j;
                    oj[e] = (int32_t)p;
                    ow[e] = w;
                }
            }
            // carry: last run start seen in this chunk
            int cs = start ? i : -1;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) cs = max(cs, __shfl_xor(cs, o, 64));
            if (cs >= 0) carry_start = cs;
        }
        runs += __popcll(sm);
    }
    return runs;
}

// Pass 1 (emit=false): cnt[j] = #partners > j, overflow nodes appended to ov.
// Pass 2 (emit=true): write edges at eoff[j].
template <bool EMIT>
__global__ __launch_bounds__(64 * SNN_WAVES) void snn_node_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, int k, int type,
    const int64_t* __restrict__ hoff, const int2* __restrict__ hosts,
    int64_t* __restrict__ cnt_or_off, int* __restrict__ ov_list, int* __restrict__ ov_count,
    int64_t cap, int32_t* __restrict__ oi, int32_t* __restrict__ oj, double* __restrict__ ow) {
    __shared__ unsigned long long lds_all[SNN_WAVES][SNN_CAP];
    const int wv = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    unsigned long long* lds = lds_all[wv];
    for (int64_t j = (int64_t)blockIdx.x * SNN_WAVES + wv; j < n; j += (int64_t)gridDim.x * SNN_WAVES) {
        const int c = snn_gather(j, knn, kstride, k, hoff, hosts, lds);
        if (c > SNN_CAP) {
            if (!EMIT && lane == 0) {
                int p = atomicAdd(ov_count, 1);
                ov_list[p] = (int)j;
            }
            continue;  // dense path handles this node in both passes
        }
        WAVE_LDS_SYNC();
        wave_sort_lds(lds, c);
        if (!EMIT) {
            int64_t r = snn_reduce_runs(lds, c, j, k, type, false, 0, 0, oi, oj, ow);
            if (lane == 0) cnt_or_off[j] = r;
        } else {
            snn_reduce_runs(lds, c, j, k, type, true, cnt_or_off[j], cap, oi, oj, ow);
        }
        WAVE_LDS_SYNC();
    }
}

// Dense path for overflow nodes: one block per node, dense int array of n.
template <bool EMIT>
__global__ __launch_bounds__(256) void snn_dense_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, int k, int type,
    const int64_t* __restrict__ hoff, const int2* __restrict__ hosts,
    const int* __restrict__ ov_list, const int* __restrict__ ov_count, int* __restrict__ dense_all,
    int64_t* __restrict__ cnt_or_off, int64_t cap, int32_t* __restrict__ oi,
    int32_t* __restrict__ oj, double* __restrict__ ow) {
    __shared__ int64_t wsum[4];
    int* dense = dense_all + (int64_t)blockIdx.x * n;
    const int nov = *ov_count;
    const int EMPTY = (type == CCG_SNN_NUMBER) ? 0 : 0x7fffffff;
    for (int f = blockIdx.x; f < nov; f += gridDim.x) {
        const int64_t j = ov_list[f];
        for (int64_t p = j + 1 + threadIdx.x; p < n; p += 256)
            __hip_atomic_store(&dense[p], EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (int i = 0; i <= k; ++i) {
            const int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
            const int64_t h0 = hoff[cur];
            const int64_t len = hoff[cur + 1] - h0 + 1;
            for (int64_t o = threadIdx.x; o < len; o += 256) {
                int p, val;
                if (o == len - 1) {
                    p = cur;
                    val = i;
                } else {
                    int2 hr = hosts[h0 + o];
                    p = hr.x;
                    val = hr.y + i;
                }
                if (p > j) {
                    if (type == CCG_SNN_NUMBER) atomicAdd(&dense[p], 1);
                    else atomicMin(&dense[p], val);
                }
            }
        }
        __syncthreads();
        int64_t base = EMIT ? cnt_or_off[j] : 0;
        int64_t total = 0;
        for (int64_t p0 = j + 1; p0 < n; p0 += 256) {
            const int64_t p = p0 + threadIdx.x;
            const int v = (p < n) ? __hip_atomic_load(&dense[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : EMPTY;
            const bool hit = v != EMPTY;
            const unsigned long long m = __ballot(hit);
            const int wv = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) wsum[wv] = __popcll(m);
            __syncthreads();
            int64_t before = 0, tot = 0;
            for (int w = 0; w < 4; ++w) {
                if (w < wv) before += wsum[w];
                tot += wsum[w];
            }
            if (EMIT && hit) {
                const int64_t e = base + total + before + __popcll(m & lanemask_lt());
                if (e < cap) {
                    double w;
                    if (type == CCG_SNN_NUMBER) w = (double)v;
                    else {
                        w = (double)k - 0.5 * (double)v;
                        w = w < 1e-6 ? 1e-6 : w;
                    }
                    oi[e] = (int32_t)j;
                    oj[e] = (int32_t)p;
                    ow[e] = w;
                }
            }
            total += tot;
            __syncthreads();
        }
        if (!EMIT && threadIdx.x == 0) cnt_or_off[j] = total;
        __syncthreads();
    }
}

__global__ void snn_copy_total(const int64_t* __restrict__ off, int64_t n, int64_t* __restrict__ dst) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *dst = off[n];
}

extern "C" int ccg_snn_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, int k,
                           int type, int32_t* out_i, int32_t* out_j, double* out_w, int64_t cap,
                           int64_t* d_nedges, void* stream) {
    CCG_REQUIRE(ctx && knn && d_nedges, "ccg_snn_dev: NULL argument");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31), "ccg_snn_dev: bad n");
    CCG_REQUIRE(k >= 1 && k <= kstride, "ccg_snn_dev: need 1 <= k <= kstride");
    CCG_REQUIRE(type == CCG_SNN_NUMBER || type == CCG_SNN_RANK, "ccg_snn_dev: bad type");
    CCG_REQUIRE(cap == 0 || (out_i && out_j && out_w), "ccg_snn_dev: NULL outputs with cap > 0");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    // layout of WS_SNN_A: hcnt/hoff [n+1] i64 | cursor [n+1] i64 | misc
    int64_t* hoff = (int64_t*)ccg_ws(ctx, WS_SNN_A, sizeof(int64_t) * (2 * (n + 1) + 16));
    int2* hosts = (int2*)ccg_ws(ctx, WS_SNN_B, sizeof(int2) * (n * k + 1));
    int64_t* cnt = (int64_t*)ccg_ws(ctx, WS_SNN_C, sizeof(int64_t) * (n + 1));
    int* ov = (int*)ccg_ws(ctx, WS_SNN_E, sizeof(int) * (n + 16));
    int* dense = (int*)ccg_ws(ctx, WS_SNN_D, sizeof(int) * n * SNN_DENSE_BLOCKS);
    if (!hoff || !hosts || !cnt || !ov || !dense) return CCG_ENOMEM;
    unsigned long long* cursor = (unsigned long long*)(hoff + (n + 1));
    int* err = (int*)(hoff + 2 * (n + 1));
    int* ov_count = ov + n;
    const int64_t nk = n * k;
    const int t_all = ccg_timer_start(ctx, CCG_KT_SNN, st);
    CCG_HIP(hipMemsetAsync(hoff, 0, sizeof(int64_t) * (n + 1) + 0, st));
    CCG_HIP(hipMemsetAsync(err, 0, sizeof(int) * 4, st));
    CCG_HIP(hipMemsetAsync(ov_count, 0, sizeof(int), st));
    snn_count_hosts<<<(unsigned)ccg_cdiv(nk, 256), 256, 0, st>>>(knn, n, kstride, k,
                                                                 (unsigned long long*)hoff, err);
    int rc = ccg_scan_i64(ctx, hoff, hoff, n, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(cursor, hoff, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, st));
    snn_fill_hosts<<<(unsigned)ccg_cdiv(nk, 256), 256, 0, st>>>(knn, n, kstride, k, cursor, hosts);
    const unsigned nblk = (unsigned)std::min<int64_t>(ccg_cdiv(n, SNN_WAVES), 8192);
    snn_node_kernel<false><<<nblk, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, k, type, hoff, hosts,
                                                           cnt, ov, ov_count, 0, out_i, out_j, out_w);
    snn_dense_kernel<false><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, k, type, hoff, hosts,
                                                             ov, ov_count, dense, cnt, 0, out_i,
                                                             out_j, out_w);
    rc = ccg_scan_i64(ctx, cnt, cnt, n, st);
    if (rc) return rc;
    if (cap > 0) {
        snn_node_kernel<true><<<nblk, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, k, type, hoff, hosts,
                                                              cnt, ov, ov_count, cap, out_i, out_j,
                                                              out_w);
        snn_dense_kernel<true><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, k, type, hoff,
                                                                hosts, ov, ov_count, dense, cnt, cap,
                                                                out_i, out_j, out_w);
    }
    snn_copy_total<<<1, 64, 0, st>>>(cnt, n, d_nedges);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_snn(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, int k, int type,
                       int32_t* out_i, int32_t* out_j, double* out_w, int64_t cap,
                       int64_t* nedges) {
    CCG_REQUIRE(ctx && knn && nedges, "ccg_snn: NULL argument");
    CCG_REQUIRE(n >= 1 && kstride >= 1, "ccg_snn: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    for (int64_t t = 0; t < n * kstride; ++t)
        CCG_REQUIRE(knn[t] >= 0 && knn[t] < n && knn[t] != t / kstride,
                    "ccg_snn: neighbour index out of range or self at %lld", (long long)t);
    int32_t* dknn = (int32_t*)ccg_ws(ctx, WS_HOST_A, sizeof(int32_t) * n * kstride);
    int64_t* dne = (int64_t*)ccg_ws(ctx, WS_HOST_E, 64);
    int32_t* di = cap > 0 ? (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * cap) : nullptr;
    int32_t* dj = cap > 0 ? (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * cap) : nullptr;
    double* dw = cap > 0 ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * cap) : nullptr;
    if (!dknn || !dne || (cap > 0 && (!di || !dj || !dw))) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dknn, knn, sizeof(int32_t) * n * kstride, hipMemcpyHostToDevice, st));
    int rc = ccg_snn_dev(ctx, dknn, n, kstride, k, type, di, dj, dw, cap, dne, st);
    if (rc) return rc;
    int64_t ne = 0;
    CCG_HIP(hipMemcpyAsync(&ne, dne, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    *nedges = ne;
    if (ne > cap) {
        ccg_set_error("ccg_snn: capacity %lld < required %lld edges", (long long)cap, (long long)ne);
        return CCG_ECAP;
    }
    if (ne > 0) {
        CCG_HIP(hipMemcpyAsync(out_i, di, sizeof(int32_t) * ne, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipMemcpyAsync(out_j, dj, sizeof(int32_t) * ne, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipMemcpyAsync(out_w, dw, sizeof(double) * ne, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
    }
    return CCG_OK;
}
