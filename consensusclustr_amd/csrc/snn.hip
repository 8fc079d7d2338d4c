// Shared-nearest-neighbour graphs on gfx950.
//
// Reference path: bluster::neighborsToSNNGraph(index, type="number") inside
// SNNGraphParam (R/consensusClust.R:656-658) for each k of kNum (:653), and
// type="rank" on the consensus kNN (:426); bluster's C++ build_snn_number /
// build_snn_rank.
//
// For node j, every member s of N+(j) = {j} u knn(j) is shared with each
// partner p in {s} u hosts(s) (hosts(s) = nodes listing s as a neighbour).
// NUMBER counts shared members; RANK keeps min(rank_j(s) + rank_p(s)), self
// rank 0.  Because the k-lists are prefixes of the kmax list, one pass over
// the kmax graph serves every k in kNum: a shared member with ranks
// (rj, rp) belongs to graph k iff max(rj, rp) <= k.  Per graph t the value
// lives in byte t of a 32-bit word (counts <= 33, rank sums <= 64).
//
// Pipeline (every step deterministic):
//   1. host lists: the kNN entries radix-sorted (stable) by neighbour, so
//      every hosts(s) is in ascending host order; back-pointers bp (where h
//      sits in hosts(knn[h][r])) and split[x] (hosts of x below x).
//   2. capacity: per node the number M_j of (partner, member) items with
//      partner p > j; a scan gives every node a row of M_j slots.
//   3. build: the items of a node are gathered, sorted by partner and
//      merged (sum for NUMBER, bytewise min for RANK) into the node's row of
//      (partner, packed per-graph values), ascending partner -- the union
//      graph (the largest k) in CSR form with per-graph counts.  Tiers by
//      size: a register bitonic sort, one wave per node (<= 2048 items) or
//      one 4-wave block per hub node (<= 4096); a 16K-slot block hash table;
//      an exact O(n) dense pass.
//   4. per-graph edge lists (i < j sorted by (i, j)) are streamed from the
//      rows when the caller wants them (ccg_snn_multi_dev).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ccg_internal.h"

#define WAVE_LDS_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)

#define SNN_MAXK 4           // graphs per pass (|kNum| <= 4)
#define SNN_WAVES 4          // waves per block in the wave kernels
#define SNN_BT 16384         // block table slots (overflow path)
#define SNN_DENSE_BLOCKS 64  // concurrent dense-path nodes
#define SNN_EMPTY (-1)
#define SNN_BITONIC_MAX 4096  // items of the largest bitonic-tier node

struct SnnSpec {
    int nk;
    int kk[SNN_MAXK];  // ascending
    int type;
    unsigned init;     // empty value word (0 for NUMBER, 0xFFFFFFFF for RANK)
};

// Per-graph edge outputs (ccg_snn_multi_dev).
struct SnnOut {
    int32_t* oi[SNN_MAXK];
    int32_t* oj[SNN_MAXK];
    double* ow[SNN_MAXK];
    int64_t cap[SNN_MAXK];
};

// Node rows: row j = [roff[j], roff[j] + rlen[j]) of (nbr, wpk), capacity
// roff[j+1] - roff[j]; written only when roff[n] <= cap.
struct SnnRows {
    const int64_t* roff;
    int32_t* rlen;
    int32_t* nbr;
    uint32_t* wpk;
    int64_t cap;
};

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Contribution of one shared member with ranks (rj, rp) to the packed word
// (branch-free: byte t is live iff max(rj, rp) <= kk[t]).
__device__ __forceinline__ unsigned snn_contrib(const SnnSpec& sp, int rj, int rp) {
    const int m = rj > rp ? rj : rp;
    unsigned live = 0;
#pragma unroll
    for (int t = 0; t < SNN_MAXK; ++t) live |= (t < sp.nk && m <= sp.kk[t]) ? (0xFFu << (8 * t)) : 0u;
    const unsigned num = live & 0x01010101u;
    const unsigned rank = (((unsigned)(rj + rp) * 0x01010101u) & live) | ~live;
    return sp.type == CCG_SNN_NUMBER ? num : rank;
}

__device__ __forceinline__ unsigned bytewise_min(unsigned a, unsigned b) {
    unsigned r = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const unsigned x = (a >> (8 * t)) & 0xFFu, y = (b >> (8 * t)) & 0xFFu;
        r |= (x < y ? x : y) << (8 * t);
    }
    return r;
}

__device__ __forceinline__ unsigned snn_combine(int type, unsigned a, unsigned b) {
    return type == CCG_SNN_NUMBER ? a + b : bytewise_min(a, b);  // per-byte counts never carry
}

template <typename V>
__device__ __forceinline__ void snn_update(const SnnSpec& sp, V* v, unsigned c) {
    if (sp.type == CCG_SNN_NUMBER) {
        atomicAdd(v, c);
    } else {
        unsigned old = __hip_atomic_load(v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            const unsigned nw = bytewise_min(old, c);
            if (nw == old) break;
            const unsigned prev = atomicCAS(v, old, nw);
            if (prev == old) break;
            old = prev;
        }
    }
}

__device__ __forceinline__ unsigned snn_hash(int p, int bits) {
    return ((unsigned)p * 2654435761u) >> (32 - bits);
}

__device__ __forceinline__ bool graph_has(const SnnSpec& sp, unsigned v, int t) {
    const unsigned b = (v >> (8 * t)) & 0xFFu;
    return sp.type == CCG_SNN_NUMBER ? b != 0u : b != 0xFFu;
}

__device__ __forceinline__ double graph_weight(const SnnSpec& sp, unsigned v, int t) {
    const unsigned b = (v >> (8 * t)) & 0xFFu;
    if (sp.type == CCG_SNN_NUMBER) return (double)b;
    double w = (double)sp.kk[t] - 0.5 * (double)b;
    return w < 1e-6 ? 1e-6 : w;
}

// --------------------------------------------------------- host lists --
// Entry t = h*kmax + r of the kNN (h lists x at rank r+1) becomes the pair
// (x, t); invalid neighbours (out of range, self) get key n, sort to the end
// and raise CCG_DERR_SNN_INDEX.
__global__ void snn_pairs_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride, int kmax,
                                 int32_t* __restrict__ keys, int32_t* __restrict__ vals, int* __restrict__ err) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kmax) return;
    const int64_t h = t / kmax;
    const int r = (int)(t - h * kmax);
    const int32_t x = knn[h * kstride + r];
    const bool ok = x >= 0 && x < n && x != h;
    if (!ok) atomicOr(err, CCG_DERR_SNN_INDEX);
    keys[t] = ok ? x : (int32_t)n;
    vals[t] = (int32_t)t;
}

// hoff[x] = first sorted position with key >= x (x = 0..n).
__global__ void snn_hoff_kernel(const int32_t* __restrict__ skey, int64_t total, int64_t n,
                                int64_t* __restrict__ hoff) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x > n) return;
    int64_t lo = 0, hi = total;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (skey[mid] < x) lo = mid + 1; else hi = mid;
    }
    hoff[x] = lo;
}

// hosts_s[p] = (host, rank); bp[t] = position of the host in its list.
__global__ void snn_hosts_kernel(const int32_t* __restrict__ skey, const int32_t* __restrict__ sval, int kmax,
                                 const int64_t* __restrict__ hoff, int64_t n, int2* __restrict__ hosts_s,
                                 int* __restrict__ bp) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= hoff[n]) return;
    const int32_t x = skey[p], t = sval[p];
    const int h = t / kmax, r = t - h * kmax;
    hosts_s[p] = make_int2(h, r + 1);
    bp[t] = (int)(p - hoff[x]);
}

// split[x] = number of hosts of x below x (hosts are ascending).
__global__ void snn_split_kernel(const int64_t* __restrict__ hoff, const int2* __restrict__ hosts_s, int64_t n,
                                 int* __restrict__ split) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    int64_t lo = hoff[x], hi = hoff[x + 1];
    const int64_t base = lo;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (hosts_s[mid].x < x) lo = mid + 1; else hi = mid;
    }
    split[x] = (int)(lo - base);
}

// ------------------------------------------------------------- members --
// Member i of node j (lane i <= kmax): i = 0 is j itself, starting at its
// first host above j; i >= 1 is s = knn[j][i-1], starting at the entry
// after j in hosts(s), plus s itself (rank 0) when s > j.  Items are the
// partners p > j only.
struct SnnMember {
    int cur;
    int len;
    long long h0, hend;
};

__device__ __forceinline__ SnnMember snn_member(const int32_t* __restrict__ knn, int64_t n, int kstride, int kmax,
                                                int64_t j, int lane, const int64_t* __restrict__ hoff,
                                                const int* __restrict__ bp, const int* __restrict__ split) {
    SnnMember m{0, 0, 0, 0};
    if (lane > kmax) return m;
    if (lane == 0) {
        m.cur = (int)j;
        m.h0 = hoff[j] + split[j];
        m.hend = hoff[j + 1];
        m.len = (int)(m.hend - m.h0);
    } else {
        const int c = knn[j * kstride + lane - 1];
        if ((unsigned)c < (unsigned)n && c != j) {
            const int q = bp[j * kmax + lane - 1];
            m.cur = c;
            m.h0 = hoff[c] + q + 1;
            m.hend = hoff[c + 1];
            m.len = (int)(m.hend - m.h0) + (c > j ? 1 : 0);
        } else {
            m.cur = (int)j;  // invalid input (reported via CCG_DERR_SNN_INDEX): no items
        }
    }
    return m;
}

// Items M_j of every node: the row capacities.  kmax <= 31 (PACK): two nodes
// per wave, one per 32-lane half (members in lanes 0..kmax of the half).
template <bool PACK>
__global__ __launch_bounds__(256) void snn_items_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        int kmax, const int64_t* __restrict__ hoff,
                                                        const int* __restrict__ bp, const int* __restrict__ split,
                                                        int64_t* __restrict__ cap) {
    constexpr int WL = PACK ? 32 : 64;  // lanes per node
    constexpr int NPW = 64 / WL;        // nodes per wave
    const int lane = threadIdx.x & (WL - 1);
    const int64_t stride = (int64_t)gridDim.x * 4 * NPW;
    for (int64_t jb = (int64_t)blockIdx.x * 4 * NPW; jb < n; jb += stride) {
        const int64_t j = jb + (threadIdx.x / WL);
        SnnMember m{0, 0, 0, 0};
        if (j < n) m = snn_member(knn, n, kstride, kmax, j, lane, hoff, bp, split);
        int v = m.len;
        for (int o = WL / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WL);
        if (lane == 0 && j < n) cap[j] = v;
    }
}

// Write the per-graph counts of a finished row.
__device__ __forceinline__ void snn_row_counts(const SnnSpec& sp, int64_t (&c4)[SNN_MAXK], int64_t n, int64_t j,
                                               int lane, int64_t* __restrict__ cnt) {
#pragma unroll
    for (int t = 0; t < SNN_MAXK; ++t) {
        int64_t v = c4[t];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0 && t < sp.nk) cnt[(int64_t)t * (n + 1) + j] = v;
    }
}

// Size class of every node from its capacity (items): packed one-hot counts
// (class c in bits 21c..21c+20) for one scan that ranks every class at once.
// Classes 0..2 in 21-bit fields (n < 2^21); class 3's rank is the node index
// minus the other three.
#define SNN_CLS_BITS 21
// (also zeroes the per-graph counts cnt[nk][n+1] and the overflow counters,
// which the build tiers fill: one launch instead of two memsets)
// Copy nodes (src[j] >= 0, snn_src_kernel) join class 3, whose fixed-grid
// kernel skips them: the copy pass writes their rows.
// (ucount: class-level build -- entries past the u classes are in no list)
__global__ void snn_class_kernel(const int64_t* __restrict__ roff, int64_t n, int64_t* __restrict__ cls,
                                 int64_t* __restrict__ cnt, int nk, int* __restrict__ ov_count,
                                 const int* __restrict__ src, const int64_t* __restrict__ ucount) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < 64) ov_count[j] = 0;
    if (j <= n)
        for (int t = 0; t < nk; ++t) cnt[(int64_t)t * (n + 1) + j] = 0;
    if (j >= n) return;
    const int64_t M = roff[j + 1] - roff[j];
    int c = (src && src[j] >= 0) ? 3 : (M <= 512 ? 0 : (M <= 1024 ? 1 : (M <= 2048 ? 2 : 3)));
    if (ucount && j >= *ucount) c = 3;  // not a class (the scatter lists class 3 only below u)
    cls[j] = c < 3 ? 1LL << (SNN_CLS_BITS * c) : 0;
}

// Lists of each class in node order; counts[c] = class size.
__global__ void snn_class_scatter_kernel(const int64_t* __restrict__ cls_scan, int64_t n, int* __restrict__ lists,
                                         int64_t* __restrict__ counts, const int64_t* __restrict__ ucount) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    const int64_t jl = ucount ? min(j, *ucount) : j;  // entries past u are in no class
    const int64_t mask = (1LL << SNN_CLS_BITS) - 1;
    const int64_t v = cls_scan[j];
    int64_t r[4];
    r[0] = v & mask;
    r[1] = (v >> SNN_CLS_BITS) & mask;
    r[2] = (v >> (2 * SNN_CLS_BITS)) & mask;
    r[3] = jl - r[0] - r[1] - r[2];
    if (j == n) {
        for (int c = 0; c < 4; ++c) counts[c] = r[c];
        return;
    }
    if (j != jl) return;  // past u (class-level build): no list
    const int64_t d = cls_scan[j + 1] - v;  // this node's one-hot class (0 for class 3)
    const int c = d == 1 ? 0 : (d == (1LL << SNN_CLS_BITS) ? 1 : (d == (1LL << (2 * SNN_CLS_BITS)) ? 2 : 3));
    lists[c * n + r[c]] = (int)j;
}

// ------------------------------------------------------- bitonic tier --
// Nodes with at most 64*E items (E = 4, 8, 16, 32): one wave per node.
// Every item (partner p > j, member rank rj, host rank rp) becomes one key
// that orders by p and carries all its merge needs:
//   NUMBER: p << 6 | m, m = max(rj, rp)                      (32-bit)
//   RANK:   p << 32 | (rj + rp) << 8 | m                     (64-bit)
// Items are gathered element-major (item t = 64 e + lane, so host reads are
// coalesced), transposed through LDS to lane-major (lane l holds items
// E l .. E l + E - 1), bitonic-sorted in registers (in-lane stages are
// min/max pairs; cross-lane stages one shuffle per element), and every run
// of equal p is combined by a segmented scan (in lane, then across lanes by
// DPP); the last item of each run writes the row entry.  No LDS round trip
// sits inside a loop, so the tier is bound by VALU issue, not by latency.

// Inclusive wave scans over lanes 0..lane (DPP row shifts, then the row
// broadcasts of lanes 15 and 31).
#define SNN_DPP_SHR(n) (0x110 | (n))
#define SNN_DPP_BCAST15 0x142
#define SNN_DPP_BCAST31 0x143
__device__ __forceinline__ int snn_scan_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_SHR(1), 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_SHR(2), 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_SHR(4), 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_SHR(8), 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_BCAST15, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, SNN_DPP_BCAST31, 0xC, 0xF, false));
    return v;
}
__device__ __forceinline__ int snn_scan_add(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_SHR(1), 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_SHR(2), 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_SHR(4), 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_SHR(8), 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_BCAST15, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, SNN_DPP_BCAST31, 0xC, 0xF, false);
    return v;
}

// Value of lane (lane ^ MSK) for the masks the bitonic network uses, without
// an LDS address round trip where the hardware has a direct path: DPP
// quad_perm / row (half-)mirror for 1, 2, 3, 7, 15; ds_swizzle (bit mode,
// within 32 lanes) for 4, 8, 16, 31; v_permlane32_swap for 32 (and 63 = 32
// then 31).
template <int MSK>
__device__ __forceinline__ unsigned snn_xlane(unsigned v) {
    if constexpr (MSK == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (MSK == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (MSK == 3) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);
    else if constexpr (MSK == 7) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    else if constexpr (MSK == 15) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    else if constexpr (MSK == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    } else if constexpr (MSK == 63) {
        return snn_xlane<31>(snn_xlane<32>(v));
    } else {
        static_assert(MSK == 4 || MSK == 8 || MSK == 16 || MSK == 31, "unsupported lane mask");
        return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (MSK << 10));
    }
}

template <typename K>
struct SnnKeyT;
template <>
struct SnnKeyT<uint32_t> {
    static constexpr int PS = 6;  // p << 6 | m
    __device__ static uint32_t make(int p, int rj, int rp) { return ((uint32_t)p << 6) | (uint32_t)max(rj, rp); }
    __device__ static int m(uint32_t k) { return (int)(k & 63u); }
    __device__ static int rs(uint32_t) { return 0; }
    template <int MSK>
    __device__ static uint32_t shx(uint32_t v) { return snn_xlane<MSK>(v); }
};
template <>
struct SnnKeyT<unsigned long long> {
    static constexpr int PS = 32;  // p << 32 | (rj + rp) << 8 | m
    __device__ static unsigned long long make(int p, int rj, int rp) {
        return ((unsigned long long)(unsigned)p << 32) | ((unsigned)(rj + rp) << 8) | (unsigned)max(rj, rp);
    }
    __device__ static int m(unsigned long long k) { return (int)(k & 0xFFu); }
    __device__ static int rs(unsigned long long k) { return (int)((k >> 8) & 0xFFu); }
    template <int MSK>
    __device__ static unsigned long long shx(unsigned long long v) {
        const unsigned lo = snn_xlane<MSK>((unsigned)v), hi = snn_xlane<MSK>((unsigned)(v >> 32));
        return ((unsigned long long)hi << 32) | lo;
    }
};

// Packed per-graph contribution of one item from its key (snn_contrib's
// value: byte t live iff m <= kk[t]).
// Class-level items (row classes, below): key = H << PS | 4-bit fields,
// field t = min(t_R(c), t_H(c)) for graph t -- the rows of the shared class c
// that both N+ sets hold.  32-bit keys carry 3 graphs (partner < 2^20);
// 64-bit keys 4 graphs.
template <typename K>
struct SnnClsKeyT;
template <>
struct SnnClsKeyT<uint32_t> {
    static constexpr int PS = 12;
};
template <>
struct SnnClsKeyT<unsigned long long> {
    static constexpr int PS = 32;
};
template <typename K, bool CS>
__host__ __device__ constexpr int snn_ps() {
    return CS ? SnnClsKeyT<K>::PS : SnnKeyT<K>::PS;
}
__device__ __forceinline__ unsigned snn_min4(unsigned a, unsigned b) {
    unsigned r = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const unsigned x = (a >> (4 * t)) & 15u, y = (b >> (4 * t)) & 15u;
        r |= (x < y ? x : y) << (4 * t);
    }
    return r;
}
__host__ __device__ __forceinline__ unsigned snn_nib2byte(unsigned v) {  // 4-bit fields -> bytes
    return (v & 0xFu) | ((v & 0xF0u) << 4) | ((v & 0xF00u) << 8) | ((v & 0xF000u) << 12);
}

template <typename K, bool CS = false>
__device__ __forceinline__ unsigned snn_key_contrib(const SnnSpec& sp, K key) {
    if constexpr (CS) {
        constexpr int PS = SnnClsKeyT<K>::PS;
        constexpr unsigned mask = PS >= 16 ? 0xFFFFu : ((1u << PS) - 1u);
        return snn_nib2byte((unsigned)key & mask);
    }
    const int m = SnnKeyT<K>::m(key);
    unsigned live = 0;
#pragma unroll
    for (int t = 0; t < SNN_MAXK; ++t) live |= (t < sp.nk && m <= sp.kk[t]) ? (0xFFu << (8 * t)) : 0u;
    if (sp.type == CCG_SNN_NUMBER) return live & 0x01010101u;
    return (((unsigned)SnnKeyT<K>::rs(key) * 0x01010101u) & live) | ~live;
}

template <typename K>
__device__ __forceinline__ void snn_ce(K& a, K& b) {  // (a, b) <- (min, max)
    const K lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Bitonic sort (all compare-exchanges ascending: each merge starts with the
// mirror stage i ^ (k - 1), then i ^ j for j = k/4 .. 1) of the 64*E keys in
// lane-major order, element i = E*lane + e.  snn_bitonic_xor runs the xor
// stages j = J .. 1 of one merge (J < 64*E).
template <int E, typename K, int J>
__device__ __forceinline__ void snn_bitonic_xor(K (&x)[E], int lane) {
    if constexpr (J < E) {
#pragma unroll
        for (int e = 0; e < E; ++e)
            if ((e & J) == 0) snn_ce(x[e], x[e ^ J]);
    } else {
        const bool lower = (lane & (J / E)) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const K o = SnnKeyT<K>::template shx<J / E>(x[e]);
            const K lo = x[e] < o ? x[e] : o, hi = x[e] < o ? o : x[e];
            x[e] = lower ? lo : hi;
        }
    }
    if constexpr (J > 1) snn_bitonic_xor<E, K, J / 2>(x, lane);
}

template <int E, typename K, int k>
__device__ __forceinline__ void snn_bitonic_merge(K (&x)[E], int lane) {
    if constexpr (k <= E) {  // mirror stage inside the lane
#pragma unroll
        for (int e = 0; e < E; ++e)
            if ((e & (k / 2)) == 0) snn_ce(x[e], x[e ^ (k - 1)]);
    } else {  // mirror stage across lanes: lane ^ (k/E - 1), element E-1-e
        const bool lower = (lane & (k / (2 * E))) == 0;
        K o[E];
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] = SnnKeyT<K>::template shx<k / E - 1>(x[E - 1 - e]);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const K lo = x[e] < o[e] ? x[e] : o[e], hi = x[e] < o[e] ? o[e] : x[e];
            x[e] = lower ? lo : hi;
        }
    }
    if constexpr (k >= 4) snn_bitonic_xor<E, K, k / 4>(x, lane);
    if constexpr (k < 64 * E) snn_bitonic_merge<E, K, 2 * k>(x, lane);
}

template <int E, typename K>
__device__ __forceinline__ void snn_bitonic(K (&x)[E], int lane) {
    snn_bitonic_merge<E, K, 2>(x, lane);
}

// Ascending bitonic network over N keys in one lane's registers (compile-
// time indices: min/max pairs only).
template <int N, typename K>
__device__ __forceinline__ void snn_sort_regs(K (&y)[N]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1)
#pragma unroll
        for (int jj = k >> 1; jj > 0; jj >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ jj;
                if (l > i) {
                    const K a = y[i], b = y[l];
                    const K lo = a < b ? a : b, hi = a < b ? b : a;
                    y[i] = (i & k) == 0 ? lo : hi;
                    y[l] = (i & k) == 0 ? hi : lo;
                }
            }
}

// Bucket tier of the sort (one wave, W = 1): the node's M keys (element-major
// in x, item t = 64 e + lane) are split by partner into 64 buckets of equal
// partner range (lane b owns bucket b; a node's partners are spread evenly
// over (j, n)), ranked by LDS atomics, scattered to LDS, and every lane sorts
// its bucket (<= CAP keys) in registers; x then holds the sorted keys lane-
// major (element E lane + e), padding ~0 last, as the bitonic tier leaves
// them.  A wave-level bitonic sort of 64 E slots costs ~log^2(64 E) / 2
// exchange stages per key, most across lanes; this is one register network
// of CAP keys per lane plus a few LDS passes.  Returns false (x untouched)
// when a bucket holds more than CAP keys: the caller sorts bitonically.
template <int E, int CAP, typename K, bool CS = false>
__device__ __forceinline__ bool snn_bucket_sort(K (&x)[E], int M, int lane, int* hist, K* buf) {
    constexpr int PS = snn_ps<K, CS>();
    K kmin = ~(K)0, kmax = 0;
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (64 * e + lane < M) {
            kmin = x[e] < kmin ? x[e] : kmin;
            kmax = x[e] > kmax ? x[e] : kmax;
        }
    int pmin = (int)(kmin >> PS), pmax = (int)(kmax >> PS);
    if (64 * 0 + lane >= M) pmin = INT_MAX, pmax = INT_MIN;  // (M >= 1: lane 0 holds a key)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pmin = min(pmin, __shfl_xor(pmin, o, 64));
        pmax = max(pmax, __shfl_xor(pmax, o, 64));
    }
    const float sc = 64.0f / (float)(pmax - pmin + 1);
    hist[lane] = 0;
    WAVE_LDS_SYNC();
    int b[E], r[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        b[e] = 0;
        r[e] = 0;
        if (64 * e + lane < M) {
            b[e] = min(63, (int)((float)((int)(x[e] >> PS) - pmin) * sc));
            r[e] = atomicAdd(&hist[b[e]], 1);
        }
    }
    WAVE_LDS_SYNC();
    const int c = hist[lane];
    if (__any(c > CAP)) return false;
    const int off = snn_scan_add(c) - c;
    hist[64 + lane] = off;
    WAVE_LDS_SYNC();
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (64 * e + lane < M) buf[hist[64 + b[e]] + r[e]] = x[e];
    WAVE_LDS_SYNC();
    K y[CAP];
#pragma unroll
    for (int i = 0; i < CAP; ++i) y[i] = i < c ? buf[off + i] : ~(K)0;
    snn_sort_regs<CAP, K>(y);
#pragma unroll
    for (int i = 0; i < CAP; ++i)
        if (i < c) buf[off + i] = y[i];  // the lane's own range: no other lane reads it before the barrier
    WAVE_LDS_SYNC();
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = E * lane + e < M ? buf[E * lane + e] : ~(K)0;
    return true;
}

// LDS of one node: the member table (lane i <= kmax holds member i; packed
// for one 16-byte read per item: first host position, end, the member, first
// item), the item -> member marks / transpose stage, and the W waves'
// summaries.
template <int E, int W, typename K>
struct SnnBitonicLds {
    int4 mem[64];
    union {
        int mark[64 * E * W];  // item t -> member whose run starts at t (-1 elsewhere)
        K buf[64 * E * W];     // element-major -> lane-major transpose; cross-wave stages
    } u;
    int wfirst[W], wlast[W], wwhole[W], wcnt[W];
    unsigned wout[W];
    long long wc4[W][SNN_MAXK];
};

// The node's sorted keys x (lane-major, padding ~0 last) -> its row: runs of
// equal partner are combined (sum / bytewise min of the per-graph values) and
// the last key of each run writes (partner, packed values); per-graph counts.
// W > 1 (the hub tier) joins the waves' runs through L's wave summaries.
template <int E, int W, typename K, bool CS, typename LDS>
__device__ __forceinline__ void snn_emit_sorted(LDS& L, const SnnSpec& sp, int64_t n, int64_t j, int wv, int lane,
                                                K (&x)[E], const SnnRows& rows, int64_t* __restrict__ cnt) {
    constexpr int PS = snn_ps<K, CS>();
#define SNN_SYNC()                            \
    do {                                      \
        if constexpr (W == 1) WAVE_LDS_SYNC(); \
        else __syncthreads();                 \
    } while (0)
    // runs of equal p: forward segmented combine inside the lane
    int p[E];
    unsigned agg[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        p[e] = (int)(x[e] >> PS);
        const unsigned c = snn_key_contrib<K, CS>(sp, x[e]);
        agg[e] = (e > 0 && p[e] == p[e - 1]) ? snn_combine(sp.type, agg[e - 1], c) : c;
    }
    // across lanes: the lane's last run continues into the next lane when
    // that lane starts with the same p; segmented inclusive scan of the lane
    // tails (a lane that is one run continuing from the left is not a head)
    const int first_p = p[0], last_p = p[E - 1];
    const int prev_last = __shfl_up(last_p, 1, 64);
    const bool cont = lane > 0 && prev_last == first_p;
    unsigned out = agg[E - 1];
    int head = !(cont && first_p == last_p);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = (unsigned)__shfl_up((int)out, o, 64);
        const int fy = __shfl_up(head, o, 64);
        if (lane >= o && !head) {
            out = snn_combine(sp.type, y, out);
            head = fy;
        }
    }
    const unsigned from_left = (unsigned)__shfl_up((int)out, 1, 64);
    const int next_first = __shfl_down(first_p, 1, 64);
    const int wfirst = __builtin_amdgcn_readfirstlane(first_p);
    int wnext = INT_MAX;  // the first p of the next wave
    bool wcarry = false;
    unsigned wc = 0;
    if constexpr (W > 1) {
        if (lane == 63) {
            L.wlast[wv] = last_p;
            L.wout[wv] = out;
        }
        if (lane == 0) L.wfirst[wv] = first_p;
        SNN_SYNC();
        if (lane == 0) L.wwhole[wv] = L.wfirst[wv] == L.wlast[wv];
        SNN_SYNC();
        if (wv + 1 < W) wnext = L.wfirst[wv + 1];
        // the wave's first run continues runs ending the waves to its left
        for (int v = wv - 1; v >= 0; --v) {
            if (L.wlast[v] != wfirst) break;
            wc = wcarry ? snn_combine(sp.type, L.wout[v], wc) : L.wout[v];
            wcarry = true;
            if (!L.wwhole[v]) break;
        }
    }
    int u_lane = 0;
    bool last[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (cont && p[e] == first_p) agg[e] = snn_combine(sp.type, from_left, agg[e]);
        if (wcarry && p[e] == wfirst) agg[e] = snn_combine(sp.type, wc, agg[e]);
        const int pn = e + 1 < E ? p[e + 1] : (lane < 63 ? next_first : wnext);
        last[e] = (unsigned)p[e] < (unsigned)n && p[e] != pn;  // padding keys decode to p >= n or -1
        u_lane += last[e] ? 1 : 0;
    }
    const int u_incl = snn_scan_add(u_lane);
    int u = __builtin_amdgcn_readlane(u_incl, 63);
    int64_t ro = rows.roff[j] + (u_incl - u_lane);
    if constexpr (W > 1) {
        if (lane == 0) L.wcnt[wv] = u;
        SNN_SYNC();
        int before = 0, tot = 0;
        for (int v = 0; v < W; ++v) {
            before += v < wv ? L.wcnt[v] : 0;
            tot += L.wcnt[v];
        }
        ro += before;
        u = tot;
    }
    const bool write = rows.roff[n] <= rows.cap;
    int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
    int w = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (last[e]) {
            if (write) {
                rows.nbr[ro + w] = p[e];
                rows.wpk[ro + w] = agg[e];
            }
            ++w;
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t)
                if (t < sp.nk && graph_has(sp, agg[e], t)) ++c4[t];
        }
    }
    if constexpr (W == 1) {
        snn_row_counts(sp, c4, n, j, lane, cnt);
    } else {
#pragma unroll
        for (int t = 0; t < SNN_MAXK; ++t) {
            int64_t v = c4[t];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) L.wc4[wv][t] = v;
        }
        SNN_SYNC();
        if (wv == 0 && lane < sp.nk) {
            int64_t v = 0;
            for (int q = 0; q < W; ++q) v += L.wc4[q][lane];
            cnt[(int64_t)lane * (n + 1) + j] = v;
        }
    }
    if (wv == 0 && lane == 0) rows.rlen[j] = u;
#undef SNN_SYNC
}

// One node, W waves (W = 1: one wave; W = 4: a 256-thread block for the
// hubs); wave w holds sorted elements 64*E*w .. 64*E*(w+1) - 1.
template <int E, int W, typename K, bool BK = false, bool CS = false>
__device__ __forceinline__ void snn_bitonic_node(SnnBitonicLds<E, W, K>& L, const SnnSpec& sp, int64_t n, int64_t j,
                                                 const SnnMember& m, int wv, int lane,
                                                 const int2* __restrict__ hosts_s, const SnnRows& rows,
                                                 int64_t* __restrict__ cnt) {
    constexpr int S = 64 * E;  // elements per wave
    const int kmax = sp.kk[sp.nk - 1];
    const int incl = snn_scan_add(m.len);
    const int M = __builtin_amdgcn_readlane(incl, 63);
    const int pre = incl - m.len;
    const int base = S * wv;  // this wave's first item / element
#define SNN_SYNC()                            \
    do {                                      \
        if constexpr (W == 1) WAVE_LDS_SYNC(); \
        else __syncthreads();                 \
    } while (0)
    // gather (element-major within the wave's slice)
#pragma unroll
    for (int e = 0; e < E; ++e) L.u.mark[base + 64 * e + lane] = -1;
    if (wv == 0 && lane <= kmax) L.mem[lane] = make_int4((int)m.h0, (int)m.hend, m.cur, pre);
    SNN_SYNC();
    if (wv == 0 && lane <= kmax && m.len > 0) L.u.mark[pre] = lane;
    SNN_SYNC();
    int mi[E];
    // the member of the slice's first item when its run starts in an earlier slice
    const unsigned long long started = __ballot(lane <= kmax && m.len > 0 && pre < base);
    int carry = started ? 63 - __clzll(started) : INT_MIN;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int v = snn_scan_max(max(L.u.mark[base + 64 * e + lane], carry));
        carry = __builtin_amdgcn_readlane(v, 63);
        mi[e] = v;
    }
    int2 hv[E];
    int az[E];  // CS: the member's inclusion fields (mem.z)
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int t = base + 64 * e + lane;
        hv[e] = make_int2(0, 0);
        az[e] = 0;
        if (t < M) {
            const int4 md = L.mem[mi[e]];
            const int q = md.x + (t - md.w);
            hv[e] = q < md.y ? hosts_s[q] : make_int2(md.z, 0);
            az[e] = md.z;
        }
    }
    K x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if constexpr (CS)
            x[e] = base + 64 * e + lane < M
                       ? (((K)(unsigned)hv[e].x << snn_ps<K, true>()) | (K)snn_min4((unsigned)az[e], (unsigned)hv[e].y))
                       : ~(K)0;
        else
            x[e] = base + 64 * e + lane < M ? SnnKeyT<K>::make(hv[e].x, mi[e], hv[e].y) : ~(K)0;
    }
    SNN_SYNC();  // every mark is read
    if constexpr (BK && W == 1) {
        if (snn_bucket_sort<E, (E >= 32 ? 64 : 32), K, CS>(x, M, lane, reinterpret_cast<int*>(L.mem), L.u.buf)) {
            snn_emit_sorted<E, W, K, CS>(L, sp, n, j, wv, lane, x, rows, cnt);
            return;
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) L.u.buf[base + 64 * e + lane] = x[e];
    SNN_SYNC();
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = L.u.buf[base + E * lane + e];
    snn_bitonic<E, K>(x, lane);
    if constexpr (W > 1) {
        // merges across waves through LDS: mirror stage, then the cross-wave
        // xor stages, then the in-wave xor stages
#pragma unroll
        for (int k = 2 * S; k <= W * S; k <<= 1) {
            SNN_SYNC();
#pragma unroll
            for (int e = 0; e < E; ++e) L.u.buf[base + E * lane + e] = x[e];
            SNN_SYNC();
            {
                const int pw = wv ^ (k / S - 1);
                const bool lower = (wv & (k / (2 * S))) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const K o = L.u.buf[S * pw + E * (63 - lane) + (E - 1 - e)];
                    const K lo = x[e] < o ? x[e] : o, hi = x[e] < o ? o : x[e];
                    x[e] = lower ? lo : hi;
                }
            }
#pragma unroll
            for (int jj = k / 4; jj >= S; jj >>= 1) {
                SNN_SYNC();
#pragma unroll
                for (int e = 0; e < E; ++e) L.u.buf[base + E * lane + e] = x[e];
                SNN_SYNC();
                const int pw = wv ^ (jj / S);
                const bool lower = (wv & (jj / S)) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const K o = L.u.buf[S * pw + E * lane + e];
                    const K lo = x[e] < o ? x[e] : o, hi = x[e] < o ? o : x[e];
                    x[e] = lower ? lo : hi;
                }
            }
            snn_bitonic_xor<E, K, S / 2>(x, lane);
        }
    }
    snn_emit_sorted<E, W, K, CS>(L, sp, n, j, wv, lane, x, rows, cnt);
#undef SNN_SYNC
}


// Size classes (items M of a node): 0: M <= 512 (E = 4 or 8 per node),
// 1: <= 1024 (E = 16), 2: <= 2048 (E = 32), 3: <= 4096 (the hubs: 4 waves x
// E = 16 per node), larger: the block tier.  Classes 0..2 run one node per
// wave (4 waves per block, 2 for class 2: its LDS stage is 8-16 KB per wave);
// class 3 runs one node per 256-thread block over a fixed grid.
__host__ __device__ constexpr int snn_bitonic_wpb(int cls) { return cls == 2 ? 2 : 4; }

// Row classes (snn_cls_* below): the member slots of a class's root row.
struct SnnClsIn {
    const int* croot;      // [u] root row of each class
    const int* mcls;       // [n (kmax + 1)] member class of root slot (row, lane), -1 = none
    const unsigned* incl;  // [n (kmax + 1)] the member's packed inclusion counts (4 bits per graph)
    const int64_t* ucount;  // device: u, the number of classes
};

// Member `lane` of class c: the class of a distinct member of its root's N+
// set; its items are the hosts after the class in that member's host list.
__device__ __forceinline__ SnnMember snn_cls_member(const SnnClsIn& ci, int kmax, int64_t c, int lane,
                                                    const int64_t* __restrict__ hoff, const int* __restrict__ bp) {
    SnnMember m{0, 0, 0, 0};
    if (lane > kmax) return m;
    const int64_t slot = (int64_t)ci.croot[c] * (kmax + 1) + lane;
    const int cs = ci.mcls[slot];
    if (cs < 0) return m;
    m.cur = (int)ci.incl[slot];
    m.h0 = hoff[cs] + bp[slot] + 1;
    m.hend = hoff[cs + 1];
    m.len = (int)(m.hend - m.h0);
    return m;
}

template <int CLS, typename K, bool BUCKET = false, bool CS = false>
__global__ __launch_bounds__(64 * snn_bitonic_wpb(CLS)) void snn_bitonic_build_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp, const int64_t* __restrict__ hoff,
    const int2* __restrict__ hosts_s, const int* __restrict__ bp, const int* __restrict__ split,
    int64_t* __restrict__ cnt, SnnRows rows, const int* __restrict__ list, const int64_t* __restrict__ count,
    int* __restrict__ ov_list, int* __restrict__ ov_count, const int* __restrict__ src, SnnClsIn ci) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kmax = sp.kk[sp.nk - 1];
    auto member = [&](int64_t j) {
        if constexpr (CS) return snn_cls_member(ci, kmax, j, lane, hoff, bp);
        else return snn_member(knn, n, kstride, kmax, j, lane, hoff, bp, split);
    };
    if constexpr (CLS == 3) {
        __shared__ SnnBitonicLds<16, 4, K> lds3;
        const int64_t nl = *count;
        for (int64_t f = blockIdx.x; f < nl; f += gridDim.x) {
            const int64_t j = list[f];
            if (src && src[j] >= 0) continue;  // a copy node (snn_copy_rows_kernel)
            if (rows.roff[j + 1] - rows.roff[j] > SNN_BITONIC_MAX) {
                if (threadIdx.x == 0) ov_list[atomicAdd(ov_count, 1)] = (int)j;
                continue;
            }
            const SnnMember m = member(j);
            snn_bitonic_node<16, 4, K, false, CS>(lds3, sp, n, j, m, wv, lane, hosts_s, rows, cnt);
            __syncthreads();
        }
    } else {
        constexpr int EM = CLS == 0 ? 8 : (CLS == 1 ? 16 : 32);
        constexpr int WPB = snn_bitonic_wpb(CLS);
        __shared__ SnnBitonicLds<EM, 1, K> lds_all[WPB];
        const int64_t f = (int64_t)blockIdx.x * WPB + wv;
        if (f >= *count) return;
        const int64_t j = list[f];
        const SnnMember m = member(j);
        if constexpr (CLS == 0) {
            if (__builtin_amdgcn_readlane(snn_scan_add(m.len), 63) <= 256) {
                snn_bitonic_node<4, 1, K, false, CS>(*reinterpret_cast<SnnBitonicLds<4, 1, K>*>(&lds_all[wv]), sp, n,
                                                     j, m, 0, lane, hosts_s, rows, cnt);
                return;
            }
        }
        snn_bitonic_node<EM, 1, K, BUCKET && CLS >= 1, CS>(lds_all[wv], sp, n, j, m, 0, lane, hosts_s, rows, cnt);
    }
}

// ------------------------------------------------------- copy nodes --
// Bootstrap rows repeat cells (R/consensusClust.R:394): copies of a cell are
// at distance 0, so their kNN lists hold each other first and then the same
// rows, and their sets N+_k = {j} u knn_k(j) coincide for every k of kNum
// (whenever the zero-distance group fits in the smallest k + 1).  For NUMBER
// weights |N+_k(j) n N+_k(p)| depend on those sets only, so such a node j has
// the same weight to every partner as the node r = knn(j)[0] < j (the
// cell's lowest other row), and its row (partners p > j) is the part of r's
// row past j.  snn_src_kernel checks the sets (any input: the test is exact
// set equality); the build tiers skip these nodes and snn_copy_rows_kernel
// copies their rows after them, from the end of the src chain (the one node
// of the chain that is built).  Round 4 took r = min N+_kmin(j), which is a
// copy only when the cell's row is the smallest of the whole set: it caught
// ~23% of the copies (cfg3: ~7k of ~30k nodes skipped instead of ~30k).
template <bool PACK>
__global__ __launch_bounds__(256) void snn_src_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                      SnnSpec sp, int* __restrict__ src,
                                                      const int32_t* __restrict__ cell) {
    constexpr int WL = PACK ? 32 : 64;  // lanes per node (PACK: kmax <= 31, two nodes per wave)
    constexpr int NPW = 64 / WL;
    const int lane = threadIdx.x & (WL - 1);
    const int half = PACK ? (int)((threadIdx.x >> 5) & 1) : 0;
    const int kmax = sp.kk[sp.nk - 1];
    // this node's lanes' bits of a wave ballot
    auto mine = [&](unsigned long long b) -> unsigned long long {
        return PACK ? ((half ? b >> 32 : b) & 0xffffffffull) : b;
    };
    const unsigned long long full = PACK ? 0xffffffffull : ~0ull;
    for (int64_t jb = (int64_t)blockIdx.x * 4 * NPW; jb < n; jb += (int64_t)gridDim.x * 4 * NPW) {
        const int64_t j = jb + (threadIdx.x / WL);
        const bool live = j < n;
        int a = (int)j;
        if (live && lane >= 1 && lane <= kmax) a = knn[j * kstride + lane - 1];
        const bool bad = live && lane <= kmax && ((unsigned)a >= (unsigned)n || (lane >= 1 && a == (int)j));
        // candidate: the first neighbour (a copy of j's cell sits there: copies are at
        // distance 0, ordered by row, so it is the cell's lowest other row)
        const int r = __shfl(a, 1, WL);
        bool ok = live && r >= 0 && r < (int)j && mine(__ballot(bad)) == 0ull;
        if (cell && ok) ok = cell[r] == cell[j];  // row classes: copies of one cell only
        if (mine(__ballot(ok)) != 0ull) {  // (uniform in the node's lanes)
            int b = r;
            if (ok && lane >= 1 && lane <= kmax) b = knn[(int64_t)r * kstride + lane - 1];
            // N+_k(j) == N+_k(r) for every graph: every member of j's k-prefix is in r's
            // (both hold k + 1 distinct rows)
            for (int t = 0; t < sp.nk; ++t) {
                const int k = sp.kk[t];
                bool found = lane > k;
                for (int q = 0; q <= k; ++q) found |= a == __shfl(b, q, WL);
                ok = ok && mine(__ballot(found)) == full;
            }
        }
        if (live && lane == 0) src[j] = ok ? r : -1;
    }
}

// Walks the class-3 list (the copy nodes and the hubs; hubs are skipped), one
// wave per node: the first entry of r's row past j by a two-level search
// (64 lanes sample the row, then 64 lanes scan the chunk: two dependent loads
// instead of a ~9-step binary search), then the copy.
__global__ __launch_bounds__(256) void snn_copy_rows_kernel(int64_t n, SnnSpec sp, const int* __restrict__ src,
                                                            int64_t* __restrict__ cnt, SnnRows rows,
                                                            const int* __restrict__ list,
                                                            const int64_t* __restrict__ count) {
    if (rows.roff[n] > rows.cap) return;  // rows not written (the caller sizes and retries)
    const int lane = threadIdx.x & 63;
    const int64_t nl = *count;
    for (int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); f < nl; f += (int64_t)gridDim.x * 4) {
        const int64_t j = list[f];
        int r = src[j];
        if (r < 0) continue;  // a hub (the bitonic / block tiers)
        while (src[r] >= 0) r = src[r];  // the built end of the chain (src[x] < x: no cycles)
        const int64_t a = rows.roff[r];
        const int len = rows.rlen[r];
        // first entry of r's row with partner > j (partners ascending)
        const int step = (len + 63) >> 6;  // chunk per lane
        const int s0 = lane * step;
        const bool le0 = s0 < len && rows.nbr[a + s0] <= (int)j;
        const int nle = __popcll(__ballot(le0));  // chunks whose first entry is <= j
        int lo = 0;
        if (nle > 0) {
            const int c0 = (nle - 1) * step;  // the crossing lies in [c0, c0 + step]
            const int c1 = min(c0 + step, len);
            lo = c0;
            for (int q0 = c0; q0 < c1; q0 += 64) {  // one pass unless the row exceeds 4096 entries
                const int q = q0 + lane;
                lo += __popcll(__ballot(q < c1 && rows.nbr[a + q] <= (int)j));
            }
        }
        const int64_t o = rows.roff[j];
        int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
        for (int i = lo + lane; i < len; i += 64) {
            const unsigned w = rows.wpk[a + i];
            rows.nbr[o + i - lo] = rows.nbr[a + i];
            rows.wpk[o + i - lo] = w;
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t) c4[t] += (t < sp.nk && graph_has(sp, w, t)) ? 1 : 0;
        }
        snn_row_counts(sp, c4, n, j, lane, cnt);
        if (lane == 0) rows.rlen[j] = len - lo;
    }
}

// ------------------------------------------------------------ row classes --
// Bootstrap rows repeat cells (:394): about a third of the rows at cfg3 are
// extra copies.  A CLASS is a set of rows chained by src (equal N+_k sets for
// every graph -- snn_src_kernel -- and, when the caller passes cell ids, the
// same cell); its root, the lowest row, stands for it.  For NUMBER weights
//   w_k(x, y) = |N+_k(x) n N+_k(y)| = sum over classes c of |S_x(c) n S_y(c)|,
// S_x(c) = the rows of c in N+_k(x).  Copies of one point sit at equal
// distance from every row, ordered by row index, so S_x(c) is a PREFIX of c's
// rows in row order, and |S_x(c) n S_y(c)| = min(t_x(c), t_y(c)) with t the
// prefix lengths.  So the graph of the classes -- items (partner class H,
// per-graph min(t_R(c), t_H(c))) over the member classes c of each root R --
// carries every row-level weight: rows x in R, y in H get w(R, H), and two
// rows of one class get k + 1 (their common set).  snn_cls_members_kernel
// checks the prefix property on every root's list (an input that breaks it
// sets the status: the caller takes the row-level pass).  At cfg3 a root has
// ~14 member classes instead of 21 member rows, and the class items are ~1/3
// of the row items; the rows are expanded only on the host (ccg_snn_graphs).

// root[x]: the end of x's src chain (src[r] < r); isroot[x] for the scan that
// numbers the classes (ordinal = exclusive prefix at the root).
// (also zeroes the contract status of snn_cls_members_kernel: no memset launch)
__global__ void snn_cls_root_kernel(const int* __restrict__ src, int64_t n, int* __restrict__ root,
                                    int64_t* __restrict__ isroot, int* __restrict__ status) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x == 0) *status = 0;
    if (x >= n) return;
    int r = (int)x;
    while (src[r] >= 0) r = src[r];
    root[x] = r;
    isroot[x] = r == (int)x ? 1 : 0;
}

// Per row x: its class ordinal, its rank among its class's rows (row order:
// every row of a class is in N+_kmin of each of them), and for a root the
// class size and the ordinal -> root table.
template <bool PACK>
__global__ __launch_bounds__(256) void snn_cls_rank_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                           int kmax, const int* __restrict__ root,
                                                           const int64_t* __restrict__ ord, int* __restrict__ row_class,
                                                           int* __restrict__ crank, int* __restrict__ croot,
                                                           int* __restrict__ csize) {
    constexpr int WL = PACK ? 32 : 64;
    constexpr int NPW = 64 / WL;
    const int lane = threadIdx.x & (WL - 1);
    const int half = PACK ? (int)((threadIdx.x >> 5) & 1) : 0;
    auto mine = [&](unsigned long long b) -> unsigned long long {
        return PACK ? ((half ? b >> 32 : b) & 0xffffffffull) : b;
    };
    for (int64_t xb = (int64_t)blockIdx.x * 4 * NPW; xb < n; xb += (int64_t)gridDim.x * 4 * NPW) {
        const int64_t x = xb + (threadIdx.x / WL);
        const bool live = x < n;
        int a = (int)x;
        if (live && lane >= 1 && lane <= kmax) a = knn[x * kstride + lane - 1];
        const bool in = live && lane <= kmax && (unsigned)a < (unsigned)n;
        const int ra = in ? root[a] : -1;
        const int rx = live ? root[x] : -2;
        const int cr = __popcll(mine(__ballot(in && ra == rx && a < (int)x)));
        const int cs = __popcll(mine(__ballot(in && ra == (int)x)));
        if (live && lane == 0) {
            const int o = (int)ord[rx];
            row_class[x] = o;
            crank[x] = cr;
            if (rx == (int)x) {
                croot[o] = (int)x;
                csize[o] = cs;
            }
        }
    }
}

// Per root R (slots R (kmax + 1) + i, i = rank 0 .. kmax of N+(R)): the
// distinct member classes with their prefix lengths t_k = the class's rows at
// ranks <= k for every graph (4 bits each: a class has at most kmin + 1 <= 15
// rows), as (member class, slot) pairs for the host-list sort (other slots:
// key n, sorted past every class).  Checks the prefix property: a foreign
// class's rows appear in R's list in the class's row order.
template <bool PACK>
__global__ __launch_bounds__(256) void snn_cls_members_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                              SnnSpec sp, const int* __restrict__ root,
                                                              const int* __restrict__ row_class,
                                                              const int* __restrict__ crank, int* __restrict__ mcls,
                                                              unsigned* __restrict__ incl, int32_t* __restrict__ keys,
                                                              int32_t* __restrict__ vals, int* __restrict__ status) {
    constexpr int WL = PACK ? 32 : 64;
    constexpr int NPW = 64 / WL;
    const int lane = threadIdx.x & (WL - 1);
    const int kmax = sp.kk[sp.nk - 1];
    for (int64_t xb = (int64_t)blockIdx.x * 4 * NPW; xb < n; xb += (int64_t)gridDim.x * 4 * NPW) {
        const int64_t x = xb + (threadIdx.x / WL);
        const bool live = x < n;
        const bool isr = live && root[x] == (int)x;
        int a = (int)x;
        if (isr && lane >= 1 && lane <= kmax) a = knn[x * kstride + lane - 1];
        const bool in = isr && lane <= kmax && (unsigned)a < (unsigned)n;
        const int cs = in ? row_class[a] : -1 - lane;  // distinct dummies for idle lanes
        const int own = __shfl(cs, 0, WL);
        int before = 0;
        unsigned t4 = 0;
        for (int q = 0; q <= kmax; ++q) {
            const int o = __shfl(cs, q, WL);
            const bool same = o == cs;
            before += (same && q < lane) ? 1 : 0;
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t) t4 += (same && t < sp.nk && q <= sp.kk[t]) ? (1u << (4 * t)) : 0u;
        }
        const bool head = in && before == 0;
        if (in && cs != own && crank[a] != before) atomicOr(status, 1);  // not a prefix in row order
        if (live && lane <= kmax) {
            const int64_t slot = x * (kmax + 1) + lane;
            mcls[slot] = head ? cs : -1;
            incl[slot] = t4;
            keys[slot] = head ? cs : (int32_t)n;
            vals[slot] = (int32_t)slot;
        }
    }
}

// hosts_s[p] = (host class ordinal, its inclusion fields); bp[slot] = the
// host's position in the member class's list (hosts ascending).
__global__ void snn_cls_hosts_kernel(const int32_t* __restrict__ skey, const int32_t* __restrict__ sval, int kmax,
                                     const int64_t* __restrict__ hoff, const int64_t* __restrict__ ucount,
                                     const int* __restrict__ row_class, const unsigned* __restrict__ incl,
                                     int2* __restrict__ hosts_s, int* __restrict__ bp) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= hoff[*ucount]) return;
    const int c = skey[p], slot = sval[p];
    const int rrow = slot / (kmax + 1);
    hosts_s[p] = make_int2(row_class[rrow], (int)incl[slot]);
    bp[slot] = (int)(p - hoff[c]);
}

// hoff[c] = first sorted position with key >= c (c = 0..u); entries past u
// are unused.
__global__ void snn_cls_hoff_kernel(const int32_t* __restrict__ skey, int64_t total, const int64_t* __restrict__ ucount,
                                    int64_t* __restrict__ hoff) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > *ucount) return;
    int64_t lo = 0, hi = total;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (skey[mid] < c) lo = mid + 1; else hi = mid;
    }
    hoff[c] = lo;
}

// Items of every class (its row capacity); 0 past u.
template <bool PACK>
__global__ __launch_bounds__(256) void snn_cls_items_kernel(int64_t n, int kmax, SnnClsIn ci,
                                                            const int64_t* __restrict__ hoff,
                                                            const int* __restrict__ bp, int64_t* __restrict__ cap) {
    constexpr int WL = PACK ? 32 : 64;
    constexpr int NPW = 64 / WL;
    const int lane = threadIdx.x & (WL - 1);
    const int64_t u = *ci.ucount;
    for (int64_t cb = (int64_t)blockIdx.x * 4 * NPW; cb < n; cb += (int64_t)gridDim.x * 4 * NPW) {
        const int64_t c = cb + (threadIdx.x / WL);
        int v = 0;
        if (c < u) v = snn_cls_member(ci, kmax, c, lane, hoff, bp).len;
        for (int o = WL / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WL);
        if (lane == 0 && c < n) cap[c] = c < u ? v : 0;
    }
}

// --------------------------------------------------------- block tier --
// Nodes beyond the bitonic tier (more than SNN_BITONIC_MAX items): one
// 256-thread block and a 16K-slot LDS hash table per node; the table is
// compacted and bitonic-sorted by partner in LDS.  Nodes that overflow here
// too are appended to ov2 for the dense tier.
__device__ __forceinline__ bool table_insert_blk(int* keys, unsigned* vals, int* count, int p, unsigned c,
                                                 const SnnSpec& sp, int bits) {
    unsigned s = snn_hash(p, bits);
    for (int probe = 0; probe < SNN_BT; ++probe) {
        int k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (k == SNN_EMPTY) {
            const int prev = atomicCAS(&keys[s], SNN_EMPTY, p);
            if (prev == SNN_EMPTY) {
                atomicAdd(count, 1);
                k = p;
            } else {
                k = prev;
            }
        }
        if (k == p) {
            snn_update(sp, &vals[s], c);
            return true;
        }
        s = (s + 1) & (SNN_BT - 1);
    }
    return false;
}

// Every item (partner p > j, packed contribution c) of node j -- row-level
// (members of N+(j), their host lists) or class-level (CS: member classes
// of class j, the hosts after j) -- handed to f(p, c) by the block's threads.
template <bool CS, typename F>
__device__ __forceinline__ void snn_node_items(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                               const SnnSpec& sp, int64_t j, const int64_t* __restrict__ hoff,
                                               const int2* __restrict__ hosts, const int* __restrict__ bp,
                                               const SnnClsIn& ci, F&& f) {
    const int kmax = sp.kk[sp.nk - 1];
    for (int i = 0; i <= kmax; ++i) {
        if constexpr (CS) {
            const SnnMember m = snn_cls_member(ci, kmax, j, i, hoff, bp);
            for (int o = threadIdx.x; o < m.len; o += blockDim.x) {
                const int2 hr = hosts[m.h0 + o];
                f(hr.x, snn_nib2byte(snn_min4((unsigned)m.cur, (unsigned)hr.y)));
            }
        } else {
            const int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
            if ((unsigned)cur >= (unsigned)n || (i > 0 && cur == j)) continue;  // invalid (CCG_DERR_SNN_INDEX)
            const int64_t h0 = hoff[cur];
            const int64_t len = hoff[cur + 1] - h0 + 1;
            for (int64_t o = threadIdx.x; o < len; o += blockDim.x) {
                int p, rp;
                if (o == len - 1) {
                    p = cur;
                    rp = 0;
                } else {
                    const int2 hr = hosts[h0 + o];
                    p = hr.x;
                    rp = hr.y;
                }
                if (p > j) {
                    const unsigned c = snn_contrib(sp, i, rp);
                    if (c != sp.init) f(p, c);
                }
            }
        }
    }
}

template <bool CS>
__global__ __launch_bounds__(256) void snn_block_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        SnnSpec sp, const int64_t* __restrict__ hoff,
                                                        const int2* __restrict__ hosts, int64_t* __restrict__ cnt,
                                                        SnnRows rows, const int* __restrict__ ov_list,
                                                        const int* __restrict__ ov_count, int* __restrict__ ov2_list,
                                                        int* __restrict__ ov2_count, const int* __restrict__ bp,
                                                        SnnClsIn ci) {
    __shared__ int keys[SNN_BT];
    __shared__ unsigned vals[SNN_BT];
    __shared__ int count;
    __shared__ int full_s;
    __shared__ int u_s;
    __shared__ int tcount[256];
    __shared__ int64_t wsum[4][SNN_MAXK];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int BITS = 14;
    constexpr int PER = SNN_BT / 256;  // slots owned per thread during compaction
    const int cap_entries = SNN_BT * 3 / 4;
    const int nov = *ov_count;
    const bool write = rows.roff[n] <= rows.cap;
    for (int f = blockIdx.x; f < nov; f += gridDim.x) {
        const int64_t j = ov_list[f];
        for (int s = tid; s < SNN_BT; s += 256) {
            keys[s] = SNN_EMPTY;
            vals[s] = sp.init;
        }
        if (tid == 0) {
            count = 0;
            full_s = 0;
        }
        __syncthreads();
        snn_node_items<CS>(knn, n, kstride, sp, j, hoff, hosts, bp, ci, [&](int p, unsigned c) {
            if (!table_insert_blk(keys, vals, &count, p, c, sp, BITS)) full_s = 1;
        });
        __syncthreads();
        if (full_s || count > cap_entries) {
            if (tid == 0) ov2_list[atomicAdd(ov2_count, 1)] = (int)j;
            __syncthreads();
            continue;
        }
        // compact: thread t owns slots [t*PER, (t+1)*PER); block scan of counts
        int mine = 0;
        for (int s = tid * PER; s < tid * PER + PER; ++s) mine += keys[s] != SNN_EMPTY;
        tcount[tid] = mine;
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int t = 0; t < 256; ++t) {
                const int v = tcount[t];
                tcount[t] = acc;
                acc += v;
            }
            u_s = acc;
        }
        __syncthreads();
        // every thread reads all its slots into registers before anyone writes
        int myk[PER];
        unsigned myv[PER];
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            myk[s] = keys[tid * PER + s];
            myv[s] = vals[tid * PER + s];
        }
        __syncthreads();
        int dst = tcount[tid];
#pragma unroll
        for (int s = 0; s < PER; ++s)
            if (myk[s] != SNN_EMPTY) {
                keys[dst] = myk[s];
                vals[dst] = myv[s];
                ++dst;
            }
        const int u = u_s;
        int P = 256;
        while (P < u) P <<= 1;
        for (int s = u + tid; s < P; s += 256) keys[s] = 0x7fffffff;
        __syncthreads();
        for (int kk = 2; kk <= P; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                for (int i = tid; i < P; i += 256) {
                    const int l = i ^ jj;
                    if (l > i) {
                        const int a = keys[i], b = keys[l];
                        const bool up = (i & kk) == 0;
                        if ((a > b) == up) {
                            keys[i] = b;
                            keys[l] = a;
                            const unsigned va = vals[i];
                            vals[i] = vals[l];
                            vals[l] = va;
                        }
                    }
                }
                __syncthreads();
            }
        }
        const int64_t ro = rows.roff[j];
        int64_t c[SNN_MAXK] = {0, 0, 0, 0};
        for (int q = tid; q < u; q += 256) {
            const unsigned v = vals[q];
            if (write) {
                rows.nbr[ro + q] = keys[q];
                rows.wpk[ro + q] = v;
            }
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t)
                if (t < sp.nk && graph_has(sp, v, t)) ++c[t];
        }
#pragma unroll
        for (int t = 0; t < SNN_MAXK; ++t) {
            int64_t v = c[t];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) wsum[wv][t] = v;
        }
        __syncthreads();
        if (tid < sp.nk) cnt[(int64_t)tid * (n + 1) + j] = wsum[0][tid] + wsum[1][tid] + wsum[2][tid] + wsum[3][tid];
        if (tid == 0) rows.rlen[j] = u;
        __syncthreads();
    }
}

// --------------------------------------------------------- dense tier --
// Exact O(n) per node with a dense word per partner.  Reads/writes go
// through agent-scope atomics so the block never sees stale L1 lines.
template <bool CS>
__global__ __launch_bounds__(256) void snn_dense_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        SnnSpec sp, const int64_t* __restrict__ hoff,
                                                        const int2* __restrict__ hosts,
                                                        const int* __restrict__ ov_list,
                                                        const int* __restrict__ ov_count,
                                                        unsigned* __restrict__ dense_all, int64_t* __restrict__ cnt,
                                                        SnnRows rows, const int* __restrict__ bp, SnnClsIn ci) {
    __shared__ int64_t wsum[4];
    unsigned* dense = dense_all + (int64_t)blockIdx.x * n;
    const int nov = *ov_count;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool write = rows.roff[n] <= rows.cap;
    for (int f = blockIdx.x; f < nov; f += gridDim.x) {
        const int64_t j = ov_list[f];
        for (int64_t p = j + 1 + threadIdx.x; p < n; p += 256)
            __hip_atomic_store(&dense[p], sp.init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        snn_node_items<CS>(knn, n, kstride, sp, j, hoff, hosts, bp, ci,
                           [&](int p, unsigned c) { snn_update(sp, &dense[p], c); });
        __syncthreads();
        // the row: partners of the union graph (the largest k) in ascending p
        const int64_t ro = rows.roff[j];
        const int tu = sp.nk - 1;
        int64_t total = 0;
        int64_t c[SNN_MAXK] = {0, 0, 0, 0};
        for (int64_t p0 = j + 1; p0 < n; p0 += 256) {
            const int64_t p = p0 + threadIdx.x;
            const unsigned v = (p < n) ? __hip_atomic_load(&dense[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : sp.init;
            const bool hit = (p < n) && graph_has(sp, v, tu);
            const unsigned long long m = __ballot(hit);
            if (lane == 0) wsum[wv] = __popcll(m);
            __syncthreads();
            int64_t before = 0, tot = 0;
            for (int w = 0; w < 4; ++w) {
                if (w < wv) before += wsum[w];
                tot += wsum[w];
            }
            if (hit) {
                const int64_t e = ro + total + before + __popcll(m & lanemask_lt());
                if (write) {
                    rows.nbr[e] = (int32_t)p;
                    rows.wpk[e] = v;
                }
#pragma unroll
                for (int t = 0; t < SNN_MAXK; ++t)
                    if (t < sp.nk && graph_has(sp, v, t)) ++c[t];
            }
            total += tot;
            __syncthreads();
        }
#pragma unroll
        for (int t = 0; t < SNN_MAXK; ++t) {
            int64_t v = c[t];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) wsum[wv] = v;
            __syncthreads();
            if (threadIdx.x == 0 && t < sp.nk) cnt[(int64_t)t * (n + 1) + j] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            __syncthreads();
        }
        if (threadIdx.x == 0) rows.rlen[j] = (int32_t)total;
        __syncthreads();
    }
}

// ------------------------------------------------- per-graph edge lists --
// Graph t's edges of node j are the row entries with byte t present, already
// in ascending partner order; off = ONE exclusive scan of the graphs' counts
// laid end to end (block t = [t (n+1), (t+1)(n+1)), slot n zero), so graph
// t's offsets are off[t (n+1) + j] - off[t (n+1)].
__global__ __launch_bounds__(256) void snn_emit_kernel(int64_t n, SnnSpec sp, const int64_t* __restrict__ off,
                                                       SnnRows rows, SnnOut out) {
    const int lane = threadIdx.x & 63;
    if (rows.roff[n] > rows.cap) return;  // rows were not written (reported through the totals)
    for (int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (int64_t)gridDim.x * 4) {
        const int u = rows.rlen[j];
        const int64_t ro = rows.roff[j];
        for (int t = 0; t < sp.nk; ++t) {
            if (out.cap[t] <= 0) continue;
            int64_t e = off[(int64_t)t * (n + 1) + j] - off[(int64_t)t * (n + 1)];
            for (int c0 = 0; c0 < u; c0 += 64) {
                const int c = c0 + lane;
                const unsigned v = c < u ? rows.wpk[ro + c] : sp.init;
                const bool has = c < u && graph_has(sp, v, t);
                const unsigned long long m = __ballot(has);
                if (has) {
                    const int64_t pos = e + __popcll(m & lanemask_lt());
                    if (pos < out.cap[t]) {
                        out.oi[t][pos] = (int32_t)j;
                        out.oj[t][pos] = rows.nbr[ro + c];
                        out.ow[t][pos] = graph_weight(sp, v, t);
                    }
                }
                e += __popcll(m);
            }
        }
    }
}

// Totals per graph; -(required row capacity) when the rows did not fit.
__global__ void snn_copy_totals(const int64_t* __restrict__ cnt, int64_t n, int nk, const int64_t* __restrict__ roff,
                                int64_t rcap, int64_t* d0, int64_t* d1, int64_t* d2, int64_t* d3) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t* ds[4] = {d0, d1, d2, d3};
    const bool fit = roff[n] <= rcap;
    for (int t = 0; t < nk; ++t)
        if (ds[t]) *ds[t] = fit ? cnt[(int64_t)t * (n + 1) + n] - cnt[(int64_t)t * (n + 1)] : -roff[n];
}

// --------------------------------------------------------------- driver --
static int snn_spec(const int* ks, int nk, int type, int kstride, SnnSpec* sp) {
    CCG_REQUIRE(ks, "SNN: NULL ks");
    CCG_REQUIRE(nk >= 1 && nk <= SNN_MAXK, "SNN: 1 <= nk <= %d", SNN_MAXK);
    CCG_REQUIRE(type == CCG_SNN_NUMBER || type == CCG_SNN_RANK, "SNN: bad type");
    sp->nk = nk;
    sp->type = type;
    sp->init = type == CCG_SNN_NUMBER ? 0u : 0xFFFFFFFFu;
    for (int t = 0; t < SNN_MAXK; ++t) sp->kk[t] = t < nk ? ks[t] : 0;
    for (int t = 0; t < nk; ++t)
        CCG_REQUIRE(ks[t] >= 1 && ks[t] <= kstride && ks[t] <= 32 && (t == 0 || ks[t] > ks[t - 1]),
                    "SNN: ks must be ascending in [1, min(kstride, 32)]");
    return CCG_OK;
}

// Builds the node rows (union graph) and per-graph counts; on return
// cnt[t (n+1) + j] holds one exclusive scan of all graphs' counts (graph t's edge
// offsets and total relative to cnt[t (n+1)]).
// roff: n+1 row offsets (capacity-based), from the workspace when NULL.
static int snn_build(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const SnnSpec& sp, hipStream_t st,
                     int32_t* nbr, uint32_t* wpk, int64_t cap, int64_t* roff, int32_t* rlen, int64_t** cnt_out,
                     const int64_t** roff_out) {
    const int kmax = sp.kk[sp.nk - 1];
    const int64_t nkk = n * kmax;
    CCG_REQUIRE(nkk < (1LL << 31) - 1, "SNN: n*kmax too large");
    int64_t* hoff = (int64_t*)ccg_ws(ctx, WS_SNN_A, sizeof(int64_t) * (2 * (n + 1) + 16));
    int2* hosts_s = (int2*)ccg_ws(ctx, WS_SNN_B, sizeof(int2) * (nkk + 1));
    int64_t* cnt = (int64_t*)ccg_ws(ctx, WS_SNN_C, sizeof(int64_t) * (sp.nk * (n + 1) + 1));
    int* ov = (int*)ccg_ws(ctx, WS_SNN_E, sizeof(int) * (5 * n + 64));
    unsigned* dense = (unsigned*)ccg_ws(ctx, WS_SNN_D, sizeof(unsigned) * n * SNN_DENSE_BLOCKS);
    int32_t* pairs = (int32_t*)ccg_ws(ctx, WS_SNN_F, sizeof(int32_t) * 4 * (nkk + 16));
    int* bp = (int*)ccg_ws(ctx, WS_SNN_G, sizeof(int) * (nkk + n + 64));
    if (!hoff || !hosts_s || !cnt || !ov || !dense || !pairs || !bp) return CCG_ENOMEM;
    int* split = bp + nkk;
    int32_t* keys = pairs;
    int32_t* vals = pairs + (nkk + 16);
    int32_t* skey = vals + (nkk + 16);
    int32_t* sval = skey + (nkk + 16);
    int* ov2_list = ov + 4 * n;
    int* ov_count = ov + 5 * n;  // [1] block tier, [2] dense tier
    if (!roff) roff = hoff + (n + 1);
    // 1. host lists
    int bits = 1;
    while ((1LL << bits) <= n) ++bits;
    snn_pairs_kernel<<<(unsigned)ccg_cdiv(nkk, 256), 256, 0, st>>>(knn, n, kstride, kmax, keys, vals, ctx->d_err);
    int rc = ccg_sort_pairs_i32(ctx, keys, skey, vals, sval, nkk, bits, st);
    if (rc) return rc;
    snn_hoff_kernel<<<(unsigned)ccg_cdiv(n + 1, 256), 256, 0, st>>>(skey, nkk, n, hoff);
    snn_hosts_kernel<<<(unsigned)ccg_cdiv(nkk, 256), 256, 0, st>>>(skey, sval, kmax, hoff, n, hosts_s, bp);
    snn_split_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(hoff, hosts_s, n, split);
    // 2. row capacities
    const unsigned nblk = (unsigned)std::min<int64_t>(ccg_cdiv(n, SNN_WAVES), 16384);
    if (kmax <= 31)
        snn_items_kernel<true><<<(unsigned)std::min<int64_t>(ccg_cdiv(n, 8), 16384), 256, 0, st>>>(
            knn, n, kstride, kmax, hoff, bp, split, roff);
    else snn_items_kernel<false><<<nblk, 256, 0, st>>>(knn, n, kstride, kmax, hoff, bp, split, roff);
    rc = ccg_scan_i64(ctx, roff, roff, n, st);
    if (rc) return rc;
    // 3. build: sort tier -> hash tier -> block tier -> dense tier
    SnnRows rows{roff, rlen, nbr, wpk, cap};

    // size classes -> node lists (scan of packed one-hot class counts)
    CCG_REQUIRE(n < (1LL << SNN_CLS_BITS), "SNN: n must be below 2^%d", SNN_CLS_BITS);
    int64_t* cls = (int64_t*)ccg_ws(ctx, WS_SNN_H, sizeof(int64_t) * (n + 1 + 8) + sizeof(int) * 4 * n);
    if (!cls) return CCG_ENOMEM;
    int64_t* ccount = cls + (n + 1);
    int* lists = (int*)(ccount + 8);
    // copy nodes (NUMBER graphs only: RANK weights depend on the ranks)
    int* src = sp.type == CCG_SNN_NUMBER ? ov : nullptr;
    if (src) {
        if (kmax <= 31)
            snn_src_kernel<true><<<(unsigned)std::min<int64_t>(ccg_cdiv(n, 8), 16384), 256, 0, st>>>(knn, n, kstride,
                                                                                                      sp, src, nullptr);
        else
            snn_src_kernel<false><<<nblk, 256, 0, st>>>(knn, n, kstride, sp, src, nullptr);
    }
    snn_class_kernel<<<(unsigned)ccg_cdiv(std::max<int64_t>(n + 1, 64), 256), 256, 0, st>>>(roff, n, cls, cnt, sp.nk,
                                                                                           ov_count, src, nullptr);
    rc = ccg_scan_i64(ctx, cls, cls, n, st);
    if (rc) return rc;
    snn_class_scatter_kernel<<<(unsigned)ccg_cdiv(n + 1, 256), 256, 0, st>>>(cls, n, lists, ccount, nullptr);
    int* ov_list = ov + 3 * n;
#define SNN_BITONIC(CLS_, K_, GRID_, BK_)                                                                      \
    snn_bitonic_build_kernel<CLS_, K_, BK_><<<(GRID_), 64 * snn_bitonic_wpb(CLS_), 0, st>>>(                  \
        knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt, rows, lists + (CLS_) * n, ccount + (CLS_), ov_list, \
        ov_count + 1, src, SnnClsIn{})
#define SNN_BITONIC_ALL(K_)                                                   \
    do {                                                                      \
        SNN_BITONIC(0, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(0)), false); \
        SNN_BITONIC(1, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(1)), true);  \
        SNN_BITONIC(2, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(2)), true);  \
        SNN_BITONIC(3, K_, 1024u, false);                                     \
    } while (0)
    // classes 1-2 sort through the bucket tier (64 partner-range buckets, one
    // register network per lane; a bucket over its cap takes the wave-wide
    // bitonic sort): classes 1 / 2 172.5 -> 162.6 / 156.4 -> 154.7 us at cfg3.
    // (Round 4's merge-path tier of the sorted host runs measured slower --
    // 136 / 251 / 249 against 97 / 170 / 156 us per class -- and is gone.)
    if (sp.type == CCG_SNN_NUMBER) SNN_BITONIC_ALL(uint32_t);
    else SNN_BITONIC_ALL(unsigned long long);
#undef SNN_BITONIC_ALL
#undef SNN_BITONIC
    // nodes with more than SNN_BITONIC_MAX items: the block tier, then dense
    snn_block_kernel<false><<<256, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, cnt, rows, ov_list,
                                                 ov_count + 1, ov2_list, ov_count + 2, bp, SnnClsIn{});
    snn_dense_kernel<false><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, ov2_list,
                                                              ov_count + 2, dense, cnt, rows, bp, SnnClsIn{});
    if (src) snn_copy_rows_kernel<<<nblk, 256, 0, st>>>(n, sp, src, cnt, rows, lists + 3 * n, ccount + 3);
    rc = ccg_scan_i64(ctx, cnt, cnt, (int64_t)sp.nk * (n + 1), st);  // every graph's offsets in one scan
    if (rc) return rc;
    *cnt_out = cnt;
    *roff_out = roff;
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// Info of a class-level build (ccg_snn_classes_dev's d_info): u, status,
// required row capacity, then per graph its class-edge count (or -(required
// capacity) when the rows did not fit).
__global__ void snn_cls_info_kernel(const int64_t* __restrict__ ucount, const int* __restrict__ status,
                                    const int64_t* __restrict__ cnt, int64_t n, int nk,
                                    const int64_t* __restrict__ roff, int64_t rcap, int64_t* __restrict__ info) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const bool fit = roff[n] <= rcap;
    info[0] = *ucount;
    info[1] = *status;
    info[2] = roff[n];
    for (int t = 0; t < nk; ++t) info[3 + t] = fit ? cnt[(int64_t)t * (n + 1) + n] - cnt[(int64_t)t * (n + 1)] : -roff[n];
}

// Whether the class-level build serves these graphs: NUMBER weights, and the
// 4-bit prefix fields hold every class (a class has at most kmin + 1 rows).
static bool snn_cls_ok(const SnnSpec& sp) { return sp.type == CCG_SNN_NUMBER && sp.kk[0] <= 14; }

// The class-level graph (row classes above).  row_class[n] (class ordinal of
// every row), croot[n] (root row of ordinal c < u); class rows over ordinals:
// roff[n + 1] capacity-based (entries past u are empty), rlen, nbr (partner
// classes > c, ascending), wpk (per-graph packed weights), written when
// roff[n] <= cap.  *cnt_out: per-graph exclusive scans of the class rows'
// edge counts; *u_out: device u; *status_out: device int, nonzero when the
// input breaks the class contract (a prefix check failed: take the row pass).
static int snn_build_cls(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                         const SnnSpec& sp, hipStream_t st, int32_t* row_class, int32_t* croot, int64_t* roff,
                         int32_t* rlen, int32_t* nbr, uint32_t* wpk, int64_t cap, int64_t** cnt_out,
                         const int64_t** u_out, const int** status_out) {
    const int kmax = sp.kk[sp.nk - 1];
    const int64_t S = n * (kmax + 1);  // member slots (root row, rank)
    CCG_REQUIRE(S < (1LL << 31) - 64, "SNN: n*(kmax+1) too large");
    CCG_REQUIRE(n < (1LL << SNN_CLS_BITS), "SNN: n must be below 2^%d", SNN_CLS_BITS);
    int64_t* A = (int64_t*)ccg_ws(ctx, WS_SNN_A, sizeof(int64_t) * (2 * (n + 1) + 16));
    int2* hosts_s = (int2*)ccg_ws(ctx, WS_SNN_B, sizeof(int2) * (S + 1));
    int64_t* cnt = (int64_t*)ccg_ws(ctx, WS_SNN_C, sizeof(int64_t) * (sp.nk * (n + 1) + 1));
    int* ov = (int*)ccg_ws(ctx, WS_SNN_E, sizeof(int) * (6 * n + 192));
    unsigned* dense = (unsigned*)ccg_ws(ctx, WS_SNN_D, sizeof(unsigned) * n * SNN_DENSE_BLOCKS);
    int32_t* pairs = (int32_t*)ccg_ws(ctx, WS_SNN_F, sizeof(int32_t) * 4 * (S + 16));
    int* G = (int*)ccg_ws(ctx, WS_SNN_G, sizeof(int) * 3 * (S + 64));
    int64_t* cls = (int64_t*)ccg_ws(ctx, WS_SNN_H, sizeof(int64_t) * (n + 1 + 8) + sizeof(int) * 4 * n);
    if (!A || !hosts_s || !cnt || !ov || !dense || !pairs || !G || !cls) return CCG_ENOMEM;
    int64_t* hoff = A;            // [n + 1] (u + 1 used)
    int64_t* ord = A + (n + 1);   // [n + 1] isroot -> exclusive scan; ord[n] = u
    const int64_t* ucount = ord + n;
    int* src = ov;                // [n]
    int* root = ov + n;           // [n]
    int* crank = ov + 2 * n;      // [n]
    int* csize = ov + 3 * n;      // [n]
    int* ov_list = ov + 4 * n;    // [n]
    int* ov2_list = ov + 5 * n;   // [n]
    int* ov_count = ov + 6 * n;   // [64] (zeroed by the class kernel)
    int* status = ov_count + 64;  // [1]
    int32_t* keys = pairs;
    int32_t* vals = pairs + (S + 16);
    int32_t* skey = vals + (S + 16);
    int32_t* sval = skey + (S + 16);
    int* bp = G;
    int* mcls = G + (S + 64);
    unsigned* incl = (unsigned*)(G + 2 * (S + 64));
    int64_t* ccount = cls + (n + 1);
    int* lists = (int*)(ccount + 8);
    const unsigned nw8 = (unsigned)std::min<int64_t>(ccg_cdiv(n, 8), 16384);  // two rows per wave (PACK)
    const unsigned nw4 = (unsigned)std::min<int64_t>(ccg_cdiv(n, 4), 16384);
    const bool pack = kmax <= 31;
    // 1. classes: src chains (equal N+ sets, same cell), roots, ordinals, ranks
    if (pack) snn_src_kernel<true><<<nw8, 256, 0, st>>>(knn, n, kstride, sp, src, cell);
    else snn_src_kernel<false><<<nw4, 256, 0, st>>>(knn, n, kstride, sp, src, cell);
    snn_cls_root_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(src, n, root, ord, status);
    int rc = ccg_scan_i64(ctx, ord, ord, n, st);
    if (rc) return rc;
    if (pack)
        snn_cls_rank_kernel<true><<<nw8, 256, 0, st>>>(knn, n, kstride, kmax, root, ord, row_class, crank, croot, csize);
    else
        snn_cls_rank_kernel<false><<<nw4, 256, 0, st>>>(knn, n, kstride, kmax, root, ord, row_class, crank, croot,
                                                         csize);
    // 2. member classes of every root, the hosts of every class
    if (pack)
        snn_cls_members_kernel<true><<<nw8, 256, 0, st>>>(knn, n, kstride, sp, root, row_class, crank, mcls, incl,
                                                           keys, vals, status);
    else
        snn_cls_members_kernel<false><<<nw4, 256, 0, st>>>(knn, n, kstride, sp, root, row_class, crank, mcls, incl,
                                                            keys, vals, status);
    int bits = 1;
    while ((1LL << bits) <= n) ++bits;
    rc = ccg_sort_pairs_i32(ctx, keys, skey, vals, sval, S, bits, st);
    if (rc) return rc;
    snn_cls_hoff_kernel<<<(unsigned)ccg_cdiv(n + 1, 256), 256, 0, st>>>(skey, S, ucount, hoff);
    snn_cls_hosts_kernel<<<(unsigned)ccg_cdiv(S, 256), 256, 0, st>>>(skey, sval, kmax, hoff, ucount, row_class, incl,
                                                                     hosts_s, bp);
    // 3. capacities, size classes, build
    const SnnClsIn ci{croot, mcls, incl, ucount};
    if (pack) snn_cls_items_kernel<true><<<nw8, 256, 0, st>>>(n, kmax, ci, hoff, bp, roff);
    else snn_cls_items_kernel<false><<<nw4, 256, 0, st>>>(n, kmax, ci, hoff, bp, roff);
    rc = ccg_scan_i64(ctx, roff, roff, n, st);
    if (rc) return rc;
    SnnRows rows{roff, rlen, nbr, wpk, cap};
    snn_class_kernel<<<(unsigned)ccg_cdiv(std::max<int64_t>(n + 1, 64), 256), 256, 0, st>>>(roff, n, cls, cnt, sp.nk,
                                                                                           ov_count, nullptr, ucount);
    rc = ccg_scan_i64(ctx, cls, cls, n, st);
    if (rc) return rc;
    snn_class_scatter_kernel<<<(unsigned)ccg_cdiv(n + 1, 256), 256, 0, st>>>(cls, n, lists, ccount, ucount);
#define SNN_CBUILD(CLS_, K_, GRID_, BK_)                                                                         \
    snn_bitonic_build_kernel<CLS_, K_, BK_, true><<<(GRID_), 64 * snn_bitonic_wpb(CLS_), 0, st>>>(              \
        knn, n, kstride, sp, hoff, hosts_s, bp, nullptr, cnt, rows, lists + (CLS_) * n, ccount + (CLS_), ov_list, \
        ov_count + 1, nullptr, ci)
#define SNN_CBUILD_ALL(K_)                                                   \
    do {                                                                     \
        SNN_CBUILD(0, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(0)), false); \
        SNN_CBUILD(1, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(1)), true);  \
        SNN_CBUILD(2, K_, (unsigned)ccg_cdiv(n, snn_bitonic_wpb(2)), true);  \
        SNN_CBUILD(3, K_, 1024u, false);                                     \
    } while (0)
    // 32-bit keys (partner << 12 | three 4-bit fields) when they fit
    if (sp.nk <= 3 && n < (1LL << 20)) SNN_CBUILD_ALL(uint32_t);
    else SNN_CBUILD_ALL(unsigned long long);
#undef SNN_CBUILD_ALL
#undef SNN_CBUILD
    snn_block_kernel<true><<<256, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, cnt, rows, ov_list, ov_count + 1,
                                                ov2_list, ov_count + 2, bp, ci);
    snn_dense_kernel<true><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, ov2_list,
                                                             ov_count + 2, dense, cnt, rows, bp, ci);
    rc = ccg_scan_i64(ctx, cnt, cnt, (int64_t)sp.nk * (n + 1), st);
    if (rc) return rc;
    *cnt_out = cnt;
    *u_out = ucount;
    *status_out = status;
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_snn_classes_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                                   const int* ks, int nk, int32_t* row_class, int32_t* class_root, int64_t* class_off,
                                   int32_t* class_len, int32_t* nbr, uint32_t* wpk, int64_t cap, int64_t* d_info,
                                   void* stream) {
    CCG_REQUIRE(ctx && knn && ks && row_class && class_root && class_off && class_len && d_info,
                "ccg_snn_classes_dev: NULL argument");
    CCG_REQUIRE(cap == 0 || (nbr && wpk), "ccg_snn_classes_dev: NULL rows with cap > 0");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) - 1, "ccg_snn_classes_dev: bad n");
    SnnSpec sp;
    int rc = snn_spec(ks, nk, CCG_SNN_NUMBER, kstride, &sp);
    if (rc) return rc;
    CCG_REQUIRE(snn_cls_ok(sp), "ccg_snn_classes_dev: the smallest k must be <= 14 (4-bit class prefix fields)");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int t_all = ccg_timer_start(ctx, CCG_KT_SNN, st);
    int64_t* cnt = nullptr;
    const int64_t* u = nullptr;
    const int* status = nullptr;
    rc = snn_build_cls(ctx, knn, n, kstride, cell, sp, st, row_class, class_root, class_off, class_len, nbr, wpk, cap,
                       &cnt, &u, &status);
    if (rc) return rc;
    snn_cls_info_kernel<<<1, 64, 0, st>>>(u, status, cnt, n, nk, class_off, cap, d_info);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// Default row reservation of the per-graph API: entries per node per (kmax + 1).
#define SNN_ROW_RESERVE 40

extern "C" int ccg_snn_multi_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks,
                                 int nk, int type, int32_t* const* out_i, int32_t* const* out_j,
                                 double* const* out_w, const int64_t* caps, int64_t* const* d_nedges,
                                 void* stream) {
    CCG_REQUIRE(ctx && knn && ks && d_nedges, "ccg_snn_multi_dev: NULL argument");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) - 1, "ccg_snn_multi_dev: bad n");
    SnnSpec sp;
    int rc = snn_spec(ks, nk, type, kstride, &sp);
    if (rc) return rc;
    SnnOut out;
    for (int t = 0; t < SNN_MAXK; ++t) {
        out.cap[t] = 0;
        out.oi[t] = nullptr;
        out.oj[t] = nullptr;
        out.ow[t] = nullptr;
    }
    for (int t = 0; t < nk; ++t) {
        out.cap[t] = caps ? caps[t] : 0;
        if (out.cap[t] > 0) {
            CCG_REQUIRE(out_i && out_j && out_w && out_i[t] && out_j[t] && out_w[t],
                        "ccg_snn_multi_dev: NULL outputs with cap > 0");
            out.oi[t] = out_i[t];
            out.oj[t] = out_j[t];
            out.ow[t] = out_w[t];
        }
    }
    const int kmax = ks[nk - 1];
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int t_all = ccg_timer_start(ctx, CCG_KT_SNN, st);
    const int64_t rcap =
        ctx->snn_row_reserve > 0 ? ctx->snn_row_reserve : (int64_t)SNN_ROW_RESERVE * n * (kmax + 1);
    char* rbuf =
        (char*)ccg_ws(ctx, WS_SNN_ROWS, (sizeof(int32_t) + sizeof(uint32_t)) * rcap + sizeof(int32_t) * (n + 64));
    if (!rbuf) return CCG_ENOMEM;
    int32_t* nbr = (int32_t*)rbuf;
    uint32_t* wpk = (uint32_t*)(nbr + rcap);
    int32_t* rlen = (int32_t*)(wpk + rcap);
    int64_t* cnt = nullptr;
    const int64_t* roff = nullptr;
    rc = snn_build(ctx, knn, n, kstride, sp, st, nbr, wpk, rcap, nullptr, rlen, &cnt, &roff);
    if (rc) return rc;
    bool any_cap = false;
    for (int t = 0; t < nk; ++t) any_cap |= out.cap[t] > 0;
    if (any_cap) {
        SnnRows rows{roff, rlen, nbr, wpk, rcap};
        snn_emit_kernel<<<(unsigned)std::min<int64_t>(ccg_cdiv(n, 4), 16384), 256, 0, st>>>(n, sp, cnt, rows, out);
    }
    snn_copy_totals<<<1, 64, 0, st>>>(cnt, n, nk, roff, rcap, d_nedges[0], nk > 1 ? d_nedges[1] : nullptr,
                                      nk > 2 ? d_nedges[2] : nullptr, nk > 3 ? d_nedges[3] : nullptr);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_snn_rows_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks, int nk,
                                int type, int64_t* row_off, int32_t* row_len, int32_t* nbr, uint32_t* wpk,
                                int64_t cap, int64_t* d_nedges, void* stream) {
    CCG_REQUIRE(ctx && knn && ks && row_off && row_len && d_nedges, "ccg_snn_rows_dev: NULL argument");
    CCG_REQUIRE(cap == 0 || (nbr && wpk), "ccg_snn_rows_dev: NULL rows with cap > 0");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) - 1, "ccg_snn_rows_dev: bad n");
    SnnSpec sp;
    int rc = snn_spec(ks, nk, type, kstride, &sp);
    if (rc) return rc;
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int t_all = ccg_timer_start(ctx, CCG_KT_SNN, st);
    int64_t* cnt = nullptr;
    const int64_t* roff = nullptr;
    rc = snn_build(ctx, knn, n, kstride, sp, st, nbr, wpk, cap, row_off, row_len, &cnt, &roff);
    if (rc) return rc;
    snn_copy_totals<<<1, 64, 0, st>>>(cnt, n, nk, roff, cap, d_nedges, nk > 1 ? d_nedges + 1 : nullptr,
                                      nk > 2 ? d_nedges + 2 : nullptr, nk > 3 ? d_nedges + 3 : nullptr);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_snn_reserve(ccg_ctx* ctx, int64_t entries) {
    CCG_REQUIRE(ctx && entries >= 0, "ccg_snn_reserve: bad argument");
    ctx->snn_row_reserve = entries;
    return CCG_OK;
}

// ------------------------------------------------ host consumers (R, Python) --
// What a host clustering call (igraph::make_graph + cluster_leiden, :656-658)
// needs is every kNum graph as an edge list.  The device builds the graph
// ONCE -- for NUMBER graphs the class-level rows (snn_build_cls: the kernels
// of ccg_snn_classes_dev, which bench.py times), otherwise (RANK, or an input
// that breaks the class contract) the union graph's rows (snn_build: the
// kernels of ccg_snn_rows_dev) -- and copies the rows (8 B per class / union
// edge: partner + packed per-graph values), the per-graph row offsets and the
// row -> class map to pinned host memory the context owns.  Each graph's
// row-level (i, j, w) list is decoded from them on the host, sorted by (i, j).
// No per-graph edge list is formed on the device.
struct SnnStage {
    int64_t n = 0;
    SnnSpec sp{};
    bool classes = false;      // class-level rows (u classes) or row-level union rows
    int64_t u = 0;
    int64_t* roff = nullptr;   // n + 1 capacity-based row offsets (rows or class ordinals)
    int32_t* rlen = nullptr;   // n used lengths
    int64_t* cnt = nullptr;    // nk (n + 1): per-graph exclusive scans of the row edge counts
    int32_t* nbr = nullptr;    // roff[n] partners
    uint32_t* wpk = nullptr;   // roff[n] packed per-graph values
    int32_t* rcls = nullptr;   // n: class ordinal of every row (classes)
    size_t cap_n = 0, cap_l = 0, cap_e = 0, cap_w = 0, cap_c = 0, cap_r = 0;
    int64_t ne[SNN_MAXK] = {0, 0, 0, 0};  // row-level edges per graph
    // classes: the rows of every class (ascending) and the symmetric class
    // adjacency over the entries present in any graph (partner, packed
    // values), built once per pass for every graph's fetch
    std::vector<int64_t> mstart;
    std::vector<int32_t> mrows;
    std::vector<int64_t> aoff;
    std::vector<int32_t> adj;
    std::vector<uint32_t> av;
    bool valid = false;
};

static void snn_stage_release(SnnStage* s) {
    for (void* p : {(void*)s->roff, (void*)s->rlen, (void*)s->cnt, (void*)s->nbr, (void*)s->wpk, (void*)s->rcls})
        if (p) (void)hipHostFree(p);
    s->roff = nullptr;
    s->rlen = nullptr;
    s->cnt = nullptr;
    s->nbr = nullptr;
    s->wpk = nullptr;
    s->rcls = nullptr;
    s->cap_n = s->cap_l = s->cap_e = s->cap_w = s->cap_c = s->cap_r = 0;
}

void ccg_snn_stage_free(ccg_ctx* ctx) {
    if (!ctx || !ctx->snn_stage) return;
    SnnStage* s = (SnnStage*)ctx->snn_stage;
    snn_stage_release(s);
    delete s;
    ctx->snn_stage = nullptr;
}

template <typename T>
static int snn_host_grow(T** p, size_t* cap, size_t want) {
    if (*cap >= want && *p) return CCG_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t w = want + want / 8 + 64;
    CCG_HIP(hipHostMalloc((void**)p, sizeof(T) * w, hipHostMallocDefault));
    *cap = w;
    return CCG_OK;
}

static double snn_host_weight(const SnnSpec& sp, unsigned v, int t) {
    const unsigned b = (v >> (8 * t)) & 0xFFu;
    if (sp.type == CCG_SNN_NUMBER) return (double)b;
    const double w = (double)sp.kk[t] - 0.5 * (double)b;
    return w < 1e-6 ? 1e-6 : w;
}

static bool snn_host_has(const SnnSpec& sp, unsigned v, int t) {
    const unsigned b = (v >> (8 * t)) & 0xFFu;
    return sp.type == CCG_SNN_NUMBER ? b != 0u : b != 0xFFu;
}

// Host threads for the decode (the split does not change the output).
static unsigned snn_host_threads(int64_t work) {
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    return work < (1 << 16) ? 1u : nt;
}

template <typename F>
static void snn_host_parallel(int64_t n, unsigned nt, F&& f) {
    if (nt <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned q = 0; q < nt; ++q) th.emplace_back(f, n * q / nt, n * (q + 1) / nt);
    for (auto& x : th) x.join();
}

// The same with the thread's index: f(q, lo, hi) for q < nt.
template <typename F>
static void snn_host_parallel_q(int64_t n, unsigned nt, F&& f) {
    if (nt <= 1) {
        f(0u, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned q = 0; q < nt; ++q) th.emplace_back(f, q, n * q / nt, n * (q + 1) / nt);
    for (auto& x : th) x.join();
}

// Phase times of the host decode on stderr when CCG_SNN_HOST_PROFILE is set
// (tools and tuning only).
struct SnnHostClock {
    bool on = std::getenv("CCG_SNN_HOST_PROFILE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ccg snn host] %-28s %8.2f ms\n", what,
                     std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

// Class-level staging (NUMBER graphs): the rows of every class, the
// symmetric class adjacency over the entries present in any graph, and the
// row-level edge count of every graph, on host threads.  The adjacency's
// order within a class depends on the thread schedule; the fetch sorts each
// output row, so the edge lists do not.
static void snn_stage_classes(SnnStage* S, unsigned nt) {
    const int64_t n = S->n, u = S->u;
    const SnnSpec& sp = S->sp;
    const int nk = sp.nk;
    S->mstart.assign(u + 1, 0);
    for (int64_t x = 0; x < n; ++x) S->mstart[S->rcls[x] + 1]++;
    for (int64_t c = 0; c < u; ++c) S->mstart[c + 1] += S->mstart[c];
    S->mrows.resize(n);
    {
        std::vector<int64_t> cur(S->mstart.begin(), S->mstart.end() - 1);
        for (int64_t x = 0; x < n; ++x) S->mrows[cur[S->rcls[x]]++] = (int32_t)x;  // ascending within a class
    }
    const int64_t* ms = S->mstart.data();
    // A counting sort by class without atomics: thread q owns classes
    // [u q / nt, u (q + 1) / nt) and counts the entries naming each class in
    // its own histogram; a class's adjacency is its own present entries, then
    // the entries naming it in thread order (deterministic).
    std::vector<int64_t> own(u, 0);
    std::vector<int64_t> hist((size_t)nt * u, 0);
    snn_host_parallel_q(u, nt, [&](unsigned q, int64_t c0, int64_t c1) {
        int64_t* hq = hist.data() + (size_t)q * u;
        for (int64_t c = c0; c < c1; ++c) {
            int64_t k = 0;
            for (int r = 0; r < S->rlen[c]; ++r) {
                const int64_t e = S->roff[c] + r;
                if (S->wpk[e] == 0u) continue;  // (NUMBER: no graph has this pair)
                ++k;
                hq[S->nbr[e]]++;
            }
            own[c] = k;
        }
    });
    S->aoff.assign(u + 1, 0);
    for (int64_t c = 0; c < u; ++c) {  // offsets; the histograms become each thread's fill cursors
        int64_t base = S->aoff[c] + own[c];
        for (unsigned q = 0; q < nt; ++q) {
            const int64_t h = hist[(size_t)q * u + c];
            hist[(size_t)q * u + c] = base;
            base += h;
        }
        S->aoff[c + 1] = base;
    }
    S->adj.resize(S->aoff[u]);
    S->av.resize(S->aoff[u]);
    std::atomic<int64_t> netot[SNN_MAXK];
    for (auto& z : netot) z.store(0, std::memory_order_relaxed);
    snn_host_parallel_q(u, nt, [&](unsigned q, int64_t c0, int64_t c1) {
        int64_t* hq = hist.data() + (size_t)q * u;
        int64_t tot[SNN_MAXK] = {0, 0, 0, 0};
        for (int64_t c = c0; c < c1; ++c) {
            const int64_t mc = ms[c + 1] - ms[c];
            int64_t sm[SNN_MAXK] = {0, 0, 0, 0};
            int64_t a = S->aoff[c];
            for (int r = 0; r < S->rlen[c]; ++r) {
                const int64_t e = S->roff[c] + r;
                const unsigned v = S->wpk[e];
                if (v == 0u) continue;
                const int32_t h = S->nbr[e];
                S->adj[a] = h;
                S->av[a++] = v;
                const int64_t b = hq[h]++;
                S->adj[b] = (int32_t)c;
                S->av[b] = v;
                const int64_t mh = ms[h + 1] - ms[h];
                for (int t = 0; t < nk; ++t)
                    if (snn_host_has(sp, v, t)) sm[t] += mh;
            }
            // row-level edges: m_C m_H per class edge, m_C (m_C - 1) / 2 inside a class
            for (int t = 0; t < nk; ++t) tot[t] += mc * (mc - 1) / 2 + mc * sm[t];
        }
        for (int t = 0; t < nk; ++t) netot[t].fetch_add(tot[t], std::memory_order_relaxed);
    });
    for (int t = 0; t < nk; ++t) S->ne[t] = netot[t].load();
}

// One device pass + the copy to the host staging (rows or classes).
static int snn_graphs_stage(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                            const SnnSpec& sp, SnnStage* S, bool try_classes) {
    hipStream_t st = ctx->stream;
    const int nk = sp.nk, kmax = sp.kk[nk - 1];
    int32_t* dknn = (int32_t*)ccg_ws(ctx, WS_HOST_A, sizeof(int32_t) * n * kstride);
    int32_t* dcell = cell ? (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * n) : nullptr;
    int32_t* dcls = (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * 2 * n + 64);
    int64_t* dinfo = (int64_t*)ccg_ws(ctx, WS_HOST_E, 256);
    if (!dknn || (cell && !dcell) || !dcls || !dinfo) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dknn, knn, sizeof(int32_t) * n * kstride, hipMemcpyHostToDevice, st));
    if (cell) CCG_HIP(hipMemcpyAsync(dcell, cell, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
    int rc = snn_host_grow(&S->roff, &S->cap_n, (size_t)n + 1);
    if (!rc) rc = snn_host_grow(&S->rlen, &S->cap_l, (size_t)n);
    if (!rc) rc = snn_host_grow(&S->cnt, &S->cap_c, (size_t)nk * (n + 1));
    if (!rc) rc = snn_host_grow(&S->rcls, &S->cap_r, (size_t)n);
    if (rc) return rc;
    bool classes = try_classes && snn_cls_ok(sp);
    for (int attempt = 0; attempt < 3; ++attempt) {
        const int64_t rcap =
            ctx->snn_row_reserve > 0 ? ctx->snn_row_reserve : (int64_t)SNN_ROW_RESERVE * n * (kmax + 1);
        char* rbuf = (char*)ccg_ws(ctx, WS_SNN_ROWS,
                                   (sizeof(int32_t) + sizeof(uint32_t)) * rcap + sizeof(int32_t) * (n + 64));
        if (!rbuf) return CCG_ENOMEM;
        int32_t* nbr = (int32_t*)rbuf;
        uint32_t* wpk = (uint32_t*)(nbr + rcap);
        int32_t* rlen = (int32_t*)(wpk + rcap);
        int64_t* cnt = nullptr;
        const int64_t* roff = nullptr;
        int64_t info[3] = {0, 0, 0};
        if (classes) {
            int64_t* droff = (int64_t*)ccg_ws(ctx, WS_HOST_D, sizeof(int64_t) * (n + 1));
            if (!droff) return CCG_ENOMEM;
            const int64_t* u = nullptr;
            const int* status = nullptr;
            rc = snn_build_cls(ctx, dknn, n, kstride, dcell, sp, st, dcls, dcls + n, droff, rlen, nbr, wpk, rcap,
                               &cnt, &u, &status);
            if (rc) return rc;
            snn_cls_info_kernel<<<1, 64, 0, st>>>(u, status, cnt, n, nk, droff, rcap, dinfo);
            CCG_HIP(hipGetLastError());
            CCG_HIP(hipMemcpyAsync(info, dinfo, sizeof(info), hipMemcpyDeviceToHost, st));
            roff = droff;
        } else {
            rc = snn_build(ctx, dknn, n, kstride, sp, st, nbr, wpk, rcap, nullptr, rlen, &cnt, &roff);
            if (rc) return rc;
        }
        CCG_HIP(hipMemcpyAsync(S->roff, roff, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, st));
        rc = ccg_take_device_error(ctx);  // synchronises; an invalid index raised on the device fails here
        if (rc) return rc;
        if (classes && info[1] != 0) {  // the input breaks the class contract: the row-level pass
            classes = false;
            continue;
        }
        const int64_t need = S->roff[n];
        if (need > rcap) {  // the rows did not fit the reservation: grow it and rerun
            ctx->snn_row_reserve = need + need / 8;
            continue;
        }
        rc = snn_host_grow(&S->nbr, &S->cap_e, (size_t)std::max<int64_t>(need, 1));
        if (!rc) rc = snn_host_grow(&S->wpk, &S->cap_w, (size_t)std::max<int64_t>(need, 1));
        if (rc) return rc;
        CCG_HIP(hipMemcpyAsync(S->rlen, rlen, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipMemcpyAsync(S->cnt, cnt, sizeof(int64_t) * nk * (n + 1), hipMemcpyDeviceToHost, st));
        if (classes) CCG_HIP(hipMemcpyAsync(S->rcls, dcls, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
        if (need > 0) {
            CCG_HIP(hipMemcpyAsync(S->nbr, nbr, sizeof(int32_t) * need, hipMemcpyDeviceToHost, st));
            CCG_HIP(hipMemcpyAsync(S->wpk, wpk, sizeof(uint32_t) * need, hipMemcpyDeviceToHost, st));
        }
        CCG_HIP(hipStreamSynchronize(st));
        S->n = n;
        S->sp = sp;
        S->classes = classes;
        S->u = classes ? info[0] : n;
        S->mstart.clear();
        S->mrows.clear();
        S->aoff.clear();
        S->adj.clear();
        S->av.clear();
        if (!classes) {
            for (int t = 0; t < nk; ++t) S->ne[t] = S->cnt[(int64_t)t * (n + 1) + n] - S->cnt[(int64_t)t * (n + 1)];
        } else {
            SnnHostClock clk;
            snn_stage_classes(S, snn_host_threads(need * nk));
            clk.lap("stage: classes + adjacency");
        }
        S->valid = true;
        return CCG_OK;
    }
    ccg_set_error("ccg_snn_graphs: row reservation could not be satisfied");
    return CCG_ENOMEM;
}

extern "C" int ccg_snn_graphs_cells(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int32_t* cell,
                                    const int* ks, int nk, int type, int64_t* nedges) {
    CCG_REQUIRE(ctx && knn && ks && nedges, "ccg_snn_graphs: NULL argument");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) - 1 && kstride >= 1, "ccg_snn_graphs: bad sizes");
    SnnSpec sp;
    int rc = snn_spec(ks, nk, type, kstride, &sp);
    if (rc) return rc;
    for (int64_t t = 0; t < n * kstride; ++t)
        CCG_REQUIRE(knn[t] >= 0 && knn[t] < n && knn[t] != t / kstride,
                    "ccg_snn_graphs: neighbour index out of range or self at %lld", (long long)t);
    CCG_HIP(hipSetDevice(ctx->device));
    if (!ctx->snn_stage) ctx->snn_stage = new SnnStage();
    SnnStage* S = (SnnStage*)ctx->snn_stage;
    S->valid = false;
    rc = snn_graphs_stage(ctx, knn, n, kstride, cell, sp, S, true);
    if (rc) return rc;
    for (int t = 0; t < nk; ++t) nedges[t] = S->ne[t];
    return CCG_OK;
}

extern "C" int ccg_snn_graphs(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks, int nk,
                              int type, int64_t* nedges) {
    return ccg_snn_graphs_cells(ctx, knn, n, kstride, nullptr, ks, nk, type, nedges);
}

extern "C" int ccg_snn_graph_fetch(ccg_ctx* ctx, int t, int32_t* out_i, int32_t* out_j, double* out_w,
                                   int64_t cap) {
    CCG_REQUIRE(ctx, "ccg_snn_graph_fetch: NULL ctx");
    SnnStage* S = (SnnStage*)ctx->snn_stage;
    CCG_REQUIRE(S && S->valid, "ccg_snn_graph_fetch: no graphs staged (call ccg_snn_graphs first)");
    CCG_REQUIRE(t >= 0 && t < S->sp.nk, "ccg_snn_graph_fetch: graph %d of %d", t, S->sp.nk);
    const int64_t n = S->n;
    const int64_t ne = S->ne[t];
    if (cap < ne) {
        ccg_set_error("ccg_snn_graph_fetch: capacity %lld < %lld edges", (long long)cap, (long long)ne);
        return CCG_ECAP;
    }
    const SnnSpec sp = S->sp;
    const unsigned nt = snn_host_threads(ne);
    if (!S->classes) {
        // union rows: graph t's entries of row j, already ascending, at the
        // row's per-graph offset
        const int64_t* c = S->cnt + (int64_t)t * (n + 1);
        auto work = [&](int64_t j0, int64_t j1) {
            for (int64_t j = j0; j < j1; ++j) {
                int64_t e = c[j] - c[0];
                const int64_t ro = S->roff[j];
                const int u = S->rlen[j];
                for (int q = 0; q < u; ++q) {
                    const unsigned v = S->wpk[ro + q];
                    if (!snn_host_has(sp, v, t)) continue;
                    if (out_i) out_i[e] = (int32_t)j;
                    if (out_j) out_j[e] = S->nbr[ro + q];
                    if (out_w) out_w[e] = snn_host_weight(sp, v, t);
                    ++e;
                }
            }
        };
        snn_host_parallel(n, nt, work);
        return CCG_OK;
    }
    // classes: per row x of class C every row y > x of C (weight k + 1: one
    // common set) and of each class adjacent to C in graph t (the staged
    // adjacency's entries present in t), sorted by y
    SnnHostClock clk;
    const int64_t* ms = S->mstart.data();
    const int32_t* mr = S->mrows.data();
    const int64_t* aoff = S->aoff.data();
    const int32_t* adj = S->adj.data();
    const uint32_t* av = S->av.data();
    const unsigned wself = (unsigned)(sp.kk[t] + 1);
    // rows of class h above x: [first, end) of its ascending member list
    auto above = [&](int64_t h, int32_t x) {
        const int32_t* b = mr + ms[h];
        const int32_t* e = mr + ms[h + 1];
        if (e - b > 16) return std::make_pair(std::upper_bound(b, e, x), e);
        while (b < e && *b <= x) ++b;  // (a class is mostly a handful of rows: a linear scan)
        return std::make_pair(b, e);
    };
    std::vector<int64_t> roff(n + 1, 0);
    snn_host_parallel(n, nt, [&](int64_t x0, int64_t x1) {
        for (int64_t x = x0; x < x1; ++x) {
            const int64_t c = S->rcls[x];
            auto r = above(c, (int32_t)x);
            int64_t k = r.second - r.first;
            for (int64_t a = aoff[c]; a < aoff[c + 1]; ++a) {
                if (!snn_host_has(sp, av[a], t)) continue;
                auto q = above(adj[a], (int32_t)x);
                k += q.second - q.first;
            }
            roff[x + 1] = k;
        }
    });
    for (int64_t x = 0; x < n; ++x) roff[x + 1] += roff[x];
    clk.lap("fetch: row counts");
    if (roff[n] != ne) {
        ccg_set_error("ccg_snn_graph_fetch: internal count mismatch (%lld vs %lld)", (long long)roff[n], (long long)ne);
        return CCG_EINVAL;
    }
    snn_host_parallel(n, nt, [&](int64_t x0, int64_t x1) {
        std::vector<uint64_t> buf;  // y << 8 | weight: one 64-bit sort key per edge
        for (int64_t x = x0; x < x1; ++x) {
            buf.clear();
            const int64_t c = S->rcls[x];
            auto r = above(c, (int32_t)x);
            for (auto p = r.first; p < r.second; ++p) buf.push_back((uint64_t)*p << 8 | wself);
            for (int64_t a = aoff[c]; a < aoff[c + 1]; ++a) {
                const unsigned v = av[a];
                if (!snn_host_has(sp, v, t)) continue;
                const uint64_t w = (v >> (8 * t)) & 0xFFu;
                auto q = above(adj[a], (int32_t)x);
                for (auto p = q.first; p < q.second; ++p) buf.push_back((uint64_t)*p << 8 | w);
            }
            std::sort(buf.begin(), buf.end());
            const int64_t e = roff[x];
            const int64_t m = (int64_t)buf.size();
            if (out_i) std::fill(out_i + e, out_i + e + m, (int32_t)x);
            if (out_j)
                for (int64_t z = 0; z < m; ++z) out_j[e + z] = (int32_t)(buf[z] >> 8);
            if (out_w)
                for (int64_t z = 0; z < m; ++z) out_w[e + z] = (double)(buf[z] & 0xFFu);
        }
    });
    clk.lap("fetch: rows");
    return CCG_OK;
}

extern "C" int ccg_snn_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, int k, int type,
                           int32_t* out_i, int32_t* out_j, double* out_w, int64_t cap, int64_t* d_nedges,
                           void* stream) {
    CCG_REQUIRE(k >= 1 && k <= kstride, "ccg_snn_dev: need 1 <= k <= kstride");
    int32_t* oi[1] = {out_i};
    int32_t* oj[1] = {out_j};
    double* ow[1] = {out_w};
    int64_t caps[1] = {cap};
    int64_t* dn[1] = {d_nedges};
    return ccg_snn_multi_dev(ctx, knn, n, kstride, &k, 1, type, oi, oj, ow, caps, dn, stream);
}

extern "C" int ccg_snn(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, int k, int type,
                       int32_t* out_i, int32_t* out_j, double* out_w, int64_t cap, int64_t* nedges) {
    CCG_REQUIRE(ctx && knn && nedges, "ccg_snn: NULL argument");
    CCG_REQUIRE(n >= 1 && kstride >= 1, "ccg_snn: bad sizes");
    CCG_REQUIRE(k >= 1 && k <= kstride, "ccg_snn: need 1 <= k <= kstride");
    int64_t ne = 0;
    int rc = ccg_snn_graphs(ctx, knn, n, kstride, &k, 1, type, &ne);
    if (rc) return rc;
    *nedges = ne;
    if (ne > cap) {
        ccg_set_error("ccg_snn: capacity %lld < required %lld edges", (long long)cap, (long long)ne);
        return CCG_ECAP;
    }
    return ccg_snn_graph_fetch(ctx, 0, out_i, out_j, out_w, cap);
}

extern "C" int ccg_snn_multi(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks, int nk, int type,
                             int32_t* const* out_i, int32_t* const* out_j, double* const* out_w, const int64_t* caps,
                             int64_t* nedges) {
    CCG_REQUIRE(ctx && knn && ks && nedges, "ccg_snn_multi: NULL argument");
    CCG_REQUIRE(n >= 1 && kstride >= 1 && nk >= 1 && nk <= SNN_MAXK, "ccg_snn_multi: bad sizes");
    int rc = ccg_snn_graphs(ctx, knn, n, kstride, ks, nk, type, nedges);
    if (rc) return rc;
    bool short_cap = false;
    for (int t = 0; t < nk; ++t) short_cap |= !caps || nedges[t] > caps[t];
    if (short_cap) {
        ccg_set_error("ccg_snn_multi: capacities smaller than the edge counts (reported in nedges)");
        return CCG_ECAP;
    }
    for (int t = 0; t < nk; ++t) {
        rc = ccg_snn_graph_fetch(ctx, t, out_i ? out_i[t] : nullptr, out_j ? out_j[t] : nullptr,
                                 out_w ? out_w[t] : nullptr, caps[t]);
        if (rc) return rc;
    }
    return CCG_OK;
}
