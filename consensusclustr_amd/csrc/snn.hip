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
//   3. build, one wave per node: the items are gathered, ordered by partner
//      and merged (sum for NUMBER, bytewise min for RANK) into the node's row
//      of (partner, packed per-graph values), ascending partner -- the union
//      graph (the largest k) in CSR form with per-graph counts.  Tiers by
//      size: register/LDS bucket sort (<= 1024 items), a 2048-slot LDS hash
//      table, a 16K-slot block table, an exact O(n) dense pass.
//   4. per-graph edge lists (i < j sorted by (i, j)) are streamed from the
//      rows when the caller wants them (ccg_snn_multi_dev).
#include <algorithm>
#include <cstdlib>

#include "ccg_internal.h"

#define WAVE_LDS_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)

#define SNN_MAXK 4           // graphs per pass (|kNum| <= 4)
#define SNN_WT 2048          // wave hash-table slots
#define SNN_WAVES 4          // waves per block in the wave kernels
#define SNN_BT 16384         // block table slots (overflow path)
#define SNN_DENSE_BLOCKS 64  // concurrent dense-path nodes
#define SNN_EMPTY (-1)

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

// Items M_j of every node: the row capacities.
__global__ __launch_bounds__(256) void snn_items_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        int kmax, const int64_t* __restrict__ hoff,
                                                        const int* __restrict__ bp, const int* __restrict__ split,
                                                        int64_t* __restrict__ cap) {
    const int lane = threadIdx.x & 63;
    for (int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (int64_t)gridDim.x * 4) {
        const SnnMember m = snn_member(knn, n, kstride, kmax, j, lane, hoff, bp, split);
        int v = m.len;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) cap[j] = v;
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

// ------------------------------------------------------- sort (ESC) tier --
// Nodes with at most 64*R items: the items are gathered to registers (all
// host loads of the node in flight at once), bucketed by partner into an LDS
// stage (histogram, wave scan, scatter), ranked inside their bucket by
// (partner, stage slot) and rewritten in order; one pass over the sorted
// stage merges equal partners and writes the row.  R is chosen per node
// (4, 8, 12 or 16 rounds of 64 items) so a node pays for its own size only.
#ifndef SNN_SNB
#define SNN_SNB 240   // buckets
#endif
#define SNN_SI 1024   // items staged per wave (largest sort-tier node)

template <int SI>
struct SnnSortLds {
    unsigned long long stage[SI];
    union {
        struct {  // gather phase: member headers
            long long h0[64];
            long long hend[64];
            int cur[64];
            int pre[65];
        } g;
        struct {  // bucket phase
            int hist[SNN_SNB];
            int bst[SNN_SNB + 1];
        } s;
    } u;
};

template <int R, int SI>
__device__ __forceinline__ void snn_sort_node(SnnSortLds<SI>& L, const SnnSpec& sp, int64_t n, int64_t j, int M,
                                              int lane, const int2* __restrict__ hosts_s,
                                              const SnnRows& rows, int64_t* __restrict__ cnt) {
    unsigned long long* stage = L.stage;
    // gather: every host load of the node is issued before any is used;
    // item r is held as (p << 32 | member << 8 | host rank) until its
    // contribution is known, then as (p << 32 | packed contribution)
    unsigned long long e[R];
    int mi = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int t = 64 * r + lane;
        e[r] = ~0ull;
        if (t < M) {
            while (L.u.g.pre[mi + 1] <= t) ++mi;
            const long long q = L.u.g.h0[mi] + (t - L.u.g.pre[mi]);
            int p = L.u.g.cur[mi], rp = 0;
            if (q < L.u.g.hend[mi]) {
                const int2 h = hosts_s[q];
                p = h.x;
                rp = h.y;
            }
            e[r] = ((unsigned long long)(unsigned)p << 32) | (unsigned)(mi << 8) | (unsigned)rp;
        }
    }
    WAVE_LDS_SYNC();
    int* hist = L.u.s.hist;
    int* bst = L.u.s.bst;
    for (int b = lane; b < SNN_SNB; b += 64) hist[b] = 0;
    WAVE_LDS_SYNC();
    const float inv = (float)SNN_SNB / (float)(n - j);
    int bk[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bk[r] = -1;
        if (e[r] != ~0ull) {
            const unsigned lo = (unsigned)e[r];
            const unsigned c = snn_contrib(sp, (int)(lo >> 8), (int)(lo & 0xFFu));
            const int p = (int)(e[r] >> 32);
            if (c != sp.init) {
                e[r] = ((unsigned long long)(unsigned)p << 32) | c;
                bk[r] = min(SNN_SNB - 1, (int)((float)(p - (int)j - 1) * inv));
                atomicAdd(&hist[bk[r]], 1);
            } else {
                e[r] = ~0ull;
            }
        }
    }
    WAVE_LDS_SYNC();
    // bucket starts: lane owns buckets BPL*lane .. BPL*lane+BPL-1
    constexpr int BPL = (SNN_SNB + 63) / 64;
    int hv[BPL], hs = 0;
#pragma unroll
    for (int i = 0; i < BPL; ++i) {
        const int b = BPL * lane + i;
        hv[i] = b < SNN_SNB ? hist[b] : 0;
        hs += hv[i];
    }
    int sc = hs;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(sc, o);
        if (lane >= o) sc += y;
    }
    const int V = __shfl(sc, 63);
    int run = sc - hs;
    WAVE_LDS_SYNC();
#pragma unroll
    for (int i = 0; i < BPL; ++i) {
        const int b = BPL * lane + i;
        if (b < SNN_SNB) {
            bst[b] = run;
            hist[b] = run;  // scatter cursor
        }
        run += hv[i];
    }
    if (lane == 0) bst[SNN_SNB] = V;
    WAVE_LDS_SYNC();
    int pos[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        pos[r] = 0;
        if (bk[r] >= 0) {
            pos[r] = atomicAdd(&hist[bk[r]], 1);
            stage[pos[r]] = e[r];
        }
    }
    WAVE_LDS_SYNC();
    // rank inside the bucket by (p, slot)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (bk[r] >= 0) {
            const int b0 = bst[bk[r]], b1 = bst[bk[r] + 1];
            const unsigned key = (unsigned)(e[r] >> 32);
            int rank = 0;
            for (int q = b0; q < b1; ++q) {
                const unsigned kq = (unsigned)(stage[q] >> 32);
                rank += (kq < key || (kq == key && q < pos[r])) ? 1 : 0;
            }
            pos[r] = b0 + rank;
        }
    }
    WAVE_LDS_SYNC();
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (bk[r] >= 0) stage[pos[r]] = e[r];
    WAVE_LDS_SYNC();
    // unique partners: the first of each run of equal keys merges the run
    const bool write = rows.roff[n] <= rows.cap;
    const int64_t ro = rows.roff[j];
    int u = 0;
    int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
    for (int q0 = 0; q0 < V; q0 += 64) {
        const int q = q0 + lane;
        unsigned key = 0, agg = 0;
        bool first = false;
        if (q < V) {
            const unsigned long long x = stage[q];
            key = (unsigned)(x >> 32);
            first = q == 0 || (unsigned)(stage[q - 1] >> 32) != key;
            if (first) {
                agg = (unsigned)x;
                for (int q2 = q + 1; q2 < V; ++q2) {
                    const unsigned long long y = stage[q2];
                    if ((unsigned)(y >> 32) != key) break;
                    agg = snn_combine(sp.type, agg, (unsigned)y);
                }
            }
        }
        const unsigned long long m = __ballot(first);
        if (first) {
            if (write) {
                const int64_t o = ro + u + __popcll(m & lanemask_lt());
                rows.nbr[o] = (int32_t)key;
                rows.wpk[o] = agg;
            }
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t)
                if (t < sp.nk && graph_has(sp, agg, t)) ++c4[t];
        }
        u += __popcll(m);
    }
    snn_row_counts(sp, c4, n, j, lane, cnt);
    if (lane == 0) rows.rlen[j] = u;
}

// Three size classes, each its own kernel over its own node list (built by a
// scan, so in ascending node order): CLS 0 sorts the nodes with <= 320 items
// (R = 3 or 5), CLS 1 those with 321..640 (R = 8 or 10), CLS 2 641..1024
// (R = 12 or 16).  The LDS stage is sized to the class, so small nodes --
// the majority -- run at more waves per SIMD to hide the gather latency.  One
// node per wave: no node loop whose invariants the compiler would hoist into
// the item registers.
template <int CLS>
__global__ __launch_bounds__(64 * SNN_WAVES, CLS == 0 ? 8 : (CLS == 1 ? 6 : 4)) void snn_sort_build_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp, const int64_t* __restrict__ hoff,
    const int2* __restrict__ hosts_s, const int* __restrict__ bp, const int* __restrict__ split,
    int64_t* __restrict__ cnt, SnnRows rows, const int* __restrict__ list, const int64_t* __restrict__ count) {
    constexpr int SI = CLS == 0 ? 320 : (CLS == 1 ? 640 : 1024);
    __shared__ SnnSortLds<SI> lds_all[SNN_WAVES];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SnnSortLds<SI>& L = lds_all[wv];
    const int kmax = sp.kk[sp.nk - 1];
    const int64_t f = (int64_t)blockIdx.x * SNN_WAVES + wv;
    if (f >= *count) return;
    const int64_t j = list[f];
    const SnnMember m = snn_member(knn, n, kstride, kmax, j, lane, hoff, bp, split);
    int incl = m.len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int M = __shfl(incl, 63);
    if (lane <= kmax) {
        L.u.g.pre[lane] = incl - m.len;
        L.u.g.h0[lane] = m.h0;
        L.u.g.hend[lane] = m.hend;
        L.u.g.cur[lane] = m.cur;
    }
    if (lane == 0) L.u.g.pre[kmax + 1] = M;
    WAVE_LDS_SYNC();
    if (CLS == 0) {
        if (M <= 192) snn_sort_node<3>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
        else snn_sort_node<5>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
    } else if (CLS == 1) {
        if (M <= 512) snn_sort_node<8>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
        else snn_sort_node<10>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
    } else {
        if (M <= 768) snn_sort_node<12>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
        else snn_sort_node<16>(L, sp, n, j, M, lane, hosts_s, rows, cnt);
    }
}

// Size class of every node from its capacity (items): packed one-hot counts
// (class c in bits 21c..21c+20) for one scan that ranks every class at once.
// Classes 0..2 in 21-bit fields (n < 2^21); class 3's rank is the node index
// minus the other three.
#define SNN_CLS_BITS 21
__global__ void snn_class_kernel(const int64_t* __restrict__ roff, int64_t n, int64_t* __restrict__ cls) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t M = roff[j + 1] - roff[j];
    const int c = M <= 320 ? 0 : (M <= 640 ? 1 : (M <= SNN_SI ? 2 : 3));
    cls[j] = c < 3 ? 1LL << (SNN_CLS_BITS * c) : 0;
}

// Lists of each class in node order; counts[c] = class size.
__global__ void snn_class_scatter_kernel(const int64_t* __restrict__ cls_scan, int64_t n, int* __restrict__ lists,
                                         int64_t* __restrict__ counts) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    const int64_t mask = (1LL << SNN_CLS_BITS) - 1;
    const int64_t v = cls_scan[j];
    int64_t r[4];
    r[0] = v & mask;
    r[1] = (v >> SNN_CLS_BITS) & mask;
    r[2] = (v >> (2 * SNN_CLS_BITS)) & mask;
    r[3] = j - r[0] - r[1] - r[2];
    if (j == n) {
        for (int c = 0; c < 4; ++c) counts[c] = r[c];
        return;
    }
    const int64_t d = cls_scan[j + 1] - v;  // this node's one-hot class (0 for class 3)
    const int c = d == 1 ? 0 : (d == (1LL << SNN_CLS_BITS) ? 1 : (d == (1LL << (2 * SNN_CLS_BITS)) ? 2 : 3));
    lists[c * n + r[c]] = (int)j;
}

// ---------------------------------------------------------- hash tier --
// Nodes with more items: one wave per node builds an LDS hash table of
// 64-bit slots (partner p << 32 | packed per-graph values): a new partner
// costs one CAS, a repeat one add.  The table is compacted, sorted by p and
// written to the row.  Nodes beyond its capacity go to the block tier.
#define SNN_EMPTY64 (~0ull)

__device__ __forceinline__ bool table_insert64(unsigned long long* tab, int p, unsigned c, const SnnSpec& sp,
                                               int bits, int T) {
    unsigned s = snn_hash(p, bits);
    const unsigned long long want = ((unsigned long long)(unsigned)p << 32) | c;
    for (int probe = 0; probe < T; ++probe) {
        unsigned long long cur = __hip_atomic_load(&tab[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == SNN_EMPTY64) {
            const unsigned long long old = atomicCAS(&tab[s], SNN_EMPTY64, want);
            if (old == SNN_EMPTY64) return true;
            cur = old;
        }
        if ((unsigned)(cur >> 32) == (unsigned)p) {
            if (sp.type == CCG_SNN_NUMBER) {
                atomicAdd(&tab[s], (unsigned long long)c);  // per-byte counts never carry
            } else {
                while (true) {
                    const unsigned nv = bytewise_min((unsigned)cur, c);
                    if (nv == (unsigned)cur) break;
                    const unsigned long long nw = (cur & 0xFFFFFFFF00000000ull) | nv;
                    const unsigned long long old = atomicCAS(&tab[s], cur, nw);
                    if (old == cur) break;
                    cur = old;
                }
            }
            return true;
        }
        s = (s + 1) & (T - 1);
    }
    return false;
}

template <int WT>
constexpr int snn_log2() {
    int b = 0;
    while ((1 << b) < WT) ++b;
    return b;
}

// Sort a node's u compacted entries (tab[0..u), distinct partners p in (j, n))
// by p and store them to the row.  Each lane holds entries c = r*64 + lane
// in registers; a 128-bucket split on p (monotone in p) gives every entry its
// bucket's start by a histogram + wave scan, the entries are scattered into
// bucket order in tab, and each entry's final place is its bucket start plus
// the number of smaller partners in its (small) bucket.
#define SNN_NB 128
template <int RMAX>
__device__ __forceinline__ void snn_bucket_store(unsigned long long* tab, int u, int lane, int64_t j, int64_t n,
                                                 int* hist, int* bst, int32_t* __restrict__ nbr,
                                                 uint32_t* __restrict__ wpk, bool write) {
    unsigned long long e[RMAX];
    int bk[RMAX];
    const float inv = (float)SNN_NB / (float)(n - j - 1);
    for (int b = lane; b < SNN_NB; b += 64) hist[b] = 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
        const int c = r * 64 + lane;
        e[r] = c < u ? tab[c] : SNN_EMPTY64;
        const int p = (int)(e[r] >> 32);
        bk[r] = min(SNN_NB - 1, (int)((float)(p - (int)j - 1) * inv));
    }
    WAVE_LDS_SYNC();
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
        if (r * 64 + lane < u) atomicAdd(&hist[bk[r]], 1);
    WAVE_LDS_SYNC();
    const int h0 = hist[2 * lane], h1 = hist[2 * lane + 1];
    int incl = h0 + h1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int excl = incl - h0 - h1;
    bst[2 * lane] = excl;
    bst[2 * lane + 1] = excl + h0;
    hist[2 * lane] = excl;  // hist becomes the scatter cursor
    hist[2 * lane + 1] = excl + h0;
    if (lane == 0) bst[SNN_NB] = u;
    WAVE_LDS_SYNC();
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
        if (r * 64 + lane < u) tab[atomicAdd(&hist[bk[r]], 1)] = e[r];
    WAVE_LDS_SYNC();
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
        if (r * 64 + lane < u) {
            const int b0 = bst[bk[r]], b1 = bst[bk[r] + 1];
            const unsigned p = (unsigned)(e[r] >> 32);
            int rank = 0;
            for (int i = b0; i < b1; ++i) rank += (unsigned)(tab[i] >> 32) < p;
            if (write) {
                nbr[b0 + rank] = (int32_t)p;
                wpk[b0 + rank] = (uint32_t)e[r];
            }
        }
    }
}

template <int WT>
struct SnnWaveLds {
    unsigned long long tab[WT];
    union {
        struct {  // gather phase: member headers
            long long h0[64];
            long long hend[64];
            int cur[64];
            int pre[65];
        } g;
        struct {  // sort phase: bucket histogram / starts
            int hist[SNN_NB];
            int bst[SNN_NB + 1];
        } s;
    } u;
};

template <int WT>
__global__ __launch_bounds__(64 * SNN_WAVES, 2) void snn_wave_build_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp, const int64_t* __restrict__ hoff,
    const int2* __restrict__ hosts_s, const int* __restrict__ bp, const int* __restrict__ split,
    int64_t* __restrict__ cnt, SnnRows rows, const int* __restrict__ in_list, const int64_t* __restrict__ in_count,
    int* __restrict__ ov_list, int* __restrict__ ov_count) {
    __shared__ SnnWaveLds<WT> lds_all[SNN_WAVES];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SnnWaveLds<WT>& L = lds_all[wv];
    unsigned long long* tab = L.tab;
    const int kmax = sp.kk[sp.nk - 1];
    constexpr int CAP = WT * 3 / 4;
    const bool write = rows.roff[n] <= rows.cap;
    const int64_t nn = *in_count;
    for (int64_t f = (int64_t)blockIdx.x * SNN_WAVES + wv; f < nn; f += (int64_t)gridDim.x * SNN_WAVES) {
        const int64_t j = in_list[f];
        for (int s = lane; s < WT; s += 64) tab[s] = SNN_EMPTY64;
        // Flat gather over the partners p > j; host entries are fetched one
        // round ahead so their latency hides behind the current LDS inserts.
        const SnnMember mem = snn_member(knn, n, kstride, kmax, j, lane, hoff, bp, split);
        int incl = mem.len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int M = __shfl(incl, 63);
        if (lane <= kmax) {
            L.u.g.pre[lane] = incl - mem.len;
            L.u.g.h0[lane] = mem.h0;
            L.u.g.hend[lane] = mem.hend;
            L.u.g.cur[lane] = mem.cur;
        }
        if (lane == 0) L.u.g.pre[kmax + 1] = M;
        WAVE_LDS_SYNC();
        int mi = 0;
        auto fetch = [&](int t, int& p, int& rp, int& ii) {
            p = -1;
            rp = 0;
            ii = 0;
            if (t < M) {
                while (L.u.g.pre[mi + 1] <= t) ++mi;
                ii = mi;
                const long long q = L.u.g.h0[mi] + (t - L.u.g.pre[mi]);
                if (q < L.u.g.hend[mi]) {
                    const int2 hr = hosts_s[q];
                    p = hr.x;
                    rp = hr.y;
                } else {
                    p = L.u.g.cur[mi];
                }
            }
        };
        int p, rp, ii;
        fetch(lane, p, rp, ii);
        bool full = false;
        for (int t0 = 0; t0 < M; t0 += 64) {
            int np, nrp, nii;
            fetch(t0 + 64 + lane, np, nrp, nii);
            bool ok = true;
            if (p >= 0) {
                const unsigned c = snn_contrib(sp, ii, rp);
                if (c != sp.init) ok = table_insert64(tab, p, c, sp, snn_log2<WT>(), WT);
            }
            full = __any(!ok);
            if (full) break;
            p = np;
            rp = nrp;
            ii = nii;
        }
        WAVE_LDS_SYNC();
        // Compact: every lane reads its WT/64 slots (slot r*64 + lane) to
        // registers first, so the in-place writes cannot overtake a pending read.
        int u = 0;
        if (!full) {
            unsigned long long e[WT / 64];
#pragma unroll
            for (int r = 0; r < WT / 64; ++r) e[r] = tab[r * 64 + lane];
            WAVE_LDS_SYNC();
#pragma unroll
            for (int r = 0; r < WT / 64; ++r) {
                const bool occ = e[r] != SNN_EMPTY64;
                const unsigned long long m = __ballot(occ);
                if (occ) tab[u + __popcll(m & lanemask_lt())] = e[r];
                u += __popcll(m);
            }
            WAVE_LDS_SYNC();
        }
        if (full || u > CAP) {
            if (lane == 0) ov_list[atomicAdd(ov_count, 1)] = (int)j;
            continue;
        }
        const int64_t ro = rows.roff[j];
        const int R = (u + 63) >> 6;
        int* hist = L.u.s.hist;
        int* bst = L.u.s.bst;
        if (u == 0) {
        } else if (R <= 4) snn_bucket_store<4>(tab, u, lane, j, n, hist, bst, rows.nbr + ro, rows.wpk + ro, write);
        else if (R <= 8) snn_bucket_store<8>(tab, u, lane, j, n, hist, bst, rows.nbr + ro, rows.wpk + ro, write);
        else if (R <= 12) snn_bucket_store<12>(tab, u, lane, j, n, hist, bst, rows.nbr + ro, rows.wpk + ro, write);
        else snn_bucket_store<CAP / 64>(tab, u, lane, j, n, hist, bst, rows.nbr + ro, rows.wpk + ro, write);
        WAVE_LDS_SYNC();
        int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
        for (int c = lane; c < u; c += 64) {
            const unsigned v = (unsigned)tab[c];
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t)
                if (t < sp.nk && graph_has(sp, v, t)) ++c4[t];
        }
        snn_row_counts(sp, c4, n, j, lane, cnt);
        if (lane == 0) rows.rlen[j] = u;
        WAVE_LDS_SYNC();
    }
}

// --------------------------------------------------------- block tier --
// Same algorithm with one 256-thread block and a 16K-slot table per node,
// for the overflow list of the hash tier; the table is compacted and
// bitonic-sorted by partner in LDS.  Nodes that overflow here too are
// appended to ov2 for the dense tier.
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

__global__ __launch_bounds__(256) void snn_block_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        SnnSpec sp, const int64_t* __restrict__ hoff,
                                                        const int2* __restrict__ hosts, int64_t* __restrict__ cnt,
                                                        SnnRows rows, const int* __restrict__ ov_list,
                                                        const int* __restrict__ ov_count, int* __restrict__ ov2_list,
                                                        int* __restrict__ ov2_count) {
    __shared__ int keys[SNN_BT];
    __shared__ unsigned vals[SNN_BT];
    __shared__ int count;
    __shared__ int full_s;
    __shared__ int u_s;
    __shared__ int tcount[256];
    __shared__ int64_t wsum[4][SNN_MAXK];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int kmax = sp.kk[sp.nk - 1];
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
        for (int i = 0; i <= kmax; ++i) {
            const int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
            if ((unsigned)cur >= (unsigned)n || (i > 0 && cur == j)) continue;  // invalid (CCG_DERR_SNN_INDEX)
            const int64_t h0 = hoff[cur];
            const int64_t len = hoff[cur + 1] - h0 + 1;
            for (int64_t o = tid; o < len; o += 256) {
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
                    if (c != sp.init && !table_insert_blk(keys, vals, &count, p, c, sp, BITS)) full_s = 1;
                }
            }
        }
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
__global__ __launch_bounds__(256) void snn_dense_kernel(const int32_t* __restrict__ knn, int64_t n, int kstride,
                                                        SnnSpec sp, const int64_t* __restrict__ hoff,
                                                        const int2* __restrict__ hosts,
                                                        const int* __restrict__ ov_list,
                                                        const int* __restrict__ ov_count,
                                                        unsigned* __restrict__ dense_all, int64_t* __restrict__ cnt,
                                                        SnnRows rows) {
    __shared__ int64_t wsum[4];
    unsigned* dense = dense_all + (int64_t)blockIdx.x * n;
    const int nov = *ov_count;
    const int kmax = sp.kk[sp.nk - 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool write = rows.roff[n] <= rows.cap;
    for (int f = blockIdx.x; f < nov; f += gridDim.x) {
        const int64_t j = ov_list[f];
        for (int64_t p = j + 1 + threadIdx.x; p < n; p += 256)
            __hip_atomic_store(&dense[p], sp.init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (int i = 0; i <= kmax; ++i) {
            const int32_t cur = (i == 0) ? (int32_t)j : knn[j * kstride + i - 1];
            if ((unsigned)cur >= (unsigned)n || (i > 0 && cur == j)) continue;  // invalid (CCG_DERR_SNN_INDEX)
            const int64_t h0 = hoff[cur];
            const int64_t len = hoff[cur + 1] - h0 + 1;
            for (int64_t o = threadIdx.x; o < len; o += 256) {
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
                    if (c != sp.init) snn_update(sp, &dense[p], c);
                }
            }
        }
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
// in ascending partner order; off_t = exclusive scan of the per-graph counts.
__global__ __launch_bounds__(256) void snn_emit_kernel(int64_t n, SnnSpec sp, const int64_t* __restrict__ off,
                                                       SnnRows rows, SnnOut out) {
    const int lane = threadIdx.x & 63;
    if (rows.roff[n] > rows.cap) return;  // rows were not written (reported through the totals)
    for (int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (int64_t)gridDim.x * 4) {
        const int u = rows.rlen[j];
        const int64_t ro = rows.roff[j];
        for (int t = 0; t < sp.nk; ++t) {
            if (out.cap[t] <= 0) continue;
            int64_t e = off[(int64_t)t * (n + 1) + j];
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
        if (ds[t]) *ds[t] = fit ? cnt[(int64_t)t * (n + 1) + n] : -roff[n];
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
// cnt[t][0..n] holds their exclusive scans (graph t's edge offsets and total).
// roff: n+1 row offsets (capacity-based), from the workspace when NULL.
static int snn_build(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const SnnSpec& sp, hipStream_t st,
                     int32_t* nbr, uint32_t* wpk, int64_t cap, int64_t* roff, int32_t* rlen, int64_t** cnt_out,
                     const int64_t** roff_out) {
    const int kmax = sp.kk[sp.nk - 1];
    const int64_t nkk = n * kmax;
    CCG_REQUIRE(nkk < (1LL << 31) - 1, "SNN: n*kmax too large");
    int64_t* hoff = (int64_t*)ccg_ws(ctx, WS_SNN_A, sizeof(int64_t) * (2 * (n + 1) + 16));
    int2* hosts_s = (int2*)ccg_ws(ctx, WS_SNN_B, sizeof(int2) * (nkk + 1));
    int64_t* cnt = (int64_t*)ccg_ws(ctx, WS_SNN_C, sizeof(int64_t) * sp.nk * (n + 1));
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
    int* ov_list = ov + 3 * n;
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
    snn_items_kernel<<<nblk, 256, 0, st>>>(knn, n, kstride, kmax, hoff, bp, split, roff);
    rc = ccg_scan_i64(ctx, roff, roff, n, st);
    if (rc) return rc;
    // 3. build: sort tier -> hash tier -> block tier -> dense tier
    SnnRows rows{roff, rlen, nbr, wpk, cap};
    CCG_HIP(hipMemsetAsync(ov_count, 0, sizeof(int) * 64, st));
    CCG_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * sp.nk * (n + 1), st));
    // size classes -> node lists (scan of packed one-hot class counts)
    CCG_REQUIRE(n < (1LL << SNN_CLS_BITS), "SNN: n must be below 2^%d", SNN_CLS_BITS);
    int64_t* cls = (int64_t*)ccg_ws(ctx, WS_SNN_H, sizeof(int64_t) * (n + 1 + 8) + sizeof(int) * 4 * n);
    if (!cls) return CCG_ENOMEM;
    int64_t* ccount = cls + (n + 1);
    int* lists = (int*)(ccount + 8);
    snn_class_kernel<<<(unsigned)ccg_cdiv(n, 256), 256, 0, st>>>(roff, n, cls);
    rc = ccg_scan_i64(ctx, cls, cls, n, st);
    if (rc) return rc;
    snn_class_scatter_kernel<<<(unsigned)ccg_cdiv(n + 1, 256), 256, 0, st>>>(cls, n, lists, ccount);
    const unsigned nsb = (unsigned)ccg_cdiv(n, SNN_WAVES);
    snn_sort_build_kernel<0><<<nsb, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt, rows,
                                                             lists, ccount);
    snn_sort_build_kernel<1><<<nsb, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt, rows,
                                                             lists + n, ccount + 1);
    snn_sort_build_kernel<2><<<nsb, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt, rows,
                                                             lists + 2 * n, ccount + 2);
    snn_wave_build_kernel<SNN_WT><<<(unsigned)std::min<int64_t>(nsb, 1024), 64 * SNN_WAVES, 0, st>>>(
        knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt, rows, lists + 3 * n, ccount + 3, ov_list, ov_count + 1);
    snn_block_kernel<<<256, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, cnt, rows, ov_list, ov_count + 1,
                                          ov2_list, ov_count + 2);
    snn_dense_kernel<<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, ov2_list, ov_count + 2,
                                                       dense, cnt, rows);
    for (int t = 0; t < sp.nk; ++t) {
        rc = ccg_scan_i64(ctx, cnt + (int64_t)t * (n + 1), cnt + (int64_t)t * (n + 1), n, st);
        if (rc) return rc;
    }
    *cnt_out = cnt;
    *roff_out = roff;
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
    int64_t ne = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        int rc = ccg_snn_dev(ctx, dknn, n, kstride, k, type, di, dj, dw, cap, dne, st);
        if (rc) return rc;
        CCG_HIP(hipMemcpyAsync(&ne, dne, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        if (ne >= 0) break;
        ctx->snn_row_reserve = -ne + (-ne) / 8;  // rows did not fit the reservation: grow and rerun
    }
    CCG_REQUIRE(ne >= 0, "ccg_snn: row reservation could not be satisfied");
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
