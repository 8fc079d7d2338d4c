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
// Each undirected edge is emitted by its smaller endpoint (partners p > j).
// Per node one wave builds an LDS open-addressing hash table of its
// partners (key p, packed per-graph values), then (pass 2) compacts it,
// bitonic-sorts by p and emits each graph's edges in (i, j) order at offsets
// from a device scan of pass-1 counts -- deterministic and sorted, no
// scratch.  Nodes with more partners than the wave table holds use a
// 256-thread table of 16K slots; beyond that an exact O(n) dense path.
#include <algorithm>
#include <cstdlib>

#include "ccg_internal.h"

#define WAVE_LDS_SYNC() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)

#define SNN_MAXK 4           // graphs per pass (|kNum| <= 4)
#define SNN_WT 2048          // wave table slots
#define SNN_WAVES 4          // waves per block in the wave kernel
#define SNN_BT 16384         // block table slots (overflow path)
#define SNN_DENSE_BLOCKS 64  // concurrent dense-path nodes
#define SNN_EMPTY (-1)

struct SnnSpec {
    int nk;
    int kk[SNN_MAXK];  // ascending
    int type;
    unsigned init;     // empty value word (0 for NUMBER, 0xFFFFFFFF for RANK)
};

struct SnnOut {
    int32_t* oi[SNN_MAXK];
    int32_t* oj[SNN_MAXK];
    double* ow[SNN_MAXK];
    int64_t cap[SNN_MAXK];
};

__global__ void snn_count_hosts(const int32_t* __restrict__ knn, int64_t n, int kstride, int k,
                                unsigned long long* __restrict__ hcnt, int* __restrict__ err) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * k) return;
    int64_t h = t / k;
    int r = (int)(t - h * k);
    int32_t x = knn[h * kstride + r];
    if (x < 0 || x >= n || x == h) {
        atomicOr(err, CCG_DERR_SNN_INDEX);
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

// Sort every host list by host id (one wave per list; rank of each entry =
// number of smaller ids, ids in a list are distinct) into hosts_s, and record
// where each kNN entry landed: bp[h * kmax + r - 1] = position of h in
// hosts_s(knn[h][r - 1]), split[x] = number of hosts of x below x.  The
// build then starts member s of node j at the entry after j itself, so it
// only ever fetches partners p > j.
#define SNN_SORT_LDS 512
__global__ __launch_bounds__(256) void snn_sort_hosts(const int64_t* __restrict__ hoff, int64_t n, int kmax,
                                                      const int2* __restrict__ hosts, int2* __restrict__ hosts_s,
                                                      int* __restrict__ bp, int* __restrict__ split) {
    __shared__ int buf_all[4][SNN_SORT_LDS];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int* buf = buf_all[wv];
    for (int64_t x = (int64_t)blockIdx.x * 4 + wv; x < n; x += (int64_t)gridDim.x * 4) {
        const int64_t h0 = hoff[x];
        const int len = (int)(hoff[x + 1] - h0);
        const int2* src = hosts + h0;
        const bool in_lds = len <= SNN_SORT_LDS;
        if (in_lds)
            for (int c = lane; c < len; c += 64) buf[c] = src[c].x;
        WAVE_LDS_SYNC();
        int below = 0;
        for (int c = lane; c < len; c += 64) {
            const int2 e = src[c];
            int rank = 0;
            if (in_lds)
                for (int i = 0; i < len; ++i) rank += buf[i] < e.x;
            else
                for (int i = 0; i < len; ++i) rank += src[i].x < e.x;
            hosts_s[h0 + rank] = e;
            bp[(int64_t)e.x * kmax + e.y - 1] = rank;
            below += e.x < x;
        }
        for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
        if (lane == 0) split[x] = below;
        WAVE_LDS_SYNC();
    }
}

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

// Insert partner p with contribution c; returns false when the table is full.
template <int T>
__device__ __forceinline__ bool table_insert(int* keys, unsigned* vals, int* count, int p, unsigned c,
                                             const SnnSpec& sp, int bits) {
    unsigned s = snn_hash(p, bits);
    for (int probe = 0; probe < T; ++probe) {
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
        s = (s + 1) & (T - 1);
    }
    return false;
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

// ---------------------------------------------------------------- wave path --
// Pass 1 (build): one wave per node builds an LDS hash table of 64-bit slots
// (partner p << 32 | packed per-graph values): a new partner costs one CAS, a
// repeat one add.  The table is compacted, sorted by p and parked in a
// fixed-capacity scratch row; per-graph edge counts go to cnt[t][j].  It
// serves the nodes the sort path below cannot stage (more than 1024 items);
// nodes beyond its capacity go to the block path.
// Pass 2 (emit) streams the sorted rows into the caller's edge arrays.
#define SNN_WCAP (SNN_WT * 3 / 4)
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

// One item per active lane into a WT-slot table, probing with CAS only (a
// CAS on an empty slot inserts, a returned equal key means the partner is
// already there).  The loop runs while any lane still has its item, so the
// control flow stays wave-uniform.  Returns false on lanes that found no slot.
template <int WT>
__device__ __forceinline__ bool wave_insert64(unsigned long long* tab, int p, unsigned c, bool active, int type) {
    unsigned s = snn_hash(p, snn_log2<WT>());
    const unsigned long long want = ((unsigned long long)(unsigned)p << 32) | c;
    int probes = 0;
    bool ok = true;
    while (__any(active)) {
        if (active) {
            unsigned long long old = atomicCAS(&tab[s], SNN_EMPTY64, want);
            if (old == SNN_EMPTY64) {
                active = false;
            } else if ((unsigned)(old >> 32) == (unsigned)p) {
                if (type == CCG_SNN_NUMBER) {
                    atomicAdd(&tab[s], (unsigned long long)c);  // per-byte counts never carry
                } else {
                    while (true) {
                        const unsigned nv = bytewise_min((unsigned)old, c);
                        if (nv == (unsigned)old) break;
                        const unsigned long long nw = (old & 0xFFFFFFFF00000000ull) | nv;
                        const unsigned long long prev = atomicCAS(&tab[s], old, nw);
                        if (prev == old) break;
                        old = prev;
                    }
                }
                active = false;
            } else {
                s = (s + 1) & (WT - 1);
                if (++probes == WT) {
                    active = false;
                    ok = false;
                }
            }
        }
    }
    return ok;
}

// Sort a node's u compacted entries (tab[0..u), distinct partners p in (j, n))
// by p and store them to dst[0..u).  Each lane holds entries c = r*64 + lane
// in registers; a 128-bucket split on p (monotone in p) gives every entry its
// bucket's start by a histogram + wave scan, the entries are scattered into
// bucket order in tab, and each entry's final place is its bucket start plus
// the number of smaller partners in its (small) bucket.
#define SNN_NB 128
template <int RMAX>
__device__ __forceinline__ void snn_bucket_store(unsigned long long* tab, int u, int lane, int64_t j, int64_t n,
                                                 int* hist, int* bst, unsigned long long* __restrict__ dst) {
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
            dst[b0 + rank] = e[r];
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

// Tier kernel: WT-slot tables (WT = 1024: 4 waves/SIMD, fits ~96% of nodes at
// cfg3; WT = 2048 for the overflow list of the first tier).  in_list = nullptr
// walks every node, else the in_count nodes of in_list.
template <int WT>
__global__ __launch_bounds__(64 * SNN_WAVES, WT <= 1024 ? 4 : 2) void snn_wave_build_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp, const int64_t* __restrict__ hoff,
    const int2* __restrict__ hosts_s, const int* __restrict__ bp, const int* __restrict__ split,
    int64_t* __restrict__ cnt, const int* __restrict__ in_list, const int* __restrict__ in_count,
    int* __restrict__ ov_list, int* __restrict__ ov_count, unsigned long long* __restrict__ scratch,
    int* __restrict__ ucount) {
    __shared__ SnnWaveLds<WT> lds_all[SNN_WAVES];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SnnWaveLds<WT>& L = lds_all[wv];
    unsigned long long* tab = L.tab;
    const int kmax = sp.kk[sp.nk - 1];
    constexpr int CAP = WT * 3 / 4;
    const int64_t nn = in_list ? (int64_t)*in_count : n;
    for (int64_t f = (int64_t)blockIdx.x * SNN_WAVES + wv; f < nn; f += (int64_t)gridDim.x * SNN_WAVES) {
        const int64_t j = in_list ? (int64_t)in_list[f] : f;
        for (int s = lane; s < WT; s += 64) tab[s] = SNN_EMPTY64;
        // Flat gather over the partners p > j only: member 0 (j itself) from
        // its first host above j, member i (s = knn[j][i-1]) from the entry
        // after j in the sorted hosts(s), plus s itself (rank 0) when s > j.
        // Item t of M = sum of member lengths; host entries are fetched one
        // round ahead so their latency hides behind the current LDS inserts.
        int mcur = 0, mlen = 0;
        long long mh0 = 0, mend = 0;
        if (lane <= kmax) {
            if (lane == 0) {
                mcur = (int)j;
                mh0 = hoff[j] + split[j];
                mend = hoff[j + 1];
                mlen = (int)(mend - mh0);
            } else {
                mcur = knn[j * kstride + lane - 1];
                if ((unsigned)mcur < (unsigned)n && mcur != j) {
                    const int q = bp[j * kmax + lane - 1];
                    mh0 = hoff[mcur] + q + 1;
                    mend = hoff[mcur + 1];
                    mlen = (int)(mend - mh0) + (mcur > j ? 1 : 0);
                } else {
                    mcur = (int)j;  // invalid input (reported via CCG_DERR_SNN_INDEX): no items
                }
            }
        }
        int incl = mlen;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int M = __shfl(incl, 63);
        if (lane <= kmax) {
            L.u.g.pre[lane] = incl - mlen;
            L.u.g.h0[lane] = mh0;
            L.u.g.hend[lane] = mend;
            L.u.g.cur[lane] = mcur;
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
            if (lane == 0) {
                const int q = atomicAdd(ov_count, 1);
                ov_list[q] = (int)j;
            }
            continue;
        }
        // Sort by partner and park the row in scratch (bucket split + in-bucket rank).
        unsigned long long* dst = scratch + j * SNN_WCAP;
        const int R = (u + 63) >> 6;
        int* hist = L.u.s.hist;
        int* bst = L.u.s.bst;
        if (u == 0) {
        } else if (R <= 4) snn_bucket_store<4>(tab, u, lane, j, n, hist, bst, dst);
        else if (R <= 8) snn_bucket_store<8>(tab, u, lane, j, n, hist, bst, dst);
        else if (R <= 12) snn_bucket_store<12>(tab, u, lane, j, n, hist, bst, dst);
        else if constexpr (CAP > 768) snn_bucket_store<CAP / 64>(tab, u, lane, j, n, hist, bst, dst);
        WAVE_LDS_SYNC();
        int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
        for (int c = lane; c < u; c += 64) {
            const unsigned v = (unsigned)tab[c];
#pragma unroll
            for (int t = 0; t < SNN_MAXK; ++t)
                if (t < sp.nk && graph_has(sp, v, t)) ++c4[t];
        }
#pragma unroll
        for (int t = 0; t < SNN_MAXK; ++t) {
            int64_t v = c4[t];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0 && t < sp.nk) cnt[(int64_t)t * (n + 1) + j] = v;
        }
        if (lane == 0) ucount[j] = u;
        WAVE_LDS_SYNC();
    }
}

// ------------------------------------------------------- sort (ESC) path --
// Nodes with at most SI items (partners p > j, with multiplicity) skip the
// hash table: the items are gathered to registers (all host loads in flight
// at once), bucketed by p into an LDS stage (histogram, scan, scatter),
// ranked inside their bucket by (p, stage slot) and rewritten in sorted
// order; one pass over the sorted stage then merges equal partners (sum for
// NUMBER, bytewise min for RANK) and writes the row.  Every item costs a
// fixed handful of LDS operations instead of a probe sequence.
#define SNN_SNB 240  // buckets: SI*8 + 2*SNN_SNB*4 + 4 bytes of LDS per wave

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

__device__ __forceinline__ unsigned snn_combine(int type, unsigned a, unsigned b) {
    return type == CCG_SNN_NUMBER ? a + b : bytewise_min(a, b);  // per-byte counts never carry
}

template <int SI>
__global__ __launch_bounds__(64 * SNN_WAVES, SI <= 1024 ? 4 : 2) void snn_sort_build_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp, const int64_t* __restrict__ hoff,
    const int2* __restrict__ hosts_s, const int* __restrict__ bp, const int* __restrict__ split,
    int64_t* __restrict__ cnt, const int* __restrict__ in_list, const int* __restrict__ in_count,
    int* __restrict__ ov_list, int* __restrict__ ov_count, unsigned long long* __restrict__ scratch,
    int* __restrict__ ucount) {
    constexpr int R = SI / 64;
    __shared__ SnnSortLds<SI> lds_all[SNN_WAVES];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SnnSortLds<SI>& L = lds_all[wv];
    unsigned long long* stage = L.stage;
    const int kmax = sp.kk[sp.nk - 1];
    const int64_t nn = in_list ? (int64_t)*in_count : n;
    for (int64_t f = (int64_t)blockIdx.x * SNN_WAVES + wv; f < nn; f += (int64_t)gridDim.x * SNN_WAVES) {
        const int64_t j = in_list ? (int64_t)in_list[f] : f;
        // members: as in snn_wave_build_kernel (partners p > j only)
        int mcur = 0, mlen = 0;
        long long mh0 = 0, mend = 0;
        if (lane <= kmax) {
            if (lane == 0) {
                mcur = (int)j;
                mh0 = hoff[j] + split[j];
                mend = hoff[j + 1];
                mlen = (int)(mend - mh0);
            } else {
                mcur = knn[j * kstride + lane - 1];
                if ((unsigned)mcur < (unsigned)n && mcur != j) {
                    const int q = bp[j * kmax + lane - 1];
                    mh0 = hoff[mcur] + q + 1;
                    mend = hoff[mcur + 1];
                    mlen = (int)(mend - mh0) + (mcur > j ? 1 : 0);
                } else {
                    mcur = (int)j;  // invalid input (reported via CCG_DERR_SNN_INDEX): no items
                }
            }
        }
        int incl = mlen;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int M = __shfl(incl, 63);
        if (M > SI) {
            if (lane == 0) {
                const int q = atomicAdd(ov_count, 1);
                ov_list[q] = (int)j;
            }
            continue;
        }
        if (lane <= kmax) {
            L.u.g.pre[lane] = incl - mlen;
            L.u.g.h0[lane] = mh0;
            L.u.g.hend[lane] = mend;
            L.u.g.cur[lane] = mcur;
        }
        if (lane == 0) L.u.g.pre[kmax + 1] = M;
        WAVE_LDS_SYNC();
        // gather: every host load of the node is issued before any is used
        int2 hr[R];
        int im[R];
        int mi = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int t = 64 * r + lane;
            im[r] = -1;
            hr[r] = make_int2(-1, 0);
            if (t < M) {
                while (L.u.g.pre[mi + 1] <= t) ++mi;
                im[r] = mi;
                const long long q = L.u.g.h0[mi] + (t - L.u.g.pre[mi]);
                if (q < L.u.g.hend[mi]) hr[r] = hosts_s[q];
                else hr[r] = make_int2(L.u.g.cur[mi], 0);
            }
        }
        WAVE_LDS_SYNC();
        int* hist = L.u.s.hist;
        int* bst = L.u.s.bst;
        for (int b = lane; b < SNN_SNB; b += 64) hist[b] = 0;
        WAVE_LDS_SYNC();
        const float inv = (float)SNN_SNB / (float)(n - j);
        unsigned long long e[R];
        int bk[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            e[r] = SNN_EMPTY64;
            bk[r] = -1;
            if (im[r] >= 0) {
                const unsigned c = snn_contrib(sp, im[r], hr[r].y);
                if (c != sp.init) {
                    e[r] = ((unsigned long long)(unsigned)hr[r].x << 32) | c;
                    bk[r] = min(SNN_SNB - 1, (int)((float)(hr[r].x - (int)j - 1) * inv));
                    atomicAdd(&hist[bk[r]], 1);
                }
            }
        }
        WAVE_LDS_SYNC();
        // bucket starts: lane owns buckets 4*lane .. 4*lane+3
        int hv[4], hs = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int b = 4 * lane + i;
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
        for (int i = 0; i < 4; ++i) {
            const int b = 4 * lane + i;
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
        // unique partners: first of each run of equal keys
        auto is_first = [&](int q, unsigned& key) {
            const unsigned long long x = stage[q];
            key = (unsigned)(x >> 32);
            return q == 0 || (unsigned)(stage[q - 1] >> 32) != key;
        };
        if constexpr (SI > SNN_WCAP) {
            int uu = 0;
            for (int q0 = 0; q0 < V; q0 += 64) {
                unsigned key;
                const bool first = q0 + lane < V && is_first(q0 + lane, key);
                uu += __popcll(__ballot(first));
            }
            if (uu > SNN_WCAP) {
                if (lane == 0) {
                    const int q = atomicAdd(ov_count, 1);
                    ov_list[q] = (int)j;
                }
                WAVE_LDS_SYNC();
                continue;
            }
        }
        unsigned long long* dst = scratch + j * SNN_WCAP;
        int u = 0;
        int64_t c4[SNN_MAXK] = {0, 0, 0, 0};
        for (int q0 = 0; q0 < V; q0 += 64) {
            const int q = q0 + lane;
            unsigned key = 0, agg = 0;
            const bool first = q < V && is_first(q, key);
            if (first) {
                agg = (unsigned)stage[q];
                for (int q2 = q + 1; q2 < V; ++q2) {
                    const unsigned long long y = stage[q2];
                    if ((unsigned)(y >> 32) != key) break;
                    agg = snn_combine(sp.type, agg, (unsigned)y);
                }
            }
            const unsigned long long m = __ballot(first);
            if (first) {
                dst[u + __popcll(m & lanemask_lt())] = ((unsigned long long)key << 32) | agg;
#pragma unroll
                for (int t = 0; t < SNN_MAXK; ++t)
                    if (t < sp.nk && graph_has(sp, agg, t)) ++c4[t];
            }
            u += __popcll(m);
        }
#pragma unroll
        for (int t = 0; t < SNN_MAXK; ++t) {
            int64_t v = c4[t];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0 && t < sp.nk) cnt[(int64_t)t * (n + 1) + j] = v;
        }
        if (lane == 0) ucount[j] = u;
        WAVE_LDS_SYNC();
    }
}

__global__ __launch_bounds__(256) void snn_wave_emit_kernel(int64_t n, SnnSpec sp, const int64_t* __restrict__ off,
                                                            const int* __restrict__ ov_flag,
                                                            const unsigned long long* __restrict__ scratch,
                                                            const int* __restrict__ ucount, SnnOut out) {
    const int lane = threadIdx.x & 63;
    for (int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (int64_t)gridDim.x * 4) {
        if (ov_flag[j]) continue;
        const int u = ucount[j];
        const unsigned long long* src = scratch + j * SNN_WCAP;
        for (int t = 0; t < sp.nk; ++t) {
            int64_t e = off[(int64_t)t * (n + 1) + j];
            for (int c0 = 0; c0 < u; c0 += 64) {
                const int c = c0 + lane;
                const unsigned long long x = c < u ? src[c] : 0ull;
                const unsigned v = (unsigned)x;
                const bool has = c < u && graph_has(sp, v, t);
                const unsigned long long m = __ballot(has);
                if (has) {
                    const int64_t pos = e + __popcll(m & lanemask_lt());
                    if (pos < out.cap[t]) {
                        out.oi[t][pos] = (int32_t)j;
                        out.oj[t][pos] = (int32_t)(x >> 32);
                        out.ow[t][pos] = graph_weight(sp, v, t);
                    }
                }
                e += __popcll(m);
            }
        }
    }
}

// --------------------------------------------------------------- block path --
// Same algorithm with one 256-thread block and a 16K-slot table per node, for
// the overflow list of the wave path.  Nodes that overflow here too are
// appended to ov2 for the dense path.
template <bool EMIT>
__global__ __launch_bounds__(256) void snn_block_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp,
    const int64_t* __restrict__ hoff, const int2* __restrict__ hosts, int64_t* __restrict__ cnt,
    const int* __restrict__ ov_list, const int* __restrict__ ov_count, int* __restrict__ ov2_list,
    int* __restrict__ ov2_count, const int* __restrict__ ov2_flag, SnnOut out) {
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
    for (int f = blockIdx.x; f < nov; f += gridDim.x) {
        const int64_t j = ov_list[f];
        if (EMIT && ov2_flag[j]) continue;  // uniform across the block
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
                    if (c != sp.init && !table_insert<SNN_BT>(keys, vals, &count, p, c, sp, BITS)) full_s = 1;
                }
            }
        }
        __syncthreads();
        if (full_s || count > cap_entries) {
            if (!EMIT && tid == 0) {
                const int q = atomicAdd(ov2_count, 1);
                ov2_list[q] = (int)j;
            }
            __syncthreads();
            continue;
        }
        if (!EMIT) {
            int64_t c[SNN_MAXK] = {0, 0, 0, 0};
            for (int s = tid; s < SNN_BT; s += 256)
                if (keys[s] != SNN_EMPTY) {
                    const unsigned v = vals[s];
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
            if (tid < sp.nk)
                cnt[(int64_t)tid * (n + 1) + j] = wsum[0][tid] + wsum[1][tid] + wsum[2][tid] + wsum[3][tid];
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
        for (int t = 0; t < sp.nk; ++t) {
            int64_t e = cnt[(int64_t)t * (n + 1) + j];
            for (int c0 = 0; c0 < u; c0 += 256) {
                const int c = c0 + tid;
                const bool in = c < u;
                const unsigned v = in ? vals[c] : sp.init;
                const bool has = in && graph_has(sp, v, t);
                const unsigned long long m = __ballot(has);
                if (lane == 0) wsum[wv][0] = __popcll(m);
                __syncthreads();
                int64_t before = 0, tot = 0;
                for (int w = 0; w < 4; ++w) {
                    if (w < wv) before += wsum[w][0];
                    tot += wsum[w][0];
                }
                if (has) {
                    const int64_t pos = e + before + __popcll(m & lanemask_lt());
                    if (pos < out.cap[t]) {
                        out.oi[t][pos] = (int32_t)j;
                        out.oj[t][pos] = keys[c];
                        out.ow[t][pos] = graph_weight(sp, v, t);
                    }
                }
                e += tot;
                __syncthreads();
            }
        }
        __syncthreads();
    }
}

// --------------------------------------------------------------- dense path --
// Exact O(n) per node with a dense word per partner.  Reads/writes go
// through agent-scope atomics so the block never sees stale L1 lines.
template <bool EMIT>
__global__ __launch_bounds__(256) void snn_dense_kernel(
    const int32_t* __restrict__ knn, int64_t n, int kstride, SnnSpec sp,
    const int64_t* __restrict__ hoff, const int2* __restrict__ hosts, const int* __restrict__ ov_list,
    const int* __restrict__ ov_count, unsigned* __restrict__ dense_all, int64_t* __restrict__ cnt,
    SnnOut out) {
    __shared__ int64_t wsum[4];
    unsigned* dense = dense_all + (int64_t)blockIdx.x * n;
    const int nov = *ov_count;
    const int kmax = sp.kk[sp.nk - 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
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
        for (int t = 0; t < sp.nk; ++t) {
            int64_t base = EMIT ? cnt[(int64_t)t * (n + 1) + j] : 0;
            int64_t total = 0;
            for (int64_t p0 = j + 1; p0 < n; p0 += 256) {
                const int64_t p = p0 + threadIdx.x;
                const unsigned v = (p < n) ? __hip_atomic_load(&dense[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : sp.init;
                const bool hit = (p < n) && graph_has(sp, v, t);
                const unsigned long long m = __ballot(hit);
                if (lane == 0) wsum[wv] = __popcll(m);
                __syncthreads();
                int64_t before = 0, tot = 0;
                for (int w = 0; w < 4; ++w) {
                    if (w < wv) before += wsum[w];
                    tot += wsum[w];
                }
                if (EMIT && hit) {
                    const int64_t e = base + total + before + __popcll(m & lanemask_lt());
                    if (e < out.cap[t]) {
                        out.oi[t][e] = (int32_t)j;
                        out.oj[t][e] = (int32_t)p;
                        out.ow[t][e] = graph_weight(sp, v, t);
                    }
                }
                total += tot;
                __syncthreads();
            }
            if (!EMIT && threadIdx.x == 0) cnt[(int64_t)t * (n + 1) + j] = total;
            __syncthreads();
        }
    }
}

__global__ void snn_mark_kernel(const int* __restrict__ list, const int* __restrict__ count,
                                int* __restrict__ flag) {
    const int nl = *count;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x) flag[list[i]] = 1;
}

__global__ void snn_copy_totals(const int64_t* __restrict__ cnt, int64_t n, int nk, int64_t* d0, int64_t* d1,
                                int64_t* d2, int64_t* d3) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t* ds[4] = {d0, d1, d2, d3};
    for (int t = 0; t < nk; ++t)
        if (ds[t]) *ds[t] = cnt[(int64_t)t * (n + 1) + n];
}

extern "C" int ccg_snn_multi_dev(ccg_ctx* ctx, const int32_t* knn, int64_t n, int kstride, const int* ks,
                                 int nk, int type, int32_t* const* out_i, int32_t* const* out_j,
                                 double* const* out_w, const int64_t* caps, int64_t* const* d_nedges,
                                 void* stream) {
    CCG_REQUIRE(ctx && knn && ks && d_nedges, "ccg_snn_multi_dev: NULL argument");
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) - 1, "ccg_snn_multi_dev: bad n");
    CCG_REQUIRE(nk >= 1 && nk <= SNN_MAXK, "ccg_snn_multi_dev: 1 <= nk <= %d", SNN_MAXK);
    CCG_REQUIRE(type == CCG_SNN_NUMBER || type == CCG_SNN_RANK, "ccg_snn_multi_dev: bad type");
    SnnSpec sp;
    sp.nk = nk;
    sp.type = type;
    sp.init = type == CCG_SNN_NUMBER ? 0u : 0xFFFFFFFFu;
    SnnOut out;
    for (int t = 0; t < SNN_MAXK; ++t) {
        sp.kk[t] = t < nk ? ks[t] : 0;
        out.cap[t] = 0;
        out.oi[t] = nullptr;
        out.oj[t] = nullptr;
        out.ow[t] = nullptr;
    }
    for (int t = 0; t < nk; ++t) {
        CCG_REQUIRE(ks[t] >= 1 && ks[t] <= kstride && ks[t] <= 32 && (t == 0 || ks[t] > ks[t - 1]),
                    "ccg_snn_multi_dev: ks must be ascending in [1, min(kstride, 32)]");
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
    int64_t* hoff = (int64_t*)ccg_ws(ctx, WS_SNN_A, sizeof(int64_t) * (2 * (n + 1) + 16));
    int2* hosts = (int2*)ccg_ws(ctx, WS_SNN_B, sizeof(int2) * 2 * (n * kmax + 1));
    int64_t* cnt = (int64_t*)ccg_ws(ctx, WS_SNN_C, sizeof(int64_t) * nk * (n + 1));
    int* ov = (int*)ccg_ws(ctx, WS_SNN_E, sizeof(int) * (5 * n + 64));
    unsigned* dense = (unsigned*)ccg_ws(ctx, WS_SNN_D, sizeof(unsigned) * n * SNN_DENSE_BLOCKS);
    unsigned long long* scratch =
        (unsigned long long*)ccg_ws(ctx, WS_SNN_F, sizeof(unsigned long long) * n * SNN_WCAP + sizeof(int) * (n + 64));
    int* bp = (int*)ccg_ws(ctx, WS_SNN_G, sizeof(int) * (n * kmax + n + 64));
    if (!hoff || !hosts || !cnt || !ov || !dense || !scratch || !bp) return CCG_ENOMEM;
    int2* hosts_s = hosts + (n * kmax + 1);
    int* split = bp + n * kmax;
    int* ucount = (int*)(scratch + n * SNN_WCAP);
    unsigned long long* cursor = (unsigned long long*)(hoff + (n + 1));
    int* err = ctx->d_err;
    int* ov_list = ov;  // nodes for the block path (overflowed both wave tiers)
    int* ov2_list = ov + n;
    int* flag1 = ov + 2 * n;
    int* flag2 = ov + 3 * n;
    int* ova_list = ov + 4 * n;  // more than 1024 items -> 2048-slot hash tier
    int* ov_count = ov + 5 * n;
    int* ov2_count = ov_count + 1;
    int* ova_count = ov_count + 2;
    const int64_t nkk = (int64_t)n * kmax;
    const int t_all = ccg_timer_start(ctx, CCG_KT_SNN, st);
    CCG_HIP(hipMemsetAsync(hoff, 0, sizeof(int64_t) * (n + 1), st));
    CCG_HIP(hipMemsetAsync(flag1, 0, sizeof(int) * 2 * n, st));
    CCG_HIP(hipMemsetAsync(ov_count, 0, sizeof(int) * 64, st));
    CCG_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * nk * (n + 1), st));
    snn_count_hosts<<<(unsigned)ccg_cdiv(nkk, 256), 256, 0, st>>>(knn, n, kstride, kmax,
                                                                  (unsigned long long*)hoff, err);
    int rc = ccg_scan_i64(ctx, hoff, hoff, n, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(cursor, hoff, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, st));
    snn_fill_hosts<<<(unsigned)ccg_cdiv(nkk, 256), 256, 0, st>>>(knn, n, kstride, kmax, cursor, hosts);
    snn_sort_hosts<<<(unsigned)std::min<int64_t>(ccg_cdiv(n, 4), 16384), 256, 0, st>>>(hoff, n, kmax, hosts,
                                                                                      hosts_s, bp, split);
    const unsigned nblk = (unsigned)std::min<int64_t>(ccg_cdiv(n, SNN_WAVES), 16384);
    // pass 1: per-graph counts (sort tier for nodes with <= 1024 items, 2048-slot hash tables,
    // then block tables, then dense)
    snn_sort_build_kernel<1024><<<nblk, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt,
                                                                 nullptr, nullptr, ova_list, ova_count, scratch,
                                                                 ucount);
    const unsigned nblk2 = (unsigned)std::min<int64_t>(ccg_cdiv(n, SNN_WAVES), 1024);
    snn_wave_build_kernel<2048><<<nblk2, 64 * SNN_WAVES, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, bp, split, cnt,
                                                                  ova_list, ova_count, ov_list, ov_count, scratch,
                                                                  ucount);
    snn_block_kernel<false><<<256, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, cnt, ov_list, ov_count,
                                                 ov2_list, ov2_count, flag2, out);
    snn_dense_kernel<false><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, ov2_list,
                                                             ov2_count, dense, cnt, out);
    snn_mark_kernel<<<64, 256, 0, st>>>(ov_list, ov_count, flag1);
    snn_mark_kernel<<<64, 256, 0, st>>>(ov2_list, ov2_count, flag2);
    for (int t = 0; t < nk; ++t) {
        rc = ccg_scan_i64(ctx, cnt + (int64_t)t * (n + 1), cnt + (int64_t)t * (n + 1), n, st);
        if (rc) return rc;
    }
    bool any_cap = false;
    for (int t = 0; t < nk; ++t) any_cap |= out.cap[t] > 0;
    if (any_cap) {
        snn_wave_emit_kernel<<<(unsigned)std::min<int64_t>(ccg_cdiv(n, 4), 16384), 256, 0, st>>>(
            n, sp, cnt, flag1, scratch, ucount, out);
        snn_block_kernel<true><<<256, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, cnt, ov_list, ov_count,
                                                    ov2_list, ov2_count, flag2, out);
        snn_dense_kernel<true><<<SNN_DENSE_BLOCKS, 256, 0, st>>>(knn, n, kstride, sp, hoff, hosts_s, ov2_list,
                                                                ov2_count, dense, cnt, out);
    }
    snn_copy_totals<<<1, 64, 0, st>>>(cnt, n, nk, d_nedges[0], nk > 1 ? d_nedges[1] : nullptr,
                                      nk > 2 ? d_nedges[2] : nullptr, nk > 3 ? d_nedges[3] : nullptr);
    ccg_timer_stop(ctx, t_all, st);
    CCG_HIP(hipGetLastError());
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
