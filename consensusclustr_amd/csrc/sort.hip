// Stable LSD radix sort of (int32 key, int32 value) pairs, hand-written for
// gfx950.  Used where the per-bootstrap path groups entries by a bounded key:
// the distinct-cell kNN groups bootstrap rows by cell (keys < N, knn.hip) and
// the SNN build lists every node's hosts (keys < n, snn.hip); both need the
// equal keys in input order (rows / hosts ascending).
//
// One pass per digit of <= 9 bits (the key bits split evenly, so 17-bit keys
// take two 9/8-bit passes), three launches per pass:
//   rs_hist    : per tile of 256 * IPT pairs, the digit histogram (LDS atomics),
//                written digit-major: cnt[digit * ntiles + tile];
//   scan       : the library's two-launch multi-block scan (ccg_scan_i64) of
//                that matrix -> every (digit, tile) pair's first output
//                position (digit-major = stable).  A single-block scan here
//                waited for a free CU behind the co-scheduled streams' kernels
//                (~150 us per launch in the bench against ~5 us alone);
//   rs_scatter : each tile ranks its pairs stably -- a wave takes a contiguous
//                run of 64 * RS_IPT pairs, lanes along consecutive pairs, peers
//                of equal digit found by one ballot per digit bit, running
//                per-wave digit counts in LDS -- puts the tile in digit order
//                in LDS and writes it out with consecutive threads on
//                consecutive positions of each digit's run.
// Keys outside [0, 2^key_bits) are the caller's contract (only the low
// key_bits bits are looked at).
#include "ccg_internal.h"

#define RS_THREADS 256
#define RS_WAVES (RS_THREADS / 64)
#define RS_MAXBITS 9
// pairs per thread per tile (IPT = 1..16, tiles of 256 * IPT pairs): chosen per
// sort so that about 256 or more tiles fill the GPU (the bootstrap's 90k-row
// grouping ran 22 tiles of 4096 pairs, each a long serial chain)
#define RS_TILES_MIN 256
#ifndef RS_ADAPT
#define RS_ADAPT 1  // tools only: 0 = tiles of 4096 pairs always (A/B)
#endif

// Block b runs on XCD b mod 8; each XCD takes a contiguous range of tiles so
// neighbouring tiles' histogram columns and output runs (adjacent in the
// digit-major order) are written through one L2 instead of eight.
__device__ __forceinline__ int rs_tile(int b, int ntiles) {
    const int full = ntiles >> 3, rem = ntiles & 7, x = b & 7;
    return x * full + min(x, rem) + (b >> 3);
}

template <int RS_IPT>
__global__ __launch_bounds__(RS_THREADS) void rs_hist(const int32_t* __restrict__ keys, int64_t n, int shift,
                                                      int bits, int ntiles, int64_t* __restrict__ cnt) {
    __shared__ int h[1 << RS_MAXBITS];
    const int nb = 1 << bits;
    for (int t = threadIdx.x; t < nb; t += RS_THREADS) h[t] = 0;
    __syncthreads();
    const int tile = rs_tile(blockIdx.x, ntiles);
    const int64_t base = (int64_t)tile * (RS_THREADS * RS_IPT);
#pragma unroll 4
    for (int i = 0; i < RS_IPT; ++i) {
        const int64_t e = base + (int64_t)i * RS_THREADS + threadIdx.x;
        if (e < n) atomicAdd(&h[((unsigned)keys[e] >> shift) & (nb - 1)], 1);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nb; t += RS_THREADS) cnt[(int64_t)t * ntiles + tile] = h[t];
}

__device__ __forceinline__ unsigned long long rs_lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <int RS_IPT>
__global__ __launch_bounds__(RS_THREADS) void rs_scatter(const int32_t* __restrict__ kin,
                                                         const int32_t* __restrict__ vin, int64_t n, int shift,
                                                         int bits, int ntiles, const int64_t* __restrict__ off,
                                                         int32_t* __restrict__ kout, int32_t* __restrict__ vout) {
    __shared__ int wcnt[RS_WAVES][1 << RS_MAXBITS];  // per-wave running digit counts, then prefixes
    __shared__ int goff[1 << RS_MAXBITS];
    __shared__ int dstart[1 << RS_MAXBITS];  // tile-local first position of each digit
    __shared__ int wsum[RS_WAVES];
    __shared__ int2 stage[RS_THREADS * RS_IPT];
    const int nb = 1 << bits;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tile = rs_tile(blockIdx.x, ntiles);
    for (int t = threadIdx.x; t < RS_WAVES * nb; t += RS_THREADS) wcnt[t / nb][t % nb] = 0;
    for (int t = threadIdx.x; t < nb; t += RS_THREADS) goff[t] = (int)off[(int64_t)t * ntiles + tile];
    __syncthreads();
    // wave w's run: pairs [base, base + 64 * RS_IPT), item i at base + 64 i + lane
    const int64_t base = (int64_t)tile * (RS_THREADS * RS_IPT) + (int64_t)w * 64 * RS_IPT;
    int kk[RS_IPT], vv[RS_IPT], rk[RS_IPT];
    const unsigned long long lt = rs_lanemask_lt();
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
        const int64_t e = base + 64 * i + lane;
        const bool ok = e < n;
        kk[i] = ok ? kin[e] : 0;
        vv[i] = ok ? vin[e] : 0;
    }
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
        const bool ok = base + 64 * i + lane < n;
        const unsigned dg = ((unsigned)kk[i] >> shift) & (unsigned)(nb - 1);
        unsigned long long peers = __ballot(ok);
        for (int b = 0; b < bits; ++b) {
            const bool bit = (dg >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int before = ok ? wcnt[w][dg] : 0;  // every lane reads before the leader's update below
        __builtin_amdgcn_wave_barrier();
        rk[i] = before + __popcll(peers & lt);
        if (ok && (peers & lt) == 0) wcnt[w][dg] = before + __popcll(peers);  // the lowest peer updates
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // per digit: exclusive prefix over the waves (tile order = wave order);
    // the digit's tile total goes to dstart
    for (int t = threadIdx.x; t < nb; t += RS_THREADS) {
        int s = 0;
#pragma unroll
        for (int ww = 0; ww < RS_WAVES; ++ww) {
            const int c = wcnt[ww][t];
            wcnt[ww][t] = s;
            s += c;
        }
        dstart[t] = s;
    }
    __syncthreads();
    {  // dstart -> exclusive prefix over the digits (two digits per thread)
        const int d0 = 2 * threadIdx.x;
        const int c0 = d0 < nb ? dstart[d0] : 0, c1 = d0 + 1 < nb ? dstart[d0 + 1] : 0;
        int x = c0 + c1;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int ex = x - c0 - c1;
        for (int ww = 0; ww < w; ++ww) ex += wsum[ww];
        if (d0 < nb) dstart[d0] = ex;
        if (d0 + 1 < nb) dstart[d0 + 1] = ex + c0;
    }
    __syncthreads();
    // the tile in digit order through LDS, then written out by consecutive
    // threads (a digit's run of the tile is contiguous in the output)
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
        if (base + 64 * i + lane >= n) continue;
        const unsigned dg = ((unsigned)kk[i] >> shift) & (unsigned)(nb - 1);
        stage[dstart[dg] + wcnt[w][dg] + rk[i]] = make_int2(kk[i], vv[i]);
    }
    __syncthreads();
    const int64_t tbase = (int64_t)tile * (RS_THREADS * RS_IPT);
    const int tn = (int)min((int64_t)(RS_THREADS * RS_IPT), n - tbase);
    for (int j = threadIdx.x; j < tn; j += RS_THREADS) {
        const int2 kv = stage[j];
        const unsigned dg = ((unsigned)kv.x >> shift) & (unsigned)(nb - 1);
        const int pos = goff[dg] + (j - dstart[dg]);
        kout[pos] = kv.x;
        vout[pos] = kv.y;
    }
}

int ccg_sort_pairs_i32(ccg_ctx* ctx, const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                       int32_t* vals_out, int64_t n, int key_bits, hipStream_t st) {
    CCG_REQUIRE(n >= 0 && n < (1LL << 31), "ccg_sort_pairs_i32: n out of range");
    CCG_REQUIRE(key_bits >= 0 && key_bits <= 31, "ccg_sort_pairs_i32: key_bits out of range");
    if (n == 0) return CCG_OK;
    int ipt = 16;
    while (RS_ADAPT && ipt > 1 && ccg_cdiv(n, (int64_t)RS_THREADS * ipt) < RS_TILES_MIN) ipt >>= 1;
    const int ntiles = (int)ccg_cdiv(n, (int64_t)RS_THREADS * ipt);
    if (key_bits == 0) {  // one digit value: the input order
        CCG_HIP(hipMemcpyAsync(keys_out, keys_in, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
        CCG_HIP(hipMemcpyAsync(vals_out, vals_in, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
        return CCG_OK;
    }
    const int npass = (key_bits + RS_MAXBITS - 1) / RS_MAXBITS;
    const size_t cnt_ints = (size_t)(1 << RS_MAXBITS) * ntiles;
    char* ws = (char*)ccg_ws(ctx, WS_SORT, sizeof(int64_t) * (cnt_ints + 1) + sizeof(int32_t) * 2 * (size_t)n + 256);
    if (!ws) return CCG_ENOMEM;
    int64_t* cnt = (int64_t*)ws;
    int32_t* tk = (int32_t*)(ws + ccg_cdiv(sizeof(int64_t) * (cnt_ints + 1), 256) * 256);
    int32_t* tv = tk + n;
    // pass p writes out when (npass - 1 - p) is even, so the last pass lands in out
    const int32_t* ck = keys_in;
    const int32_t* cv = vals_in;
    int shift = 0;
    for (int p = 0; p < npass; ++p) {
        const int bits = (key_bits - shift + (npass - p) - 1) / (npass - p);  // the remaining bits split evenly
        int32_t* ok = ((npass - 1 - p) % 2 == 0) ? keys_out : tk;
        int32_t* ov = ((npass - 1 - p) % 2 == 0) ? vals_out : tv;
#define RS_PASS(IPT_)                                                                              \
    do {                                                                                           \
        rs_hist<IPT_><<<ntiles, RS_THREADS, 0, st>>>(ck, n, shift, bits, ntiles, cnt);             \
        const int rc = ccg_scan_i64(ctx, cnt, cnt, (int64_t)(1 << bits) * ntiles, st);            \
        if (rc) return rc;                                                                         \
        rs_scatter<IPT_><<<ntiles, RS_THREADS, 0, st>>>(ck, cv, n, shift, bits, ntiles, cnt, ok, ov);       \
    } while (0)
        if (ipt == 16) RS_PASS(16);
        else if (ipt == 8) RS_PASS(8);
        else if (ipt == 4) RS_PASS(4);
        else if (ipt == 2) RS_PASS(2);
        else RS_PASS(1);
#undef RS_PASS
        ck = ok;
        cv = ov;
        shift += bits;
    }
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

extern "C" int ccg_sort_pairs_dev(ccg_ctx* ctx, const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                                  int32_t* vals_out, int64_t n, int key_bits, void* stream) {
    CCG_REQUIRE(ctx && (n == 0 || (keys_in && keys_out && vals_in && vals_out)), "ccg_sort_pairs_dev: NULL argument");
    CCG_REQUIRE(keys_in != keys_out && vals_in != vals_out, "ccg_sort_pairs_dev: in-place sorting is not supported");
    return ccg_sort_pairs_i32(ctx, keys_in, keys_out, vals_in, vals_out, n, key_bits, ccg_pick_stream(ctx, stream));
}

extern "C" int ccg_scan_i64_dev(ccg_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, void* stream) {
    CCG_REQUIRE(ctx && (n <= 0 || in) && out, "ccg_scan_i64_dev: NULL argument");
    CCG_REQUIRE(n >= 0, "ccg_scan_i64_dev: n=%lld", (long long)n);
    return ccg_scan_i64(ctx, in, out, n, ccg_pick_stream(ctx, stream));
}
