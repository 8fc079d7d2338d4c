// Context, error reporting, workspace and a device scan for libccg.so.
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <chrono>

#include "ccg_internal.h"

static thread_local char g_err[1024] = "";

void ccg_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int ccg_hip_fail(hipError_t e, const char* what, const char* file, int line) {
    ccg_set_error("HIP error '%s' (%d) in %s at %s:%d", hipGetErrorString(e),
                  (int)e, what, file, line);
    return e == hipErrorOutOfMemory ? CCG_ENOMEM : CCG_EHIP;
}

extern "C" int ccg_abi_version(void) { return CCG_ABI_VERSION; }
extern "C" const char* ccg_last_error(void) { return g_err; }

extern "C" int ccg_open(const ccg_config* cfg, ccg_ctx** out) {
    if (!out) {
        ccg_set_error("ccg_open: out is NULL");
        return CCG_EINVAL;
    }
    *out = nullptr;
    int dev = cfg ? cfg->device : 0;
    int ndev = 0;
    CCG_HIP(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) {
        ccg_set_error("ccg_open: device %d out of range (%d devices)", dev, ndev);
        return CCG_EINVAL;
    }
    CCG_HIP(hipSetDevice(dev));
    ccg_ctx* c = new ccg_ctx();
    memset(c->ws, 0, sizeof(c->ws));
    memset(c->ws_bytes, 0, sizeof(c->ws_bytes));
    c->device = dev;
    c->last_stats.queries = 0;
    c->last_stats.fallback = 0;
    c->timing = 0;
    c->timers = nullptr;
    c->ntimers = c->cap_timers = c->used_timers = 0;
    c->d_err = nullptr;
    c->snn_row_reserve = 0;
    c->snn_stage = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return ccg_hip_fail(e, "hipStreamCreate", __FILE__, __LINE__);
    }
    e = hipMalloc(&c->d_err, 64);
    if (e == hipSuccess) e = hipMemset(c->d_err, 0, 64);
    c->scan_nstreams = 0;
    if (e == hipSuccess) e = hipMalloc(&c->d_scan, (size_t)SCAN_LB_BYTES * CCG_SCAN_SLOTS);
    if (e == hipSuccess) e = hipMemset(c->d_scan, 0, (size_t)SCAN_LB_BYTES * CCG_SCAN_SLOTS);
    if (e != hipSuccess) {
        if (c->d_err) (void)hipFree(c->d_err);
        if (c->d_scan) (void)hipFree(c->d_scan);
        (void)hipStreamDestroy(c->stream);
        delete c;
        return ccg_hip_fail(e, "hipMalloc(d_err, d_scan)", __FILE__, __LINE__);
    }
    *out = c;
    return CCG_OK;
}

extern "C" int ccg_close(ccg_ctx* ctx) {
    if (!ctx) return CCG_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (int s = 0; s < WS_NSLOTS; ++s)
        if (ctx->ws[s]) (void)hipFree(ctx->ws[s]);
    for (int t = 0; t < ctx->ntimers; ++t) {
        (void)hipEventDestroy(ctx->timers[t].start);
        (void)hipEventDestroy(ctx->timers[t].stop);
    }
    free(ctx->timers);
    for (int s = 0; s < CCG_PIN_RING; ++s) {
        if (ctx->pin_buf[s]) (void)hipHostFree(ctx->pin_buf[s]);
        if (ctx->pin_ev[s]) (void)hipEventDestroy(ctx->pin_ev[s]);
    }
    ccg_snn_stage_free(ctx);
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->d_scan) (void)hipFree(ctx->d_scan);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return CCG_OK;
}

int ccg_h2d_staged(ccg_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes == 0) return CCG_OK;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    CCG_HIP(hipStreamIsCapturing(st, &cap));
    if (cap != hipStreamCaptureStatusNone) {
        // the ring slot's event wait cannot be captured, and a replay would
        // copy whatever a later call left in the slot
        ccg_set_error("this entry point uploads a host table (segment offsets / pointer tables) and cannot be "
                      "captured into a HIP graph; launch it eagerly");
        return CCG_EINVAL;
    }
    const int s = ctx->pin_next;
    ctx->pin_next = (s + 1) % CCG_PIN_RING;
    if (!ctx->pin_ev[s]) CCG_HIP(hipEventCreateWithFlags(&ctx->pin_ev[s], hipEventDisableTiming));
    else if (hipEventQuery(ctx->pin_ev[s]) == hipErrorNotReady) {  // the slot's previous copy has not run
        (void)hipGetLastError();  // (not-ready is a status, not an error: keep it out of the next launch check)
        const auto t0 = std::chrono::steady_clock::now();
        CCG_HIP(hipEventSynchronize(ctx->pin_ev[s]));
        ctx->pin_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ctx->pin_waits++;
    }
    if (ctx->pin_bytes[s] < bytes) {
        if (ctx->pin_buf[s]) CCG_HIP(hipHostFree(ctx->pin_buf[s]));
        ctx->pin_buf[s] = nullptr;
        ctx->pin_bytes[s] = 0;
        // at least 64 KB, powers of two: a slot almost never grows after its
        // first use (hipHostFree synchronises the device: a regrowth inside a
        // launch loop leaves the GPU idle while the host waits)
        size_t want = 65536;
        while (want < bytes) want *= 2;
        CCG_HIP(hipHostMalloc(&ctx->pin_buf[s], want, hipHostMallocDefault));
        ctx->pin_bytes[s] = want;
    }
    memcpy(ctx->pin_buf[s], src, bytes);
    CCG_HIP(hipMemcpyAsync(dst, ctx->pin_buf[s], bytes, hipMemcpyHostToDevice, st));
    CCG_HIP(hipEventRecord(ctx->pin_ev[s], st));
    return CCG_OK;
}

int ccg_take_device_error(ccg_ctx* ctx) {
    int bits = 0;
    CCG_HIP(hipSetDevice(ctx->device));
    CCG_HIP(hipDeviceSynchronize());
    CCG_HIP(hipMemcpy(&bits, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (!bits) return CCG_OK;
    CCG_HIP(hipMemset(ctx->d_err, 0, sizeof(int)));
    if (bits & CCG_DERR_LABEL_RANGE) {
        ccg_set_error("cluster label exceeds the assignment matrix's label width (use label_bits=16)");
        return CCG_ERANGE;
    }
    if (bits & CCG_DERR_CLUSTER_INDEX) {
        ccg_set_error("cluster position outside [0, K)");
        return CCG_EINVAL;
    }
    if (bits & CCG_DERR_SCAN_RANGE) {
        ccg_set_error("scan: a tile sum or prefix outside [0, 2^62)");
        return CCG_ERANGE;
    }
    if (bits & CCG_DERR_KNN_UNIQUE) {
        ccg_set_error("ccg_knn_boot_dev: n_unique is not the number of distinct cells in idx");
        return CCG_EINVAL;
    }
    ccg_set_error("SNN: neighbour index out of range or equal to the row itself");
    return CCG_EINVAL;
}

extern "C" int ccg_synchronize(ccg_ctx* ctx) {
    CCG_REQUIRE(ctx, "ccg_synchronize: NULL ctx");
    return ccg_take_device_error(ctx);
}

extern "C" int ccg_check_errors(ccg_ctx* ctx) {
    CCG_REQUIRE(ctx, "ccg_check_errors: NULL ctx");
    return ccg_take_device_error(ctx);
}

extern "C" void* ccg_stream(ccg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

extern "C" int ccg_ctx_device(const ccg_ctx* ctx, int* device) {
    CCG_REQUIRE(ctx && device, "ccg_ctx_device: NULL argument");
    *device = ctx->device;
    return CCG_OK;
}

void* ccg_ws(ccg_ctx* ctx, int slot, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (ctx->ws_bytes[slot] >= bytes) return ctx->ws[slot];
    // Growth: let in-flight work that may still read the old buffer finish.
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    // state that points into the old buffer goes with it: the kNN's zeroed-
    // counter marks (re-zeroed on the next call) and the exact-search row list
    // of ccg_knn_last_fallback
    const char* old = (const char*)ctx->ws[slot];
    const size_t oldb = ctx->ws_bytes[slot];
    auto inside = [&](const void* p) { return old && p && (const char*)p >= old && (const char*)p < old + oldb; };
    if (inside(ctx->kb_zeroed)) ctx->kb_zeroed = nullptr;
    if (inside(ctx->fx_zeroed)) ctx->fx_zeroed = nullptr;
    if (inside(ctx->last_fail_list) || inside(ctx->last_fail_count)) {
        ctx->last_fail_list = nullptr;
        ctx->last_fail_count = nullptr;
    }
    if (ctx->ws[slot]) (void)hipFree(ctx->ws[slot]);
    ctx->ws[slot] = nullptr;
    ctx->ws_bytes[slot] = 0;
    size_t want = bytes + bytes / 8;  // headroom for slowly growing sizes
    want = (want + 255) & ~(size_t)255;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        ccg_set_error("workspace allocation of %zu bytes failed (slot %d): %s",
                      want, slot, hipGetErrorString(e));
        return nullptr;
    }
    ctx->ws[slot] = p;
    ctx->ws_bytes[slot] = want;
    return p;
}

// ---------------------------------------------------------------- timing --
int ccg_timer_start(ccg_ctx* ctx, int which, hipStream_t st) {
    if (!ctx->timing) return -1;
    if (ctx->used_timers == ctx->ntimers) {
        if (ctx->ntimers == ctx->cap_timers) {
            int nc = ctx->cap_timers ? 2 * ctx->cap_timers : 256;
            ccg_timer_rec* nt = (ccg_timer_rec*)realloc(ctx->timers, sizeof(ccg_timer_rec) * nc);
            if (!nt) return -1;
            ctx->timers = nt;
            ctx->cap_timers = nc;
        }
        ccg_timer_rec& r = ctx->timers[ctx->ntimers];
        if (hipEventCreate(&r.start) != hipSuccess) return -1;
        if (hipEventCreate(&r.stop) != hipSuccess) return -1;
        ctx->ntimers++;
    }
    int h = ctx->used_timers++;
    ctx->timers[h].which = which;
    (void)hipEventRecord(ctx->timers[h].start, st);
    return h;
}

void ccg_timer_stop(ccg_ctx* ctx, int handle, hipStream_t st) {
    if (handle < 0) return;
    (void)hipEventRecord(ctx->timers[handle].stop, st);
}

extern "C" int ccg_timing_enable(ccg_ctx* ctx, int enable) {
    CCG_REQUIRE(ctx, "ccg_timing_enable: NULL ctx");
    ctx->timing = enable ? 1 : 0;
    return CCG_OK;
}

extern "C" int ccg_timing_read(ccg_ctx* ctx, int which, double* total_ms, int64_t* launches) {
    CCG_REQUIRE(ctx && total_ms && launches, "ccg_timing_read: NULL argument");
    if (which == CCG_KT_HOST_RING_WAIT) {  // host-side accounting, read and reset
        *total_ms = ctx->pin_wait_ms;
        *launches = ctx->pin_waits;
        ctx->pin_wait_ms = 0.0;
        ctx->pin_waits = 0;
        return CCG_OK;
    }
    CCG_REQUIRE(which >= 0 && which < CCG_KT_COUNT, "ccg_timing_read: bad kernel id");
    double tot = 0.0;
    int64_t n = 0;
    int keep = 0;
    for (int t = 0; t < ctx->used_timers; ++t) {
        ccg_timer_rec r = ctx->timers[t];
        if (r.which == which) {
            CCG_HIP(hipEventSynchronize(r.stop));
            float ms = 0.f;
            CCG_HIP(hipEventElapsedTime(&ms, r.start, r.stop));
            tot += ms;
            ++n;
        } else {
            ctx->timers[t] = ctx->timers[keep];  // compact unread records to the front
            ctx->timers[keep] = r;
            ++keep;
        }
    }
    ctx->used_timers = keep;
    *total_ms = tot;
    *launches = n;
    return CCG_OK;
}

// ------------------------------------------------------------------ scan --
#define SCAN_T 256
#ifndef SCAN_TILE
#define SCAN_TILE 2048  // 8 elements per thread
#endif

__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t* total) {
    const int t = threadIdx.x;
    const int lane = t & 63, wv = t >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    int64_t woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_T / 64; ++w) {
        int64_t s = sh[w];
        if (w < wv) woff += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return woff + x - v;
}

__global__ __launch_bounds__(SCAN_T) void scan_tile_sums(const int64_t* __restrict__ in,
                                                         int64_t n, int64_t* __restrict__ bsum) {
    __shared__ int64_t sh[SCAN_T / 64];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t s = 0;
#pragma unroll
    for (int e = 0; e < SCAN_TILE / SCAN_T; ++e) {
        int64_t i = base + threadIdx.x * (SCAN_TILE / SCAN_T) + e;
        if (i < n) s += in[i];
    }
    int64_t tot;
    block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void scan_block_sums(int64_t* __restrict__ bsum, int64_t nb) {
    __shared__ int64_t sh[SCAN_T / 64];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += SCAN_T) {
        int64_t i = b0 + threadIdx.x;
        int64_t v = i < nb ? bsum[i] : 0;
        int64_t tot;
        int64_t ex = block_excl_scan(v, sh, &tot);
        if (i < nb) bsum[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

__global__ __launch_bounds__(SCAN_T) void scan_tiles(const int64_t* in, int64_t* out, int64_t n,
                                                     const int64_t* __restrict__ bsum, int64_t nb) {
    __shared__ int64_t sh[SCAN_T / 64];
    constexpr int E = SCAN_TILE / SCAN_T;
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * E;
    int64_t v[E];
    int64_t s = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        v[e] = (base + e < n) ? in[base + e] : 0;
        s += v[e];
    }
    int64_t tot;
    int64_t ex = block_excl_scan(s, sh, &tot) + bsum[blockIdx.x];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (base + e < n) out[base + e] = ex;
        ex += v[e];
    }
    if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = bsum[nb];
}

// Single pass for up to SCAN_LB_MAX tiles (decoupled look-back): block b
// scans its tile and publishes a status word, (1 << 62) | aggregate, then
// walks back over the words of the tiles before it -- adding aggregates
// until it meets an inclusive prefix, (2 << 62) | prefix -- and publishes
// its own inclusive prefix; wave 0 reads 64 predecessors' words per round
// (one per lane: one word per round took ~1 us per predecessor, the words
// being read past the L2).  One launch instead of the tile-sums pass plus
// the tile pass (two launches on the critical path of each of a bootstrap's
// ~8 scans).  Status and value share one 64-bit word, so relaxed
// device-scope atomics suffice: no release / acquire fences (their L2
// write-back and invalidate cost a first version of this kernel 21 us per
// call under three streams).  A block waits only on lower-numbered blocks,
// which the dispatcher starts first.  The last block to finish (the
// finished count) clears the words for the next call, so the kernel needs no
// per-call epoch and replays from a HIP graph.  Tile sums and prefixes must
// lie in [0, 2^62): the library scans counts.
#define SCAN_ST_AGG (1ull << 62)
#define SCAN_ST_INC (2ull << 62)
#define SCAN_VAL_MASK ((1ull << 62) - 1)
__global__ __launch_bounds__(SCAN_T) void scan_onepass(const int64_t* in, int64_t* out, int64_t n, int nb,
                                                       unsigned long long* __restrict__ stat,
                                                       unsigned* __restrict__ done, int* __restrict__ err) {
    __shared__ int64_t sh[SCAN_T / 64];
    __shared__ int64_t pref;
    constexpr int E = SCAN_TILE / SCAN_T;
    const int b = blockIdx.x;
    const int64_t base = (int64_t)b * SCAN_TILE + threadIdx.x * E;
    int64_t v[E];
    int64_t s = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        v[e] = (base + e < n) ? in[base + e] : 0;
        s += v[e];
    }
    int64_t tot;
    int64_t ex = block_excl_scan(s, sh, &tot);
    // the status words hold 62-bit values: a negative or too large tile sum
    // (a caller's contract violation) is reported, not silently wrapped
    if (threadIdx.x == 0 && (uint64_t)tot >> 62) atomicOr(err, CCG_DERR_SCAN_RANGE);
    if (threadIdx.x < 64) {  // wave 0: the look-back, 64 predecessors per round (one per lane)
        const int lane = threadIdx.x;
        unsigned long long run = 0;
        if (b == 0) {
            if (lane == 0)
                __hip_atomic_store(&stat[0], SCAN_ST_INC | ((unsigned long long)tot & SCAN_VAL_MASK),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&stat[b], SCAN_ST_AGG | ((unsigned long long)tot & SCAN_VAL_MASK),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int j0 = b - 1;;) {
                const int j = j0 - lane;  // (j < 0 reads as a prefix past tile 0's, which is never reached)
                const unsigned long long w =
                    j >= 0 ? __hip_atomic_load(&stat[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : SCAN_ST_INC;
                const unsigned long long st2 = w >> 62;
                const unsigned long long inc = __ballot(st2 == 2);
                const int lim = inc ? __ffsll((long long)inc) - 1 : 64;  // the nearest inclusive prefix
                const unsigned long long need = lim == 64 ? ~0ull : ((2ull << lim) - 1);
                if (__ballot(st2 == 0) & need) {  // a tile before it has not published yet (wave-uniform)
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                unsigned long long v = lane <= lim ? (w & SCAN_VAL_MASK) : 0ull;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
                run += v;
                if (lim < 64) break;
                j0 -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&stat[b], SCAN_ST_INC | ((run + (unsigned long long)tot) & SCAN_VAL_MASK),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) pref = (int64_t)run;
    }
    __syncthreads();
    ex += pref;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (base + e < n) out[base + e] = ex;
        ex += v[e];
    }
    if (b == nb - 1 && threadIdx.x == 0) {
        out[n] = pref + tot;
        if ((uint64_t)(pref + tot) >> 62) atomicOr(err, CCG_DERR_SCAN_RANGE);
    }
    if (threadIdx.x == 0) {
        // every block counted here has finished its look-back
        const unsigned t = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == (unsigned)nb - 1) {
            for (int j = 0; j < nb; ++j) __hip_atomic_store(&stat[j], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int ccg_scan_i64(ccg_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, hipStream_t st) {
    if (n <= 0) {
        CCG_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), st));
        return CCG_OK;
    }
    int64_t nb = ccg_cdiv(n, SCAN_TILE);
    // the stream's own slice of the single-pass state: two streams' scans
    // never share status words (a shared word could make a tile of one wait
    // on a word the other's last tile already cleared: a hang); a context
    // used from more than CCG_SCAN_SLOTS streams takes the two-pass scan
    int slot = -1;
    for (int i = 0; i < ctx->scan_nstreams; ++i)
        if (ctx->scan_stream[i] == st) slot = i;
    if (slot < 0 && ctx->scan_nstreams < CCG_SCAN_SLOTS) {
        slot = ctx->scan_nstreams++;
        ctx->scan_stream[slot] = st;
    }
    if (nb <= SCAN_LB_MAX && slot >= 0) {
        unsigned long long* stat = (unsigned long long*)((char*)ctx->d_scan + (size_t)slot * SCAN_LB_BYTES);
        scan_onepass<<<(unsigned)nb, SCAN_T, 0, st>>>(in, out, n, (int)nb, stat, (unsigned*)(stat + SCAN_LB_MAX),
                                                      ctx->d_err);
        CCG_HIP(hipGetLastError());
        return CCG_OK;
    }
    int64_t* bsum = (int64_t*)ccg_ws(ctx, WS_SCAN, sizeof(int64_t) * (nb + 1));
    if (!bsum) return CCG_ENOMEM;
    scan_tile_sums<<<(unsigned)nb, SCAN_T, 0, st>>>(in, n, bsum);
    scan_block_sums<<<1, SCAN_T, 0, st>>>(bsum, nb);
    scan_tiles<<<(unsigned)nb, SCAN_T, 0, st>>>(in, out, n, bsum, nb);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}
