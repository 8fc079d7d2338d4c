// Context, error reporting, workspace and a device scan for libccg.so.
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

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
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return ccg_hip_fail(e, "hipStreamCreate", __FILE__, __LINE__);
    }
    e = hipMalloc(&c->d_err, 64);
    if (e == hipSuccess) e = hipMemset(c->d_err, 0, 64);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return ccg_hip_fail(e, "hipMalloc(d_err)", __FILE__, __LINE__);
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
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
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
#define SCAN_TILE 2048  // 8 elements per thread

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

// One-pass scan (decoupled look-back): every block takes the next tile id
// from a ticket (so a tile's predecessors are always running or done),
// publishes its tile sum, looks back over the predecessors' published sums
// until one carries its inclusive prefix, publishes its own inclusive prefix
// and writes its outputs.  One launch per scan instead of two.  A status word
// holds (call sequence << 2 | state), state 1 = tile sum, 2 = inclusive
// prefix, so no reset is needed between calls; the value is stored before
// the word (release) and read after it (acquire).  The block that takes the
// last id returns the ticket to 0 for the next call.
struct ScanStatus {
    unsigned* ticket;
    unsigned* flag;
    int64_t* aggr;
    int64_t* incl;
};

__global__ __launch_bounds__(SCAN_T) void scan_onepass(const int64_t* in, int64_t* out, int64_t n, int64_t nb,
                                                       ScanStatus ss, unsigned seq) {
    __shared__ int64_t sh[SCAN_T / 64];
    __shared__ int64_t sh_pre;
    __shared__ unsigned sh_tile;
    if (threadIdx.x == 0) {
        const unsigned t = atomicAdd(ss.ticket, 1u);
        if (t == (unsigned)nb - 1) __hip_atomic_store(ss.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_tile = t;
    }
    __syncthreads();
    const int64_t tile = sh_tile;
    constexpr int E = SCAN_TILE / SCAN_T;
    const int64_t base = tile * SCAN_TILE + threadIdx.x * E;
    int64_t v[E];
    int64_t s = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        v[e] = (base + e < n) ? in[base + e] : 0;
        s += v[e];
    }
    int64_t tot;
    const int64_t ex = block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) {
        int64_t pre = 0;
        if (tile == 0) {
            __hip_atomic_store(&ss.incl[0], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ss.flag[0], (seq << 2) | 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&ss.aggr[tile], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ss.flag[tile], (seq << 2) | 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            for (int64_t p = tile - 1; p >= 0;) {
                const unsigned f = __hip_atomic_load(&ss.flag[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if ((f >> 2) != seq) {  // not published yet in this call
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if ((f & 3u) == 2u) {
                    pre += __hip_atomic_load(&ss.incl[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                pre += __hip_atomic_load(&ss.aggr[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                --p;
            }
            __hip_atomic_store(&ss.incl[tile], pre + tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ss.flag[tile], (seq << 2) | 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        sh_pre = pre;
    }
    __syncthreads();
    int64_t x = ex + sh_pre;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (base + e < n) out[base + e] = x;
        x += v[e];
    }
    if (tile == nb - 1 && threadIdx.x == 0) out[n] = sh_pre + tot;
}

int ccg_scan_i64(ccg_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, hipStream_t st) {
    if (n <= 0) {
        CCG_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), st));
        return CCG_OK;
    }
    const int64_t nb = ccg_cdiv(n, SCAN_TILE);
    // status of up to max(nb, 2^16) tiles: ticket, flags, tile sums, inclusive prefixes
    const int64_t cap = std::max<int64_t>(nb, 1 << 16);
    const size_t fb = (size_t)ccg_cdiv(sizeof(unsigned) * (cap + 4), 16) * 16;
    char* ws = (char*)ccg_ws(ctx, WS_SCAN, fb + 2 * sizeof(int64_t) * (size_t)cap);
    if (!ws) return CCG_ENOMEM;
    if (ctx->scan_zeroed != (void*)ws || ctx->scan_cap < cap) {  // fresh buffer: ticket and flags zero
        CCG_HIP(hipMemsetAsync(ws, 0, fb, st));
        ctx->scan_zeroed = (void*)ws;
        ctx->scan_cap = (ctx->ws_bytes[WS_SCAN] - fb) / (2 * sizeof(int64_t));
        ctx->scan_seq = 0;
    }
    ctx->scan_seq = (ctx->scan_seq % 0x3FFFFFFFu) + 1;  // 30-bit call sequence, never 0
    ScanStatus ss{(unsigned*)ws, (unsigned*)ws + 4, (int64_t*)(ws + fb), (int64_t*)(ws + fb) + cap};
    scan_onepass<<<(unsigned)nb, SCAN_T, 0, st>>>(in, out, n, nb, ss, ctx->scan_seq);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}
