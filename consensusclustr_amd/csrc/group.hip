// Multi-GPU layer of libccg.so: a device group = one engine context (HIP
// stream + workspaces) per local device and one RCCL communicator per device.
//
// The reference is single-node CPU (BiocParallel workers over bootstraps,
// RcppParallel threads inside parDist, R/consensusClust.R:391-421); its
// multi-GPU form here (north_star subsystem 4):
//   * bootstraps are independent: contiguous blocks per rank (ccg_boot_shard),
//     no communication for gather / kNN / SNN / silhouette / map-back;
//   * the co-clustering step needs every rank's assignment columns: ONE
//     all-gather over xGMI (ccg_allgather_columns, RCCL);
//   * the packed co/both/dist triangle is split into row slabs balanced by
//     pair count (ccg_row_slabs), each slab computed and kept by one device
//     (ccg_cocluster_sharded_dev);
//   * the fused consensus kNN splits full rows evenly (ccg_rect_slabs) and
//     all-gathers the N x k neighbour matrix (ccg_consensus_knn_sharded_dev).
// Two ways to form a group: one process driving several devices
// (ccg_group_open, ncclCommInitAll -- what an R session uses) or one process
// per device (ccg_group_open_rank with an id from ccg_group_unique_id that
// the caller broadcasts -- what a torchrun launch uses).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ccg_internal.h"

struct ccg_group {
    int nlocal = 0;  // devices driven by this process
    int nranks = 0;  // devices in the communicator
    int rank0 = 0;   // global rank of local device 0
    std::vector<ccg_ctx*> ctx;
    std::vector<ncclComm_t> comm;
};

static int nccl_fail(ncclResult_t r, const char* what) {
    ccg_set_error("RCCL error '%s' (%d) in %s", ncclGetErrorString(r), (int)r, what);
    return CCG_EHIP;
}

#define CCG_NCCL(x)                                        \
    do {                                                   \
        ncclResult_t ccg_r_ = (x);                         \
        if (ccg_r_ != ncclSuccess) return nccl_fail(ccg_r_, #x); \
    } while (0)

// Runs fn(l) for every local device, on its own host thread when the group
// drives several devices (so per-device host synchronisation -- e.g. the
// uint16 slot-table sizing of the co-cluster -- does not serialise devices).
// The first failing device's status and message are returned.
template <class F>
static int for_each_local(ccg_group* g, F fn) {
    if (g->nlocal == 1) {
        CCG_HIP(hipSetDevice(g->ctx[0]->device));
        return fn(0);
    }
    std::vector<int> rc(g->nlocal, CCG_OK);
    std::vector<std::string> msg(g->nlocal);
    std::vector<std::thread> th;
    th.reserve(g->nlocal);
    for (int l = 0; l < g->nlocal; ++l)
        th.emplace_back([&, l] {
            hipError_t e = hipSetDevice(g->ctx[l]->device);
            rc[l] = e == hipSuccess ? fn(l) : ccg_hip_fail(e, "hipSetDevice", __FILE__, __LINE__);
            if (rc[l]) msg[l] = ccg_last_error();
        });
    for (auto& t : th) t.join();
    for (int l = 0; l < g->nlocal; ++l)
        if (rc[l]) {
            ccg_set_error("device %d: %s", g->ctx[l]->device, msg[l].c_str());
            return rc[l];
        }
    return CCG_OK;
}

// ------------------------------------------------------------- planning --
extern "C" int ccg_row_slabs(int64_t N, int G, int64_t* cuts) {
    CCG_REQUIRE(cuts && N >= 0 && G >= 1, "ccg_row_slabs: bad arguments");
    // Row i of the packed triangle holds N-1-i pairs, so equal pair counts put
    // cut g at N (1 - sqrt(1 - g/G)); interior cuts are rounded to the
    // co-cluster tile height and kept <= the last aligned row.
    const int64_t A = CCG_COCLUSTER_ROW_ALIGN;
    const int64_t top = (N / A) * A;
    cuts[0] = 0;
    for (int g = 1; g < G; ++g) {
        const double r = (double)N * (1.0 - std::sqrt(1.0 - (double)g / (double)G));
        int64_t c = (int64_t)std::llround(r / (double)A) * A;
        cuts[g] = std::min(std::max(c, cuts[g - 1]), top);
    }
    cuts[G] = N;
    return CCG_OK;
}

extern "C" int ccg_rect_slabs(int64_t N, int G, int64_t* cuts) {
    CCG_REQUIRE(cuts && N >= 0 && G >= 1, "ccg_rect_slabs: bad arguments");
    // Full rows cost N each (consensus kNN): equal row counts, aligned.
    const int64_t A = CCG_COCLUSTER_ROW_ALIGN;
    const int64_t top = (N / A) * A;
    cuts[0] = 0;
    for (int g = 1; g < G; ++g) {
        int64_t c = (int64_t)std::llround((double)N * g / G / (double)A) * A;
        cuts[g] = std::min(std::max(c, cuts[g - 1]), top);
    }
    cuts[G] = N;
    return CCG_OK;
}

extern "C" int ccg_boot_shard(int64_t nboots, int G, int rank, int64_t* b0, int64_t* b1) {
    CCG_REQUIRE(b0 && b1 && nboots >= 0 && G >= 1 && rank >= 0 && rank < G, "ccg_boot_shard: bad arguments");
    const int64_t base = nboots / G, rem = nboots % G;
    *b0 = rank * base + std::min<int64_t>(rank, rem);
    *b1 = *b0 + base + (rank < rem ? 1 : 0);
    return CCG_OK;
}

// The collective plan of group_allgather_rows, host only (no device, no RCCL):
// offsets = exclusive prefix of the counts; equal counts -> one ncclAllGather;
// unequal -> one ncclBroadcast per rank with rows to send, in rank order.
extern "C" int ccg_allgather_plan(int nranks, const int64_t* counts, int64_t* offsets, int* equal, int* roots,
                                  int* nroots) {
    CCG_REQUIRE(nranks >= 1 && counts && offsets && equal && nroots, "ccg_allgather_plan: bad arguments");
    offsets[0] = 0;
    int eq = 1, nr = 0;
    for (int r = 0; r < nranks; ++r) {
        CCG_REQUIRE(counts[r] >= 0, "ccg_allgather_plan: negative count for rank %d", r);
        offsets[r + 1] = offsets[r] + counts[r];
        eq = eq && counts[r] == counts[0];
    }
    for (int r = 0; r < nranks; ++r)
        if (!eq && counts[r] > 0) {
            if (roots) roots[nr] = r;
            ++nr;
        }
    *equal = eq;
    *nroots = eq ? 0 : nr;
    return CCG_OK;
}

// ------------------------------------------------------------ lifecycle --
extern "C" int ccg_group_unique_id(uint8_t* id) {
    CCG_REQUIRE(id, "ccg_group_unique_id: NULL id");
    ncclUniqueId u;
    CCG_NCCL(ncclGetUniqueId(&u));
    static_assert(sizeof(u) == CCG_GROUP_ID_BYTES, "RCCL unique id size");
    memcpy(id, &u, sizeof(u));
    return CCG_OK;
}

static void group_free(ccg_group* g) {
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    for (ccg_ctx* c : g->ctx) (void)ccg_close(c);
    delete g;
}

extern "C" int ccg_group_open(const int* devices, int ndev, ccg_group** out) {
    CCG_REQUIRE(out && devices && ndev >= 1, "ccg_group_open: bad arguments");
    *out = nullptr;
    for (int a = 0; a < ndev; ++a)
        for (int b = a + 1; b < ndev; ++b)
            CCG_REQUIRE(devices[a] != devices[b], "ccg_group_open: device %d listed twice", devices[a]);
    ccg_group* g = new ccg_group();
    g->nlocal = g->nranks = ndev;
    g->rank0 = 0;
    for (int l = 0; l < ndev; ++l) {
        ccg_config cfg = {devices[l], 0};
        ccg_ctx* c = nullptr;
        int rc = ccg_open(&cfg, &c);
        if (rc) {
            group_free(g);
            return rc;
        }
        g->ctx.push_back(c);
    }
    g->comm.assign(ndev, nullptr);
    ncclResult_t r = ncclCommInitAll(g->comm.data(), ndev, devices);
    if (r != ncclSuccess) {
        g->comm.assign(ndev, nullptr);
        group_free(g);
        return nccl_fail(r, "ncclCommInitAll");
    }
    *out = g;
    return CCG_OK;
}

extern "C" int ccg_group_open_rank(int device, int nranks, int rank, const uint8_t* id, ccg_group** out) {
    CCG_REQUIRE(out && id && nranks >= 1 && rank >= 0 && rank < nranks, "ccg_group_open_rank: bad arguments");
    *out = nullptr;
    ccg_config cfg = {device, 0};
    ccg_ctx* c = nullptr;
    int rc = ccg_open(&cfg, &c);
    if (rc) return rc;
    ccg_group* g = new ccg_group();
    g->nlocal = 1;
    g->nranks = nranks;
    g->rank0 = rank;
    g->ctx.push_back(c);
    g->comm.assign(1, nullptr);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    (void)hipSetDevice(device);
    ncclResult_t r = ncclCommInitRank(&g->comm[0], nranks, u, rank);
    if (r != ncclSuccess) {
        g->comm[0] = nullptr;
        group_free(g);
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = g;
    return CCG_OK;
}

extern "C" int ccg_group_close(ccg_group* g) {
    if (!g) return CCG_OK;
    for (ccg_ctx* c : g->ctx) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    group_free(g);
    return CCG_OK;
}

extern "C" int ccg_group_info(const ccg_group* g, int* nlocal, int* nranks, int* first_rank) {
    CCG_REQUIRE(g, "ccg_group_info: NULL group");
    if (nlocal) *nlocal = g->nlocal;
    if (nranks) *nranks = g->nranks;
    if (first_rank) *first_rank = g->rank0;
    return CCG_OK;
}

extern "C" int ccg_group_ctx(ccg_group* g, int local, ccg_ctx** out) {
    CCG_REQUIRE(g && out && local >= 0 && local < g->nlocal, "ccg_group_ctx: bad arguments");
    *out = g->ctx[local];
    return CCG_OK;
}

extern "C" int ccg_group_synchronize(ccg_group* g) {
    CCG_REQUIRE(g, "ccg_group_synchronize: NULL group");
    int first = CCG_OK;
    for (ccg_ctx* c : g->ctx) {
        int rc = ccg_synchronize(c);
        if (rc && !first) first = rc;
    }
    return first;
}

// ---------------------------------------------------------- collectives --
// Variable-count all-gather of row blocks: rank r contributes counts[r] rows
// of `row_bytes` bytes; every device receives all blocks in rank order.
// Equal counts use one ncclAllGather (ring over xGMI); unequal counts one
// broadcast per root, fused in a single RCCL group.  src may alias the
// rank's own block of dst.
static int group_allgather_rows(ccg_group* g, const void* const* src, const int64_t* counts, size_t row_bytes,
                                void* const* dst) {
    std::vector<int64_t> off(g->nranks + 1, 0);
    std::vector<int> roots(g->nranks);
    int eq = 0, nroots = 0;
    int rc = ccg_allgather_plan(g->nranks, counts, off.data(), &eq, roots.data(), &nroots);
    if (rc) return rc;
    const bool equal = eq != 0;
    for (int l = 0; l < g->nlocal; ++l)
        CCG_REQUIRE(dst[l] && (src[l] || counts[g->rank0 + l] == 0), "allgather: NULL buffer on local device %d", l);
    if (off[g->nranks] == 0) return CCG_OK;
    CCG_NCCL(ncclGroupStart());
    for (int l = 0; l < g->nlocal; ++l) {
        const int me = g->rank0 + l;
        char* d = (char*)dst[l];
        if (equal) {
            const size_t cnt = (size_t)counts[0] * row_bytes;
            ncclResult_t r = ncclAllGather(src[l], d, cnt, ncclUint8, g->comm[l], g->ctx[l]->stream);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_fail(r, "ncclAllGather");
            }
            continue;
        }
        for (int t = 0; t < nroots; ++t) {
            const int root = roots[t];
            char* recv = d + (size_t)off[root] * row_bytes;
            const void* send = root == me ? src[l] : recv;
            ncclResult_t r = ncclBroadcast(send, recv, (size_t)counts[root] * row_bytes, ncclUint8, root, g->comm[l],
                                           g->ctx[l]->stream);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_fail(r, "ncclBroadcast");
            }
        }
    }
    CCG_NCCL(ncclGroupEnd());
    return CCG_OK;
}

extern "C" int ccg_allgather_columns(ccg_group* g, const void* const* local_A, const int64_t* counts, int64_t N,
                                     int label_bits, void* const* A) {
    CCG_REQUIRE(g && local_A && counts && A, "ccg_allgather_columns: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_allgather_columns: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 1, "ccg_allgather_columns: bad N");
    return group_allgather_rows(g, local_A, counts, (size_t)N * (label_bits / 8), A);
}

// ------------------------------------------------------ sharded compute --
static int64_t tri_off(int64_t N, int64_t i) { return i * N - i * (i + 1) / 2; }

extern "C" int ccg_cocluster_sharded_dev(ccg_group* g, const void* const* A, int label_bits, int64_t N, int64_t B,
                                         uint16_t* const* co, uint16_t* const* both, double* const* dist,
                                         int64_t* cuts) {
    CCG_REQUIRE(g && A, "ccg_cocluster_sharded_dev: NULL argument");
    std::vector<int64_t> cut(g->nranks + 1);
    int rc = ccg_row_slabs(N, g->nranks, cut.data());
    if (rc) return rc;
    if (cuts) std::copy(cut.begin(), cut.end(), cuts);
    return for_each_local(g, [&](int l) {
        const int r = g->rank0 + l;
        return ccg_cocluster_dev(g->ctx[l], A[l], label_bits, N, B, cut[r], cut[r + 1], co ? co[l] : nullptr,
                                 both ? both[l] : nullptr, dist ? dist[l] : nullptr, g->ctx[l]->stream);
    });
}

extern "C" int ccg_consensus_knn_sharded_dev(ccg_group* g, const void* const* A, int label_bits, int64_t N,
                                             int64_t B, int k, int32_t* const* out_idx, int32_t* const* d_nan_flag) {
    CCG_REQUIRE(g && A && out_idx && d_nan_flag, "ccg_consensus_knn_sharded_dev: NULL argument");
    std::vector<int64_t> cut(g->nranks + 1), rows(g->nranks);
    int rc = ccg_rect_slabs(N, g->nranks, cut.data());
    if (rc) return rc;
    for (int r = 0; r < g->nranks; ++r) rows[r] = cut[r + 1] - cut[r];
    rc = for_each_local(g, [&](int l) {
        const int r = g->rank0 + l;
        return ccg_consensus_knn_assign_dev(g->ctx[l], A[l], label_bits, N, B, k, cut[r], cut[r + 1], out_idx[l],
                                            d_nan_flag[l], g->ctx[l]->stream);
    });
    if (rc) return rc;
    // every device gets the whole N x k matrix (in place: each rank's rows are
    // already at their final offset) and the OR of the NaN flags
    std::vector<const void*> src(g->nlocal);
    std::vector<void*> dst(g->nlocal);
    for (int l = 0; l < g->nlocal; ++l) {
        src[l] = out_idx[l] + cut[g->rank0 + l] * k;
        dst[l] = out_idx[l];
    }
    rc = group_allgather_rows(g, src.data(), rows.data(), sizeof(int32_t) * k, dst.data());
    if (rc) return rc;
    CCG_NCCL(ncclGroupStart());
    for (int l = 0; l < g->nlocal; ++l) {
        ncclResult_t r = ncclAllReduce(d_nan_flag[l], d_nan_flag[l], 1, ncclInt32, ncclMax, g->comm[l],
                                       g->ctx[l]->stream);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return nccl_fail(r, "ncclAllReduce");
        }
    }
    CCG_NCCL(ncclGroupEnd());
    return CCG_OK;
}

// ------------------------------------------------------- host flavours --
// Single-process groups only (every rank local): the entry points an R
// session binds.  A is uploaded once to device 0 and broadcast over xGMI.
static int upload_broadcast(ccg_group* g, const void* A, size_t abytes, std::vector<void*>& dA) {
    dA.assign(g->nlocal, nullptr);
    for (int l = 0; l < g->nlocal; ++l) {
        CCG_HIP(hipSetDevice(g->ctx[l]->device));
        dA[l] = ccg_ws(g->ctx[l], WS_HOST_A, abytes);
        if (!dA[l]) return CCG_ENOMEM;
    }
    CCG_HIP(hipSetDevice(g->ctx[0]->device));
    CCG_HIP(hipMemcpyAsync(dA[0], A, abytes, hipMemcpyHostToDevice, g->ctx[0]->stream));
    if (g->nlocal == 1) return CCG_OK;
    CCG_NCCL(ncclGroupStart());
    for (int l = 0; l < g->nlocal; ++l) {
        ncclResult_t r = ncclBroadcast(dA[l], dA[l], abytes, ncclUint8, 0, g->comm[l], g->ctx[l]->stream);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return nccl_fail(r, "ncclBroadcast");
        }
    }
    CCG_NCCL(ncclGroupEnd());
    return CCG_OK;
}

extern "C" int ccg_group_cocluster(ccg_group* g, const void* A, int label_bits, int64_t N, int64_t B, uint16_t* co,
                                   uint16_t* both, double* dist) {
    CCG_REQUIRE(g && A, "ccg_group_cocluster: NULL argument");
    CCG_REQUIRE(g->nlocal == g->nranks, "ccg_group_cocluster: needs a single-process group (use the _dev form per rank)");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_group_cocluster: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && B >= 1, "ccg_group_cocluster: bad sizes");
    std::vector<void*> dA;
    int rc = upload_broadcast(g, A, (size_t)(B * N) * (label_bits / 8), dA);
    if (rc) return rc;
    std::vector<int64_t> cut(g->nranks + 1);
    ccg_row_slabs(N, g->nranks, cut.data());
    return for_each_local(g, [&](int l) {
        ccg_ctx* c = g->ctx[l];
        const int64_t r0 = cut[l], r1 = cut[l + 1];
        const int64_t o = tri_off(N, r0), P = tri_off(N, r1) - o;
        if (P == 0) return (int)CCG_OK;
        uint16_t* dco = co ? (uint16_t*)ccg_ws(c, WS_HOST_B, sizeof(uint16_t) * P) : nullptr;
        uint16_t* dboth = both ? (uint16_t*)ccg_ws(c, WS_HOST_C, sizeof(uint16_t) * P) : nullptr;
        double* ddist = dist ? (double*)ccg_ws(c, WS_HOST_D, sizeof(double) * P) : nullptr;
        if ((co && !dco) || (both && !dboth) || (dist && !ddist)) return (int)CCG_ENOMEM;
        int rc2 = ccg_cocluster_dev(c, dA[l], label_bits, N, B, r0, r1, dco, dboth, ddist, c->stream);
        if (rc2) return rc2;
        if (co) CCG_HIP(hipMemcpyAsync(co + o, dco, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, c->stream));
        if (both) CCG_HIP(hipMemcpyAsync(both + o, dboth, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, c->stream));
        if (dist) CCG_HIP(hipMemcpyAsync(dist + o, ddist, sizeof(double) * P, hipMemcpyDeviceToHost, c->stream));
        CCG_HIP(hipStreamSynchronize(c->stream));
        return (int)CCG_OK;
    });
}

extern "C" int ccg_group_consensus_knn_assign(ccg_group* g, const void* A, int label_bits, int64_t N, int64_t B,
                                              int k, int32_t* out_idx) {
    CCG_REQUIRE(g && A && out_idx, "ccg_group_consensus_knn_assign: NULL argument");
    CCG_REQUIRE(g->nlocal == g->nranks,
                "ccg_group_consensus_knn_assign: needs a single-process group (use the _dev form per rank)");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_group_consensus_knn_assign: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && B >= 1 && k >= 1, "ccg_group_consensus_knn_assign: bad sizes");
    std::vector<void*> dA;
    int rc = upload_broadcast(g, A, (size_t)(B * N) * (label_bits / 8), dA);
    if (rc) return rc;
    std::vector<int32_t*> dout(g->nlocal), dflag(g->nlocal);
    for (int l = 0; l < g->nlocal; ++l) {
        CCG_HIP(hipSetDevice(g->ctx[l]->device));
        dout[l] = (int32_t*)ccg_ws(g->ctx[l], WS_HOST_B, sizeof(int32_t) * N * k + 64);
        if (!dout[l]) return CCG_ENOMEM;
        dflag[l] = dout[l] + N * k;
    }
    rc = ccg_consensus_knn_sharded_dev(g, (const void* const*)dA.data(), label_bits, N, B, k, dout.data(),
                                       dflag.data());
    if (rc) return rc;
    ccg_ctx* c = g->ctx[0];
    int flag = 0;
    CCG_HIP(hipSetDevice(c->device));
    CCG_HIP(hipMemcpyAsync(&flag, dflag[0], sizeof(int), hipMemcpyDeviceToHost, c->stream));
    CCG_HIP(hipMemcpyAsync(out_idx, dout[0], sizeof(int32_t) * N * k, hipMemcpyDeviceToHost, c->stream));
    rc = ccg_group_synchronize(g);
    if (rc) return rc;
    if (flag) {
        ccg_set_error("ccg_group_consensus_knn_assign: data/distances cannot contain NAs (a pair was never co-sampled)");
        return CCG_ENAN;
    }
    return CCG_OK;
}

extern "C" int ccg_group_knn_boot(ccg_group* g, const double* pcs, int64_t N, int d, const int32_t* boot_idx,
                                  int64_t n, int nb, int kmax, int32_t* out_idx, double* out_dist,
                                  ccg_knn_stats* stats) {
    CCG_REQUIRE(g && pcs && boot_idx && out_idx, "ccg_group_knn_boot: NULL argument");
    CCG_REQUIRE(nb >= 0 && n >= 1 && kmax >= 1, "ccg_group_knn_boot: bad sizes");
    // bootstraps split in contiguous blocks over the local devices
    std::vector<ccg_knn_stats> st(g->nlocal, ccg_knn_stats{0, 0});
    int rc = for_each_local(g, [&](int l) {
        int64_t b0, b1;
        ccg_boot_shard(nb, g->nlocal, l, &b0, &b1);
        if (b1 == b0) return (int)CCG_OK;
        return ccg_knn_boot(g->ctx[l], pcs, N, d, boot_idx + b0 * n, n, (int)(b1 - b0), kmax,
                            out_idx + b0 * n * kmax, out_dist ? out_dist + b0 * n * kmax : nullptr, &st[l]);
    });
    if (rc) return rc;
    if (stats) {
        stats->queries = stats->fallback = 0;
        for (auto& s : st) {
            stats->queries += s.queries;
            stats->fallback += s.fallback;
        }
    }
    return CCG_OK;
}
