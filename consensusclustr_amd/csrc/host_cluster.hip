// Host community detection for the Python drop-in (no device code).
//
// The reference clusters every bootstrap's SNN graphs with
// igraph::cluster_leiden on the host (R/consensusClust.R:656-658 through
// bluster, :430-433 directly), and the R drop-in keeps igraph.  python-igraph
// is not in this image, so the Python mirror needs a host clusterer of its
// own; cluster_host.py's pure-Python Louvain takes seconds per graph at
// cfg2's 18k rows.  This is the same algorithm (Louvain local moving with
// igraph's resolution-scaled modularity gain, then aggregation, at most 16
// levels of at most 32 sweeps) in C++, callable from host threads (ctypes
// releases the GIL, so the 60 clusterings of a bootstrap run in parallel).
// It is a stand-in, not igraph's Leiden: the labels differ from igraph's, as
// the Python version's do.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "ccg_internal.h"

namespace {

uint64_t lv_mix(uint64_t x) {  // splitmix64
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct LvGraph {  // symmetric CSR (both directions of every edge) + self weights
    int64_t n = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> nbr;
    std::vector<double> wt;
    std::vector<double> self;
};

// CSR of an undirected edge list (a != b); self weights given separately.
void lv_build(LvGraph& g, int64_t n, int64_t ne, const int32_t* a, const int32_t* b, const double* w) {
    g.n = n;
    g.ptr.assign(n + 1, 0);
    for (int64_t e = 0; e < ne; ++e) {
        g.ptr[a[e] + 1]++;
        g.ptr[b[e] + 1]++;
    }
    for (int64_t i = 0; i < n; ++i) g.ptr[i + 1] += g.ptr[i];
    g.nbr.resize(g.ptr[n]);
    g.wt.resize(g.ptr[n]);
    std::vector<int64_t> cur(g.ptr.begin(), g.ptr.end() - 1);
    for (int64_t e = 0; e < ne; ++e) {
        g.nbr[cur[a[e]]] = b[e];
        g.wt[cur[a[e]]++] = w[e];
        g.nbr[cur[b[e]]] = a[e];
        g.wt[cur[b[e]]++] = w[e];
    }
}

// One level of local moving; comm renumbered 0..nc-1 in order of first
// appearance.  Returns whether any node moved.
bool lv_level(const LvGraph& g, double gamma, uint64_t seed, std::vector<int32_t>& comm, int32_t& nc) {
    const int64_t n = g.n;
    std::vector<double> k(n), tot(n);
    double m2 = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double s = 2.0 * g.self[i];
        for (int64_t e = g.ptr[i]; e < g.ptr[i + 1]; ++e) s += g.wt[e];
        k[i] = s;
        m2 += s;
    }
    comm.resize(n);
    for (int64_t i = 0; i < n; ++i) comm[i] = (int32_t)i;
    nc = (int32_t)n;
    if (m2 <= 0.0) return false;
    tot = k;
    std::vector<int32_t> order(n);
    for (int64_t i = 0; i < n; ++i) order[i] = (int32_t)i;
    for (int64_t i = n - 1; i > 0; --i) {  // Fisher-Yates from the seed
        const int64_t j = (int64_t)(lv_mix(seed ^ (uint64_t)i) % (uint64_t)(i + 1));
        std::swap(order[i], order[j]);
    }
    std::vector<double> link(n, 0.0);
    std::vector<int32_t> touched;
    touched.reserve(64);
    bool moved = false;
    for (int sweep = 0; sweep < 32; ++sweep) {
        bool improved = false;
        for (int64_t oi = 0; oi < n; ++oi) {
            const int32_t i = order[oi];
            const int32_t ci = comm[i];
            touched.clear();
            for (int64_t e = g.ptr[i]; e < g.ptr[i + 1]; ++e) {
                const int32_t c = comm[g.nbr[e]];
                if (link[c] == 0.0) touched.push_back(c);
                link[c] += g.wt[e];
            }
            tot[ci] -= k[i];
            int32_t best = ci;
            double bg = link[ci] - gamma * k[i] * tot[ci] / m2;
            for (const int32_t c : touched) {
                const double gn = link[c] - gamma * k[i] * tot[c] / m2;
                if (gn > bg + 1e-12) {
                    bg = gn;
                    best = c;
                }
            }
            tot[best] += k[i];
            if (best != ci) {
                comm[i] = best;
                improved = moved = true;
            }
            for (const int32_t c : touched) link[c] = 0.0;
        }
        if (!improved) break;
    }
    std::vector<int32_t> ren(n, -1);
    nc = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (ren[comm[i]] < 0) ren[comm[i]] = nc++;
        comm[i] = ren[comm[i]];
    }
    return moved;
}

// The graph of the communities: intra-community weight to self, the rest
// summed per community pair.
void lv_aggregate(const LvGraph& g, const std::vector<int32_t>& comm, int32_t nc, LvGraph& out) {
    std::vector<double> self(nc, 0.0);
    std::vector<uint64_t> key;
    std::vector<double> kw;
    for (int64_t i = 0; i < g.n; ++i) {
        self[comm[i]] += g.self[i];
        for (int64_t e = g.ptr[i]; e < g.ptr[i + 1]; ++e) {
            const int32_t j = g.nbr[e];
            if (j <= i) continue;  // each undirected edge once
            const int32_t a = comm[i], b = comm[j];
            if (a == b) {
                self[a] += g.wt[e];
            } else {
                key.push_back((uint64_t)std::min(a, b) << 32 | (uint32_t)std::max(a, b));
                kw.push_back(g.wt[e]);
            }
        }
    }
    std::vector<int64_t> idx(key.size());
    for (size_t t = 0; t < idx.size(); ++t) idx[t] = (int64_t)t;
    std::sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return key[x] < key[y] || (key[x] == key[y] && x < y); });
    std::vector<int32_t> ea, eb;
    std::vector<double> ew;
    for (size_t t = 0; t < idx.size(); ++t) {
        const uint64_t kk = key[idx[t]];
        if (t > 0 && kk == key[idx[t - 1]]) {
            ew.back() += kw[idx[t]];
            continue;
        }
        ea.push_back((int32_t)(kk >> 32));
        eb.push_back((int32_t)(kk & 0xFFFFFFFFu));
        ew.push_back(kw[idx[t]]);
    }
    lv_build(out, nc, (int64_t)ea.size(), ea.data(), eb.data(), ew.data());
    out.self = std::move(self);
}

}  // namespace

extern "C" int ccg_host_louvain(int64_t n, int64_t ne, const int32_t* ei, const int32_t* ej, const double* w,
                                double resolution, uint64_t seed, int32_t* labels) {
    CCG_REQUIRE(n >= 1 && n < (1LL << 31) && ne >= 0 && labels, "ccg_host_louvain: bad sizes or NULL labels");
    CCG_REQUIRE(ne == 0 || (ei && ej && w), "ccg_host_louvain: NULL edge list");
    for (int64_t e = 0; e < ne; ++e)
        CCG_REQUIRE(ei[e] >= 0 && ei[e] < n && ej[e] >= 0 && ej[e] < n && ei[e] != ej[e] && w[e] >= 0.0,
                    "ccg_host_louvain: edge %lld out of range, a self loop or a negative weight", (long long)e);
    LvGraph g;
    lv_build(g, n, ne, ei, ej, w);
    g.self.assign(n, 0.0);
    std::vector<int32_t> member(n);
    for (int64_t i = 0; i < n; ++i) member[i] = (int32_t)i;
    std::vector<int32_t> comm;
    for (int level = 0; level < 16; ++level) {
        int32_t nc = 0;
        const bool moved = lv_level(g, resolution, lv_mix(seed + 0x1000003ull * (uint64_t)level), comm, nc);
        for (int64_t i = 0; i < n; ++i) member[i] = comm[member[i]];
        if (!moved) break;
        LvGraph next;
        lv_aggregate(g, comm, nc, next);
        g = std::move(next);
    }
    // labels 1..C in order of first appearance over the nodes
    std::vector<int32_t> ren(n, 0);
    int32_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!ren[member[i]]) ren[member[i]] = ++c;
        labels[i] = ren[member[i]];
    }
    return CCG_OK;
}
