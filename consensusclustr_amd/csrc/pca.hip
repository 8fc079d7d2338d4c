// Normalisation + PCA of a cell subset: the producer of
// every (sub)cluster's PC matrix, R/consensusClust.R:287 (shifted_log_transform
// with pseudo_count 1 = log1p(counts / sf)), :339 / :369 / :790
// (prcomp_irlba(t(norm), npc, center = rowMeans2(norm), scale = rowSds(norm))).
//
// Device path (fp64 throughout):
//   1. gather the selected genes x cells, y = log1p(c / sf)     [cells x genes]
//   2. per-gene mean and sample sd (two passes), z = (y - mean) / sd
//   3. covariance C = Z^T Z / (n - 1)                             [genes x genes]
//   4. block subspace iteration on C with CholeskyQR2 re-orthonormalisation
//      and Rayleigh-Ritz every few steps, until every wanted Ritz pair has a
//      relative residual below 1e-11 (irlba stops at 1e-5; this is the exact
//      PCA up to rounding)
//   5. scores x = Z V, sdev = sqrt(eigenvalues of C)
// The small dense factorisations (p x p Cholesky and symmetric eigen, p <=
// npc + 16) run on the host in plain C; everything of size genes or cells
// runs on the GPU.  Signs: a component is oriented so that its
// largest-|loading| gene is positive (irlba's signs depend on its random
// start vector, so parity on the scores is up to sign per component).
#include <algorithm>
#include <cmath>
#include <vector>

#include "ccg_internal.h"

// ------------------------------------------------------------ DGEMM --
// C[m][n] = alpha * sum_k A(m, k) B(k, n) (+ beta C), A(m, k) = A[m*sam + k*sak],
// B(k, n) = B[k*sbk + n*sbn], C row-major with ldc.  64 x 64 tile per 256
// threads (4 x 4 outputs each), K staged through LDS in steps of 16.
#define PG_T 64
#define PG_K 16
__global__ __launch_bounds__(256) void pca_dgemm_kernel(int64_t M, int64_t N, int64_t K, const double* __restrict__ A,
                                                        int64_t sam, int64_t sak, const double* __restrict__ B,
                                                        int64_t sbk, int64_t sbn, double* __restrict__ C,
                                                        int64_t ldc, double alpha, double beta) {
    __shared__ double As[PG_K][PG_T + 1];
    __shared__ double Bs[PG_K][PG_T + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t m0 = (int64_t)blockIdx.y * PG_T, n0 = (int64_t)blockIdx.x * PG_T;
    double acc[4][4] = {};
    for (int64_t k0 = 0; k0 < K; k0 += PG_K) {
        // 1024 elements of each tile, 4 per thread; the fastest index follows
        // the operand's unit stride where it has one
        for (int e = threadIdx.x; e < PG_K * PG_T; e += 256) {
            int kk, mm;
            if (sam == 1) { mm = e % PG_T; kk = e / PG_T; } else { kk = e % PG_K; mm = e / PG_K; }
            const int64_t gm = m0 + mm, gk = k0 + kk;
            As[kk][mm] = (gm < M && gk < K) ? A[gm * sam + gk * sak] : 0.0;
            int kb, nn;
            if (sbn == 1) { nn = e % PG_T; kb = e / PG_T; } else { kb = e % PG_K; nn = e / PG_K; }
            const int64_t gn = n0 + nn, gkb = k0 + kb;
            Bs[kb][nn] = (gn < N && gkb < K) ? B[gkb * sbk + gn * sbn] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < PG_K; ++kk) {
            double a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t gm = m0 + ty + 16 * i, gn = n0 + tx + 16 * j;
            if (gm < M && gn < N) {
                double* c = C + gm * ldc + gn;
                *c = beta == 0.0 ? alpha * acc[i][j] : alpha * acc[i][j] + beta * *c;
            }
        }
}

static int pca_gemm(int64_t M, int64_t N, int64_t K, const double* A, int64_t sam, int64_t sak, const double* B,
                    int64_t sbk, int64_t sbn, double* C, int64_t ldc, double alpha, double beta, hipStream_t st) {
    const dim3 g((unsigned)ccg_cdiv(N, PG_T), (unsigned)ccg_cdiv(M, PG_T));
    pca_dgemm_kernel<<<g, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, alpha, beta);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------ normalisation --
// Z[i][g] = log1p(counts[genes[g] + cells[i] * G] / sf[cells[i]])
__global__ __launch_bounds__(256) void pca_gather_kernel(const double* __restrict__ counts, int64_t G,
                                                         const double* __restrict__ sf,
                                                         const int32_t* __restrict__ genes, int ng,
                                                         const int32_t* __restrict__ cells, int64_t nc,
                                                         double* __restrict__ Z) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nc * ng) return;
    const int64_t i = t / ng, g = t - i * ng;
    const int64_t c = cells[i];
    Z[t] = log1p(counts[(int64_t)genes[g] + c * G] / sf[c]);
}

// One block per gene: mean, then the sample sd of the deviations, then
// standardise in place.  sd == 0 flags the gene (prcomp_irlba cannot scale it).
__global__ __launch_bounds__(256) void pca_standardize_kernel(double* __restrict__ Z, int64_t nc, int ng,
                                                              int* __restrict__ zero_var) {
    __shared__ double red[256];
    const int g = blockIdx.x;
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < nc; i += 256) s += Z[i * ng + g];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double mu = red[0] / (double)nc;
    __syncthreads();
    double v = 0.0;
    for (int64_t i = threadIdx.x; i < nc; i += 256) {
        const double e = Z[i * ng + g] - mu;
        v += e * e;
    }
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double sd = sqrt(red[0] / (double)(nc - 1));
    if (!(sd > 0.0)) {
        if (threadIdx.x == 0) atomicOr(zero_var, 1);
        return;
    }
    const double inv = 1.0 / sd;
    for (int64_t i = threadIdx.x; i < nc; i += 256) Z[i * ng + g] = (Z[i * ng + g] - mu) * inv;
}

// deterministic start block: a hash of (row, column) in [-1, 1)
__global__ void pca_start_kernel(double* __restrict__ V, int64_t ng, int p) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ng * p) return;
    uint64_t x = (uint64_t)t * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    V[t] = (double)(x >> 11) * 0x1p-52 - 1.0;
}

// ------------------------------------------------- small host linear algebra
// Cholesky of a p x p SPD matrix (row-major, lower factor in place); false if
// not positive definite.
static bool host_cholesky(std::vector<double>& a, int p) {
    for (int j = 0; j < p; ++j) {
        double s = a[j * p + j];
        for (int k = 0; k < j; ++k) s -= a[j * p + k] * a[j * p + k];
        if (!(s > 0.0)) return false;
        const double d = std::sqrt(s);
        a[j * p + j] = d;
        for (int i = j + 1; i < p; ++i) {
            double t = a[i * p + j];
            for (int k = 0; k < j; ++k) t -= a[i * p + k] * a[j * p + k];
            a[i * p + j] = t / d;
        }
        for (int i = 0; i < j; ++i) a[i * p + j] = 0.0;
    }
    return true;
}

// inverse of the upper factor R = L^T (p x p row-major), returned row-major
static std::vector<double> host_inv_upper_from_lower(const std::vector<double>& L, int p) {
    std::vector<double> Ri(p * p, 0.0);  // R^{-1}, upper triangular
    for (int j = p - 1; j >= 0; --j) {
        Ri[j * p + j] = 1.0 / L[j * p + j];
        for (int i = j - 1; i >= 0; --i) {
            double s = 0.0;
            for (int k = i + 1; k <= j; ++k) s += L[k * p + i] * Ri[k * p + j];  // R[i][k] = L[k][i]
            Ri[i * p + j] = -s / L[i * p + i];
        }
    }
    return Ri;
}

// Cyclic Jacobi eigen-decomposition of a symmetric p x p matrix (row-major):
// eigenvalues in w, eigenvectors as the columns of Q.
static void host_jacobi(std::vector<double> a, int p, std::vector<double>& w, std::vector<double>& Q) {
    Q.assign(p * p, 0.0);
    for (int i = 0; i < p; ++i) Q[i * p + i] = 1.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int i = 0; i < p; ++i)
            for (int j = 0; j < p; ++j) {
                tot += a[i * p + j] * a[i * p + j];
                if (i != j) off += a[i * p + j] * a[i * p + j];
            }
        if (off <= 1e-30 * tot) break;
        for (int r = 0; r < p - 1; ++r)
            for (int c = r + 1; c < p; ++c) {
                const double arc = a[r * p + c];
                if (std::fabs(arc) < 1e-300) continue;
                const double theta = (a[c * p + c] - a[r * p + r]) / (2.0 * arc);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double cs = 1.0 / std::sqrt(t * t + 1.0), sn = t * cs;
                for (int k = 0; k < p; ++k) {  // columns r, c
                    const double akr = a[k * p + r], akc = a[k * p + c];
                    a[k * p + r] = cs * akr - sn * akc;
                    a[k * p + c] = sn * akr + cs * akc;
                }
                for (int k = 0; k < p; ++k) {  // rows r, c
                    const double ark = a[r * p + k], ack = a[c * p + k];
                    a[r * p + k] = cs * ark - sn * ack;
                    a[c * p + k] = sn * ark + cs * ack;
                }
                for (int k = 0; k < p; ++k) {
                    const double qkr = Q[k * p + r], qkc = Q[k * p + c];
                    Q[k * p + r] = cs * qkr - sn * qkc;
                    Q[k * p + c] = sn * qkr + cs * qkc;
                }
            }
    }
    w.resize(p);
    for (int i = 0; i < p; ++i) w[i] = a[i * p + i];
}

// ------------------------------------------------------------ driver --
#define PCA_TOL 1e-11        // converged: every wanted ||C v - theta v|| <= PCA_TOL * theta_1
#define PCA_TOL_LOOSE 1e-6   // accepted at the iteration cap (irlba's default tol is 1e-5)
#define PCA_MAX_ITERS 3000
#define PCA_RR_EVERY 8

extern "C" int ccg_pca_dev(ccg_ctx* ctx, const double* counts, int64_t G, int64_t N, const double* sf,
                           const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc, double* x,
                           double* sdev, void* stream) {
    CCG_REQUIRE(ctx && counts && sf && genes && cells && x && sdev, "ccg_pca_dev: NULL argument");
    CCG_REQUIRE(G >= 1 && N >= 1 && ng >= 2 && nc >= 3, "ccg_pca_dev: need >= 2 genes and >= 3 cells");
    CCG_REQUIRE(npc >= 1 && npc < ng && npc < nc, "ccg_pca_dev: need 1 <= npc < min(genes, cells)");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    const int p = std::min<int>(ng, npc + 16);  // block width (oversampled)
    const size_t nz = (size_t)nc * ng, ncv = (size_t)ng * ng, nv = (size_t)ng * p, np = (size_t)p * p;
    double* ws = (double*)ccg_ws(ctx, WS_PCA, sizeof(double) * (nz + ncv + 4 * nv + 2 * np) + 64);
    if (!ws) return CCG_ENOMEM;
    // Z: cells x genes; C: genes x genes; V: basis; W = C V; T1, T2: scratch
    double *Z = ws, *C = Z + nz, *V = C + ncv, *W = V + nv, *T1 = W + nv, *T2 = T1 + nv, *S = T2 + nv, *S2 = S + np;
    int* flag = (int*)(S2 + np);
    CCG_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
    pca_gather_kernel<<<(unsigned)ccg_cdiv((int64_t)nz, 256), 256, 0, st>>>(counts, G, sf, genes, ng, cells, nc, Z);
    pca_standardize_kernel<<<(unsigned)ng, 256, 0, st>>>(Z, nc, ng, flag);
    CCG_HIP(hipGetLastError());
    int zero_var = 0;
    CCG_HIP(hipMemcpyAsync(&zero_var, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (zero_var) {
        ccg_set_error("ccg_pca: a selected gene has zero variance among the cells (prcomp_irlba cannot scale it)");
        return CCG_ENAN;
    }
    // C = Z^T Z / (nc - 1): A(g, i) = Z[i ng + g], B(i, h) = Z[i ng + h]
    int rc = pca_gemm(ng, ng, nc, Z, 1, ng, Z, ng, 1, C, ng, 1.0 / (double)(nc - 1), 0.0, st);
    if (rc) return rc;
    std::vector<double> hS(np), w, Q;
    // one CholeskyQR step: S = src^T src = L L^T, dst = src L^{-T}
    auto cholqr = [&](const double* src, double* dst) -> int {
        int r2 = pca_gemm(p, p, ng, src, 1, p, src, p, 1, S, p, 1.0, 0.0, st);
        if (r2) return r2;
        CCG_HIP(hipMemcpyAsync(hS.data(), S, sizeof(double) * np, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        if (!host_cholesky(hS, p)) {
            ccg_set_error("ccg_pca: the iterated subspace lost rank (%d vectors, %d genes)", p, ng);
            return CCG_EINVAL;
        }
        const std::vector<double> Ri = host_inv_upper_from_lower(hS, p);
        CCG_HIP(hipMemcpyAsync(S2, Ri.data(), sizeof(double) * np, hipMemcpyHostToDevice, st));
        return pca_gemm(ng, p, p, src, p, 1, S2, p, 1, dst, p, 1.0, 0.0, st);
    };
    // CholeskyQR2 of src (!= T1) into dst
    auto orthonormalise = [&](const double* src, double* dst) -> int {
        int r2 = cholqr(src, T1);
        return r2 ? r2 : cholqr(T1, dst);
    };
    pca_start_kernel<<<(unsigned)ccg_cdiv((int64_t)nv, 256), 256, 0, st>>>(T2, ng, p);
    rc = orthonormalise(T2, V);
    if (rc) return rc;
    std::vector<double> hv(nv), hw(nv), res(npc);
    for (int it = 1;; ++it) {
        rc = pca_gemm(ng, p, ng, C, ng, 1, V, p, 1, W, p, 1.0, 0.0, st);  // W = C V
        if (rc) return rc;
        if (it % PCA_RR_EVERY != 0) {
            rc = orthonormalise(W, V);  // power step
            if (rc) return rc;
            continue;
        }
        // Rayleigh-Ritz on span(V): T = V^T C V = V^T W, eigenpairs sorted descending
        rc = pca_gemm(p, p, ng, V, 1, p, W, p, 1, S, p, 1.0, 0.0, st);
        if (rc) return rc;
        CCG_HIP(hipMemcpyAsync(hS.data(), S, sizeof(double) * np, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        for (int a = 0; a < p; ++a)
            for (int b = 0; b < a; ++b) hS[a * p + b] = hS[b * p + a] = 0.5 * (hS[a * p + b] + hS[b * p + a]);
        host_jacobi(hS, p, w, Q);
        std::vector<int> ord(p);
        for (int a = 0; a < p; ++a) ord[a] = a;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] > w[b]; });
        std::vector<double> Qs(np);
        for (int a = 0; a < p; ++a)
            for (int b = 0; b < p; ++b) Qs[a * p + b] = Q[a * p + ord[b]];
        CCG_HIP(hipMemcpyAsync(S2, Qs.data(), sizeof(double) * np, hipMemcpyHostToDevice, st));
        rc = pca_gemm(ng, p, p, V, p, 1, S2, p, 1, T1, p, 1.0, 0.0, st);  // Ritz vectors
        if (rc) return rc;
        rc = pca_gemm(ng, p, p, W, p, 1, S2, p, 1, T2, p, 1.0, 0.0, st);  // C times them
        if (rc) return rc;
        CCG_HIP(hipMemcpyAsync(hv.data(), T1, sizeof(double) * nv, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipMemcpyAsync(hw.data(), T2, sizeof(double) * nv, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        const double th0 = std::fabs(w[ord[0]]);
        double worst = 0.0;
        for (int j = 0; j < npc; ++j) {
            const double th = w[ord[j]];
            double r = 0.0;
            for (int g = 0; g < ng; ++g) {
                const double e = hw[(size_t)g * p + j] - th * hv[(size_t)g * p + j];
                r += e * e;
            }
            worst = std::max(worst, std::sqrt(r) / th0);
        }
        const bool cap = it >= PCA_MAX_ITERS;
        if (worst <= PCA_TOL || (cap && worst <= PCA_TOL_LOOSE)) {
            for (int j = 0; j < npc; ++j) sdev[j] = std::sqrt(std::max(w[ord[j]], 0.0));
            // orientation: the largest-|loading| gene of each component positive
            std::vector<double> sgn(np, 0.0);
            for (int j = 0; j < p; ++j) {
                int best = 0;
                for (int g = 1; g < ng; ++g)
                    if (std::fabs(hv[(size_t)g * p + j]) > std::fabs(hv[(size_t)best * p + j])) best = g;
                sgn[j * p + j] = hv[(size_t)best * p + j] < 0 ? -1.0 : 1.0;
            }
            CCG_HIP(hipMemcpyAsync(S2, sgn.data(), sizeof(double) * np, hipMemcpyHostToDevice, st));
            rc = pca_gemm(ng, p, p, T1, p, 1, S2, p, 1, T2, p, 1.0, 0.0, st);
            if (rc) return rc;
            // x (nc x npc column-major) = Z V_k, as x^T (npc x nc row-major) = V_k^T Z^T
            rc = pca_gemm(npc, nc, ng, T2, 1, p, Z, 1, ng, x, nc, 1.0, 0.0, st);
            if (rc) return rc;
            CCG_HIP(hipStreamSynchronize(st));
            return CCG_OK;
        }
        if (cap) {
            ccg_set_error("ccg_pca: subspace iteration did not converge in %d steps (residual %.3g)", PCA_MAX_ITERS,
                          worst);
            return CCG_EINVAL;
        }
        rc = orthonormalise(T2, V);  // power step on the rotated basis: V = orth(C V Q)
        if (rc) return rc;
    }
}

extern "C" int ccg_pca(ccg_ctx* ctx, const double* counts, int64_t G, int64_t N, const double* sf,
                       const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc, double* x,
                       double* sdev) {
    CCG_REQUIRE(ctx && counts && sf && genes && cells && x && sdev, "ccg_pca: NULL argument");
    CCG_REQUIRE(G >= 1 && N >= 1 && ng >= 2 && nc >= 3, "ccg_pca: need >= 2 genes and >= 3 cells");
    for (int g = 0; g < ng; ++g) CCG_REQUIRE(genes[g] >= 0 && genes[g] < G, "ccg_pca: gene index out of range");
    for (int64_t i = 0; i < nc; ++i) CCG_REQUIRE(cells[i] >= 0 && cells[i] < N, "ccg_pca: cell index out of range");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t cbytes = sizeof(double) * (size_t)(G * N);
    double* dC = (double*)ccg_ws(ctx, WS_HOST_A, cbytes);
    double* dsf = (double*)ccg_ws(ctx, WS_HOST_B, sizeof(double) * N + sizeof(int32_t) * (ng + nc) + 64);
    double* dx = (double*)ccg_ws(ctx, WS_HOST_C, sizeof(double) * (size_t)(nc * npc));
    if (!dC || !dsf || !dx) return CCG_ENOMEM;
    int32_t* dg = (int32_t*)(dsf + N);
    int32_t* dcell = dg + ng;
    CCG_HIP(hipMemcpyAsync(dC, counts, cbytes, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dsf, sf, sizeof(double) * N, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dg, genes, sizeof(int32_t) * ng, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dcell, cells, sizeof(int32_t) * nc, hipMemcpyHostToDevice, st));
    int rc = ccg_pca_dev(ctx, dC, G, N, dsf, dg, ng, dcell, nc, npc, dx, sdev, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(x, dx, sizeof(double) * (size_t)(nc * npc), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}
