// Normalisation + PCA of a cell subset: the producer of
// every (sub)cluster's PC matrix, R/consensusClust.R:287 (shifted_log_transform
// with pseudo_count 1 = log1p(counts / sf)), :339 / :369 / :790
// (prcomp_irlba(t(norm), npc, center = rowMeans2(norm), scale = rowSds(norm))).
//
// Device path (fp64 throughout):
//   1. gather the selected genes x cells, y = log1p(c / sf)     [cells x genes]
//   2. per-gene mean and sample sd (two passes), z = (y - mean) / sd
//   3. covariance C = Z^T Z / (n - 1)                             [genes x genes]
//   4. Chebyshev-filtered block subspace iteration on C (degree 24 between
//      Rayleigh-Ritz steps, CholeskyQR every step), until every wanted Ritz
//      pair has a relative residual below 1e-11 (irlba stops at 1e-5; this is
//      the exact PCA up to rounding)
//   5. scores x = Z V, sdev = sqrt(eigenvalues of C)
// The small dense factorisations (p <= npc + 16): the Cholesky and
// triangular inverse of every CholeskyQR step in one device block (no host
// round trip per filter step; the host C code for p > 90), the Rayleigh-Ritz
// eigenproblem every 24 matvecs on the host in plain C; everything of size
// genes or cells runs on the GPU.  Signs: a component is oriented so that its
// largest-|loading| gene is positive (irlba's signs depend on its random
// start vector, so parity on the scores is up to sign per component).
#include <algorithm>
#include <cmath>
#include <vector>

#include "ccg_internal.h"

// ------------------------------------------------------------ DGEMM --
// C[m][n] = alpha * sum_k A(m, k) B(k, n) (+ beta C), A(m, k) = A[m*sam + k*sak],
// B(k, n) = B[k*sbk + n*sbn], C row-major with ldc, on the fp64 matrix core
// (v_mfma_f64_16x16x4f64).  A 64 x 64 tile per 256 threads: each wave owns a
// 32 x 32 quarter (2 x 2 MFMA tiles); K is staged through LDS 16 at a time,
// the next stage's panels in registers while the current one is consumed.
// Lane (g, j) = (lane >> 4, lane & 15) feeds A[m = j][k = g] and
// B[k = g][n = j] of a 16 x 16 x 4 step, and holds D[m = g + 4 i][n = j] in
// accumulator i.  sym: C is symmetric (A(m, k) = B(k, m)): only the tiles on
// or above the diagonal are computed, pca_mirror_kernel copies the rest.
#define PM_T 64
#define PM_K 16
#define PM_LD (PM_T + 2)  // LDS row pad: the 16 lanes of a fragment read hit distinct banks
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pca_mfma_gemm_kernel(int64_t M, int64_t N, int64_t K,
                                                            const double* __restrict__ A, int64_t sam, int64_t sak,
                                                            const double* __restrict__ B, int64_t sbk, int64_t sbn,
                                                            double* __restrict__ C, int64_t ldc, double alpha,
                                                            double beta, int sym, int64_t kchunk, int64_t cz) {
    __shared__ double As[PM_K][PM_LD];
    __shared__ double Bs[PM_K][PM_LD];
    const int64_t m0 = (int64_t)blockIdx.y * PM_T, n0 = (int64_t)blockIdx.x * PM_T;
    // split K: slice z sums k in [z kchunk, (z + 1) kchunk) into C + z cz
    const int64_t kb = (int64_t)blockIdx.z * kchunk;
    K = min(K, kb + kchunk);
    C += (int64_t)blockIdx.z * cz;
    if (sym && n0 + PM_T <= m0) return;  // strictly below the diagonal
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    // panel element e of a stage: (k, m) with the fastest index along the
    // operand's unit stride where it has one (coalesced loads)
    auto a_idx = [&](int e, int& kk, int& mm) {
        if (sam == 1) { mm = e & (PM_T - 1); kk = e >> 6; } else { kk = e & (PM_K - 1); mm = e >> 4; }
    };
    auto b_idx = [&](int e, int& kk, int& nn) {
        if (sbn == 1) { nn = e & (PM_T - 1); kk = e >> 6; } else { kk = e & (PM_K - 1); nn = e >> 4; }
    };
    double pa[4], pb[4];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = r * 256 + tid;
            int kk, mm, kb, nn;
            a_idx(e, kk, mm);
            b_idx(e, kb, nn);
            const int64_t gm = m0 + mm, gk = k0 + kk, gn = n0 + nn, gkb = k0 + kb;
            pa[r] = (gm < M && gk < K) ? A[gm * sam + gk * sak] : 0.0;
            pb[r] = (gn < N && gkb < K) ? B[gkb * sbk + gn * sbn] : 0.0;
        }
    };
    f64x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (f64x4){0.0, 0.0, 0.0, 0.0};
    load(kb);
    for (int64_t k0 = kb; k0 < K; k0 += PM_K) {
        __syncthreads();  // the previous stage's reads are done
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = r * 256 + tid;
            int kk, mm, kb, nn;
            a_idx(e, kk, mm);
            b_idx(e, kb, nn);
            As[kk][mm] = pa[r];
            Bs[kb][nn] = pb[r];
        }
        __syncthreads();
        if (k0 + PM_K < K) load(k0 + PM_K);  // in flight during the MFMAs
#pragma unroll
        for (int ks = 0; ks < PM_K / 4; ++ks) {
            const int kk = ks * 4 + g;
            const double a0 = As[kk][wm + j], a1 = As[kk][wm + 16 + j];
            const double b0 = Bs[kk][wn + j], b1 = Bs[kk][wn + 16 + j];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
        }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t gm = m0 + wm + mt * 16 + g + 4 * i, gn = n0 + wn + nt * 16 + j;
                if (gm < M && gn < N && (!sym || gn >= gm)) {
                    double* c = C + gm * ldc + gn;
                    *c = beta == 0.0 ? alpha * acc[mt][nt][i] : alpha * acc[mt][nt][i] + beta * *c;
                }
            }
}

// lower triangle of a symmetric n x n matrix from its upper triangle
__global__ void pca_mirror_kernel(double* __restrict__ C, int64_t n, int64_t ldc) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * n) return;
    const int64_t r = t / n, c = t - r * n;
    if (c < r) C[r * ldc + c] = C[c * ldc + r];
}

static int pca_gemm(int64_t M, int64_t N, int64_t K, const double* A, int64_t sam, int64_t sak, const double* B,
                    int64_t sbk, int64_t sbn, double* C, int64_t ldc, double alpha, double beta, hipStream_t st,
                    bool sym = false) {
    const dim3 g((unsigned)ccg_cdiv(N, PM_T), (unsigned)ccg_cdiv(M, PM_T));
    pca_mfma_gemm_kernel<<<g, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, alpha, beta, sym ? 1 : 0, K,
                                            0);
    if (sym) pca_mirror_kernel<<<(unsigned)ccg_cdiv(M * M, 256), 256, 0, st>>>(C, M, ldc);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// The same product as `slices` partial sums over contiguous K ranges, slice z
// into C + z * M * ldc (alpha 1, beta 0): enough workgroups for the thin
// products of the subspace iteration (N = p columns); the consumer adds the
// slices in a fixed order (deterministic).  sym: upper triangle only, no mirror.
static int pca_gemm_split(int64_t M, int64_t N, int64_t K, const double* A, int64_t sam, int64_t sak,
                          const double* B, int64_t sbk, int64_t sbn, double* C, int64_t ldc, int slices,
                          hipStream_t st, bool sym = false) {
    const int64_t kc = ccg_cdiv(ccg_cdiv(K, slices), PM_K) * PM_K;
    const dim3 g((unsigned)ccg_cdiv(N, PM_T), (unsigned)ccg_cdiv(M, PM_T), (unsigned)ccg_cdiv(K, kc));
    pca_mfma_gemm_kernel<<<g, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, 1.0, 0.0, sym ? 1 : 0, kc,
                                            M * ldc);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------ normalisation --
// Z[i][g] = log1p(counts[genes[g] + cells[i] * G] / sf[cells[i]])  (dense G x N)
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

// Sparse counts (dgCMatrix: column c's nonzeros are x[p[c] .. p[c+1]) at
// gene rows ri[]): Z starts at log1p(0) = 0 and one wave per selected cell
// scatters its nonzeros of selected genes (gpos[gene] = position or -1).
__global__ __launch_bounds__(256) void pca_gather_csc_kernel(const double* __restrict__ xv,
                                                             const int32_t* __restrict__ ri,
                                                             const int64_t* __restrict__ cp,
                                                             const double* __restrict__ sf,
                                                             const int32_t* __restrict__ gpos,
                                                             const int32_t* __restrict__ cells, int64_t nc, int ng,
                                                             double* __restrict__ Z) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= nc) return;
    const int lane = threadIdx.x & 63;
    const int64_t c = cells[i];
    const double s = sf[c];
    for (int64_t e = cp[c] + lane; e < cp[c + 1]; e += 64) {
        const int pos = gpos[ri[e]];
        if (pos >= 0) Z[i * ng + pos] = log1p(xv[e] / s);
    }
}

__global__ void pca_fill_kernel(double* __restrict__ Z, int64_t n, double v) {
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) Z[t] = v;
}

// Per-gene column statistics with lanes along the genes (coalesced rows of
// Z): block (gx, cy) sums genes [256 gx, +256) over the cells of slice cy;
// pca_colstat_finish adds the slices in a fixed order (deterministic).
// pass 0: partial sums of z; pass 1: partial sums of (z - mean)^2.
#define PCA_SLICES 64
__global__ __launch_bounds__(256) void pca_colstat_kernel(const double* __restrict__ Z, int64_t nc, int ng,
                                                          const double* __restrict__ mean, int pass,
                                                          double* __restrict__ part) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= ng) return;
    const int64_t per = ccg_cdiv(nc, PCA_SLICES);
    const int64_t i0 = (int64_t)blockIdx.y * per, i1 = min(nc, i0 + per);
    const double mu = pass ? mean[g] : 0.0;
    double s0 = 0.0, s1 = 0.0;  // two chains: more loads in flight
    int64_t i = i0;
    for (; i + 1 < i1; i += 2) {
        const double a = Z[i * ng + g] - mu, b = Z[(i + 1) * ng + g] - mu;
        s0 += pass ? a * a : a;
        s1 += pass ? b * b : b;
    }
    if (i < i1) {
        const double a = Z[i * ng + g] - mu;
        s0 += pass ? a * a : a;
    }
    part[(int64_t)blockIdx.y * ng + g] = s0 + s1;
}

// pass 0: mean[g] = sum / nc; pass 1: inv_sd[g] = 1 / sample sd (flag 0 sd)
__global__ void pca_colstat_finish(const double* __restrict__ part, int64_t nc, int ng, int pass,
                                   double* __restrict__ mean, double* __restrict__ inv_sd,
                                   int* __restrict__ zero_var) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= ng) return;
    double s = 0.0;
    for (int y = 0; y < PCA_SLICES; ++y) s += part[(int64_t)y * ng + g];
    if (pass == 0) {
        mean[g] = s / (double)nc;
    } else {
        const double sd = sqrt(s / (double)(nc - 1));
        if (!(sd > 0.0)) {
            atomicOr(zero_var, 1);
            inv_sd[g] = 0.0;
        } else {
            inv_sd[g] = 1.0 / sd;
        }
    }
}

__global__ void pca_scale_kernel(double* __restrict__ Z, int64_t nc, int ng, const double* __restrict__ mean,
                                 const double* __restrict__ inv_sd) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nc * ng) return;
    const int g = (int)(t % ng);
    Z[t] = (Z[t] - mean[g]) * inv_sd[g];
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

// The same factorisation on the device, one 256-thread block with the Gram
// matrix in LDS (p <= PCA_DEV_CHOL), so a CholeskyQR step needs no host round
// trip: S = sum of the `nsl` split-K partials (upper triangles, fixed order)
// -> Ri = (L^T)^{-1} (row-major, upper), S = L L^T.  Symmetric Gaussian
// elimination on [S | I] with one barrier per column: step j reads row j of
// the upper triangle (l_ij = S_ji / S_jj by symmetry) and writes only the
// trailing upper block and rows > j of the right part, which ends as
// L_u^{-1} (S = L_u D L_u^T, unit lower L_u); then L^{-1} = D^{-1/2} L_u^{-1}
// and Ri = (L^{-1})^T.  A non-positive pivot sets *flag (the subspace lost
// rank; the host reports it at its next check).
#define PCA_SPLIT_MV 8       // split-K slices of the C Y matvec (ng x p output)
#define PCA_SPLIT_GRAM 16    // split-K slices of the p x p Gram matrices
#define PCA_DEV_CHOL 90      // 2 p^2 doubles of static LDS (127 KB at p = 90; gfx950 has 160 KB)
__global__ __launch_bounds__(256) void pca_chol_kernel(const double* __restrict__ Sp, int nsl, int p,
                                                       double* __restrict__ Ri, int* __restrict__ flag) {
    __shared__ double La[PCA_DEV_CHOL * PCA_DEV_CHOL];  // [p][p], upper triangle
    __shared__ double Ms[PCA_DEV_CHOL * PCA_DEV_CHOL];  // [p][p], unit lower: L_u^{-1}
    __shared__ double dinv[PCA_DEV_CHOL];
    const int tid = threadIdx.x, pp = p * p;
    const int ty = tid >> 4, tx = tid & 15;
    for (int i = ty; i < p; i += 16)
        for (int k = tx; k < p; k += 16) {
            if (k >= i) {  // the slices' loads all in flight
                double v[PCA_SPLIT_GRAM];
#pragma unroll
                for (int z = 0; z < PCA_SPLIT_GRAM; ++z) v[z] = z < nsl ? Sp[(size_t)z * pp + i * p + k] : 0.0;
                double s = 0.0;
#pragma unroll
                for (int z = 0; z < PCA_SPLIT_GRAM; ++z) s += v[z];
                La[i * p + k] = s;
            }
            Ms[i * p + k] = i == k ? 1.0 : 0.0;
        }
    __syncthreads();
    for (int j = 0; j + 1 < p; ++j) {
        const double piv = La[j * p + j];
        const double rp = piv > 0.0 ? 1.0 / piv : 0.0;  // lost pivot: flagged below
        const double* Lj = La + j * p;
        const double* Mj = Ms + j * p;
        for (int i = j + 1 + ty; i < p; i += 16) {
            const double li = Lj[i] * rp;  // S_ij / S_jj
            double* Li = La + i * p;
            for (int k = i + tx; k < p; k += 16) Li[k] -= li * Lj[k];
            double* Mi = Ms + i * p;
            for (int c = tx; c <= j; c += 16) Mi[c] -= li * Mj[c];
        }
        __syncthreads();
    }
    if (tid < p) {
        const double d = La[tid * p + tid];
        if (!(d > 0.0)) atomicOr(flag, 1);
        dinv[tid] = d > 0.0 ? 1.0 / sqrt(d) : 1.0;
    }
    __syncthreads();
    for (int t = tid; t < pp; t += 256) {  // Ri[r][j] = L^{-1}[j][r] = Ms[j][r] / sqrt(d_j)
        const int r = t / p, j = t - r * p;
        Ri[t] = r <= j ? Ms[j * p + r] * dinv[j] : 0.0;
    }
}

// One Chebyshev recurrence step of the filtered subspace iteration, fused
// with the split-K reduction of the matvec: top = s1 (sum_z Wp[z]) - s2 A -
// s3 B, bot = A (the pair moves down).  A / B / bot may be NULL.
__global__ void pca_cheb_kernel(const double* __restrict__ Wp, int nsl, int64_t nv, const double* __restrict__ A,
                                const double* __restrict__ B, double s1, double s2, double s3,
                                double* __restrict__ top, double* __restrict__ bot) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nv) return;
    double w = 0.0;
    for (int z = 0; z < nsl; ++z) w += Wp[(int64_t)z * nv + t];
    const double a = A ? A[t] : 0.0;
    double r = s1 * w - s2 * a;
    if (B) r -= s3 * B[t];
    top[t] = r;
    if (bot) bot[t] = a;
}

// Symmetric eigen-decomposition of a p x p matrix (row-major) by Householder
// reduction to tridiagonal form with the transformations accumulated, then
// implicit QL with Wilkinson-type shifts on the tridiagonal (O(p^3), ~10x
// fewer flops than cyclic Jacobi at p = 64): eigenvalues in w, eigenvectors as
// the columns of Q (Q[k p + i] = component k of vector i).
static void host_symeig(const std::vector<double>& a, int p, std::vector<double>& w, std::vector<double>& Q) {
    const int n = p;
    Q = a;
    w.assign(n, 0.0);
    std::vector<double> e(n, 0.0);
    double* V = Q.data();
    double* d = w.data();
    auto at = [&](int r, int c) -> double& { return V[(size_t)r * n + c]; };
    for (int j = 0; j < n; ++j) d[j] = at(n - 1, j);
    for (int i = n - 1; i > 0; --i) {  // Householder step on row i
        double scale = 0.0, h = 0.0;
        for (int k = 0; k < i; ++k) scale += std::fabs(d[k]);
        if (scale == 0.0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; ++j) {
                d[j] = at(i - 1, j);
                at(i, j) = 0.0;
                at(j, i) = 0.0;
            }
        } else {
            for (int k = 0; k < i; ++k) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1], g = std::sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h -= f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; ++j) e[j] = 0.0;
            for (int j = 0; j < i; ++j) {
                f = d[j];
                at(j, i) = f;
                g = e[j] + at(j, j) * f;
                for (int k = j + 1; k <= i - 1; ++k) {
                    g += at(k, j) * d[k];
                    e[k] += at(k, j) * f;
                }
                e[j] = g;
            }
            f = 0.0;
            for (int j = 0; j < i; ++j) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            const double hh = f / (h + h);
            for (int j = 0; j < i; ++j) e[j] -= hh * d[j];
            for (int j = 0; j < i; ++j) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; ++k) at(k, j) -= (f * e[k] + g * d[k]);
                d[j] = at(i - 1, j);
                at(i, j) = 0.0;
            }
        }
        d[i] = h;
    }
    for (int i = 0; i < n - 1; ++i) {  // accumulate the transformations
        at(n - 1, i) = at(i, i);
        at(i, i) = 1.0;
        const double h = d[i + 1];
        if (h != 0.0) {
            for (int k = 0; k <= i; ++k) d[k] = at(k, i + 1) / h;
            for (int j = 0; j <= i; ++j) {
                double g = 0.0;
                for (int k = 0; k <= i; ++k) g += at(k, i + 1) * at(k, j);
                for (int k = 0; k <= i; ++k) at(k, j) -= g * d[k];
            }
        }
        for (int k = 0; k <= i; ++k) at(k, i + 1) = 0.0;
    }
    for (int j = 0; j < n; ++j) {
        d[j] = at(n - 1, j);
        at(n - 1, j) = 0.0;
    }
    at(n - 1, n - 1) = 1.0;
    e[0] = 0.0;
    // the QL rotations combine columns i, i + 1 of V: work on V^T (rows contiguous)
    std::vector<double> T((size_t)n * n);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) T[(size_t)c * n + r] = V[(size_t)r * n + c];
    // implicit QL on the tridiagonal (d, e), rotations applied to the columns of V
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    double f = 0.0, tst1 = 0.0;
    const double eps = 0x1p-52;
    for (int l = 0; l < n; ++l) {
        tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
        int m = l;
        while (m < n - 1 && std::fabs(e[m]) > eps * tst1) ++m;
        if (m > l) {
            for (int iter = 0; iter < 64; ++iter) {
                double g = d[l];
                double pp = (d[l + 1] - g) / (2.0 * e[l]);
                double r = std::hypot(pp, 1.0);
                if (pp < 0) r = -r;
                d[l] = e[l] / (pp + r);
                d[l + 1] = e[l] * (pp + r);
                const double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; ++i) d[i] -= h;
                f += h;
                pp = d[m];
                double c = 1.0, c2 = c, c3 = c, s = 0.0, s2 = 0.0;
                const double el1 = e[l + 1];
                for (int i = m - 1; i >= l; --i) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * pp;
                    r = std::hypot(pp, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = pp / r;
                    pp = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    double* ti = T.data() + (size_t)i * n;
                    double* tj = ti + n;
                    for (int k = 0; k < n; ++k) {
                        const double hk = tj[k], gk = ti[k];
                        tj[k] = s * gk + c * hk;
                        ti[k] = c * gk - s * hk;
                    }
                }
                pp = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * pp;
                d[l] = c * pp;
                if (!(std::fabs(e[l]) > eps * tst1)) break;
            }
        }
        d[l] += f;
        e[l] = 0.0;
    }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) V[(size_t)r * n + c] = T[(size_t)c * n + r];
}

// ------------------------------------------------------------ driver --
#define PCA_TOL 1e-11        // converged: every wanted ||C v - theta v|| <= PCA_TOL * theta_1
#define PCA_TOL_LOOSE 1e-6   // accepted at the iteration cap (irlba's default tol is 1e-5)
#define PCA_CHEB_DEG 24      // matvecs per filter (between Rayleigh-Ritz steps)
#define PCA_MAX_OUTER 250    // Rayleigh-Ritz steps (x PCA_CHEB_DEG matvecs)

// block width: npc + 16 (oversampled), trimmed to a multiple of the 64-column
// GEMM tile when that keeps >= 12 extra vectors (a 66-wide block pays for two
// column tiles)
static int pca_block_width(int ng, int npc) {
    int p = npc + 16;
    if (p > 64 && p % 64 <= 4) p -= p % 64;
    return std::min(ng, p);
}

static int pca_nslices(int64_t K, int slices) {
    const int64_t kc = ccg_cdiv(ccg_cdiv(K, slices), PM_K) * PM_K;
    return (int)ccg_cdiv(K, kc);
}

// Workspace of one PCA: Z (cells x genes), C (genes x genes), V / W / T1 / T2
// (genes x p), the filter's stacked pairs P / Q (2 genes x p), the matvec's
// split-K slices Wp, S / S2 (p x p), the Gram slices Sp, then the per-gene
// statistics and the flags.
struct PcaWs {
    double *Z, *C, *V, *W, *T1, *T2, *P, *Q, *Wp, *S, *S2, *Sp, *mean, *inv_sd, *part;
    int* flag;
};
static int pca_workspace(ccg_ctx* ctx, int64_t nc, int ng, int p, PcaWs* w) {
    const size_t nz = (size_t)nc * ng, ncv = (size_t)ng * ng, nv = (size_t)ng * p, np = (size_t)p * p;
    const size_t nd = nz + ncv + (8 + PCA_SPLIT_MV) * nv + (2 + PCA_SPLIT_GRAM) * np + (size_t)(PCA_SLICES + 2) * ng;
    double* ws = (double*)ccg_ws(ctx, WS_PCA, sizeof(double) * nd + 64);
    if (!ws) return CCG_ENOMEM;
    w->Z = ws;
    w->C = w->Z + nz;
    w->V = w->C + ncv;
    w->W = w->V + nv;
    w->T1 = w->W + nv;
    w->T2 = w->T1 + nv;
    w->P = w->T2 + nv;
    w->Q = w->P + 2 * nv;
    w->Wp = w->Q + 2 * nv;
    w->S = w->Wp + PCA_SPLIT_MV * nv;
    w->S2 = w->S + np;
    w->Sp = w->S2 + np;
    w->mean = w->Sp + PCA_SPLIT_GRAM * np;
    w->inv_sd = w->mean + ng;
    w->part = w->inv_sd + ng;
    w->flag = (int*)(w->part + (size_t)PCA_SLICES * ng);
    return CCG_OK;
}

// Steps 2-5 on the gathered Z (cells x genes of y = log1p(c / sf)).
//
// Step 4 is a Chebyshev-filtered subspace iteration: after each Rayleigh-Ritz
// step (Ritz values theta, descending), the block is multiplied by the degree-
// PCA_CHEB_DEG Chebyshev polynomial of C mapped so that [0, a] -> [-1, 1],
// a = theta_{p-1} (C is PSD, so 0 bounds the spectrum below): every unwanted
// direction stays bounded by 1 while a wanted eigenvalue lambda grows like
// cosh(deg acosh(2 lambda / a - 1)).  On a flat spectrum (lambda_50 /
// lambda_66 = 1.007 on the production shape's synthetic counts) that is
// ~0.16 per matvec in the log of the error against ~0.007 for the plain power
// step: ~220 matvecs instead of > 3000.  The three-term recurrence
// Y_{k+1} = (2 / e)(C - c) Y_k - Y_{k-1} is re-orthonormalised every step:
// CholeskyQR of Y_{k+1} with the same R^{-1} applied to Y_k (linear, so the
// span is the filtered one) -- the block's condition number never exceeds one
// step's growth (~4 theta_1 / a).
static int pca_from_z(ccg_ctx* ctx, const PcaWs& ws, int64_t nc, int ng, int npc, double* x, double* sdev,
                      hipStream_t st) {
    const int p = pca_block_width(ng, npc);
    const size_t nv = (size_t)ng * p, np = (size_t)p * p;
    double *Z = ws.Z, *C = ws.C, *V = ws.V, *W = ws.W, *T1 = ws.T1, *T2 = ws.T2, *S2 = ws.S2;
    double *P = ws.P, *Q = ws.Q, *Wp = ws.Wp, *Sp = ws.Sp;
    int* flag = ws.flag;
    // per-gene mean and sample sd (two passes, deterministic slice order), standardise
    CCG_HIP(hipMemsetAsync(flag, 0, 2 * sizeof(int), st));  // [0] zero variance, [1] lost rank (device Cholesky)
    const dim3 gs((unsigned)ccg_cdiv(ng, 256), PCA_SLICES);
    const unsigned gf = (unsigned)ccg_cdiv(ng, 256);
    pca_colstat_kernel<<<gs, 256, 0, st>>>(Z, nc, ng, ws.mean, 0, ws.part);
    pca_colstat_finish<<<gf, 256, 0, st>>>(ws.part, nc, ng, 0, ws.mean, ws.inv_sd, flag);
    pca_colstat_kernel<<<gs, 256, 0, st>>>(Z, nc, ng, ws.mean, 1, ws.part);
    pca_colstat_finish<<<gf, 256, 0, st>>>(ws.part, nc, ng, 1, ws.mean, ws.inv_sd, flag);
    pca_scale_kernel<<<(unsigned)ccg_cdiv(nc * (int64_t)ng, 256), 256, 0, st>>>(Z, nc, ng, ws.mean, ws.inv_sd);
    CCG_HIP(hipGetLastError());
    int zero_var = 0;
    CCG_HIP(hipMemcpyAsync(&zero_var, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (zero_var) {
        ccg_set_error("ccg_pca: a selected gene has zero variance among the cells (prcomp_irlba cannot scale it)");
        return CCG_ENAN;
    }
    // C = Z^T Z / (nc - 1): A(g, i) = Z[i ng + g], B(i, h) = Z[i ng + h]; symmetric
    int rc = pca_gemm(ng, ng, nc, Z, 1, ng, Z, ng, 1, C, ng, 1.0 / (double)(nc - 1), 0.0, st, true);
    if (rc) return rc;
    std::vector<double> hS(np), hSp, w, Q_;
    const bool dev_chol = p <= PCA_DEV_CHOL;
    const int nsl_g = pca_nslices(ng, PCA_SPLIT_GRAM), nsl_mv = pca_nslices(ng, PCA_SPLIT_MV);
    const unsigned gv = (unsigned)ccg_cdiv((int64_t)nv, 256);
    // one CholeskyQR step over `rows` rows of src (the Gram matrix of its first
    // ng rows): S = src^T src = L L^T, dst = src L^{-T}
    auto cqr = [&](const double* src, int64_t rows, double* dst) -> int {
        int r2 = pca_gemm_split(p, p, ng, src, 1, p, src, p, 1, Sp, p, PCA_SPLIT_GRAM, st, true);
        if (r2) return r2;
        if (dev_chol) {
            pca_chol_kernel<<<1, 256, 0, st>>>(Sp, nsl_g, p, S2, flag + 1);
            CCG_HIP(hipGetLastError());
        } else {
            hSp.resize((size_t)nsl_g * np);
            CCG_HIP(hipMemcpyAsync(hSp.data(), Sp, sizeof(double) * hSp.size(), hipMemcpyDeviceToHost, st));
            CCG_HIP(hipStreamSynchronize(st));
            for (int i = 0; i < p; ++i)
                for (int k = i; k < p; ++k) {
                    double v = 0.0;
                    for (int z = 0; z < nsl_g; ++z) v += hSp[(size_t)z * np + i * p + k];
                    hS[i * p + k] = hS[k * p + i] = v;
                }
            if (!host_cholesky(hS, p)) {
                ccg_set_error("ccg_pca: the iterated subspace lost rank (%d vectors, %d genes)", p, ng);
                return CCG_EINVAL;
            }
            const std::vector<double> Ri = host_inv_upper_from_lower(hS, p);
            CCG_HIP(hipMemcpyAsync(S2, Ri.data(), sizeof(double) * np, hipMemcpyHostToDevice, st));
            CCG_HIP(hipStreamSynchronize(st));  // Ri is a stack temporary
        }
        return pca_gemm(rows, p, p, src, p, 1, S2, p, 1, dst, p, 1.0, 0.0, st);
    };
    auto matvec = [&](const double* src) -> int {  // Wp slices of C src
        return pca_gemm_split(ng, p, ng, C, ng, 1, src, p, 1, Wp, p, PCA_SPLIT_MV, st);
    };
    pca_start_kernel<<<gv, 256, 0, st>>>(T2, ng, p);
    rc = cqr(T2, ng, T1);
    if (!rc) rc = cqr(T1, ng, V);  // CholeskyQR2
    if (rc) return rc;
    std::vector<double> hv(nv), hw(nv), res(npc);
    for (int it = 1;; ++it) {
        rc = matvec(V);  // W = C V
        if (rc) return rc;
        pca_cheb_kernel<<<gv, 256, 0, st>>>(Wp, nsl_mv, (int64_t)nv, nullptr, nullptr, 1.0, 0.0, 0.0, W, nullptr);
        // Rayleigh-Ritz on span(V): T = V^T C V = V^T W, eigenpairs sorted descending
        rc = pca_gemm_split(p, p, ng, V, 1, p, W, p, 1, Sp, p, PCA_SPLIT_GRAM, st);
        if (rc) return rc;
        hSp.resize((size_t)nsl_g * np);
        CCG_HIP(hipMemcpyAsync(hSp.data(), Sp, sizeof(double) * hSp.size(), hipMemcpyDeviceToHost, st));
        int lost = 0;
        if (dev_chol) CCG_HIP(hipMemcpyAsync(&lost, flag + 1, sizeof(int), hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        if (lost) {
            ccg_set_error("ccg_pca: the iterated subspace lost rank (%d vectors, %d genes)", p, ng);
            return CCG_EINVAL;
        }
        for (size_t t = 0; t < np; ++t) {  // the slices in a fixed order
            double v = 0.0;
            for (int z = 0; z < nsl_g; ++z) v += hSp[(size_t)z * np + t];
            hS[t] = v;
        }
        for (int a = 0; a < p; ++a)
            for (int b = 0; b < a; ++b) hS[a * p + b] = hS[b * p + a] = 0.5 * (hS[a * p + b] + hS[b * p + a]);
        host_symeig(hS, p, w, Q_);
        std::vector<int> ord(p);
        for (int a = 0; a < p; ++a) ord[a] = a;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] > w[b]; });
        std::vector<double> Qs(np);
        for (int a = 0; a < p; ++a)
            for (int b = 0; b < p; ++b) Qs[a * p + b] = Q_[a * p + ord[b]];
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
        const bool cap = it >= PCA_MAX_OUTER;
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
            ccg_set_error("ccg_pca: subspace iteration did not converge in %d steps (residual %.3g)",
                          PCA_MAX_OUTER * PCA_CHEB_DEG, worst);
            return CCG_EINVAL;
        }
        // the filter on [0, a] (a bounded away from 0: one step's growth ~4 theta_1 / a stays well inside
        // CholeskyQR's range)
        const double a = std::max(w[ord[p - 1]], 1e-7 * th0), c = 0.5 * a, e = 0.5 * a;
        // Y_1 = (C - c) Y_0 / e from the Ritz pairs (T2 = C T1), Y_0 = T1: Q = [Y_1; Y_0]
        pca_cheb_kernel<<<gv, 256, 0, st>>>(T2, 1, (int64_t)nv, T1, nullptr, 1.0 / e, c / e, 0.0, Q, Q + nv);
        rc = cqr(Q, 2 * (int64_t)ng, P);
        if (rc) return rc;
        for (int k = 2; k <= PCA_CHEB_DEG; ++k) {
            rc = matvec(P);
            if (rc) return rc;
            pca_cheb_kernel<<<gv, 256, 0, st>>>(Wp, nsl_mv, (int64_t)nv, P, P + nv, 2.0 / e, 2.0 * c / e, 1.0, Q,
                                                 Q + nv);
            rc = cqr(Q, 2 * (int64_t)ng, P);
            if (rc) return rc;
        }
        rc = cqr(P, ng, V);  // the second CholeskyQR pass of the filtered block
        if (rc) return rc;
    }
}

extern "C" int ccg_pca_dev(ccg_ctx* ctx, const double* counts, int64_t G, int64_t N, const double* sf,
                           const int32_t* genes, int ng, const int32_t* cells, int64_t nc, int npc, double* x,
                           double* sdev, void* stream) {
    CCG_REQUIRE(ctx && counts && sf && genes && cells && x && sdev, "ccg_pca_dev: NULL argument");
    CCG_REQUIRE(G >= 1 && N >= 1 && ng >= 2 && nc >= 3, "ccg_pca_dev: need >= 2 genes and >= 3 cells");
    CCG_REQUIRE(npc >= 1 && npc < ng && npc < nc, "ccg_pca_dev: need 1 <= npc < min(genes, cells)");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    PcaWs ws;
    int rc = pca_workspace(ctx, nc, ng, pca_block_width(ng, npc), &ws);
    if (rc) return rc;
    const int64_t nz = nc * (int64_t)ng;
    pca_gather_kernel<<<(unsigned)ccg_cdiv(nz, 256), 256, 0, st>>>(counts, G, sf, genes, ng, cells, nc, ws.Z);
    CCG_HIP(hipGetLastError());
    return pca_from_z(ctx, ws, nc, ng, npc, x, sdev, st);
}

extern "C" int ccg_pca_csc_dev(ccg_ctx* ctx, const double* xv, const int32_t* ri, const int64_t* cp, int64_t G,
                               int64_t N, const double* sf, const int32_t* gpos, int ng, const int32_t* cells,
                               int64_t nc, int npc, double* x, double* sdev, void* stream) {
    CCG_REQUIRE(ctx && cp && sf && gpos && cells && x && sdev, "ccg_pca_csc_dev: NULL argument");
    CCG_REQUIRE(G >= 1 && N >= 1 && ng >= 2 && nc >= 3, "ccg_pca_csc_dev: need >= 2 genes and >= 3 cells");
    CCG_REQUIRE(npc >= 1 && npc < ng && npc < nc, "ccg_pca_csc_dev: need 1 <= npc < min(genes, cells)");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    PcaWs ws;
    int rc = pca_workspace(ctx, nc, ng, pca_block_width(ng, npc), &ws);
    if (rc) return rc;
    const int64_t nz = nc * (int64_t)ng;
    pca_fill_kernel<<<(unsigned)std::min<int64_t>(ccg_cdiv(nz, 256), 4096), 256, 0, st>>>(ws.Z, nz, 0.0);
    pca_gather_csc_kernel<<<(unsigned)ccg_cdiv(nc, 4), 256, 0, st>>>(xv, ri, cp, sf, gpos, cells, nc, ng, ws.Z);
    CCG_HIP(hipGetLastError());
    return pca_from_z(ctx, ws, nc, ng, npc, x, sdev, st);
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

extern "C" int ccg_pca_csc(ccg_ctx* ctx, const double* xv, const int32_t* ri, const int64_t* cp, int64_t G,
                           int64_t N, const double* sf, const int32_t* genes, int ng, const int32_t* cells, int64_t nc,
                           int npc, double* x, double* sdev) {
    CCG_REQUIRE(ctx && cp && sf && genes && cells && x && sdev, "ccg_pca_csc: NULL argument");
    CCG_REQUIRE(G >= 1 && N >= 1 && ng >= 2 && nc >= 3, "ccg_pca_csc: need >= 2 genes and >= 3 cells");
    const int64_t nnz = cp[N];
    CCG_REQUIRE(cp[0] == 0 && nnz >= 0 && (nnz == 0 || (xv && ri)), "ccg_pca_csc: bad column pointers");
    for (int64_t c = 0; c < N; ++c) CCG_REQUIRE(cp[c + 1] >= cp[c], "ccg_pca_csc: column pointers must not decrease");
    for (int64_t e = 0; e < nnz; ++e) CCG_REQUIRE(ri[e] >= 0 && ri[e] < G, "ccg_pca_csc: row index out of range");
    std::vector<int32_t> gpos(G, -1);
    for (int g = 0; g < ng; ++g) {
        CCG_REQUIRE(genes[g] >= 0 && genes[g] < G, "ccg_pca_csc: gene index out of range");
        CCG_REQUIRE(gpos[genes[g]] < 0, "ccg_pca_csc: gene %d selected twice", genes[g]);
        gpos[genes[g]] = g;
    }
    for (int64_t i = 0; i < nc; ++i) CCG_REQUIRE(cells[i] >= 0 && cells[i] < N, "ccg_pca_csc: cell index out of range");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    double* dx = (double*)ccg_ws(ctx, WS_HOST_A, sizeof(double) * (size_t)std::max<int64_t>(nnz, 1));
    int32_t* dri = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1));
    int64_t* dcp = (int64_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int64_t) * (N + 1) + sizeof(double) * N +
                                                        sizeof(int32_t) * (G + nc) + 64);
    double* dout = (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * (size_t)(nc * npc));
    if (!dx || !dri || !dcp || !dout) return CCG_ENOMEM;
    double* dsf = (double*)(dcp + N + 1);
    int32_t* dgpos = (int32_t*)(dsf + N);
    int32_t* dcell = dgpos + G;
    if (nnz) {
        CCG_HIP(hipMemcpyAsync(dx, xv, sizeof(double) * nnz, hipMemcpyHostToDevice, st));
        CCG_HIP(hipMemcpyAsync(dri, ri, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, st));
    }
    CCG_HIP(hipMemcpyAsync(dcp, cp, sizeof(int64_t) * (N + 1), hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dsf, sf, sizeof(double) * N, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dgpos, gpos.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dcell, cells, sizeof(int32_t) * nc, hipMemcpyHostToDevice, st));
    int rc = ccg_pca_csc_dev(ctx, dx, dri, dcp, G, N, dsf, dgpos, ng, dcell, nc, npc, dout, sdev, st);
    if (rc) return rc;
    CCG_HIP(hipMemcpyAsync(x, dout, sizeof(double) * (size_t)(nc * npc), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}
