// Co-clustering counts and distance as a one-hot int8 MFMA GEMM on gfx950.
//
// Reference: the customDist plugin (RcppXPtrUtils::cppXPtr, R/consensusClust.R
// :411-418) evaluated by parallelDist::parDist(method="custom") and
// 1 - parDist(...) (:421):
//   overlap = #{b : A_bi == A_bj, A_bi != -1},  U = #{b : A_bi != -1, A_bj != -1}
//   jaccard = (float)overlap / (float)U  (float division), dist = 1 - jaccard.
//
// With H = one-hot(A) (N x sum_b C_b, unsampled rows all-zero) and
// S = [A != 0] (N x B):  co = H H^T,  both = S S^T.  Both are computed with
// v_mfma_i32_32x32x32_i8 on 128 x 128 output tiles of the upper triangle;
// the one-hot K-chunks (64 positions) are expanded from the uint8 labels
// straight into LDS, so H never exists in HBM (HBM traffic per tile is the
// label panels, not the one-hot matrix).  Integer accumulation makes the
// counts exact; the epilogue's division is done in fp64 and rounded once
// to fp32, which equals the correctly rounded fp32 quotient because
// 53 >= 2*24 + 2 (no double-rounding error), so the distances are bitwise
// those of the reference.
//
// The output is the packed upper triangle by rows == R's "dist" order.
#include <algorithm>

#include "ccg_internal.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define COC_BM 128
#define COC_KC 64

__global__ void coc_colmax_kernel(const uint8_t* __restrict__ A, int64_t N, int* __restrict__ colC) {
    const int b = blockIdx.y;
    const uint8_t* col = A + (int64_t)b * N;
    int mx = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N;
         i += (int64_t)gridDim.x * blockDim.x)
        mx = max(mx, (int)col[i]);
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0 && mx > 0) atomicMax(&colC[b], mx);
}

// tables layout: off[B+1] | nchunk (1) | colLo[maxch] | colHi[maxch]
__global__ __launch_bounds__(1024) void coc_tables_kernel(const int* __restrict__ colC, int64_t B,
                                                          int* __restrict__ off, int* __restrict__ nchunk,
                                                          int* __restrict__ colLo, int* __restrict__ colHi) {
    __shared__ int sh[16];
    __shared__ int carry_s;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < B; b0 += 1024) {
        const int64_t b = b0 + t;
        const int v = b < B ? colC[b] : 0;
        int x = v;
        for (int o = 1; o < 64; o <<= 1) {
            int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) sh[wv] = x;
        __syncthreads();
        int woff = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wv) woff += sh[w];
            tot += sh[w];
        }
        const int carry = carry_s;
        if (b < B) off[b] = carry + woff + x - v;
        __syncthreads();
        if (t == 0) carry_s = carry + tot;
        __syncthreads();
    }
    const int KC = carry_s;
    if (t == 0) {
        off[B] = KC;
        *nchunk = (KC + COC_KC - 1) / COC_KC;
    }
    const int nch = (KC + COC_KC - 1) / COC_KC;
    for (int ch = t; ch < nch; ch += 1024) {
        const int p0 = ch * COC_KC;
        const int p1 = min(p0 + COC_KC - 1, KC - 1);
        // largest b with off[b] <= p  (upper_bound - 1)
        int lo = 0, hi = (int)B;  // off[0] = 0 <= p
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (off[mid] <= p0) lo = mid; else hi = mid;
        }
        colLo[ch] = lo;
        lo = 0;
        hi = (int)B;
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (off[mid] <= p1) lo = mid; else hi = mid;
        }
        colHi[ch] = lo;
    }
}

__device__ __forceinline__ unsigned expand4(unsigned b) {
    return (b & 1u) | ((b & 2u) << 7) | ((b & 4u) << 14) | ((b & 8u) << 21);
}

// Store a 64-position 0/1 row (bit mask) as 64 bytes, 16-B chunks swizzled.
__device__ __forceinline__ void store_onehot_row(uint8_t* lds, int row, unsigned long long bits) {
    const int f = (row >> 2) & 3;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const unsigned s = (unsigned)(bits >> (16 * q));
        v4i v;
        v[0] = (int)expand4(s & 15u);
        v[1] = (int)expand4((s >> 4) & 15u);
        v[2] = (int)expand4((s >> 8) & 15u);
        v[3] = (int)expand4((s >> 12) & 15u);
        *(v4i*)(lds + row * 64 + ((q ^ f) << 4)) = v;
    }
}

__device__ __forceinline__ v4i load_frag(const uint8_t* lds, int row, int chunk) {
    const int f = (row >> 2) & 3;
    return *(const v4i*)(lds + row * 64 + ((chunk ^ f) << 4));
}

__device__ __forceinline__ void mfma_tile(const uint8_t* sA, const uint8_t* sB, int wr, int wc,
                                          int lane, v16i (&acc)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 2 + (lane >> 5);
        v4i a[2], b[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) a[mi] = load_frag(sA, wr * 64 + mi * 32 + (lane & 31), chunk);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) b[ni] = load_frag(sB, wc * 64 + ni * 32 + (lane & 31), chunk);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
}

__global__ __launch_bounds__(256) void coc_tile_kernel(
    const uint8_t* __restrict__ A, int64_t N, int64_t B, int64_t r0, int64_t r1, int64_t TC,
    int64_t I0, const int* __restrict__ off, const int* __restrict__ nchunk_p,
    const int* __restrict__ colLo, const int* __restrict__ colHi, uint16_t* __restrict__ co,
    uint16_t* __restrict__ both, double* __restrict__ dist) {
    __shared__ __attribute__((aligned(16))) uint8_t sA[COC_BM * COC_KC];
    __shared__ __attribute__((aligned(16))) uint8_t sB[COC_BM * COC_KC];
    // tile t -> (I, J): row tiles from I0, J in [I, TC)
    const int64_t t = blockIdx.x;
    int64_t lo = 0, hi = ccg_cdiv(r1 - r0, COC_BM);  // relative row tile in [lo, hi)
    // cum(Ir) = sum_{s<Ir} (TC - (I0+s)) = Ir*(TC-I0) - Ir*(Ir-1)/2
    auto cum = [&](int64_t Ir) { return Ir * (TC - I0) - Ir * (Ir - 1) / 2; };
    while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (cum(mid) <= t) lo = mid; else hi = mid;
    }
    const int64_t I = I0 + lo;
    const int64_t J = I + (t - cum(lo));
    const int64_t rowA0 = I * COC_BM, rowB0 = J * COC_BM;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int op = tid >> 7, row = tid & 127;
    const int64_t grow = (op ? rowB0 : rowA0) + row;
    const bool rin = grow < N;
    uint8_t* sOp = op ? sB : sA;

    v16i accC[2][2], accS[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                accC[mi][ni][r] = 0;
                accS[mi][ni][r] = 0;
            }

    // ---- co = H H^T over one-hot chunks
    const int nch = *nchunk_p;
    for (int ch = 0; ch < nch; ++ch) {
        unsigned long long bits = 0ull;
        if (rin) {
            const int p0 = ch * COC_KC;
            const int b1 = colHi[ch];
            for (int b = colLo[ch]; b <= b1; ++b) {
                const int lab = A[(int64_t)b * N + grow];
                if (lab) {
                    const int pos = off[b] + lab - 1 - p0;
                    if (pos >= 0 && pos < COC_KC) bits |= 1ull << pos;
                }
            }
        }
        store_onehot_row(sOp, row, bits);
        __syncthreads();
        mfma_tile(sA, sB, wr, wc, lane, accC);
        __syncthreads();
    }
    // ---- both = S S^T over column chunks
    const int nchB = (int)ccg_cdiv(B, COC_KC);
    for (int ch = 0; ch < nchB; ++ch) {
        unsigned long long bits = 0ull;
        if (rin) {
            const int64_t b0 = (int64_t)ch * COC_KC;
            const int nb = (int)std::min<int64_t>(COC_KC, B - b0);
            for (int kk = 0; kk < nb; ++kk)
                if (A[(b0 + kk) * N + grow]) bits |= 1ull << kk;
        }
        store_onehot_row(sOp, row, bits);
        __syncthreads();
        mfma_tile(sA, sB, wr, wc, lane, accS);
        __syncthreads();
    }
    // ---- epilogue: packed upper triangle, rows [r0, r1)
    const int64_t base = r0 * N - r0 * (r0 + 1) / 2;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t gi = rowA0 + wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int64_t gj = rowB0 + wc * 64 + ni * 32 + (lane & 31);
                if (gi < r1 && gj < N && gj > gi) {
                    const int64_t o = gi * N - gi * (gi + 1) / 2 + (gj - gi - 1) - base;
                    const int cv = accC[mi][ni][r], bv = accS[mi][ni][r];
                    if (co) co[o] = (uint16_t)cv;
                    if (both) both[o] = (uint16_t)bv;
                    if (dist) {
                        const float q = (float)((double)cv / (double)bv);
                        dist[o] = 1.0 - (double)q;
                    }
                }
            }
}

// ------------------------------------------------- fused one-hot path --
// co and both in ONE int32 accumulator: every column b gets a K range of
// S_b = ceil((C_b + 1) / 16) 16-position slots; position 0 holds the
// "sampled" flag as int8 -128 on both sides (product 16384), positions
// 1..C_b the one-hot label (product 1), so
//     acc = co + 16384 * both      (co <= B <= 16383, so the fields split)
// and K = 16 * sum_b S_b instead of sum_b C_b + B separate positions.
// A lane gets its 16-byte MFMA fragment for slot (b, s) from its row's uint8
// label through a 34-entry LDS pattern table (at most two non-zero bytes), so
// the one-hot matrix never exists -- not in HBM, not in LDS.  Labels are staged per block of
// COF_SLOTS slots (<= COF_SLOTS columns x 384 rows: 128 A-rows + 256 B-rows) in LDS,
// double-buffered through registers.
#define COF_BM 128          // output rows per block (2 waves x 64)
#define COF_BN 256          // output cols per block (2 waves x 128)
#define COF_SLOTS 32        // slots per stage (16 K-steps of v_mfma_i32_32x32x32_i8)
#define COF_ROWS (COF_BM + COF_BN)
#define COF_LOADS (COF_SLOTS * COF_ROWS / 4 / 256)  // dwords per thread per stage

// slot table: desc[k] = b << 4 | s for k < K (K padded to a multiple of
// COF_SLOTS with -1), stage_lo[st] / stage_nc[st] = the stage's column range.
__global__ __launch_bounds__(1024) void cof_slots_kernel(const int* __restrict__ colC, int64_t B,
                                                         int* __restrict__ off, int* __restrict__ nslot,
                                                         int* __restrict__ desc, int* __restrict__ stage_lo,
                                                         int* __restrict__ stage_nc) {
    __shared__ int sh[16];
    __shared__ int carry_s;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < B; b0 += 1024) {
        const int64_t b = b0 + t;
        const int v = (b < B && colC[b] > 0) ? (colC[b] + 1 + 15) / 16 : 0;
        int x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) sh[wv] = x;
        __syncthreads();
        int woff = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wv) woff += sh[w];
            tot += sh[w];
        }
        const int carry = carry_s;
        if (b < B) off[b] = carry + woff + x - v;
        __syncthreads();
        if (t == 0) carry_s = carry + tot;
        __syncthreads();
    }
    const int K = carry_s;
    const int Kp = (K + COF_SLOTS - 1) / COF_SLOTS * COF_SLOTS;
    if (t == 0) *nslot = Kp;
    for (int64_t b = t; b < B; b += 1024) {
        const int v = colC[b] > 0 ? (colC[b] + 1 + 15) / 16 : 0;
        for (int s2 = 0; s2 < v; ++s2) desc[off[b] + s2] = (int)(b << 4) | s2;
    }
    for (int k = K + t; k < Kp; k += 1024) desc[k] = -1;
    __syncthreads();
    for (int st = t; st < Kp / COF_SLOTS; st += 1024) {
        const int k0 = st * COF_SLOTS;
        int k1 = min(k0 + COF_SLOTS, K) - 1;
        const int lo = desc[k0] >> 4;
        const int hi = desc[k1] >> 4;
        stage_lo[st] = lo;
        stage_nc[st] = hi - lo + 1;
    }
}

// Fragment table (LDS, 34 x 16 B): entry i < 16 = one-hot byte i; 16 + i =
// flag (-128 in byte 0) + one-hot byte i (i >= 1); 32 = flag only; 33 = zero.
// A fragment is one conflict-free ds_read_b128 (the 16 one-hot entries span
// the 64 banks exactly once) after ~6 VALU to pick the entry.
#define COF_TAB 34
__device__ __forceinline__ int cof_entry(int lab, int sub) {
    const int pos = lab - 16 * sub;
    const int e0 = lab < 16 ? 16 + lab : 32;      // slot 0: flag (+ label if it fits)
    const int e1 = (unsigned)pos < 16u ? pos : 33;  // later slots: label or nothing
    return lab == 0 ? 33 : (sub == 0 ? e0 : e1);
}

__global__ __launch_bounds__(256, 2) void cof_tile_kernel(
    const uint8_t* __restrict__ A, int64_t N, int64_t r0, int64_t r1, int64_t TC, int64_t I0,
    const int* __restrict__ desc, const int* __restrict__ stage_lo, const int* __restrict__ stage_nc,
    const int* __restrict__ nslot_p, uint16_t* __restrict__ co, uint16_t* __restrict__ both,
    double* __restrict__ dist) {
    __shared__ __attribute__((aligned(16))) uint8_t panel[2][COF_SLOTS][COF_ROWS];
    __shared__ __attribute__((aligned(16))) v4i ftab[COF_TAB];
    __shared__ __attribute__((aligned(16))) int sdesc[2][2][COF_SLOTS / 2];  // [buf][half][k-step]
    // tile t -> (I, J): row tiles of 128 from I0, col tiles of 256 from J = I/2
    const int64_t t = blockIdx.x;
    const int64_t TR = ccg_cdiv(r1 - r0, COF_BM);
    // cum(Ir) = sum_{s<Ir} (TC - (I0+s)/2)
    auto fl = [](int64_t x) { return (x / 2) * (x / 2 - 1) + ((x & 1) ? x / 2 : 0); };  // sum_{s<x} s/2
    auto cum = [&](int64_t Ir) { return Ir * TC - (fl(I0 + Ir) - fl(I0)); };
    int64_t lo = 0, hi = TR;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (cum(mid) <= t) lo = mid; else hi = mid;
    }
    const int64_t I = I0 + lo;
    const int64_t J = I / 2 + (t - cum(lo));
    const int64_t rowA0 = I * COF_BM, rowB0 = J * COF_BN;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nstage = *nslot_p / COF_SLOTS;

    v16i acc[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0;

    // stage loader: dword p of the panel = (column c, row dword rd); rows past N read row N-4..N-1 (masked later)
    unsigned pf[COF_LOADS];
    int pdesc = -1;
    auto issue = [&](int st) {
        const int clo = stage_lo[st], nc = stage_nc[st];
#pragma unroll
        for (int i = 0; i < COF_LOADS; ++i) {
            const int p = i * 256 + tid;
            const int c = p / (COF_ROWS / 4), rd = p - c * (COF_ROWS / 4);
            int64_t row = rd < COF_BM / 4 ? rowA0 + 4 * rd : rowB0 + 4 * (rd - COF_BM / 4);
            row = row + 4 <= N ? row : N - 4;
            pf[i] = c < nc ? *reinterpret_cast<const unsigned*>(A + (int64_t)(clo + c) * N + row) : 0u;
        }
        if (tid < COF_SLOTS) {
            const int dsc = desc[(int64_t)st * COF_SLOTS + tid];
            pdesc = dsc < 0 ? -1 : (((dsc >> 4) - clo) << 4) | (dsc & 15);
        }
    };
    auto commit = [&](int bb) {
#pragma unroll
        for (int i = 0; i < COF_LOADS; ++i) reinterpret_cast<unsigned*>(&panel[bb][0][0])[i * 256 + tid] = pf[i];
        if (tid < COF_SLOTS) sdesc[bb][tid & 1][tid >> 1] = pdesc;
    };
    if (tid < COF_TAB) {
        v4i e = {0, 0, 0, 0};
        const int i = tid < 16 ? tid : (tid < 32 ? tid - 16 : -1);
        if (tid < 33 && i >= 0 && !(tid >= 16 && i == 0)) e[i >> 2] = 1 << (8 * (i & 3));
        if (tid >= 16 && tid < 33) e[0] |= 0x80;  // the flag (int8 -128) in byte 0
        ftab[tid] = e;
    }
    issue(0);
    commit(0);
    __syncthreads();
    const int ra = wr * 64 + (lane & 31);            // A rows ra, ra + 32 (panel rows 0..127)
    const int rb = COF_BM + wc * 128 + (lane & 31);  // B rows rb + 32*ni
    const int h = lane >> 5;
    for (int st = 0; st < nstage; ++st) {
        const int bb = st & 1;
        if (st + 1 < nstage) issue(st + 1);
        // software pipeline over the stage's K-steps: labels of step q+2 and
        // the fragment-table reads of step q+1 are in flight while the MFMAs
        // of step q run
        constexpr int QN = COF_SLOTS / 2;
        int dsc[QN];
#pragma unroll
        for (int q4 = 0; q4 < QN / 4; ++q4) {
            const int4 v = *reinterpret_cast<const int4*>(&sdesc[bb][h][4 * q4]);
            dsc[4 * q4 + 0] = v.x;
            dsc[4 * q4 + 1] = v.y;
            dsc[4 * q4 + 2] = v.z;
            dsc[4 * q4 + 3] = v.w;
        }
        int lab[2][6];
        auto read_labels = [&](int q, int (&L)[6]) {
            const int d = dsc[q];
            const uint8_t* col = &panel[bb][d < 0 ? 0 : d >> 4][0];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) L[mi] = d < 0 ? 0 : col[ra + 32 * mi];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) L[2 + ni] = d < 0 ? 0 : col[rb + 32 * ni];
        };
        v4i fr[2][6];
        auto read_frags = [&](int q, const int (&L)[6], v4i (&F)[6]) {
            const int sub = dsc[q] < 0 ? 0 : dsc[q] & 15;
#pragma unroll
            for (int x = 0; x < 6; ++x) F[x] = ftab[cof_entry(L[x], sub)];
        };
        read_labels(0, lab[0]);
        read_labels(1, lab[1]);
        read_frags(0, lab[0], fr[0]);
#pragma unroll
        for (int q = 0; q < QN; ++q) {
            const int cur = q & 1;
            if (q + 2 < QN) read_labels(q + 2, lab[cur]);
            if (q + 1 < QN) read_frags(q + 1, lab[cur ^ 1], fr[cur ^ 1]);
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] =
                        __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[cur][mi], fr[cur][2 + ni], acc[mi][ni], 0, 0, 0);
        }
        if (st + 1 < nstage) {
            __syncthreads();  // every wave is done with buffer bb^1 (read in stage st-1)
            commit(bb ^ 1);
            __syncthreads();
        }
    }
    // ---- epilogue: acc = co + 16384 * both; packed upper triangle, rows [r0, r1)
    const int64_t base = r0 * N - r0 * (r0 + 1) / 2;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t gi = rowA0 + wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gj = rowB0 + wc * 128 + ni * 32 + (lane & 31);
                if (gi < r1 && gj < N && gj > gi) {
                    const int64_t o = gi * N - gi * (gi + 1) / 2 + (gj - gi - 1) - base;
                    const int a = acc[mi][ni][r];
                    const int cv = a & 16383, bv = a >> 14;
                    if (co) co[o] = (uint16_t)cv;
                    if (both) both[o] = (uint16_t)bv;
                    if (dist) {
                        const float qv = (float)((double)cv / (double)bv);
                        dist[o] = 1.0 - (double)qv;
                    }
                }
            }
}

extern "C" int ccg_cocluster_dev(ccg_ctx* ctx, const uint8_t* A, int64_t N, int64_t B, int64_t r0,
                                 int64_t r1, uint16_t* co, uint16_t* both, double* dist, void* stream) {
    CCG_REQUIRE(ctx && A, "ccg_cocluster_dev: NULL argument");
    CCG_REQUIRE(N >= 2 && N < (1LL << 31), "ccg_cocluster_dev: bad N");
    CCG_REQUIRE(B >= 1 && B <= 65535, "ccg_cocluster_dev: B=%lld must be in [1, 65535] (uint16 counts)",
                (long long)B);
    CCG_REQUIRE(r0 >= 0 && r0 <= r1 && r1 <= N, "ccg_cocluster_dev: bad row range");
    CCG_REQUIRE(r0 % CCG_COCLUSTER_ROW_ALIGN == 0, "ccg_cocluster_dev: r0 must be a multiple of %d",
                CCG_COCLUSTER_ROW_ALIGN);
    hipStream_t st = ccg_pick_stream(ctx, stream);
    if (r1 == r0) return CCG_OK;
    const int64_t maxch = ccg_cdiv(B * 255, COC_KC) + 2;
    int* tab = (int*)ccg_ws(ctx, WS_COC_A, sizeof(int) * (B + (B + 1) + 1 + 2 * maxch + 8));
    if (!tab) return CCG_ENOMEM;
    int* colC = tab;
    int* off = colC + B;
    int* nchunk = off + (B + 1);
    int* colLo = nchunk + 1;
    int* colHi = colLo + maxch;
    CCG_HIP(hipMemsetAsync(colC, 0, sizeof(int) * B, st));
    coc_colmax_kernel<<<dim3((unsigned)std::min<int64_t>(ccg_cdiv(N, 256), 64), (unsigned)B), 256, 0, st>>>(
        A, N, colC);
    coc_tables_kernel<<<1, 1024, 0, st>>>(colC, B, off, nchunk, colLo, colHi);
    static const bool legacy = getenv("CCG_COC_LEGACY") != nullptr;  // A/B switch
    if (B <= 16383 && N % 4 == 0 && N >= 4 && !legacy) {
        // fused one-hot path (co + 16384*both in one accumulator)
        const int64_t maxslots = B * 16 + COF_SLOTS;
        int* ft = (int*)ccg_ws(ctx, WS_COC_B, sizeof(int) * (B + 8 + maxslots + 2 * (maxslots / COF_SLOTS + 1)));
        if (!ft) return CCG_ENOMEM;
        int* foff = ft;
        int* fnslot = foff + B;
        int* fdesc = fnslot + 8;
        int* fslo = fdesc + maxslots;
        int* fsnc = fslo + (maxslots / COF_SLOTS + 1);
        cof_slots_kernel<<<1, 1024, 0, st>>>(colC, B, foff, fnslot, fdesc, fslo, fsnc);
        const int64_t TC = ccg_cdiv(N, COF_BN);
        const int64_t I0 = r0 / COF_BM;
        const int64_t TR = ccg_cdiv(r1 - r0, COF_BM);
        auto fl = [](int64_t x) { return (x / 2) * (x / 2 - 1) + ((x & 1) ? x / 2 : 0); };
        const int64_t ntiles = TR * TC - (fl(I0 + TR) - fl(I0));
        CCG_REQUIRE(ntiles < (1LL << 31), "ccg_cocluster_dev: too many tiles");
        const int t_k = ccg_timer_start(ctx, CCG_KT_COCLUSTER, st);
        cof_tile_kernel<<<(unsigned)ntiles, 256, 0, st>>>(A, N, r0, r1, TC, I0, fdesc, fslo, fsnc, fnslot, co,
                                                         both, dist);
        ccg_timer_stop(ctx, t_k, st);
        CCG_HIP(hipGetLastError());
        return CCG_OK;
    }
    const int64_t TC = ccg_cdiv(N, COC_BM);
    const int64_t I0 = r0 / COC_BM;
    const int64_t TR = ccg_cdiv(r1 - r0, COC_BM);
    const int64_t ntiles = TR * (TC - I0) - TR * (TR - 1) / 2;
    CCG_REQUIRE(ntiles < (1LL << 31), "ccg_cocluster_dev: too many tiles");
    const int t_k = ccg_timer_start(ctx, CCG_KT_COCLUSTER, st);
    coc_tile_kernel<<<(unsigned)ntiles, 256, 0, st>>>(A, N, B, r0, r1, TC, I0, off, nchunk, colLo, colHi,
                                                     co, both, dist);
    ccg_timer_stop(ctx, t_k, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------ consensus kNN --
// One wave per row: lanes scan columns j = lane, lane+64, ...; key = the
// fp32 similarity (larger = closer, equivalent to ascending 1 - sim), ties
// by ascending j; self excluded; NaN (both == 0) raises the flag.
#define CKNN_K 32
__global__ __launch_bounds__(256) void consensus_knn_kernel(const uint16_t* __restrict__ co,
                                                            const uint16_t* __restrict__ both,
                                                            int64_t N, int k, int32_t* __restrict__ out,
                                                            int* __restrict__ nan_flag) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= N) return;
    float lv[CKNN_K];
    int li[CKNN_K];
#pragma unroll
    for (int t = 0; t < CKNN_K; ++t) {
        lv[t] = -INFINITY;
        li[t] = 0x7fffffff;
    }
    bool sawnan = false;
    for (int64_t j = lane; j < N; j += 64) {
        if (j == i) continue;
        const int64_t a = i < j ? i : j, b = i < j ? j : i;
        const int64_t o = a * N - a * (a + 1) / 2 + (b - a - 1);
        const unsigned c = co[o], u = both[o];
        if (u == 0) {
            sawnan = true;
            continue;
        }
        const float s = (float)((double)c / (double)u);
        if (!(s > lv[CKNN_K - 1])) continue;  // j ascending per lane: ties keep the earlier j
        float cv = s;
        int ci = (int)j;
#pragma unroll
        for (int t = 0; t < CKNN_K; ++t) {
            const bool sw = (cv > lv[t]) || (cv == lv[t] && ci < li[t]);
            const float tv = lv[t];
            const int ti = li[t];
            lv[t] = sw ? cv : tv;
            li[t] = sw ? ci : ti;
            cv = sw ? tv : cv;
            ci = sw ? ti : ci;
        }
    }
    if (__any(sawnan) && lane == 0) atomicOr(nan_flag, 1);
    for (int r = 0; r < k; ++r) {
        float bk = lv[0];
        int bi = li[0];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ok = __shfl_xor(bk, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ok > bk || (ok == bk && oi < bi)) {
                bk = ok;
                bi = oi;
            }
        }
        if (lane == 0) out[i * k + r] = bi;
        if (li[0] == bi) {
#pragma unroll
            for (int t = 0; t < CKNN_K - 1; ++t) {
                lv[t] = lv[t + 1];
                li[t] = li[t + 1];
            }
            lv[CKNN_K - 1] = -INFINITY;
            li[CKNN_K - 1] = 0x7fffffff;
        }
    }
}

extern "C" int ccg_consensus_knn_dev(ccg_ctx* ctx, const uint16_t* co, const uint16_t* both, int64_t N,
                                     int k, int32_t* out_idx, int32_t* d_nan_flag, void* stream) {
    CCG_REQUIRE(ctx && co && both && out_idx && d_nan_flag, "ccg_consensus_knn_dev: NULL argument");
    CCG_REQUIRE(N >= 2 && k >= 1 && k <= CKNN_K && k <= N - 1, "ccg_consensus_knn_dev: need 1 <= k <= min(32, N-1)");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    CCG_HIP(hipMemsetAsync(d_nan_flag, 0, sizeof(int32_t), st));
    consensus_knn_kernel<<<(unsigned)ccg_cdiv(N, 4), 256, 0, st>>>(co, both, N, k, out_idx, d_nan_flag);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------- host flavours --
extern "C" int ccg_cocluster(ccg_ctx* ctx, const uint8_t* A, int64_t N, int64_t B, uint16_t* co,
                             uint16_t* both, double* dist) {
    CCG_REQUIRE(ctx && A, "ccg_cocluster: NULL argument");
    CCG_REQUIRE(N >= 2 && B >= 1, "ccg_cocluster: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t P = N * (N - 1) / 2;
    uint8_t* dA = (uint8_t*)ccg_ws(ctx, WS_HOST_A, (size_t)(B * N));
    uint16_t* dco = co ? (uint16_t*)ccg_ws(ctx, WS_HOST_B, sizeof(uint16_t) * P) : nullptr;
    uint16_t* dboth = both ? (uint16_t*)ccg_ws(ctx, WS_HOST_C, sizeof(uint16_t) * P) : nullptr;
    double* ddist = dist ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * P) : nullptr;
    if (!dA || (co && !dco) || (both && !dboth) || (dist && !ddist)) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dA, A, (size_t)(B * N), hipMemcpyHostToDevice, st));
    int rc = ccg_cocluster_dev(ctx, dA, N, B, 0, N, dco, dboth, ddist, st);
    if (rc) return rc;
    if (co) CCG_HIP(hipMemcpyAsync(co, dco, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, st));
    if (both) CCG_HIP(hipMemcpyAsync(both, dboth, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, st));
    if (dist) CCG_HIP(hipMemcpyAsync(dist, ddist, sizeof(double) * P, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}

extern "C" int ccg_consensus_knn(ccg_ctx* ctx, const uint16_t* co, const uint16_t* both, int64_t N, int k,
                                 int32_t* out_idx) {
    CCG_REQUIRE(ctx && co && both && out_idx, "ccg_consensus_knn: NULL argument");
    CCG_REQUIRE(N >= 2, "ccg_consensus_knn: bad N");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t P = N * (N - 1) / 2;
    uint16_t* dco = (uint16_t*)ccg_ws(ctx, WS_HOST_A, sizeof(uint16_t) * P);
    uint16_t* dboth = (uint16_t*)ccg_ws(ctx, WS_HOST_B, sizeof(uint16_t) * P);
    int32_t* dout = (int32_t*)ccg_ws(ctx, WS_HOST_C, sizeof(int32_t) * N * k + 64);
    if (!dco || !dboth || !dout) return CCG_ENOMEM;
    int32_t* dflag = dout + N * k;
    CCG_HIP(hipMemcpyAsync(dco, co, sizeof(uint16_t) * P, hipMemcpyHostToDevice, st));
    CCG_HIP(hipMemcpyAsync(dboth, both, sizeof(uint16_t) * P, hipMemcpyHostToDevice, st));
    int rc = ccg_consensus_knn_dev(ctx, dco, dboth, N, k, dout, dflag, st);
    if (rc) return rc;
    int flag = 0;
    CCG_HIP(hipMemcpyAsync(&flag, dflag, sizeof(int), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipMemcpyAsync(out_idx, dout, sizeof(int32_t) * N * k, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (flag) {
        ccg_set_error("ccg_consensus_knn: data/distances cannot contain NAs (a pair was never co-sampled)");
        return CCG_ENAN;
    }
    return CCG_OK;
}
