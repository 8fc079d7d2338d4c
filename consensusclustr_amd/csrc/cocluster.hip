// Co-clustering counts and distance as a one-hot int8 MFMA GEMM on gfx950.
//
// Reference: the customDist plugin (RcppXPtrUtils::cppXPtr, R/consensusClust.R
// :411-418) evaluated by parallelDist::parDist(method="custom") and
// 1 - parDist(...) (:421):
//   overlap = #{b : A_bi == A_bj, A_bi != -1},  U = #{b : A_bi != -1, A_bj != -1}
//   jaccard = (float)overlap / (float)U  (float division), dist = 1 - jaccard.
//
// With H = one-hot(A) (N x sum_b C_b, unsampled rows all-zero) and
// S = [A != 0] (N x B):  co = H H^T,  both = S S^T, computed together in ONE
// int32 accumulator by v_mfma_i32_32x32x32_i8 (see "fused one-hot path"
// below).  Integer accumulation makes the counts exact; the epilogue's
// division is done in fp64 and rounded once to fp32, which equals the
// correctly rounded fp32 quotient because 53 >= 2*24 + 2 (no double-rounding
// error), so the distances are bitwise those of the reference.
//
// Outputs: the packed upper triangle by rows (== R's "dist" order) for a row
// slab [r0, r1), or (consensus kNN) full rows [r0, r1) x [0, N) packed as
// co | both << 16.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "cocluster_common.h"

template <typename T>
__global__ void coc_colmax_kernel(const T* __restrict__ A, int64_t N, int* __restrict__ colC) {
    const int b = blockIdx.y;
    const T* col = A + (int64_t)b * N;
    int mx = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N;
         i += (int64_t)gridDim.x * blockDim.x)
        mx = max(mx, (int)col[i]);
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0 && mx > 0) atomicMax(&colC[b], mx);
}

// ------------------------------------------------- fused one-hot path --
// co and both in ONE int32 accumulator.  The K dimension is cut into 8-byte
// halves: column b owns H_b = ceil((C_b + 1) / 8) consecutive halves; its
// first half holds the "sampled" flag as int8 -128 in byte 0 (product 16384
// on both sides) and labels 1..7 in bytes 1..7, half s >= 1 labels 8s..8s+7
// (product 1), so
//     acc = co + 16384 * both      (co <= B_chunk <= 16383, so the fields split)
// and K = 8 * sum_b H_b instead of sum_b C_b + B separate positions (C = 37:
// 40 positions for 38 -- 16-byte granularity took 48).
// Wider matrices (granular mode, B up to 65535) run in column chunks of at
// most 16383 whose counts are added in the epilogue of the next chunk.
// A 16-byte MFMA fragment (one slot = two halves, possibly of two columns)
// comes from an LDS pattern table: a half's state is one of 9 (zero, or the
// one-hot byte / flag pattern), a slot's entry sigma_lo + 9 sigma_hi (< 81),
// and the slot's type (which of its halves is a first half) picks one of
// four 81-entry tables -- the types of a stage's 32 slots are one 64-bit
// word.  So the one-hot matrix never exists -- not in HBM, not in LDS.  The
// entry of every (slot, row) is one byte, computed once per chunk by
// cof_entries_kernel into the entry matrix E (slots x rows).  The GEMM stages
// E per block of COF_SLOTS slots x 384 rows (128 A-rows + 256 B-rows) in LDS,
// double-buffered through registers, so its inner loop is two LDS reads per
// fragment.  Columns with no label (never sampled) own no half.
#define COF_BM 128          // output rows per block (2 waves x 64)
#define COF_BN 256          // output cols per block (2 waves x 128)
#define COF_ROWS (COF_BM + COF_BN)
#define COF_CHUNK 16383     // columns per accumulation chunk
#define COF_SB 14           // desc = column << COF_SB | half-in-column (half < 8193)
#define COF_EMAX (4LL << 30)  // bytes of the entry matrix E of one column chunk
#define COF_ENT_GRID 4096   // slot blocks (grid y) of the entry-matrix kernel

__device__ __forceinline__ int block_excl_scan1024(int v, int* sh, int* total) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
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
    __syncthreads();
    *total = tot;
    return woff + x - v;
}

// Half tables of one chunk of Bc columns (colC = the chunk's column maxima):
// ccol[c] = chunk column of the c-th non-empty column; desc[h] = c << COF_SB
// | s for the halves h < Kh (padded with -1 to 2 * nslot); *nslot = the slots
// ceil(Kh / 2) padded to a multiple of COF_SLOTS; tmask[st] = the types of
// stage st's slots, 2 bits per slot (bit 0: its low half is a column's first
// half, bit 1: its high half).
__global__ __launch_bounds__(1024) void cof_slots_kernel(const int* __restrict__ colC, int64_t Bc,
                                                         int* __restrict__ ccol, int* __restrict__ nslot,
                                                         int* __restrict__ desc,
                                                         unsigned long long* __restrict__ tmask) {
    __shared__ int sh[16];
    const int t = threadIdx.x;
    int kcar = 0, ccar = 0;
    for (int64_t b0 = 0; b0 < Bc; b0 += 1024) {
        const int64_t b = b0 + t;
        const int C = b < Bc ? colC[b] : 0;
        const int v = C > 0 ? (C + 8) / 8 : 0;  // ceil((C + 1) / 8)
        int ktot, ctot;
        const int koff = kcar + block_excl_scan1024(v, sh, &ktot);
        const int coff = ccar + block_excl_scan1024(C > 0 ? 1 : 0, sh, &ctot);
        if (C > 0) {
            ccol[coff] = (int)b;
            for (int s2 = 0; s2 < v; ++s2) desc[koff + s2] = (coff << COF_SB) | s2;
        }
        kcar += ktot;
        ccar += ctot;
    }
    const int Kh = kcar;
    const int Kp = ((Kh + 1) / 2 + COF_SLOTS - 1) / COF_SLOTS * COF_SLOTS;
    if (t == 0) *nslot = Kp;
    for (int k = Kh + t; k < 2 * Kp; k += 1024) desc[k] = -1;
    __syncthreads();  // the block's desc writes are visible to the block
    for (int st = t; st < Kp / COF_SLOTS; st += 1024) {
        unsigned long long m = 0;
        for (int j = 0; j < 2 * COF_SLOTS; ++j) {
            const int d = desc[2 * COF_SLOTS * st + j];
            if (d >= 0 && (d & ((1 << COF_SB) - 1)) == 0) m |= 1ull << j;
        }
        tmask[st] = m;
    }
}

// Fragment table (LDS, 4 x 81 x 16 B): entry type * 81 + sigma_lo + 9 sigma_hi.
// Half state sigma: 0 = zero (not sampled, or the label outside the half);
// normal half 1 + x = one-hot byte x (label 8s + x); first half 1 = the flag
// only (label >= 8), 1 + x = flag + one-hot byte x (label x = 1..7).  The flag
// is int8 -128 in byte 0.  The zero entries of the four types sit in distinct
// 16-byte bank groups.

__device__ __forceinline__ int cof_sigma(int d, int lab) {
    if (d < 0 || lab == 0) return 0;
    const int s = d & ((1 << COF_SB) - 1);
    if (s == 0) return lab < 8 ? 1 + lab : 1;
    const int x = lab - 8 * s;
    return (unsigned)x < 8u ? 1 + x : 0;
}

// Entry matrix of one chunk: E[k * Npad + i] = the table entry of row i in
// slot k (halves 2k, 2k + 1; -1 = padding: state 0), entry 0 for rows i >= N.
// Slots stride over grid y, row dwords (4 rows per thread) over grid x: no
// per-element division.
template <typename T>
__global__ __launch_bounds__(256) void cof_entries_kernel(const T* __restrict__ A, int64_t N, int64_t Npad,
                                                          const int* __restrict__ desc, const int* __restrict__ ccol,
                                                          const int* __restrict__ nslot_p, uint8_t* __restrict__ E) {
    const int nslot = *nslot_p;
    for (int k = blockIdx.y; k < nslot; k += gridDim.y) {
        const int dl = desc[2 * k], dh = desc[2 * k + 1];
        const T* cl = A + (dl < 0 ? 0 : (int64_t)ccol[dl >> COF_SB] * N);
        const T* chh = A + (dh < 0 ? 0 : (int64_t)ccol[dh >> COF_SB] * N);
        uint8_t* Ek = E + (int64_t)k * Npad;
        for (int64_t r4 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); r4 < Npad;
             r4 += 4 * (int64_t)gridDim.x * blockDim.x) {
            unsigned out = 0;
            if (dl >= 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (r4 + e >= N) continue;
                    const int en = cof_sigma(dl, (int)cl[r4 + e]) + 9 * cof_sigma(dh, (int)chh[r4 + e]);
                    out |= (unsigned)en << (8 * e);
                }
            }
            *reinterpret_cast<unsigned*>(Ek + r4) = out;
        }
    }
}

// Output modes: packed upper triangle of rows [r0, r1) (R "dist" order), or
// full rows [r0, r1) x [0, N) as one uint32 co | both << 16 per pair.

// Consensus-kNN candidate lists (COF_CAND): pair (i, j) of the triangle is
// offered to row i if sim_ij >= tau_i and to row j if sim_ij >= tau_j, where
// tau is a lower bound of each row's k-th largest similarity.  Round 5: the
// bound is a multiple of 1 / CKC_NBK, tnum / CKC_NBK (ckc_tau_kernel), so
// the test is exact in int32: co CKC_NBK >= tnum both (< 2^26 on both sides;
// tnum = -1: every pair with both > 0) -- three VALU where round 4's fp64
// test against tau - ulp/2 took two conversions, a multiply and a compare.
// A row's entries go to cand[row * cap + slot] as (the other position,
// co | both << 16); the selection maps positions to original ids (round 6:
// the epilogue no longer runs the modular reduction per push).
#define CKC_NBK 4096
struct CofCand {
    const int* tnum;
    int* cnt;
    uint2* cand;
    int cap;
    int64_t pmul, padd;  // the row permutation: original id of position p = (p * pmul + padd) mod N
    uint64_t pinv;       // floor((2^64 - 1) / N): the mod by a multiply-high (ckc_mod)
    int* flags;          // [0] a pair with both == 0, [1] a row overflowed cap
};

// x mod N for x < 2^63 by Barrett reduction with pinv = floor((2^64 - 1) / N):
// q = mulhi(x, pinv) undershoots x / N by at most 2, so two corrections at most
// (a 128-bit or 64-bit division is a long software loop on the GPU).
__device__ __forceinline__ int64_t ckc_mod(uint64_t x, int64_t N, uint64_t pinv) {
    const uint64_t q = __umul64hi(x, pinv);
    uint64_t r = x - q * (uint64_t)N;
    while (r >= (uint64_t)N) r -= (uint64_t)N;
    return (int64_t)r;
}


// COF_CAND epilogue of one wave's 64 x 128 quarter (rows ia0.., columns
// jb0..): lane (h, col) holds rows ia0 + 32 mi + (r & 3) + 8 (r >> 2) + 4 h
// against column jb0 + 32 ni + col.  A passing pair (a row keeps a few
// hundred of N columns) costs one counter add and one 8-byte store per side
// it enters; the common element two integer tests.
// Round 6: the epilogue walks groups of 4 rows x 4 column blocks; within a
// group it first issues every counter add (one per half-row per group on the
// row side, one per passing element on the column side), then the stores
// that use the returned slots -- one wait on the adds per group.  The
// round-5 form waited on each add before the next element (a push is an
// atomic whose return value addresses the store), which serialised the
// adds' latency: the candidate tile took 46.5 ms against the plain
// triangle's 40.1 at N = 100k, B = 1000.
#ifndef COF_CAND_RG
#define COF_CAND_RG 1  // rows per group (measured: 1 fastest; 4 spilled with the 128 accumulators)
#endif
template <bool INTERIOR>
__device__ __forceinline__ void cof_cand_rows(const v16i (&acc)[2][4], int64_t ia0, int64_t jb0, int64_t N,
                                              int64_t r1, const CofCand& cc, const int (&tj)[4], bool& nan) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const unsigned long long below = (1ull << lane) - 1;
    const unsigned long long half = h ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
    constexpr int RG = COF_CAND_RG;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int rg = 0; rg < 16 / RG; ++rg) {
            bool pr[RG][4], pc[RG][4];
            unsigned val[RG][4];
            int64_t gi[RG];
            int ti[RG];
#pragma unroll
            for (int q = 0; q < RG; ++q) {
                const int r = RG * rg + q;
                gi[q] = ia0 + 32 * mi + (r & 3) + 8 * (r >> 2) + 4 * h;
                ti[q] = (INTERIOR || gi[q] < r1) ? cc.tnum[gi[q]] : 0;
            }
#pragma unroll
            for (int q = 0; q < RG; ++q)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    const int a = acc[mi][ni][RG * rg + q];
                    const int cv = a & 16383, bv = a >> 14;
                    bool ok = true;
                    if (!INTERIOR) {
                        const int64_t gj = jb0 + 32 * ni + col;
                        ok = gi[q] < r1 && gj < N && gj > gi[q];
                    }
                    nan |= ok && bv == 0;
                    const int dc = cv * CKC_NBK;
                    val[q][ni] = (unsigned)cv | ((unsigned)bv << 16);
                    // (24-bit multiplies: tnum in [-1, CKC_NBK], both < 2^17 -- a
                    // full-rate v_mul_i32_i24 instead of the quarter-rate
                    // 32-bit multiply, twice per element)
                    pr[q][ni] = ok && bv > 0 && dc >= __mul24(ti[q], bv);
                    pc[q][ni] = ok && bv > 0 && dc >= __mul24(tj[ni], bv);
                }
            // row side: per row q, the half's passing elements over the 4
            // column blocks take consecutive slots (lane order within a block)
            unsigned long long hm[RG][4];
            int rbase[RG], rlead[RG];
            bool rany = false;
#pragma unroll
            for (int q = 0; q < RG; ++q) {
                int tot = 0;
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    hm[q][ni] = __ballot(pr[q][ni]);
                    tot += __popcll(hm[q][ni] & half);
                }
                // the half's first lane issues the add (lanes 0 and 32 lead)
                rlead[q] = tot;
                rbase[q] = 0;
                rany |= tot > 0;
            }
            if (__any(rany)) {  // (most groups have a passing pair somewhere)
#pragma unroll
                for (int q = 0; q < RG; ++q)
                    if (col == 0 && rlead[q] > 0) rbase[q] = atomicAdd(&cc.cnt[gi[q]], rlead[q]);
            }
            int cslot[RG][4];
#pragma unroll
            for (int q = 0; q < RG; ++q)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    cslot[q][ni] = 0;
                    if (pc[q][ni]) cslot[q][ni] = atomicAdd(&cc.cnt[jb0 + 32 * ni + col], 1);
                }
            // the stores (the first use of the returned slots)
#pragma unroll
            for (int q = 0; q < RG; ++q) {
                const int b0 = __builtin_amdgcn_readlane(rbase[q], 0), b1 = __builtin_amdgcn_readlane(rbase[q], 32);
                int off = h ? b1 : b0;
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    const unsigned long long m = hm[q][ni] & half;
                    if (pr[q][ni]) {
                        const int slot = off + __popcll(m & below);
                        const int64_t gj = jb0 + 32 * ni + col;
                        if (slot < cc.cap)
                            cc.cand[gi[q] * cc.cap + slot] = make_uint2((unsigned)gj, val[q][ni]);
                        else
                            cc.flags[1] = 1;
                    }
                    off += __popcll(m);
                }
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    if (pc[q][ni]) {
                        const int64_t gj = jb0 + 32 * ni + col;
                        if (cslot[q][ni] < cc.cap)
                            cc.cand[gj * cc.cap + cslot[q][ni]] =
                                make_uint2((unsigned)gi[q], val[q][ni]);
                        else
                            cc.flags[1] = 1;
                    }
            }
        }
}

__device__ __forceinline__ void cof_cand_epilogue(const v16i (&acc)[2][4], int64_t ia0, int64_t jb0, int64_t N,
                                                  int64_t r1, const CofCand& cc) {
    const int lane = threadIdx.x & 63, col = lane & 31;
    // the lane's 4 columns' thresholds once (not per row); an interior
    // quarter (every column above every row, inside N and the slab) needs no
    // per-element masks
    int tj[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int64_t gj = jb0 + 32 * ni + col;
        tj[ni] = gj < N ? cc.tnum[gj] : 0;  // (columns past N never pass: ok is false)
    }
    const bool interior = jb0 > ia0 + 63 && jb0 + 128 <= N && ia0 + 64 <= r1;
    bool nan = false;
    if (interior) cof_cand_rows<true>(acc, ia0, jb0, N, r1, cc, tj, nan);
    else cof_cand_rows<false>(acc, ia0, jb0, N, r1, cc, tj, nan);
    if (__any(nan) && lane == 0) cc.flags[0] = 1;
}

// Tile order (round 5).  Tiles (row tile I of 128 rows from I0, column
// tile J of 256) are grouped into supertiles of COF_ST x COF_ST: row tiles
// 8g..8g+7 of the slab and column tiles Jlo_g + 8s.. (Jlo_g = the first
// column tile of the group's first row: (I0 + 8g) / 2 in the triangle, 0 for
// full rows).  Supertile S runs on XCD S mod 8 (block b runs on XCD b mod 8),
// its 64 tiles as XCD-consecutive blocks, so the ~64 blocks an XCD holds at
// once share 8 A panels and 8 B panels of the entry matrix in that XCD's L2
// (~1 MB at cfg3).  Row-major tile order re-read every B panel from beyond
// the L2 for each row tile: 1.9e10 B per launch at N = 100k, B = 125
// (profiles/r04_pmc_cocluster_traffic.md).  Slots outside the slab, the
// column range or the triangle (J < I / 2) exit.
#define COF_ST 8
__host__ __device__ inline int64_t cof_supertiles_row(int64_t g, int64_t TC, int64_t I0, bool tri) {
    const int64_t jlo = tri ? (I0 + COF_ST * g) / 2 : 0;
    return (TC - jlo + COF_ST - 1) / COF_ST;
}
// blocks of the launch: 8 XCDs x 64 slots x the supertiles per XCD
static inline int64_t cof_tile_blocks(int64_t TR, int64_t TC, int64_t I0, bool tri) {
    int64_t ns = 0;
    for (int64_t g = 0; g < (TR + COF_ST - 1) / COF_ST; ++g) ns += cof_supertiles_row(g, TC, I0, tri);
    return 8 * (int64_t)COF_ST * COF_ST * ((ns + 7) / 8);
}
__device__ __forceinline__ bool cof_tile_of(int64_t b, int64_t TR, int64_t TC, int64_t I0, bool tri, int64_t& I,
                                            int64_t& J) {
    const int64_t k = b >> 3;
    const int64_t S = (k / (COF_ST * COF_ST)) * 8 + (b & 7);  // supertile
    const int slot = (int)(k % (COF_ST * COF_ST));
    const int64_t G = (TR + COF_ST - 1) / COF_ST;
    int64_t g = 0, cum = 0;
    for (; g < G; ++g) {  // (block-uniform scalar loop: G ~ 100 at N = 100k)
        const int64_t n = cof_supertiles_row(g, TC, I0, tri);
        if (S < cum + n) break;
        cum += n;
    }
    if (g == G) return false;
    const int64_t Ir = COF_ST * g + slot / COF_ST;
    I = I0 + Ir;
    J = (tri ? (I0 + COF_ST * g) / 2 : 0) + COF_ST * (S - cum) + slot % COF_ST;
    return Ir < TR && J < TC && (!tri || J >= I / 2);
}

// E: the chunk's entry matrix (cof_entries_kernel), Npad bytes per slot.
template <int MODE>
__global__ __launch_bounds__(256, 2) void cof_tile_kernel(
    const uint8_t* __restrict__ E, int64_t Npad, int64_t N, int64_t r0, int64_t r1, int64_t TC, int64_t I0,
    const int* __restrict__ nslot_p, const unsigned long long* __restrict__ tmask, const uint16_t* co_prev,
    const uint16_t* both_prev, uint16_t* co, uint16_t* both, double* __restrict__ dist, const uint32_t* cb_prev,
    uint32_t* cb, int64_t NB, CofCand cc) {
    constexpr int ROWD = COF_ROWS / 4;                  // dwords per staged slot
    constexpr int LOADS = COF_SLOTS * ROWD / 256;       // dwords per thread per stage
    __shared__ __attribute__((aligned(16))) uint8_t panel[2][COF_SLOTS][COF_ROWS];
    __shared__ __attribute__((aligned(16))) v4i ftab[COF_TAB];
    const int64_t TR = ccg_cdiv(r1 - r0, COF_BM);
    int64_t I, J;
    if (!cof_tile_of(blockIdx.x, TR, TC, I0, MODE != COF_RECT, I, J)) return;
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

    // Stage loader: dword p of the panel = (slot c, row dword rd) of E; rows
    // past Npad read the last dword (their outputs are masked in the
    // epilogue).  Every value loaded in an iteration is first used at that
    // iteration's commit, after the stage's MFMAs.
    unsigned pf[LOADS];
    auto issue = [&](int st) {
        const uint8_t* Es = E + (int64_t)st * COF_SLOTS * Npad;
#pragma unroll
        for (int i = 0; i < LOADS; ++i) {
            const int p = i * 256 + tid;
            const int c = p / ROWD, rd = p - c * ROWD;
            int64_t row = rd < COF_BM / 4 ? rowA0 + 4 * rd : rowB0 + 4 * (rd - COF_BM / 4);
            row = row + 4 <= Npad ? row : Npad - 4;
            pf[i] = *reinterpret_cast<const unsigned*>(Es + c * Npad + row);
        }
    };
    auto commit = [&](int bb) {
#pragma unroll
        for (int i = 0; i < LOADS; ++i) reinterpret_cast<unsigned*>(&panel[bb][0][0])[i * 256 + tid] = pf[i];
    };
    for (int x = tid; x < COF_TAB; x += 256) ftab[x] = cof_ftab_entry(x);
    if (nstage > 0) {
        issue(0);
        commit(0);
    }
    __syncthreads();
    const int ra = wr * 64 + (lane & 31);            // A rows ra, ra + 32 (panel rows 0..127)
    const int rb = COF_BM + wc * 128 + (lane & 31);  // B rows rb + 32*ni
    const int h = lane >> 5;                         // K-step q: lanes of half h take slot 2q + h
    for (int st = 0; st < nstage; ++st) {
        const int bb = st & 1;
        if (st + 1 < nstage) issue(st + 1);
        // software pipeline over the stage's K-steps: entries of step q+2 and
        // the fragment-table reads of step q+1 are in flight while the MFMAs
        // of step q run
        constexpr int QN = COF_SLOTS / 2;
        int ent[2][6];
        auto read_entries = [&](int q, int (&L)[6]) {
            const uint8_t* col = &panel[bb][2 * q + h][0];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) L[mi] = col[ra + 32 * mi];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) L[2 + ni] = col[rb + 32 * ni];
        };
        v4i fr[2][6];
        // the type of slot 2q + h picks its table: ftab + 81 * type
        const unsigned long long tm = tmask[st];
        auto read_frags = [&](int q, const int (&L)[6], v4i (&F)[6]) {
            const v4i* tb = ftab + 81 * (int)((tm >> (4 * q + 2 * h)) & 3);
#pragma unroll
            for (int x = 0; x < 6; ++x) F[x] = tb[L[x]];
        };
        read_entries(0, ent[0]);
        read_entries(1, ent[1]);
        read_frags(0, ent[0], fr[0]);
#pragma unroll
        for (int q = 0; q < QN; ++q) {
            const int cur = q & 1;
            if (q + 2 < QN) read_entries(q + 2, ent[cur]);
            if (q + 1 < QN) read_frags(q + 1, ent[cur ^ 1], fr[cur ^ 1]);
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
    if constexpr (MODE == COF_CAND) {
        cof_cand_epilogue(acc, rowA0 + wr * 64, rowB0 + wc * 128, N, r1, cc);
        return;
    }
    // ---- epilogue: acc = co + 16384 * both (+ the previous chunks' counts).
    const int64_t base = r0 * N - r0 * (r0 + 1) / 2;
    if (MODE == COF_TRI && co && both && !co_prev && !dist) {
        // interior wave quarter (every column above every row, inside N and
        // the slab): one pointer per row and immediate column offsets, no
        // per-element masks or 64-bit offset arithmetic
        const int64_t ia0 = rowA0 + wr * 64, jb0 = rowB0 + wc * 128;
        if (jb0 > ia0 + 63 && jb0 + 128 <= N && ia0 + 64 <= r1) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t gi = ia0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int64_t o = gi * N - gi * (gi + 1) / 2 - gi - 1 - base + jb0 + (lane & 31);
                    uint16_t* pc = co + o;
                    uint16_t* pb = both + o;
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni) {
                        const int a = acc[mi][ni][r];
                        pc[32 * ni] = (uint16_t)(a & 16383);
                        pb[32 * ni] = (uint16_t)(a >> 14);
                    }
                }
            return;
        }
    }
    if (MODE == COF_RECT && !cb_prev) {
        // interior wave quarter of the full rows: one pointer per row, immediate column offsets
        const int64_t ia0 = rowA0 + wr * 64, jb0 = rowB0 + wc * 128;
        if (jb0 + 128 <= NB && ia0 + 64 <= r1) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t gi = ia0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    uint32_t* pr = cb + (gi - r0) * NB + jb0 + (lane & 31);
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni) {
                        const int a = acc[mi][ni][r];
                        pr[32 * ni] = (uint32_t)(a & 16383) | ((uint32_t)(a >> 14) << 16);
                    }
                }
            return;
        }
    }
    // Loops run row-major (mi, r outer) so each of a lane's 32 rows computes
    // its packed-triangle offset once for its 4 column groups (the 64-bit
    // offset arithmetic per element dominated the small-B epilogue).  Staging
    // 8-row groups through LDS for 256-byte row stores was measured slower
    // (25.9 against 22.6 ms at N = 100k, B = 125; 95.5 against 92.3 at B = 1000).
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t gi = rowA0 + wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const bool row_ok = gi < r1;
            // TRI: o = (row gi's start in the packed triangle) + (gj - gi - 1) - base
            const int64_t rb = MODE == COF_TRI ? gi * N - gi * (gi + 1) / 2 - gi - 1 - base : (gi - r0) * NB;
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int64_t gj = rowB0 + wc * 128 + ni * 32 + (lane & 31);
                const int a = acc[mi][ni][r];
                int cv = a & 16383, bv = a >> 14;
                if (MODE == COF_TRI) {
                    if (row_ok && gj < N && gj > gi) {
                        const int64_t o = rb + gj;
                        if (co_prev) {
                            cv += co_prev[o];
                            bv += both_prev[o];
                        }
                        if (co) co[o] = (uint16_t)cv;
                        if (both) both[o] = (uint16_t)bv;
                        if (dist) {
                            const float qv = (float)((double)cv / (double)bv);
                            dist[o] = 1.0 - (double)qv;
                        }
                    }
                } else {
                    if (row_ok && gj < NB) {
                        const int64_t o = rb + gj;
                        if (cb_prev) {
                            const uint32_t pv = cb_prev[o];
                            cv += (int)(pv & 0xFFFFu);
                            bv += (int)(pv >> 16);
                        }
                        cb[o] = (uint32_t)cv | ((uint32_t)bv << 16);
                    }
                }
            }
        }
}

// Launch state shared by the triangle and full-row drivers.
struct CofPlan {
    int* colC;
    int* ccol;
    int* nslot;
    int* desc;                  // 2 * maxslots halves
    unsigned long long* tmask;  // maxslots / COF_SLOTS stages
    int64_t maxslots;
    uint8_t* E;                 // entry matrix of the current chunk (maxslots x Npad bytes)
    int64_t Npad;               // rows per slot of E (N rounded up to 4)
    std::vector<int64_t> cuts;  // column chunks [cuts[c], cuts[c + 1])
};

// Column maxima, column chunks and table space.  A chunk has at most
// COF_CHUNK columns (the 14-bit co field) and an entry matrix of at most
// COF_EMAX bytes.  8-bit labels bound the halves by 32 (slots by 16) per column; when that
// bound does not fit (and always for 16-bit labels) the column maxima are
// read back once to size the chunks exactly.
static int cof_plan(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, hipStream_t st,
                    CofPlan* pl) {
    int* colC = (int*)ccg_ws(ctx, WS_COC_A, sizeof(int) * (B + 8));
    if (!colC) return CCG_ENOMEM;
    CCG_HIP(hipMemsetAsync(colC, 0, sizeof(int) * B, st));
    const dim3 g((unsigned)std::min<int64_t>(ccg_cdiv(N, 256), 64), (unsigned)B);
    if (label_bits == 8) coc_colmax_kernel<uint8_t><<<g, 256, 0, st>>>((const uint8_t*)A, N, colC);
    else coc_colmax_kernel<uint16_t><<<g, 256, 0, st>>>((const uint16_t*)A, N, colC);
    CCG_HIP(hipGetLastError());
    const int64_t Npad = (N + 3) / 4 * 4;
    const int64_t Bc = std::min<int64_t>(B, COF_CHUNK);
    pl->cuts.clear();
    int64_t maxslots = Bc * 16 + COF_SLOTS;
    if (label_bits == 8 && maxslots * Npad <= COF_EMAX) {
        for (int64_t c0 = 0; c0 < B; c0 += COF_CHUNK) pl->cuts.push_back(c0);
        pl->cuts.push_back(B);
    } else {
        std::vector<int> h(B);
        CCG_HIP(hipMemcpyAsync(h.data(), colC, sizeof(int) * B, hipMemcpyDeviceToHost, st));
        CCG_HIP(hipStreamSynchronize(st));
        const int64_t cap = 2 * std::max<int64_t>(COF_EMAX / Npad - COF_SLOTS, 4097);  // halves per chunk
        int64_t s = 0, worst = 0, c0 = 0;
        pl->cuts.push_back(0);
        for (int64_t b = 0; b < B; ++b) {
            const int64_t v = h[b] > 0 ? (h[b] + 8) / 8 : 0;
            if (b > c0 && (b - c0 == COF_CHUNK || s + v > cap)) {
                pl->cuts.push_back(b);
                worst = std::max(worst, s);
                s = 0;
                c0 = b;
            }
            s += v;
        }
        pl->cuts.push_back(B);
        maxslots = (std::max(worst, s) + 1) / 2 + COF_SLOTS;
    }
    const int64_t nstg = maxslots / COF_SLOTS + 1;
    unsigned long long* ftm = (unsigned long long*)ccg_ws(
        ctx, WS_COC_B, sizeof(unsigned long long) * nstg + sizeof(int) * (Bc + 8 + 2 * maxslots));
    if (!ftm) return CCG_ENOMEM;
    int* ft = (int*)(ftm + nstg);
    uint8_t* E = (uint8_t*)ccg_ws(ctx, WS_COC_G, (size_t)(maxslots * Npad));
    if (!E) return CCG_ENOMEM;
    pl->colC = colC;
    pl->ccol = ft;
    pl->nslot = ft + Bc;
    pl->desc = pl->nslot + 8;
    pl->tmask = ftm;
    pl->maxslots = maxslots;
    pl->E = E;
    pl->Npad = Npad;
    return CCG_OK;
}

// One column chunk [cb0, cb0 + Bc): slot tables, entry matrix, GEMM tiles.
template <int MODE>
static void cof_launch(int label_bits, const void* A, int64_t cb0, int64_t Bc, int64_t N, int64_t r0, int64_t r1,
                       int64_t TC, int64_t I0, int64_t ntiles, const CofPlan& pl, const uint16_t* co_prev,
                       const uint16_t* both_prev, uint16_t* co, uint16_t* both, double* dist, const uint32_t* cb_prev,
                       uint32_t* cb, hipStream_t st, int64_t NB = 0, const CofCand& cc = CofCand{},
                       bool prepared = false) {
    if (!prepared) {  // (prepared: the chunk's slot tables and entry matrix are in pl from an earlier launch)
    cof_slots_kernel<<<1, 1024, 0, st>>>(pl.colC + cb0, Bc, pl.ccol, pl.nslot, pl.desc, pl.tmask);
    const dim3 eg((unsigned)std::min<int64_t>(ccg_cdiv(pl.Npad / 4, 256), 128),
                  (unsigned)std::min<int64_t>(pl.maxslots, COF_ENT_GRID));
    if (label_bits == 8)
        cof_entries_kernel<uint8_t><<<eg, 256, 0, st>>>((const uint8_t*)A + cb0 * N, N, pl.Npad, pl.desc, pl.ccol,
                                                        pl.nslot, pl.E);
    else
        cof_entries_kernel<uint16_t><<<eg, 256, 0, st>>>((const uint16_t*)A + cb0 * N, N, pl.Npad, pl.desc, pl.ccol,
                                                         pl.nslot, pl.E);
    }
    cof_tile_kernel<MODE><<<(unsigned)cof_tile_blocks(ccg_cdiv(r1 - r0, COF_BM), TC, I0, MODE != COF_RECT), 256, 0,
                            st>>>(pl.E, pl.Npad, N, r0, r1, TC, I0, pl.nslot, pl.tmask, co_prev,
                                                            both_prev, co, both, dist, cb_prev, cb, NB ? NB : N, cc);
}

extern "C" int ccg_cocluster_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, int64_t r0,
                                 int64_t r1, uint16_t* co, uint16_t* both, double* dist, void* stream) {
    CCG_REQUIRE(ctx && A, "ccg_cocluster_dev: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_cocluster_dev: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && N < (1LL << 31), "ccg_cocluster_dev: bad N");
    CCG_REQUIRE(B >= 1 && B <= 65535, "ccg_cocluster_dev: B=%lld must be in [1, 65535] (uint16 counts)",
                (long long)B);
    CCG_REQUIRE(r0 >= 0 && r0 <= r1 && r1 <= N, "ccg_cocluster_dev: bad row range");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    if (r1 == r0) return CCG_OK;
    CCG_REQUIRE(r0 % CCG_COCLUSTER_ROW_ALIGN == 0, "ccg_cocluster_dev: r0 must be a multiple of %d",
                CCG_COCLUSTER_ROW_ALIGN);
    CofPlan pl;
    int rc = cof_plan(ctx, A, label_bits, N, B, st, &pl);
    if (rc) return rc;
    const int64_t TC = ccg_cdiv(N, COF_BN);
    const int64_t I0 = r0 / COF_BM;
    const int64_t TR = ccg_cdiv(r1 - r0, COF_BM);
    auto fl = [](int64_t x) { return (x / 2) * (x / 2 - 1) + ((x & 1) ? x / 2 : 0); };
    const int64_t ntiles = TR * TC - (fl(I0 + TR) - fl(I0));
    CCG_REQUIRE(cof_tile_blocks(TR, TC, I0, true) < (1LL << 31), "ccg_cocluster_dev: too many tiles");
    const int64_t nch = (int64_t)pl.cuts.size() - 1;
    uint16_t *pco = co, *pboth = both;  // partial counts between chunks
    if (nch > 1 && (!co || !both)) {
        const int64_t P = (r1 - r0) * N - (r1 * (r1 + 1) - r0 * (r0 + 1)) / 2;
        uint16_t* scr = (uint16_t*)ccg_ws(ctx, WS_COC_C, sizeof(uint16_t) * 2 * P);
        if (!scr) return CCG_ENOMEM;
        if (!pco) pco = scr;
        if (!pboth) pboth = scr + P;
    }
    const int t_k = ccg_timer_start(ctx, CCG_KT_COCLUSTER, st);
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t cb0 = pl.cuts[c], Bc = pl.cuts[c + 1] - cb0;
        const bool last = c == nch - 1;
        cof_launch<COF_TRI>(label_bits, A, cb0, Bc, N, r0, r1, TC, I0, ntiles, pl, c ? pco : nullptr,
                            c ? pboth : nullptr, nch > 1 ? pco : co, nch > 1 ? pboth : both, last ? dist : nullptr,
                            nullptr, nullptr, st);
    }
    ccg_timer_stop(ctx, t_k, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// Rows [r0, r1) x columns [0, NB) of (co, both), packed co | both << 16 into
// cb[(i - r0) * NB + j] (diagonal included; NB = N: full rows).  Used by the
// consensus kNN on a row slab so the N x N matrix never exists.
static int ccg_cocluster_rows_packed(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, int64_t r0,
                              int64_t r1, uint32_t* cb, hipStream_t st, int64_t NB = 0) {
    if (!NB) NB = N;
    CofPlan pl;
    int rc = cof_plan(ctx, A, label_bits, N, B, st, &pl);
    if (rc) return rc;
    const int64_t TC = ccg_cdiv(NB, COF_BN);
    const int64_t I0 = r0 / COF_BM;
    const int64_t TR = ccg_cdiv(r1 - r0, COF_BM);
    const int64_t ntiles = TR * TC;
    CCG_REQUIRE(cof_tile_blocks(TR, TC, I0, false) < (1LL << 31), "ccg_cocluster_rows: too many tiles");
    const int64_t nch = (int64_t)pl.cuts.size() - 1;
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t cb0 = pl.cuts[c], Bc = pl.cuts[c + 1] - cb0;
        cof_launch<COF_RECT>(label_bits, A, cb0, Bc, N, r0, r1, TC, I0, ntiles, pl, nullptr, nullptr, nullptr, nullptr,
                             nullptr, c ? cb : nullptr, cb, st, NB);
    }
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------ consensus kNN --
// dbscan::kNN(jaccardDist, k)$id (R/consensusClust.R:425): per row, the k
// smallest D = 1 - (double)(float)(co / both) over j != i, ties by ascending
// j (R's stable order()); NaN (both == 0) makes dbscan stop().  Ascending D
// is descending fp32 similarity, so the kernels rank by (sim desc, j asc).
// One wave per row: lane l scans j = l, l + 64, ... (ascending per lane, so
// an equal value never displaces an earlier j) into a sorted register list;
// the 64 lists are merged by k rounds of wave arg-max.
#define CKNN_K 32
// (KL: the per-lane list length; any KL >= k gives the same top k -- no
// lane holds more than k of them)
template <int KL = CKNN_K>
__device__ __forceinline__ void cknn_insert(float (&lv)[KL], int (&li)[KL], float s, int j) {
    float cv = s;
    int ci = j;
#pragma unroll
    for (int t = 0; t < KL; ++t) {
        const bool sw = (cv > lv[t]) || (cv == lv[t] && ci < li[t]);
        const float tv = lv[t];
        const int ti = li[t];
        lv[t] = sw ? cv : tv;
        li[t] = sw ? ci : ti;
        cv = sw ? tv : cv;
        ci = sw ? ti : ci;
    }
}

template <int KL = CKNN_K>
__device__ __forceinline__ void cknn_merge_out(float (&lv)[KL], int (&li)[KL], int k, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
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
        if (lane == 0) out[r] = bi;
        if (li[0] == bi) {
#pragma unroll
            for (int t = 0; t < KL - 1; ++t) {
                lv[t] = lv[t + 1];
                li[t] = li[t + 1];
            }
            lv[KL - 1] = -INFINITY;
            li[KL - 1] = 0x7fffffff;
        }
    }
}

// From the packed triangle (co/both of the whole matrix).  Columns j < i come
// from column i of the triangle (strided reads); the slab path below reads
// rows only.
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
        cknn_insert(lv, li, s, (int)j);
    }
    if (__any(sawnan) && lane == 0) atomicOr(nan_flag, 1);
    cknn_merge_out(lv, li, k, out + i * k);
}

// From full rows cb[(i - r0) * N + j] = co | both << 16 (rows [r0, r1)).
__global__ __launch_bounds__(256) void consensus_knn_rows_kernel(const uint32_t* __restrict__ cb, int64_t N,
                                                                 int64_t r0, int64_t r1, int k,
                                                                 int32_t* __restrict__ out,
                                                                 int* __restrict__ nan_flag) {
    const int lane = threadIdx.x & 63;
    const int64_t i = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= r1) return;
    const uint32_t* row = cb + (i - r0) * N;
    float lv[CKNN_K];
    int li[CKNN_K];
#pragma unroll
    for (int t = 0; t < CKNN_K; ++t) {
        lv[t] = -INFINITY;
        li[t] = 0x7fffffff;
    }
    bool sawnan = false;
    for (int64_t j0 = 0; j0 < N; j0 += 256) {
        uint32_t v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t j = j0 + 64 * e + lane;
            v[e] = j < N ? row[j] : 0u;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t j = j0 + 64 * e + lane;
            if (j >= N || j == i) continue;
            const unsigned c = v[e] & 0xFFFFu, u = v[e] >> 16;
            if (u == 0) {
                sawnan = true;
                continue;
            }
            const float s = (float)((double)c / (double)u);
            if (!(s > lv[CKNN_K - 1])) continue;
            cknn_insert(lv, li, s, (int)j);
        }
    }
    if (__any(sawnan) && lane == 0) atomicOr(nan_flag, 1);
    cknn_merge_out(lv, li, k, out + i * k);
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

// ---------------------------- fused consensus kNN, triangle + candidates --
// For the whole matrix at once (rows [0, N), B <= COF_CHUNK): rows are
// visited in a fixed pseudo-random order p -> orig(p) = (p pmul + padd) mod N
// (the assignment columns permuted once), so the first CKC_SAMPLE positions
// are a spread sample of cells.
//   1. thresholds: per row, the k-th largest similarity over the sampled
//      columns (full rows against them, CKC_SAMPLE-wide) -- a lower bound of
//      the row's true k-th largest, so its k nearest all score at or above it;
//   2. the packed triangle once (half the square's MFMA work), its epilogue
//      offering each pair to both rows that it may enter (COF_CAND);
//   3. per row, the exact fp32 similarities of its candidates, ordered (sim
//      desc, original column asc) -- dbscan's stable order() -- top k.
// A row with more than CKC_CAP candidates sends the call back to the
// sub-slab path (full rows; bounded workspace).
#ifndef CKC_SAMPLE
#define CKC_SAMPLE 4096
#endif
#define CKC_CAP 2048
#define CKC_MIN_N 32768

template <typename T>
__global__ void ckc_permute_kernel(const T* __restrict__ A, int64_t N, int64_t B, int64_t pmul, int64_t padd,
                                   T* __restrict__ Ap) {
    // a thread per position p: its source cell once, then every column b
    // (round 5 divided a flat index by N per element: a 64-bit software
    // division per byte)
    const uint64_t pinv = ~0ull / (uint64_t)N;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = ckc_mod((uint64_t)p * (uint64_t)pmul + (uint64_t)padd, N, pinv);
        for (int64_t b = blockIdx.y; b < B; b += gridDim.y) Ap[b * N + p] = A[b * N + o];
    }
}

// tnum[row] for rows [a, b): tnum / CKC_NBK is a lower bound of the k-th
// largest fp32 similarity over the sampled columns q != row with both > 0
// (-1, every pair, when fewer than k are usable).  One wave per row counts
// its sampled similarities into
// CKC_NBK buckets of width 1 / CKC_NBK in LDS (bucket of the approximate
// quotient c * rcp(u), within one bucket of the exact one), finds the bucket
// bk holding the k-th largest by a suffix count, and takes (bk - 1) /
// CKC_NBK: the k values at or above bucket bk are all >= that.  Round 4 kept
// a sorted 32-entry register list per lane (a 32-step insertion chain per
// value: 5.5 ms per call at N = 100k); the bound is now looser by at most
// 2 / CKC_NBK, a few more candidates per row.
__global__ __launch_bounds__(256) void ckc_tau_kernel(const uint32_t* __restrict__ cb, int64_t a, int64_t b,
                                                      int64_t NS, int k, int* __restrict__ tnum) {
    // two 16-bit bucket counts per LDS word (a row counts at most NS <= 2^16
    // values): 8 KB per wave instead of 16, so 5 blocks per CU instead of 2
    __shared__ __attribute__((aligned(16))) unsigned hist[4][CKC_NBK / 2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t row = a + (int64_t)blockIdx.x * 4 + wv;
    if (row >= b) return;  // (whole waves: the wave's LDS slice is its own)
    unsigned* h = hist[wv];
    constexpr int PB = CKC_NBK / 64;  // buckets per lane, lane l owning [l PB, (l + 1) PB)
    constexpr int PW = PB / 2;        // their words
#pragma unroll
    for (int i = 0; i < PW; i += 4) *reinterpret_cast<uint4*>(&h[lane * PW + i]) = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const uint32_t* r = cb + (row - a) * NS;
    int usable = 0;
    // (loads 8 at a time ahead of their LDS adds: one load per iteration was a
    // latency chain)
    constexpr int TU = 8;
    for (int64_t q0 = 0; q0 < NS; q0 += 64 * TU) {
        uint32_t v[TU];
#pragma unroll
        for (int t = 0; t < TU; ++t) {
            const int64_t q = q0 + 64 * t + lane;
            v[t] = q < NS ? r[q] : 0u;
        }
#pragma unroll
        for (int t = 0; t < TU; ++t) {
            const int64_t q = q0 + 64 * t + lane;
            const unsigned c = v[t] & 0xFFFFu, u = v[t] >> 16;
            if (q == row || u == 0) continue;  // (u == 0 also past NS)
            ++usable;
            const float s = (float)c * __builtin_amdgcn_rcpf((float)u);
            const int bk = min(CKC_NBK - 1, max(0, (int)(s * (float)CKC_NBK)));
            atomicAdd(&h[bk >> 1], (bk & 1) ? 0x10000u : 1u);
        }
    }
    for (int o = 32; o > 0; o >>= 1) usable += __shfl_xor(usable, o, 64);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // the lane holding the k-th largest: suffix sums of the lanes' bucket counts
    int mine = 0;
#pragma unroll
    for (int i = 0; i < PW; i += 4) {
        const uint4 hv = *reinterpret_cast<const uint4*>(&h[lane * PW + i]);
        const unsigned lo = (hv.x & 0xFFFFu) + (hv.y & 0xFFFFu) + (hv.z & 0xFFFFu) + (hv.w & 0xFFFFu);
        mine += (int)(lo + (hv.x >> 16) + (hv.y >> 16) + (hv.z >> 16) + (hv.w >> 16));
    }
    int suf = mine;  // inclusive suffix sum over lanes >= lane
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += y;
    }
    // the highest lane whose suffix reaches k (suffix sums fall with the lane)
    const unsigned long long reach = __ballot(suf >= k);
    int t = -1;  // (fewer than k usable: every pair with both > 0 qualifies)
    if (usable >= k && reach) {
        const int L = 63 - __clzll(reach);
        int bk = 0;
        if (lane == L) {
            int acc = suf - mine;  // values above this lane's buckets
            for (int i = PB - 1; i >= 0; --i) {
                const unsigned w = h[(lane * PB + i) >> 1];
                acc += (int)((i & 1) ? (w >> 16) : (w & 0xFFFFu));
                if (acc >= k) {
                    bk = lane * PB + i;
                    break;
                }
            }
        }
        bk = __shfl(bk, L, 64);
        t = bk >= 2 ? bk - 1 : -1;  // (<= 0: every co-sampled pair qualifies)
    }
    if (lane == 0) tnum[row] = t;
}

// Per permuted row (one wave): the row's candidates, exact fp32 similarity,
// top k by (sim desc, original column asc), written to the row's original
// position.
template <int KL>
__global__ __launch_bounds__(256) void ckc_select_kernel(const uint2* __restrict__ cand, const int* __restrict__ cnt,
                                                         int cap, int64_t N, int64_t pmul, int64_t padd, uint64_t pinv,
                                                         int k, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= N) return;
    const int n = min(cnt[p], cap);
    const uint2* c = cand + p * cap;
    float lv[KL];
    int li[KL];
#pragma unroll
    for (int t = 0; t < KL; ++t) {
        lv[t] = -INFINITY;
        li[t] = 0x7fffffff;
    }
    // (4 candidates' loads per lane issued together: one load per iteration
    // was a latency chain)
    for (int e0 = 0; e0 < n; e0 += 256) {
        uint2 vv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int e = e0 + 64 * t + lane;
            vv[t] = e < n ? c[e] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint2 v = vv[t];
            const unsigned co = v.y & 0xFFFFu, u = v.y >> 16;
            if (u == 0) continue;  // (past n: a candidate always has both > 0)
            // (the correctly rounded fp32 quotient: equal to (float)((double)co / u)
            // for operands below 2^24 -- double rounding is innocuous there)
            const float s = __fdiv_rn((float)co, (float)u);
            if (s < lv[KL - 1]) continue;  // (a tie with the list's last needs the original id)
            // the candidate's original column (the epilogue stores permuted positions)
            const int j = (int)ckc_mod((uint64_t)v.x * (uint64_t)pmul + (uint64_t)padd, N, pinv);
            if (s == lv[KL - 1] && j > li[KL - 1]) continue;
            cknn_insert<KL>(lv, li, s, j);
        }
    }
    const int64_t o = ckc_mod((uint64_t)p * (uint64_t)pmul + (uint64_t)padd, N, pinv);
    cknn_merge_out<KL>(lv, li, k, out + o * k);
}

static int64_t ckc_gcd(int64_t a, int64_t b) {
    while (b) {
        const int64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// Returns CCG_OK with *done = false when a row overflowed its candidate list
// (the caller then runs the sub-slab path); synchronises the stream once.
static int ckc_run(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, int k, int32_t* out_idx,
                   int32_t* d_nan_flag, hipStream_t st, bool* done) {
    *done = false;
    const size_t lb = label_bits / 8;
    const int64_t NS = std::min<int64_t>(CKC_SAMPLE, (N / 8) / COF_BN * COF_BN);
    int64_t pmul = (int64_t)(2654435761ull % (uint64_t)N);
    if (pmul < 2) pmul = 2;
    while (ckc_gcd(pmul, N) != 1) ++pmul;
    const int64_t padd = N / 3;
    void* Ap = ccg_ws(ctx, WS_COC_D, lb * (size_t)(B * N));
    uint2* cand = (uint2*)ccg_ws(ctx, WS_COC_E, sizeof(uint2) * (size_t)N * CKC_CAP);
    char* small = (char*)ccg_ws(ctx, WS_COC_F, sizeof(double) * N + sizeof(int) * (N + 64));
    if (!Ap || !cand || !small) return CCG_ENOMEM;
    int* tnum = (int*)small;
    int* cnt = tnum + N;
    int* flags = cnt + N;  // [0] both == 0 somewhere, [1] overflow
    const dim3 pg((unsigned)std::min<int64_t>(ccg_cdiv(N, 256), 1024), (unsigned)std::min<int64_t>(B, 64));
    if (label_bits == 8) ckc_permute_kernel<uint8_t><<<pg, 256, 0, st>>>((const uint8_t*)A, N, B, pmul, padd, (uint8_t*)Ap);
    else ckc_permute_kernel<uint16_t><<<pg, 256, 0, st>>>((const uint16_t*)A, N, B, pmul, padd, (uint16_t*)Ap);
    // one column plan and entry matrix for both GEMMs (the permuted columns,
    // one chunk; round 5 built them twice, 0.7 ms per call at N = 100k)
    CofPlan pl;
    int rc = cof_plan(ctx, Ap, label_bits, N, B, st, &pl);
    if (rc) return rc;
    if (pl.cuts.size() != 2) return CCG_OK;  // more than one column chunk: not done (the sub-slab path)
    // 1. thresholds, in row chunks of <= 2 GB of sampled similarities
    int64_t R = ((2LL << 30) / (4 * NS)) / COF_BM * COF_BM;
    R = std::max<int64_t>(R, COF_BM);
    uint32_t* cb = (uint32_t*)ccg_ws(ctx, WS_COC_C, sizeof(uint32_t) * (size_t)std::min(R, N) * NS);
    if (!cb) return CCG_ENOMEM;
    for (int64_t a = 0; a < N; a += R) {
        const int64_t b = std::min(N, a + R);
        const int64_t TCs = ccg_cdiv(NS, COF_BN), I0s = a / COF_BM, TRs = ccg_cdiv(b - a, COF_BM);
        CCG_REQUIRE(cof_tile_blocks(TRs, TCs, I0s, false) < (1LL << 31), "consensus kNN: too many tiles");
        cof_launch<COF_RECT>(label_bits, Ap, 0, B, N, a, b, TCs, I0s, TRs * TCs, pl, nullptr, nullptr, nullptr, nullptr,
                             nullptr, nullptr, cb, st, NS, CofCand{}, a > 0);
        ckc_tau_kernel<<<(unsigned)ccg_cdiv(b - a, 4), 256, 0, st>>>(cb, a, b, NS, k, tnum);
    }
    // 2. the triangle with the candidate epilogue
    CCG_HIP(hipMemsetAsync(cnt, 0, sizeof(int) * (N + 64), st));
    const int64_t TC = ccg_cdiv(N, COF_BN), TR = ccg_cdiv(N, COF_BM);
    auto fl = [](int64_t x) { return (x / 2) * (x / 2 - 1) + ((x & 1) ? x / 2 : 0); };
    const int64_t ntiles = TR * TC - fl(TR);
    CCG_REQUIRE(cof_tile_blocks(TR, TC, 0, true) < (1LL << 31), "consensus kNN: too many tiles");
    CofCand cc{tnum, cnt, cand, CKC_CAP, pmul, padd, ~0ull / (uint64_t)N, flags};
    cof_launch<COF_CAND>(label_bits, Ap, 0, B, N, 0, N, TC, 0, ntiles, pl, nullptr, nullptr, nullptr, nullptr, nullptr,
                         nullptr, nullptr, st, N, cc, true);
    CCG_HIP(hipGetLastError());
    int hf[2] = {0, 0};
    CCG_HIP(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (hf[1]) return CCG_OK;  // overflow: not done
    // 3. per-row selection
    // (per-lane lists of 20 for k <= 20 -- kNum's usual maximum -- instead of 32: a shorter insertion chain)
    const uint64_t pinv = ~0ull / (uint64_t)N;
    if (k <= 20)
        ckc_select_kernel<20><<<(unsigned)ccg_cdiv(N, 4), 256, 0, st>>>(cand, cnt, CKC_CAP, N, pmul, padd, pinv, k,
                                                                        out_idx);
    else
        ckc_select_kernel<CKNN_K><<<(unsigned)ccg_cdiv(N, 4), 256, 0, st>>>(cand, cnt, CKC_CAP, N, pmul, padd, pinv, k,
                                                                            out_idx);
    CCG_HIP(hipMemcpyAsync(d_nan_flag, flags, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    CCG_HIP(hipGetLastError());
    *done = true;
    return CCG_OK;
}

// Rows per sub-slab of the fused consensus kNN: bounded by the packed-row
// scratch (CKNN_SCRATCH bytes), a multiple of the co-cluster row tile.
#define CKNN_SCRATCH (4LL << 30)

extern "C" int ccg_consensus_knn_assign_dev(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B,
                                            int k, int64_t r0, int64_t r1, int32_t* out_idx, int32_t* d_nan_flag,
                                            void* stream) {
    CCG_REQUIRE(ctx && A && out_idx && d_nan_flag, "ccg_consensus_knn_assign_dev: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_consensus_knn_assign_dev: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && N < (1LL << 31) && B >= 1 && B <= 65535, "ccg_consensus_knn_assign_dev: bad sizes");
    CCG_REQUIRE(k >= 1 && k <= CKNN_K && k <= N - 1, "ccg_consensus_knn_assign_dev: need 1 <= k <= min(32, N-1)");
    CCG_REQUIRE(r0 >= 0 && r0 <= r1 && r1 <= N, "ccg_consensus_knn_assign_dev: bad row range");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    CCG_HIP(hipMemsetAsync(d_nan_flag, 0, sizeof(int32_t), st));
    if (r0 == r1) return CCG_OK;
    CCG_REQUIRE(r0 % CCG_COCLUSTER_ROW_ALIGN == 0, "ccg_consensus_knn_assign_dev: r0 must be a multiple of %d",
                CCG_COCLUSTER_ROW_ALIGN);
    const int t_k = ccg_timer_start(ctx, CCG_KT_COCLUSTER, st);
    const char* path = getenv("CCG_CKNN_PATH");  // tools/tests: "slab" forces the sub-slab path
    if (r0 == 0 && r1 == N && N >= CKC_MIN_N && B <= COF_CHUNK && !(path && !strcmp(path, "slab"))) {
        bool done = false;
        int rc = ckc_run(ctx, A, label_bits, N, B, k, out_idx, d_nan_flag, st, &done);
        if (rc) return rc;
        if (done) {
            ccg_timer_stop(ctx, t_k, st);
            return CCG_OK;
        }
        CCG_HIP(hipMemsetAsync(d_nan_flag, 0, sizeof(int32_t), st));
    }
    int64_t R = (CKNN_SCRATCH / (4 * N)) / COF_BM * COF_BM;
    R = std::max<int64_t>(R, COF_BM);
    R = std::min<int64_t>(R, ccg_cdiv(r1 - r0, COF_BM) * COF_BM);
    uint32_t* cb = (uint32_t*)ccg_ws(ctx, WS_COC_C, sizeof(uint32_t) * R * N);
    if (!cb) return CCG_ENOMEM;
    for (int64_t a = r0; a < r1; a += R) {
        const int64_t b = std::min(r1, a + R);
        int rc = ccg_cocluster_rows_packed(ctx, A, label_bits, N, B, a, b, cb, st);
        if (rc) return rc;
        consensus_knn_rows_kernel<<<(unsigned)ccg_cdiv(b - a, 4), 256, 0, st>>>(cb, N, a, b, k, out_idx,
                                                                                d_nan_flag);
    }
    ccg_timer_stop(ctx, t_k, st);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}

// ------------------------------------------------------- host flavours --
extern "C" int ccg_cocluster(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, uint16_t* co,
                             uint16_t* both, double* dist) {
    CCG_REQUIRE(ctx && A, "ccg_cocluster: NULL argument");
    CCG_REQUIRE(N >= 2 && B >= 1, "ccg_cocluster: bad sizes");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_cocluster: label_bits must be 8 or 16");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t P = N * (N - 1) / 2;
    const size_t abytes = (size_t)(B * N) * (label_bits / 8);
    void* dA = ccg_ws(ctx, WS_HOST_A, abytes);
    uint16_t* dco = co ? (uint16_t*)ccg_ws(ctx, WS_HOST_B, sizeof(uint16_t) * P) : nullptr;
    uint16_t* dboth = both ? (uint16_t*)ccg_ws(ctx, WS_HOST_C, sizeof(uint16_t) * P) : nullptr;
    double* ddist = dist ? (double*)ccg_ws(ctx, WS_HOST_D, sizeof(double) * P) : nullptr;
    if (!dA || (co && !dco) || (both && !dboth) || (dist && !ddist)) return CCG_ENOMEM;
    CCG_HIP(hipMemcpyAsync(dA, A, abytes, hipMemcpyHostToDevice, st));
    int rc = ccg_cocluster_dev(ctx, dA, label_bits, N, B, 0, N, dco, dboth, ddist, st);
    if (rc) return rc;
    if (co) CCG_HIP(hipMemcpyAsync(co, dco, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, st));
    if (both) CCG_HIP(hipMemcpyAsync(both, dboth, sizeof(uint16_t) * P, hipMemcpyDeviceToHost, st));
    if (dist) CCG_HIP(hipMemcpyAsync(dist, ddist, sizeof(double) * P, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    return CCG_OK;
}

extern "C" int ccg_consensus_knn_assign(ccg_ctx* ctx, const void* A, int label_bits, int64_t N, int64_t B, int k,
                                        int32_t* out_idx) {
    CCG_REQUIRE(ctx && A && out_idx, "ccg_consensus_knn_assign: NULL argument");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_consensus_knn_assign: label_bits must be 8 or 16");
    CCG_REQUIRE(N >= 2 && B >= 1 && k >= 1, "ccg_consensus_knn_assign: bad sizes");
    CCG_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t abytes = (size_t)(B * N) * (label_bits / 8);
    void* dA = ccg_ws(ctx, WS_HOST_A, abytes);
    int32_t* dout = (int32_t*)ccg_ws(ctx, WS_HOST_B, sizeof(int32_t) * N * k + 64);
    if (!dA || !dout) return CCG_ENOMEM;
    int32_t* dflag = dout + N * k;
    CCG_HIP(hipMemcpyAsync(dA, A, abytes, hipMemcpyHostToDevice, st));
    int rc = ccg_consensus_knn_assign_dev(ctx, dA, label_bits, N, B, k, 0, N, dout, dflag, st);
    if (rc) return rc;
    int flag = 0;
    CCG_HIP(hipMemcpyAsync(&flag, dflag, sizeof(int), hipMemcpyDeviceToHost, st));
    CCG_HIP(hipMemcpyAsync(out_idx, dout, sizeof(int32_t) * N * k, hipMemcpyDeviceToHost, st));
    CCG_HIP(hipStreamSynchronize(st));
    if (flag) {
        ccg_set_error("ccg_consensus_knn_assign: data/distances cannot contain NAs (a pair was never co-sampled)");
        return CCG_ENAN;
    }
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
