// The co-cluster GEMM with 128 x 128 wave tiles (round 6).
//
// Same problem as cof_tile_kernel (cocluster.hip): acc = co + 16384 both over
// the entry matrix E of a column chunk, K-steps of v_mfma_i32_32x32x32_i8
// whose 16-byte fragments come from the LDS pattern table (R/consensusClust.R
// :411-421, customDist).  cof_tile_kernel gives each wave 64 x 128 outputs:
// per K-step 6 entry bytes and 6 table reads (ds_read_b128) for 8 MFMAs, and
// at 8 waves per CU the fragment reads took more LDS cycles than the MFMAs
// leave (PMC: 8.5e8 LDS instructions and 7.2e8 bank-conflict cycles per
// launch at N = 100k, B = 125; MFMA busy ~0.6).  Here a block is 256 x 256
// outputs and each of its 4 waves 128 x 128: per K-step 8 entry bytes and 8
// table reads for 16 MFMAs -- half the LDS work per MFMA.  The 256 int32
// accumulators per lane live in AGPRs (this file is built without the
// VGPR-form MFMA flag), so a SIMD holds one wave; the stage's global loads
// are issued a stage ahead and the table reads a K-step ahead.
#include "cocluster_common.h"

#define CW_B 256                 // rows and columns of a block tile
#define CW_ROWS (2 * CW_B)       // staged rows per slot (A panel then B panel)
#define CW_ST 8                  // supertile side (tiles)

// First column tile of a row tile starting at rowA0 that holds a pair j > i.
__host__ __device__ inline int64_t cw_jlo(int64_t rowA0, bool tri) { return tri ? (rowA0 + 1) / CW_B : 0; }

// Supertiles of CW_ST x CW_ST tiles: row group g (row tiles CW_ST g ..) and
// column tiles from the group's first row tile's jlo; supertile S on XCD
// S mod 8, its 64 tiles that XCD's consecutive blocks (cof_tile_of's order).
__host__ __device__ inline int64_t cw_supertiles_row(int64_t g, int64_t TC, int64_t r0, bool tri) {
    const int64_t jlo = cw_jlo(r0 + CW_ST * g * CW_B, tri);
    return jlo < TC ? (TC - jlo + CW_ST - 1) / CW_ST : 0;
}
static int64_t cw_blocks(int64_t TR, int64_t TC, int64_t r0, bool tri) {
    int64_t ns = 0;
    for (int64_t g = 0; g < (TR + CW_ST - 1) / CW_ST; ++g) ns += cw_supertiles_row(g, TC, r0, tri);
    return 8 * (int64_t)CW_ST * CW_ST * ((ns + 7) / 8);
}
__device__ __forceinline__ bool cw_tile_of(int64_t b, int64_t TR, int64_t TC, int64_t r0, bool tri, int64_t& Ir,
                                           int64_t& J) {
    const int64_t k = b >> 3;
    const int64_t S = (k / (CW_ST * CW_ST)) * 8 + (b & 7);
    const int slot = (int)(k % (CW_ST * CW_ST));
    const int64_t G = (TR + CW_ST - 1) / CW_ST;
    int64_t g = 0, cum = 0;
    for (; g < G; ++g) {  // (block-uniform scalar loop)
        const int64_t n = cw_supertiles_row(g, TC, r0, tri);
        if (S < cum + n) break;
        cum += n;
    }
    if (g == G) return false;
    Ir = CW_ST * g + slot / CW_ST;
    J = cw_jlo(r0 + CW_ST * g * CW_B, tri) + CW_ST * (S - cum) + slot % CW_ST;
    return Ir < TR && J < TC && J >= cw_jlo(r0 + Ir * CW_B, tri);
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void cof_wide_kernel(
    const uint8_t* __restrict__ E, int64_t Npad, int64_t N, int64_t r0, int64_t r1, int64_t TC,
    const int* __restrict__ nslot_p, const unsigned long long* __restrict__ tmask, const uint16_t* co_prev,
    const uint16_t* both_prev, uint16_t* co, uint16_t* both, double* __restrict__ dist, const uint32_t* cb_prev,
    uint32_t* cb, int64_t NB) {
    constexpr int ROWD = CW_ROWS / 4;              // dwords per staged slot
    constexpr int LOADS = COF_SLOTS * ROWD / 256;  // dwords per thread per stage
    __shared__ __attribute__((aligned(16))) uint8_t panel[2][COF_SLOTS][CW_ROWS];
    __shared__ __attribute__((aligned(16))) v4i ftab[COF_TAB];
    // the masked epilogue's per-wave transpose slices (32 rows x 128 columns
    // each): the registers are read with constant indices only (an
    // element loop over the accumulators put the whole array in scratch).
    // One block per CU (the accumulators), so LDS is not the limit.
    __shared__ __attribute__((aligned(16))) int eslice[4][32 * 128];
    const int64_t TR = ccg_cdiv(r1 - r0, CW_B);
    int64_t Ir, J;
    if (!cw_tile_of(blockIdx.x, TR, TC, r0, MODE == COF_TRI, Ir, J)) return;
    const int64_t rowA0 = r0 + Ir * CW_B, rowB0 = J * CW_B;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int nstage = *nslot_p / COF_SLOTS;

    v16i acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0;

    // stage loader: dword p of the panel = (slot c, row dword rd) of E; rows
    // past Npad read the last dword (their outputs are masked)
    unsigned pf[LOADS];
    auto issue = [&](int st) {
        const uint8_t* Es = E + (int64_t)st * COF_SLOTS * Npad;
#pragma unroll
        for (int i = 0; i < LOADS; ++i) {
            const int p = i * 256 + tid;
            const int c = p / ROWD, rd = p - c * ROWD;
            int64_t row = rd < CW_B / 4 ? rowA0 + 4 * rd : rowB0 + 4 * (rd - CW_B / 4);
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
    const int ra = wr * 128 + (lane & 31);         // A rows ra + 32 mi (panel rows 0..255)
    const int rb = CW_B + wc * 128 + (lane & 31);  // B rows rb + 32 ni
    const int h = lane >> 5;                       // K-step q: lanes of half h take slot 2q + h
    for (int st = 0; st < nstage; ++st) {
        const int bb = st & 1;
        if (st + 1 < nstage) issue(st + 1);
        constexpr int QN = COF_SLOTS / 2;
        int ent[2][8];
        auto read_entries = [&](int q, int (&L)[8]) {
            const uint8_t* col = &panel[bb][2 * q + h][0];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) L[mi] = col[ra + 32 * mi];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) L[4 + ni] = col[rb + 32 * ni];
        };
        v4i fr[2][8];
        const unsigned long long tm = tmask[st];
        auto read_frags = [&](int q, const int (&L)[8], v4i (&F)[8]) {
            const v4i* tb = ftab + 81 * (int)((tm >> (4 * q + 2 * h)) & 3);
#pragma unroll
            for (int x = 0; x < 8; ++x) F[x] = tb[L[x]];
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
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] =
                        __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[cur][mi], fr[cur][4 + ni], acc[mi][ni], 0, 0, 0);
        }
        if (st + 1 < nstage) {
            __syncthreads();  // every wave is done with buffer bb^1 (read in stage st-1)
            commit(bb ^ 1);
            __syncthreads();
        }
    }
    // ---- epilogue: acc = co + 16384 * both (+ the previous chunks' counts);
    // lane (h, col) holds rows ia0 + 32 mi + (r & 3) + 8 (r >> 2) + 4 h
    // against column jb0 + 32 ni + col
    const int64_t ia0 = rowA0 + wr * 128, jb0 = rowB0 + wc * 128;
    const int64_t base = r0 * N - r0 * (r0 + 1) / 2;
    if (MODE == COF_TRI && co && both && !co_prev && !dist) {
        if (jb0 > ia0 + 127 && jb0 + 128 <= N && ia0 + 128 <= r1) {  // interior quarter: no masks
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
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
        if (jb0 + 127 <= ia0) return;  // a quarter wholly below the diagonal (diagonal tiles)
    }
    if (MODE == COF_RECT && !cb_prev && jb0 + 128 <= NB && ia0 + 128 <= r1) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
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
    // masked quarters (edges, the diagonal, chunked columns, distances):
    // each 32-row slice goes through the wave's LDS slice, then a runtime
    // loop stores it row-major (consecutive lanes on consecutive columns)
    int* sl = eslice[wv];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                sl[((r & 3) + 8 * (r >> 2) + 4 * h) * 128 + 32 * ni + (lane & 31)] = acc[mi][ni][r];
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        for (int e = 0; e < 64; ++e) {
            const int idx = e * 64 + lane;
            const int64_t gi = ia0 + 32 * mi + (idx >> 7), gj = jb0 + (idx & 127);
            const int a = sl[idx];
            int cv = a & 16383, bv = a >> 14;
            if (MODE == COF_TRI) {
                if (gi < r1 && gj < N && gj > gi) {
                    const int64_t o = gi * N - gi * (gi + 1) / 2 - gi - 1 - base + gj;
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
                if (gi < r1 && gj < NB) {
                    const int64_t o = (gi - r0) * NB + gj;
                    if (cb_prev) {
                        const uint32_t pv = cb_prev[o];
                        cv += (int)(pv & 0xFFFFu);
                        bv += (int)(pv >> 16);
                    }
                    cb[o] = (uint32_t)cv | ((uint32_t)bv << 16);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");  // the slice is rewritten by the next mi
    }
}

int64_t cof_wide_blocks(int64_t N, int64_t r0, int64_t r1, int64_t NB, bool tri) {
    return cw_blocks(ccg_cdiv(r1 - r0, CW_B), ccg_cdiv(tri ? N : NB, CW_B), r0, tri);
}

void cof_wide_launch(int mode, const uint8_t* E, int64_t Npad, int64_t N, int64_t r0, int64_t r1, int64_t NB,
                     const int* nslot, const unsigned long long* tmask, const uint16_t* co_prev,
                     const uint16_t* both_prev, uint16_t* co, uint16_t* both, double* dist, const uint32_t* cb_prev,
                     uint32_t* cb, hipStream_t st) {
    const bool tri = mode == COF_TRI;
    const int64_t TC = ccg_cdiv(tri ? N : NB, CW_B);
    const unsigned nb = (unsigned)cof_wide_blocks(N, r0, r1, NB, tri);
    if (tri)
        cof_wide_kernel<COF_TRI><<<nb, 256, 0, st>>>(E, Npad, N, r0, r1, TC, nslot, tmask, co_prev, both_prev, co,
                                                     both, dist, cb_prev, cb, NB);
    else
        cof_wide_kernel<COF_RECT><<<nb, 256, 0, st>>>(E, Npad, N, r0, r1, TC, nslot, tmask, co_prev, both_prev, co,
                                                      both, dist, cb_prev, cb, NB);
}
