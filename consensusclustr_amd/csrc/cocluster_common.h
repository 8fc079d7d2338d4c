// Co-cluster constants and the fragment-table entry (cocluster.hip).
// Internal, not part of the ABI.
#pragma once
#include "ccg_internal.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#ifndef COF_SLOTS
#define COF_SLOTS 32        // slots per stage (16 K-steps of v_mfma_i32_32x32x32_i8)
#endif
#define COF_TAB (4 * 81)    // fragment tables: 4 slot types x 81 entries of 16 B
#define COF_TRI 0
#define COF_RECT 1
#define COF_CAND 2  // packed-triangle tiles whose epilogue appends consensus-kNN candidates

// Fragment table entry x = type * 81 + sigma_lo + 9 sigma_hi (cocluster.hip,
// "fused one-hot path"): the 16 bytes of one slot (two 8-byte halves) for a
// row whose half states are sigma_lo / sigma_hi.
__device__ __forceinline__ v4i cof_ftab_entry(int x) {
    const int ty = x / 81, en = x - ty * 81;
    int w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {  // half hf: dwords 2 hf, 2 hf + 1
        const int sg = hf ? en / 9 : en % 9;
        const bool first = (ty >> hf) & 1;
        if (sg >= 1 && first) w[2 * hf] |= 0x80;  // the flag
        const int ob = first ? (sg >= 2 ? sg - 1 : -1) : sg - 1;  // one-hot byte
        if (ob >= 0) w[2 * hf + (ob >> 2)] |= 1 << (8 * (ob & 3));
    }
    return (v4i){w[0], w[1], w[2], w[3]};
}
