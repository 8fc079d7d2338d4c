// Device radix sort of (int32 key, int32 value) pairs for libccg (hipCUB).
// Used by the SNN host-list build: a stable sort of the kNN entries by
// neighbour keeps every host list in ascending host order.
#include <hipcub/hipcub.hpp>

#include "ccg_internal.h"

int ccg_sort_pairs_i32(ccg_ctx* ctx, const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                       int32_t* vals_out, int64_t n, int key_bits, hipStream_t st) {
    CCG_REQUIRE(n >= 0 && n < (1LL << 31), "ccg_sort_pairs_i32: n out of range");
    if (n == 0) return CCG_OK;
    size_t tmp = 0;
    CCG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                               key_bits, st));
    void* ws = ccg_ws(ctx, WS_SORT, tmp + 256);
    if (!ws) return CCG_ENOMEM;
    CCG_HIP(hipcub::DeviceRadixSort::SortPairs(ws, tmp, keys_in, keys_out, vals_in, vals_out, (int)n, 0, key_bits,
                                               st));
    return CCG_OK;
}
