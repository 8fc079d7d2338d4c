// Per-bootstrap clustering selection and map-back to cells.
//
// Reference: getClustAssignments (R/consensusClust.R:650-692): robust score
// rules (:662-670), rank(scores, ties.method="first") / which(rank == max)
// (:684-686), assignments[match(cellOrder, names(assignments))] (:673),
// granular cbind of all clusterings (:688); NA -> -1 (:408) is encoded as 0
// in the uint8 assignment matrix; do.call(cbind, ...) (:404) = the column
// layout A[b][cell].
#include "ccg_internal.h"

// rank(ties.method="first") + which(rank == max): NaN scores rank last
// (highest) in order of appearance, so the last NaN wins; otherwise the last
// occurrence of the maximum wins.
__global__ void robust_choice_kernel(const double* __restrict__ means,
                                     const int32_t* __restrict__ nclust,
                                     const int32_t* __restrict__ minsize, int nb, int L,
                                     int min_size, int32_t* __restrict__ choice) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    int best = 0, last_nan = -1;
    double bestv = -INFINITY;
    for (int l = 0; l < L; ++l) {
        const int64_t t = (int64_t)b * L + l;
        double s;
        const bool big = minsize[t] > min_size;
        if (nclust[t] > 1 && big) s = means[t];
        else if (big) s = 0.0;
        else s = 0.15;
        if (isnan(s)) last_nan = l;
        else if (s >= bestv) {
            bestv = s;
            best = l;
        }
    }
    choice[b] = last_nan >= 0 ? last_nan : best;
}

__global__ void mapback_first_kernel(const int32_t* __restrict__ idx, int64_t n, int64_t N,
                                     int* __restrict__ first) {
    const int b = blockIdx.y;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int32_t c = idx[(int64_t)b * n + p];
    if (c >= 0 && c < N) atomicMin(&first[(int64_t)b * N + c], (int)p);
}

// Writes the chosen (robust) or every (granular) clustering's label of each
// cell's first copy; 0 = not sampled.  A label above the matrix's label width
// (255 for uint8, 65535 for uint16) or below 1 cannot be stored: the cell is
// written as 0 and CCG_DERR_LABEL_RANGE is raised (the host mirror raises
// ValueError on the same input), never a clamp that would merge clusters.
template <typename T>
__global__ void mapback_write_kernel(int mode, const int32_t* __restrict__ labels, int64_t n, int L,
                                     int64_t N, const int* __restrict__ first,
                                     const int32_t* __restrict__ choice, T* __restrict__ A,
                                     int64_t col0, int* __restrict__ err) {
    constexpr int LMAX = sizeof(T) == 1 ? 255 : 65535;
    const int b = blockIdx.y;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    const int f = first[(int64_t)b * N + c];
    const bool sampled = f < 0x7f7f7f7f;
    bool bad = false;
    const int l0 = mode == CCG_MODE_ROBUST ? choice[b] : 0;
    const int l1 = mode == CCG_MODE_ROBUST ? l0 + 1 : L;
    for (int l = l0; l < l1; ++l) {
        int lab = sampled ? labels[((int64_t)b * L + l) * n + f] : 0;
        if (sampled && (lab < 1 || lab > LMAX)) {
            bad = true;
            lab = 0;
        }
        const int64_t colx = mode == CCG_MODE_ROBUST ? col0 + b : col0 + (int64_t)b * L + l;
        A[colx * N + c] = (T)lab;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, CCG_DERR_LABEL_RANGE);
}

extern "C" int ccg_select_mapback_dev(ccg_ctx* ctx, int mode, const int32_t* labels,
                                      const int32_t* boot_idx, int64_t n, int nb, int L, int64_t N,
                                      const double* means, const int32_t* nclust,
                                      const int32_t* minsize, int min_size, void* A, int label_bits,
                                      int64_t col0, int32_t* out_choice, void* stream) {
    CCG_REQUIRE(ctx && labels && boot_idx && A, "ccg_select_mapback_dev: NULL argument");
    CCG_REQUIRE(mode == CCG_MODE_ROBUST || mode == CCG_MODE_GRANULAR, "ccg_select_mapback_dev: bad mode");
    CCG_REQUIRE(label_bits == 8 || label_bits == 16, "ccg_select_mapback_dev: label_bits must be 8 or 16");
    CCG_REQUIRE(n >= 1 && nb >= 1 && L >= 1 && N >= 1, "ccg_select_mapback_dev: bad sizes");
    CCG_REQUIRE(mode == CCG_MODE_GRANULAR || (means && nclust && minsize),
                "ccg_select_mapback_dev: robust mode needs means/nclust/minsize");
    hipStream_t st = ccg_pick_stream(ctx, stream);
    int* first = (int*)ccg_ws(ctx, WS_MAP_A, sizeof(int) * (size_t)nb * N + sizeof(int32_t) * nb + 64);
    if (!first) return CCG_ENOMEM;
    int32_t* choice = out_choice ? out_choice : (int32_t*)(first + (size_t)nb * N);
    CCG_HIP(hipMemsetAsync(first, 0x7f, sizeof(int) * (size_t)nb * N, st));
    if (mode == CCG_MODE_ROBUST)
        robust_choice_kernel<<<(unsigned)ccg_cdiv(nb, 64), 64, 0, st>>>(means, nclust, minsize, nb, L,
                                                                       min_size, choice);
    mapback_first_kernel<<<dim3((unsigned)ccg_cdiv(n, 256), nb), 256, 0, st>>>(boot_idx, n, N, first);
    const dim3 g((unsigned)ccg_cdiv(N, 256), nb);
    if (label_bits == 8)
        mapback_write_kernel<uint8_t><<<g, 256, 0, st>>>(mode, labels, n, L, N, first, choice, (uint8_t*)A, col0,
                                                         ctx->d_err);
    else
        mapback_write_kernel<uint16_t><<<g, 256, 0, st>>>(mode, labels, n, L, N, first, choice, (uint16_t*)A, col0,
                                                          ctx->d_err);
    CCG_HIP(hipGetLastError());
    return CCG_OK;
}
