// Probe of v_mfma_f64_4x4x4f64 on gfx950 (tools only): the operand / result
// lane layout and the issue rate against v_mfma_f64_16x16x4f64.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(double* out) {
    const int lane = threadIdx.x;
    // A = 100 * lane, B = 1 on one lane at a time is too many runs: instead
    // A(lane) = lane + 1, B(lane) = 1000 * (lane + 1); D = sum over k of A B
    // in each block, so each result names the lanes that fed it.
    double d = 0.0;
    for (int ka = 0; ka < 64; ++ka) {  // one nonzero A lane per pass, B all ones
        const double a = lane == ka ? 1.0 : 0.0;
        const double b = 1.0;
        const double r = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
        out[ka * 64 + lane] = r;  // which D lanes does A lane ka feed
    }
    for (int kb = 0; kb < 64; ++kb) {
        const double a = 1.0;
        const double b = lane == kb ? 1.0 : 0.0;
        const double r = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
        out[4096 + kb * 64 + lane] = r;  // which D lanes does B lane kb feed
    }
    (void)d;
}

__global__ void rate_kernel(long long* cyc, double* sink, int iters) {
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 2.0 - lane * 1e-3;
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c4, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c5, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c6, 0, 0, 0);
        c7 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c7, 0, 0, 0);
    }
    long long t1 = clock64();
    f64x4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
    for (int i = 0; i < iters; ++i) {
        e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
        e2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e2, 0, 0, 0);
        e3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e3, 0, 0, 0);
    }
    long long t2 = clock64();
    if (lane == 0) {
        cyc[blockIdx.x * 2 + 0] = (t1 - t0);  // 8 iters x 4x4x4
        cyc[blockIdx.x * 2 + 1] = (t2 - t1);  // 4 iters x 16x16x4
    }
    sink[blockIdx.x * 64 + lane] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + e0[0] + e1[1] + e2[2] + e3[3];
}

int main() {
    double* out;
    hipMalloc(&out, sizeof(double) * 8192);
    layout_kernel<<<1, 64>>>(out);
    double h[8192];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    for (int part = 0; part < 2; ++part) {
        printf("%s lane -> D lanes receiving it:\n", part ? "B" : "A");
        for (int k = 0; k < 64; ++k) {
            printf(" %2d:", k);
            for (int l = 0; l < 64; ++l)
                if (h[part * 4096 + k * 64 + l] != 0.0) printf(" %d", l);
            printf("\n");
        }
    }
    long long* cyc;
    double* sink;
    const int nb = 1;
    hipMalloc(&cyc, sizeof(long long) * 2 * nb);
    hipMalloc(&sink, sizeof(double) * 64 * nb);
    const int iters = 4096;
    rate_kernel<<<nb, 64>>>(cyc, sink, iters);
    long long hc[2];
    hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
    printf("one wave: 4x4x4 f64 %.2f clocks/instr, 16x16x4 f64 %.2f clocks/instr\n", (double)hc[0] / (8.0 * iters),
           (double)hc[1] / (4.0 * iters));
    return 0;
}
