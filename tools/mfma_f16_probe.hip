// mfma_f16_probe.hip -- checks, on gfx950, the pieces the split-f16 MFMA synthesis head uses:
//  * lane maps of v_mfma_f32_32x32x16_f16: A[m = l & 31][k = 8 (l >> 5) + j],
//    B[k = 8 (l >> 5) + j][n = l & 31], D register r of lane l = D[m = (r & 3) + 8 (r >> 2) + 4 (l >> 5)][n = l & 31];
//  * v_permlane32_swap: lanes 32..63 of the first operand trade places with lanes 0..31 of the second;
//  * the issue rate of the 32x32x16 f16 form (one wave per SIMD, independent accumulators);
//  * the error of hi/lo split products (Wh Xh + Wh Xl + Wl Xh, f32 accumulate) on random data.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f16_probe.hip -o tools/mfma_f16_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                                \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

// A (32 x 16) and B (16 x 32) row-major in global memory; D (32 x 32) row-major out.
__global__ void layout(const float *A, const float *B, float *D)
{
    const int l = threadIdx.x, h = l >> 5, r32 = l & 31;
    v8h a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)A[r32 * 16 + 8 * h + j];
        b[j] = (_Float16)B[(8 * h + j) * 32 + r32];
    }
    v16f c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + r32] = c[r];
}

__global__ void swap_probe(unsigned *out)
{
    const unsigned l = threadIdx.x;
    unsigned a = 1000 + l, b = 2000 + l;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[l] = r[0];
    out[64 + l] = r[1];
}

__global__ void rate(float *out, int iters)
{
    const int l = threadIdx.x;
    v8h a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)(1.f + l * 1e-3f);
        b[j] = (_Float16)(1.f - j * 1e-3f);
    }
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main()
{
    float hA[32 * 16], hB[16 * 32], hD[32 * 32];
    srand(1);
    for (int i = 0; i < 32 * 16; ++i) hA[i] = (float)(rand() % 17 - 8);
    for (int i = 0; i < 16 * 32; ++i) hB[i] = (float)(rand() % 13 - 6);
    float *dA, *dB, *dD;
    CHECK(hipMalloc(&dA, sizeof hA));
    CHECK(hipMalloc(&dB, sizeof hB));
    CHECK(hipMalloc(&dD, sizeof hD));
    CHECK(hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    CHECK(hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
            float s = 0.f;
            for (int k = 0; k < 16; ++k) s += hA[m * 16 + k] * hB[k * 32 + n];
            if (s != hD[m * 32 + n]) ++bad;
        }
    printf("mfma_f32_32x32x16_f16 lane map: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);

    unsigned *dS, hS[128];
    CHECK(hipMalloc(&dS, sizeof hS));
    hipLaunchKernelGGL(swap_probe, dim3(1), dim3(64), 0, 0, dS);
    CHECK(hipMemcpy(hS, dS, sizeof hS, hipMemcpyDeviceToHost));
    // expected: first result = a with lanes 32..63 replaced by b's lanes 0..31; second = b with
    // lanes 0..31 replaced by a's lanes 32..63
    int sb = 0;
    for (unsigned l = 0; l < 64; ++l) {
        const unsigned e0 = l < 32 ? 1000 + l : 2000 + (l - 32), e1 = l < 32 ? 1000 + l + 32 : 2000 + l;
        if (hS[l] != e0 || hS[64 + l] != e1) ++sb;
    }
    printf("permlane32_swap: %s (%d mismatches); lane 0/32: %u %u | %u %u\n", sb ? "FAIL" : "OK", sb, hS[0], hS[32],
           hS[64], hS[96]);

    const int blocks = 1024, iters = 20000;
    float *dout;
    CHECK(hipMalloc(&dout, sizeof(float) * 64 * blocks));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(rate, dim3(blocks), dim3(64), 0, 0, dout, iters);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(rate, dim3(blocks), dim3(64), 0, 0, dout, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = (double)blocks * iters * 4 * 32.0 * 32 * 16 * 2;
    printf("32x32x16_f16: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per wave\n", ms, flops / (ms * 1e-3) / 1e12,
           ms * 1e6 / ((double)iters * 4));

    // split-product error on random f32 data, 8-term dot products (the head's first layer)
    double worst = 0.0, worst_rel = 0.0;
    srand(7);
    for (int t = 0; t < 100000; ++t) {
        double exact = 0.0, split = 0.0, mag = 0.0;
        for (int k = 0; k < 8; ++k) {
            const float w = ((float)rand() / RAND_MAX - 0.5f) * 0.6f;
            const float x = ((float)rand() / RAND_MAX - 0.5f) * 80.f;
            const _Float16 wh = (_Float16)w, xh = (_Float16)x;
            const _Float16 wl = (_Float16)(w - (float)wh), xl = (_Float16)(x - (float)xh);
            exact += (double)w * x;
            split += (double)(float)wh * (float)xh + (double)(float)wh * (float)xl + (double)(float)wl * (float)xh;
            mag += fabs((double)w * x);
        }
        const double e = fabs(split - exact);
        if (e > worst) worst = e;
        if (e / mag > worst_rel) worst_rel = e / mag;
    }
    printf("split f16 (3 products) 8-term dot, |w| < 0.3, |x| < 40: worst abs err %.3g, worst err / sum|w x| %.3g\n",
           worst, worst_rel);
    return 0;
}
