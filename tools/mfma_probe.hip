// mfma_probe.hip -- lane map and issue rate of the f32 MFMA forms the fused synthesis head
// uses, on gfx950.  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe
//  * layout: v_mfma_f32_4x4x1_16b_f32 with distinct A / B per lane; checks that register i of
//    lane 4b+j holds A(lane 4b+i) * B(lane 4b+j) (the map the kernel relies on);
//  * rate: one wave per SIMD, 4 independent accumulators, 4x4x1_16b vs 16x16x4 (TFLOP/s).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float v4f __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                                \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

__global__ void probe_layout(const float *a, const float *b, float *d)
{
    const int l = threadIdx.x;
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

__global__ void rate_4x4(float *out, int iters)
{
    const int l = threadIdx.x;
    const float a = 1.f + l * 1e-7f, b = 1.f - l * 1e-7f;
    v4f c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ void rate_16x16(float *out, int iters)
{
    const int l = threadIdx.x;
    const float a = 1.f + l * 1e-7f, b = 1.f - l * 1e-7f;
    v4f c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main()
{
    float ha[64], hb[64], hd[256];
    for (int l = 0; l < 64; ++l) {
        ha[l] = (float)(l + 1);
        hb[l] = (float)(1000 * (l + 1));
    }
    float *da, *db, *dd, *dout;
    CHECK(hipMalloc(&da, sizeof ha));
    CHECK(hipMalloc(&db, sizeof hb));
    CHECK(hipMalloc(&dd, sizeof hd));
    CHECK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe_layout, dim3(1), dim3(64), 0, 0, da, db, dd);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
            if (hd[4 * l + r] != ha[4 * (l / 4) + r] * hb[l]) ++bad;
    printf("mfma_f32_4x4x1_16b lane map (reg i of lane 4b+j = A[4b+i] * B[4b+j]): %s (%d mismatches)\n",
           bad ? "FAIL" : "OK", bad);
    if (bad)
        for (int l = 0; l < 8; ++l)
            printf("  lane %d: %g %g %g %g\n", l, hd[4 * l], hd[4 * l + 1], hd[4 * l + 2], hd[4 * l + 3]);

    const int blocks = 1024, iters = 20000; // one wave per SIMD on 256 CUs
    CHECK(hipMalloc(&dout, sizeof(float) * 64 * blocks));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int form = 0; form < 2; ++form) {
        auto launch = [&]() {
            if (form == 0) hipLaunchKernelGGL(rate_4x4, dim3(blocks), dim3(64), 0, 0, dout, iters);
            else hipLaunchKernelGGL(rate_16x16, dim3(blocks), dim3(64), 0, 0, dout, iters);
        };
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double flop_per = form == 0 ? 16.0 * 4 * 4 * 2 : 16.0 * 16 * 4 * 2;
        const double flops = (double)blocks * iters * 4 * flop_per;
        printf("%s: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per wave\n", form == 0 ? "4x4x1_16b" : "16x16x4  ",
               ms, flops / (ms * 1e-3) / 1e12, ms * 1e6 / ((double)iters * 4));
    }
    return 0;
}
