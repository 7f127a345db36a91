// overlap_probe.hip -- does the f32 MFMA (v_mfma_f32_16x16x4_f32) run beside packed-f32 VALU
// work on gfx950, or does it hold the SIMD's vector issue for its whole 32 cycles?
// Build: hipcc --offload-arch=gfx950 -O3 tools/overlap_probe.hip -o tools/overlap_probe
// Kernels (every lane does `iters` iterations; chains independent so latency never limits):
//   mf   : 4 MFMAs per iteration (4 accumulators)
//   va   : NV v_pk_fma_f32 per iteration (8 packed accumulators)
//   both : the two bodies in one wave
//   split: the same two bodies in different waves of one workgroup (one of each per SIMD)
// If MFMA and VALU overlap, `both` ~ max(mf, va); if the MFMA blocks vector issue, ~ mf + va.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                                \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

template <int NV>
__device__ __forceinline__ void valu_body(f2 (&v)[8], f2 w)
{
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k & 7] = __builtin_elementwise_fma(v[k & 7], w, w);
}

__device__ __forceinline__ void mfma_body(v4f (&c)[4], float a, float b)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[k], 0, 0, 0);
}

template <int MODE, int NV>
__global__ __launch_bounds__(512) void probe(float *out, int iters)
{
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float a = 1.f + l * 1e-7f, b = 1.f - l * 1e-7f;
    const f2 w = f2{0.999f, 1e-4f};
    v4f c[4] = {};
    f2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = f2{a * k, b};
    const bool do_m = MODE == 0 || MODE == 2 || (MODE == 3 && wv < 4);
    const bool do_v = MODE == 1 || MODE == 2 || (MODE == 3 && wv >= 4);
    if (do_m && do_v) {
        for (int i = 0; i < iters; ++i) {
            mfma_body(c, a, b);
            valu_body<NV>(v, w);
        }
    } else if (do_m) {
        for (int i = 0; i < iters; ++i) mfma_body(c, a, b);
    } else {
        for (int i = 0; i < iters; ++i) valu_body<NV>(v, w);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += c[k][0];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k].x + v[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NV>
int run(const char *name, int blocks, int threads, int iters, float *dout)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((probe<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, dout, iters);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((probe<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, dout, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-6s NV=%2d blocks=%5d threads=%3d: %8.3f ms\n", name, NV, blocks, threads, ms);
    return 0;
}

template <int NV>
int sweep(float *dout, int iters)
{
    // 1 and 4 waves per SIMD (256 CUs x 4 SIMDs), 64-thread blocks; split uses 512-thread blocks
    for (int wps : {1, 4}) {
        const int blocks = 1024 * wps;
        if (run<0, NV>("mf", blocks, 64, iters, dout) || run<1, NV>("va", blocks, 64, iters, dout) ||
            run<2, NV>("both", blocks, 64, iters, dout))
            return 1;
    }
    if (run<3, NV>("split", 512, 512, iters, dout) || run<0, NV>("mf8", 512, 512, iters, dout) ||
        run<1, NV>("va8", 512, 512, iters, dout))
        return 1;
    return 0;
}

int main()
{
    float *dout;
    CHECK(hipMalloc(&dout, sizeof(float) * 4096 * 512));
    const int iters = 20000;
    if (sweep<16>(dout, iters) || sweep<32>(dout, iters)) return 1;
    return 0;
}
