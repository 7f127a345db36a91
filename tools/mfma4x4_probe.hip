// Layout probe for v_mfma_f32_4x4x1_16b_f32 (the head backward's weight-gradient MFMA):
// one wave, A = lane id, B = 1 -> D[bk][m][n] = A of the lane supplying row m of block bk;
// then A = 1, B = lane id -> the lane supplying column n.  Prints, per lane and register, the
// supplying lanes, and checks them against the layout train.hip assumes (mfma4x4).
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma4x4_probe.hip -o tools/ablib/mfma4x4_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(float *out)
{
    const int l = threadIdx.x;
    v4f z = {0.f, 0.f, 0.f, 0.f};
    const v4f a = __builtin_amdgcn_mfma_f32_4x4x1f32((float)l, 1.f, z, 0, 0, 0);
    const v4f b = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)l, z, 0, 0, 0);
    for (int r = 0; r < 4; ++r) {
        out[(l * 4 + r) * 2] = a[r];
        out[(l * 4 + r) * 2 + 1] = b[r];
    }
}

int main()
{
    float *d = nullptr, h[64 * 4 * 2];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            const int am = (int)h[(l * 4 + r) * 2], bn = (int)h[(l * 4 + r) * 2 + 1];
            // assumed: block bk = l >> 2, D[m = r][n = l & 3]; A row m from lane 4 bk + m,
            // B column n from lane 4 bk + n
            const int ea = 4 * (l >> 2) + r, eb = 4 * (l >> 2) + (l & 3);
            if (am != ea || bn != eb) ++bad;
            if (l < 8 || am != ea || bn != eb) printf("lane %2d reg %d: A from lane %2d, B from lane %2d\n", l, r, am, bn);
        }
    printf("mfma_f32_4x4x1_16b layout %s (%d mismatches)\n", bad ? "DIFFERS" : "as assumed", bad);
    hipFree(d);
    return bad ? 1 : 0;
}
