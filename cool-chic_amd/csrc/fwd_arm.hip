// fwd_arm.hip -- path A ARM: causal context gather + MLP + Laplace rate, float32.
//
// Replaces, for every latent of every grid of every frame in one launch:
//   quantize (quantizer.py:231-232, eval = torch.round(gain * y)),
//   _get_neighbor (arm.py:308-352: zero pad 4, 9x9 unfold, index_select of the
//                  causal context pixels, _get_non_zero_pixel_ctx_index arm.py:373-506),
//   Arm.forward (arm.py:227-268: residual Linear+ReLU x n_hidden, Linear -> (mu, log_scale),
//                scale = exp(clamp(log_scale - 4, -4.6, 5))),
//   rate (coolchic.py:419-424 with _laplace_cdf arm.py:355-370).
//
// Layout: one workgroup (256 threads, 4 waves) owns a (4 NL) x 64 tile of one grid of one
// frame.  The quantised tile plus its causal halo (4 rows above, 4 columns either
// side) is staged once in LDS; each thread evaluates the MLP for NL = 2 latents of the
// same column as one packed pair, so every weight (wave-uniform, held in SGPRs via
// scalar loads) feeds one v_pk_fma_f32 (two FMAs).  NL = 4 (two pairs per weight) was
// measured 13 % slower: 132 VGPRs, 3 waves per SIMD instead of 7.  LDS reads are lane-consecutive (conflict-free).  Grids of all resolutions
// share one launch through a tile prefix table (no per-grid launches).
#include <stdlib.h>

#include <algorithm>

#include "fwd_common.h"

using ccmi_fwd::cfloat_ptr;
using ccmi_fwd::f2;

namespace {

constexpr int kThreads = 256;
constexpr int kTX = 64;
constexpr int kRowsPerPass = kThreads / kTX; // 4
#ifndef CCMI_ARM_NL
#define CCMI_ARM_NL 2
#endif
constexpr int kNL = CCMI_ARM_NL;              // latents per thread (packed pairs)
constexpr int kNP = kNL / 2;
constexpr int kTY = kRowsPerPass * kNL;       // 8
constexpr int kHalo = 4;
constexpr int kLW = kTX + 2 * kHalo;          // 72
constexpr int kLH = kTY + kHalo;              // 12


struct ArmGeom {
    int n;
    int h[CCMI_MAX_GRIDS], w[CCMI_MAX_GRIDS], off[CCMI_MAX_GRIDS];
    int tiles_x[CCMI_MAX_GRIDS];
    int tile_start[CCMI_MAX_GRIDS + 1];
};

// Context pixel offsets (dy, dx) in the reference's gather order: flattened 9x9
// mask index k -> (k / 9 - 4, k % 9 - 4) for the indices of arm.py:373-506.
template <int D>
__device__ __forceinline__ void ctx_offset(int i, int &dy, int &dx)
{
    // clang-format off
    constexpr signed char k8[8] = {13, 22, 30, 31, 32, 37, 38, 39};
    constexpr signed char k16[16] = {13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39};
    constexpr signed char k24[24] = {4, 11, 12, 13, 14, 15, 19, 20, 21, 22, 23, 24, 25, 28, 29, 30, 31, 32, 33, 34,
                                     36, 37, 38, 39};
    constexpr signed char k32[32] = {2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 19, 20, 21, 22, 23, 24, 25, 26, 27,
                                     28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39};
    // clang-format on
    int k = D == 8 ? k8[i] : D == 16 ? k16[i] : D == 24 ? k24[i] : k32[i];
    dy = k / 9 - 4;
    dx = k % 9 - 4;
}

// inv_scale = 1 / scale (v_rcp_f32, shared by both CDF evaluations of a latent instead
// of two IEEE divisions).  expm1 of the reference is evaluated as v_exp_f32 - 1: its
// absolute error (~1 ulp of 1) is below the fp32 cancellation the reference formula
// already has in p = F(q + 1/2) - F(q - 1/2); worst rate error / tolerance of
// tests/test_forward.py over the goldens and random 720p / 1080p frames: 0.432 with
// either form (tools/rate_margin.py), ARM 5 % faster.
__device__ __forceinline__ float laplace_cdf(float x, float mu, float inv_scale)
{
    float s = x - mu;
    float sg = s > 0.f ? 1.f : (s < 0.f ? -1.f : 0.f);
    return 0.5f - 0.5f * sg * (__expf(-fabsf(s) * inv_scale) - 1.f);
}

// NH >= 0: the hidden-layer count fixed at compile time (the layer loop unrolled, so the
// next layer's scalar weight loads can be scheduled under the current layer's FMAs)
template <int D, int NH = -1>
__global__ __launch_bounds__(kThreads) void arm_fwd_kernel(
    const float *__restrict__ lat, int64_t lat_stride, ArmGeom g, float gain, int quantize, int nh,
    const float *__restrict__ params, int64_t pstride, float *__restrict__ o_mu, float *__restrict__ o_scale,
    float *__restrict__ o_log_scale, float *__restrict__ o_rate, int64_t ostride)
{
    __shared__ float tile[kLH][kLW];

    // XCD-aware tile order (ccmi_fwd::xcd_order): vertically adjacent tiles, which share the
    // 4 causal halo rows, meet in one L2
    const int wt = ccmi_fwd::xcd_order(blockIdx.x, gridDim.x);
    const int ntl = g.tile_start[g.n];
    const int b = wt / ntl;
    const int t = wt - b * ntl;
    int l = 0;
#pragma unroll
    for (int k = 1; k < CCMI_MAX_GRIDS; ++k)
        if (k < g.n && t >= g.tile_start[k]) l = k;
    const int lt = t - g.tile_start[l];
    const int H = g.h[l], W = g.w[l];
    const int y0 = (lt / g.tiles_x[l]) * kTY;
    const int x0 = (lt % g.tiles_x[l]) * kTX;
    const float *src = lat + (int64_t)b * lat_stride + g.off[l];

    // fixed trip count, unrolled: every load of the thread is in flight before the first
    // LDS store waits on one
    {
        constexpr int NU = (kLH * kLW + kThreads - 1) / kThreads;
        float lv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = threadIdx.x + u * kThreads;
            const int r = i / kLW, c = i - r * kLW;
            const int y = y0 - kHalo + r, x = x0 - kHalo + c;
            lv[u] = (i < kLH * kLW && y >= 0 && y < H && x >= 0 && x < W) ? src[y * W + x] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = threadIdx.x + u * kThreads;
            if (i < kLH * kLW) tile[i / kLW][i % kLW] = quantize ? rintf(gain * lv[u]) : lv[u];
        }
    }
    __syncthreads();

    const cfloat_ptr p = (cfloat_ptr)(size_t)(params + (int64_t)b * pstride);
    const int cx = threadIdx.x % kTX;
    const int cy0 = threadIdx.x / kTX;

    // the two latents of a thread travel as one packed pair (v_pk_fma_f32): every
    // wave-uniform weight feeds both with one instruction
    // pair q = rows cy0 + (2q) * kRowsPerPass and cy0 + (2q + 1) * kRowsPerPass
    static_assert(kNL % 2 == 0, "packed pair layout");
    f2 a[kNP][D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        int dy, dx;
        ctx_offset<D>(i, dy, dx);
#pragma unroll
        for (int q = 0; q < kNP; ++q)
            a[q][i] = f2{tile[cy0 + 2 * q * kRowsPerPass + kHalo + dy][cx + kHalo + dx],
                         tile[cy0 + (2 * q + 1) * kRowsPerPass + kHalo + dy][cx + kHalo + dx]};
    }

    if constexpr (NH >= 0) nh = NH;
#pragma unroll
    for (int layer = 0; layer < nh; ++layer) {
        const cfloat_ptr Wl = p + layer * (D * D + D);
        const cfloat_ptr bl = Wl + D * D;
        f2 o[kNP][D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            // F.linear(x) + x, then ReLU: the accumulator starts at bias + residual (one packed
            // add instead of two after the products; a different fp32 summation order, inside
            // the forward's tolerance)
            f2 acc[kNP];
#pragma unroll
            for (int q = 0; q < kNP; ++q) acc[q] = a[q][j] + f2(bl[j]);
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const f2 wji = f2(Wl[j * D + i]);
#pragma unroll
                for (int q = 0; q < kNP; ++q) acc[q] = __builtin_elementwise_fma(wji, a[q][i], acc[q]);
            }
#pragma unroll
            for (int q = 0; q < kNP; ++q) o[q][j] = __builtin_elementwise_max(acc[q], f2(0.f));
        }
#pragma unroll
        for (int q = 0; q < kNP; ++q)
#pragma unroll
            for (int j = 0; j < D; ++j) a[q][j] = o[q][j];
    }

    const cfloat_ptr Wo = p + nh * (D * D + D);
    f2 m[kNP], ls[kNP];
#pragma unroll
    for (int q = 0; q < kNP; ++q) {
        m[q] = f2(Wo[2 * D]);
        ls[q] = f2(Wo[2 * D + 1]);
    }
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const f2 w0 = f2(Wo[i]), w1 = f2(Wo[D + i]);
#pragma unroll
        for (int q = 0; q < kNP; ++q) {
            m[q] = __builtin_elementwise_fma(w0, a[q][i], m[q]);
            ls[q] = __builtin_elementwise_fma(w1, a[q][i], ls[q]);
        }
    }
#pragma unroll
    for (int n = 0; n < kNL; ++n) {
        const int y = y0 + cy0 + n * kRowsPerPass, x = x0 + cx;
        const float mn = (n & 1) ? m[n >> 1].y : m[n >> 1].x, lsn = (n & 1) ? ls[n >> 1].y : ls[n >> 1].x;
        if (y < H && x < W) {
            // v_exp_f32 / v_log_f32 directly (the clamped exponent and p in [2^-16, 1] are far
            // from the ranges the library forms guard; errors well inside the rate tolerance)
            const float sc = __expf(fminf(fmaxf(lsn - 4.f, -4.6f), 5.0f));
            const float q = tile[cy0 + n * kRowsPerPass + kHalo][cx + kHalo];
            const int64_t idx = (int64_t)b * ostride + g.off[l] + y * W + x;
            if (o_mu) o_mu[idx] = mn;
            if (o_scale) o_scale[idx] = sc;
            if (o_log_scale) o_log_scale[idx] = lsn;
            if (o_rate) {
                const float is = __builtin_amdgcn_rcpf(sc);
                const float pr = fmaxf(laplace_cdf(q + 0.5f, mn, is) - laplace_cdf(q - 0.5f, mn, is), 1.52587890625e-05f);
                o_rate[idx] = -__log2f(pr);
            }
        }
    }
}

template <int D>
__global__ __launch_bounds__(kThreads) void arm_context_kernel(const float *__restrict__ grid, int H, int W,
                                                               float *__restrict__ out)
{
    const int b = blockIdx.y;
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    const float *g = grid + (int64_t)b * H * W;
    float *o = out + ((int64_t)b * H * W + p) * D;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        int dy, dx;
        ctx_offset<D>(i, dy, dx);
        const int yy = y + dy, xx = x + dx;
        o[i] = (yy >= 0 && xx >= 0 && xx < W) ? g[yy * W + xx] : 0.f;
    }
}

template <int D>
__global__ __launch_bounds__(kThreads) void arm_mlp_kernel(const float *__restrict__ ctx, int64_t M, int nh,
                                                           const float *__restrict__ p, float *__restrict__ o_mu,
                                                           float *__restrict__ o_scale, float *__restrict__ o_ls)
{
    const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (r >= M) return;
    float a[D];
#pragma unroll
    for (int i = 0; i < D; ++i) a[i] = ctx[r * D + i];
    for (int layer = 0; layer < nh; ++layer) {
        const float *Wl = p + layer * (D * D + D);
        float o[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < D; ++i) acc = fmaf(Wl[j * D + i], a[i], acc);
            o[j] = fmaxf((acc + Wl[D * D + j]) + a[j], 0.f);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = o[j];
    }
    const float *Wo = p + nh * (D * D + D);
    float m = 0.f, ls = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        m = fmaf(Wo[i], a[i], m);
        ls = fmaf(Wo[D + i], a[i], ls);
    }
    m += Wo[2 * D];
    ls += Wo[2 * D + 1];
    if (o_mu) o_mu[r] = m;
    if (o_ls) o_ls[r] = ls;
    if (o_scale) o_scale[r] = expf(fminf(fmaxf(ls - 4.f, -4.6f), 5.0f));
}

} // namespace

extern "C" int ccmi_arm_context_f32(const float *grid, int batch, int h, int w, int dim_arm, float *out, void *stream)
{
    if (!grid || !out || batch < 1 || h < 1 || w < 1) return ccmi_set_error(CCMI_ERR_ARG, "arm_context: bad argument");
    dim3 g((unsigned)(((int64_t)h * w + kThreads - 1) / kThreads), batch);
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dim_arm) {
    case 8: hipLaunchKernelGGL(arm_context_kernel<8>, g, dim3(kThreads), 0, s, grid, h, w, out); break;
    case 16: hipLaunchKernelGGL(arm_context_kernel<16>, g, dim3(kThreads), 0, s, grid, h, w, out); break;
    case 24: hipLaunchKernelGGL(arm_context_kernel<24>, g, dim3(kThreads), 0, s, grid, h, w, out); break;
    case 32: hipLaunchKernelGGL(arm_context_kernel<32>, g, dim3(kThreads), 0, s, grid, h, w, out); break;
    default: return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "arm_context: dim_arm %d", dim_arm);
    }
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

extern "C" int ccmi_arm_mlp_f32(const float *ctx, int64_t m, int dim_arm, int n_hidden, const float *params, float *mu,
                                float *scale, float *log_scale, void *stream)
{
    if (!ctx || !params || m < 0 || n_hidden < 0 || n_hidden > 4) return ccmi_set_error(CCMI_ERR_ARG, "arm_mlp: bad argument");
    if (m == 0) return CCMI_OK;
    dim3 g((unsigned)((m + kThreads - 1) / kThreads));
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dim_arm) {
    case 8: hipLaunchKernelGGL(arm_mlp_kernel<8>, g, dim3(kThreads), 0, s, ctx, m, n_hidden, params, mu, scale, log_scale); break;
    case 16: hipLaunchKernelGGL(arm_mlp_kernel<16>, g, dim3(kThreads), 0, s, ctx, m, n_hidden, params, mu, scale, log_scale); break;
    case 24: hipLaunchKernelGGL(arm_mlp_kernel<24>, g, dim3(kThreads), 0, s, ctx, m, n_hidden, params, mu, scale, log_scale); break;
    case 32: hipLaunchKernelGGL(arm_mlp_kernel<32>, g, dim3(kThreads), 0, s, ctx, m, n_hidden, params, mu, scale, log_scale); break;
    default: return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "arm_mlp: dim_arm %d", dim_arm);
    }
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

int ccmi_launch_arm_f32(const ccmi_arm_args *a, hipStream_t s)
{
    ArmGeom g{};
    g.n = a->n_grids;
    int off = 0, tiles = 0;
    for (int l = 0; l < a->n_grids; ++l) {
        g.h[l] = a->h[l];
        g.w[l] = a->w[l];
        g.off[l] = off;
        g.tiles_x[l] = ccmi_div_up(a->w[l], kTX);
        g.tile_start[l] = tiles;
        tiles += g.tiles_x[l] * ccmi_div_up(a->h[l], kTY);
        off += a->h[l] * a->w[l];
    }
    g.tile_start[a->n_grids] = tiles;
    if ((a->latent_stride != 0 && a->latent_stride < off) || a->out_stride < off)
        return ccmi_set_error(CCMI_ERR_ARG, "arm: stride smaller than the %d latents of a frame", off);
    dim3 grid((unsigned)(tiles * a->batch));
#define CCMI_ARM_LAUNCH(DD)                                                                                     \
    hipLaunchKernelGGL(arm_fwd_kernel<DD>, grid, dim3(kThreads), 0, s, a->latent, a->latent_stride, g, a->gain, \
                       a->quantize, a->n_hidden, a->params, a->param_stride, a->mu, a->scale, a->log_scale,     \
                       a->rate, a->out_stride)
    switch (a->dim_arm) {
    case 8: CCMI_ARM_LAUNCH(8); break;
    case 16:
        // the presets' ARM (2 hidden layers): layer loop unrolled
        if (a->n_hidden == 2) {
            hipLaunchKernelGGL((arm_fwd_kernel<16, 2>), grid, dim3(kThreads), 0, s, a->latent, a->latent_stride, g, a->gain,
                               a->quantize, a->n_hidden, a->params, a->param_stride, a->mu, a->scale, a->log_scale,
                               a->rate, a->out_stride);
        } else {
            CCMI_ARM_LAUNCH(16);
        }
        break;
    case 24: CCMI_ARM_LAUNCH(24); break;
    case 32: CCMI_ARM_LAUNCH(32); break;
    default: return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "arm: dim_arm must be 8, 16, 24 or 32 (got %d)", a->dim_arm);
    }
#undef CCMI_ARM_LAUNCH
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}
