// fwd_ups.hip -- path A upsampling (Upsampling.forward, eval mode), float32.
//
// Reference (coolchic/enc/component/core/upsampling.py):
//   Upsampling.forward :476-506 -- from the coarsest grid, at each step s:
//     stack <- cat(conv2ds[s % n_pre](y_target), conv_transpose2ds[s % n_ups](stack)) ;
//   UpsamplingSeparableSymmetricConv2d.forward (eval) :205-209 -- zero-padded separable
//     cross-correlation, horizontal then vertical, plus residual;
//   UpsamplingSeparableSymmetricConvTranspose2d.forward (eval) :337-353 -- replicate pad
//     P0 = K/2, stride-2 transposed conv, crop C = K - 1 + K/2, horizontal then vertical,
//     then crop to the target size.
//
// One launch per pyramid step (coarse -> fine), all frames of the batch in the launch.
// The stride-2 transposed conv is evaluated in polyphase form: destination sample
// 2j + a reads source samples j + d with tap  a + K/2 - 1 - 2d  (derived from the
// crop offsets; the reference's padding makes border reads replicate-clamped).
// Each workgroup computes a 16 x 64 destination tile for every channel: the source
// tile (with clamped halo) and the horizontal pass are staged in LDS, then the
// vertical pass writes coalesced rows.
#include "fwd_common.h"

using namespace ccmi_fwd;

namespace {

constexpr int kThreads = 256;
constexpr int kTY = 16, kTX = 64;
constexpr int kMaxK = 16;                       // max upsampling / refine kernel taps
constexpr int kSrcW = kTX / 2 + kMaxK / 2 + 2;  // source tile row pitch (incl. halo)
constexpr int kRefH = kTY + kMaxK;              // refine rows incl. halo
constexpr int kRefW = kTX + kMaxK;


__global__ __launch_bounds__(kThreads) void ups_level_kernel(LevelArgs A)
{
    __shared__ float s_src[kRefH * kRefW]; // used for the source tile and the refine input
    __shared__ float s_h[kRefH * kTX];     // horizontal pass results

    const int b = blockIdx.y;
    const int y0 = (blockIdx.x / A.tiles_x) * kTY;
    const int x0 = (blockIdx.x % A.tiles_x) * kTX;
    const float *prm = A.params + (int64_t)b * A.pstride;
    const float *wu = prm + A.up_off;
    const float *wr = prm + A.pre_off;
    float *dst = A.dst + (int64_t)b * A.dst_stride;
    const int64_t dplane = (int64_t)A.hd * A.wd;
    const int tid = threadIdx.x;

    // ---------------- channel 0: refine(y_{k-1}) = x + sepconv(x), zero padding ----------------
    {
        const int pad = A.Kp / 2;
        const int rh = kTY + 2 * pad, rw = kTX + 2 * pad;
        const float *src = A.ref_src + (int64_t)b * A.ref_stride;
        for (int i = tid; i < rh * rw; i += kThreads) {
            const int r = i / rw, c = i - r * rw;
            const int y = y0 - pad + r, x = x0 - pad + c;
            float v = 0.f;
            if (y >= 0 && y < A.hd && x >= 0 && x < A.wd) {
                v = src[y * A.wd + x];
                if (A.ref_quant) v = rintf(A.gain * v);
            }
            s_src[r * kRefW + c] = v;
        }
        __syncthreads();
        for (int i = tid; i < rh * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            float acc = 0.f;
            for (int k = 0; k < A.Kp; ++k) acc = fmaf(wr[k], s_src[r * kRefW + c + k], acc);
            s_h[r * kTX + c] = acc;
        }
        __syncthreads();
        for (int i = tid; i < kTY * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            const int y = y0 + r, x = x0 + c;
            if (y < A.hd && x < A.wd) {
                float acc = 0.f;
                for (int k = 0; k < A.Kp; ++k) acc = fmaf(wr[k], s_h[(r + k) * kTX + c], acc);
                dst[(int64_t)y * A.wd + x] = acc + s_src[(r + pad) * kRefW + c + pad];
            }
        }
        __syncthreads();
    }

    // ---------------- channels 1..C: 2x transposed-conv upsampling of the source stack ----------------
    // source rows/cols needed: j + d for j in [y0/2, y0/2 + kTY/2), d in [dmin, dmax]
    const int K2 = A.K / 2;
    // tap = a + K2 - 1 - 2d in [0, K-1]  <=>  d in [ceil((a - K2)/2), floor((a + K2 - 1)/2)]
    const int d_lo = -((K2 + 1) / 2); // min over a in {0,1}
    const int d_hi = K2 / 2;          // max over a in {0,1}
    const int sy0 = y0 / 2 + d_lo, sx0 = x0 / 2 + d_lo;
    const int sh = kTY / 2 + d_hi - d_lo, sw = kTX / 2 + d_hi - d_lo;
    const int64_t splane = (int64_t)A.hs * A.ws;
    const float *src = A.src + (int64_t)b * A.src_stride;

    for (int c = 0; c < A.C; ++c) {
        const float *sp = src + c * splane;
        for (int i = tid; i < sh * sw; i += kThreads) {
            const int r = i / sw, cc = i - r * sw;
            const int y = clampi(sy0 + r, A.hs - 1), x = clampi(sx0 + cc, A.ws - 1);
            float v = sp[y * A.ws + x];
            if (A.src_quant) v = rintf(A.gain * v);
            s_src[r * kSrcW + cc] = v;
        }
        __syncthreads();
        // horizontal: s_h[r][c] for destination column x0 + c
        for (int i = tid; i < sh * kTX; i += kThreads) {
            const int r = i / kTX, cc = i - r * kTX;
            const int xd = x0 + cc, j = xd >> 1, a = xd & 1;
            float acc = 0.f;
            // taps in increasing source position: d from d_lo..d_hi with valid tap
            for (int d = d_lo; d <= d_hi; ++d) {
                const int tap = a + K2 - 1 - 2 * d;
                if (tap < 0 || tap >= A.K) continue;
                acc = fmaf(wu[tap], s_src[r * kSrcW + (j + d - sx0)], acc);
            }
            s_h[r * kTX + cc] = acc;
        }
        __syncthreads();
        for (int i = tid; i < kTY * kTX; i += kThreads) {
            const int r = i / kTX, cc = i - r * kTX;
            const int yd = y0 + r, xd = x0 + cc;
            if (yd < A.hd && xd < A.wd) {
                const int j = yd >> 1, a = yd & 1;
                float acc = 0.f;
                for (int d = d_lo; d <= d_hi; ++d) {
                    const int tap = a + K2 - 1 - 2 * d;
                    if (tap < 0 || tap >= A.K) continue;
                    acc = fmaf(wu[tap], s_h[(j + d - sy0) * kTX + cc], acc);
                }
                dst[(int64_t)(c + 1) * dplane + (int64_t)yd * A.wd + xd] = acc;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Specialised level kernel for compile-time kernel sizes (the reference's defaults are
// K = 8 transposed taps, KP = 7 refine taps).  Differences from the generic kernel:
//   * one channel per workgroup (grid z), small LDS footprint -> high occupancy;
//   * the polyphase loops are unrolled: a thread produces an (even, odd) output pair from
//     K/2 + 1 shared source samples, horizontally and then vertically;
//   * no per-element division: all pitches are compile-time.
// ---------------------------------------------------------------------------------------------

template <int K, int KP>
__global__ __launch_bounds__(kThreads) void ups_level_fixed(LevelArgs A)
{
    using T = UpsTile<K, KP, kTY, kTX>;
    // blockIdx.z = job: 0 -> refine channel, c >= 1 -> transposed-conv channel c.  One
    // channel per workgroup keeps LDS small (the union of the two jobs' buffers), so many
    // workgroups are resident per CU to hide the L2/HBM latency of the tile loads.
    constexpr int kRef = T::RH * T::RW + T::RH * kTX;
    constexpr int kUp = T::SH * T::SW + T::SH * kTX;
    __shared__ float s_mem[kRef > kUp ? kRef : kUp];

    const int b = blockIdx.y;
    const int job = blockIdx.z;
    const int y0 = (blockIdx.x / A.tiles_x) * kTY;
    const int x0 = (blockIdx.x % A.tiles_x) * kTX;
    const float *prm = A.params + (int64_t)b * A.pstride;
    float *dst = A.dst + (int64_t)b * A.dst_stride;
    const int64_t dplane = (int64_t)A.hd * A.wd;
    const int tid = threadIdx.x;

    if (job == 0) {
        float wr[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) wr[k] = prm[A.pre_off + k];
        float *s_ref = s_mem, *s_refh = s_mem + T::RH * T::RW;
        const float *rs = A.ref_src + (int64_t)b * A.ref_stride;
        // fixed trip counts, unrolled: all of a thread's tile loads are in flight before the
        // first LDS store waits on one (the rolled loop paid one memory latency per pass)
        {
            constexpr int NU = (T::RH * T::RW + kThreads - 1) / kThreads;
            float lv[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int i = tid + u * kThreads;
                const int r = i / T::RW, c = i - r * T::RW;
                const int y = y0 - T::PAD + r, x = x0 - T::PAD + c;
                lv[u] = (i < T::RH * T::RW && y >= 0 && y < A.hd && x >= 0 && x < A.wd) ? rs[y * A.wd + x] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int i = tid + u * kThreads;
                if (i < T::RH * T::RW) s_ref[i] = A.ref_quant ? rintf(A.gain * lv[u]) : lv[u];
            }
        }
        __syncthreads();
        for (int i = tid; i < T::RH * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            const float *p = s_ref + r * T::RW + c;
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < KP; ++k) acc = fmaf(wr[k], p[k], acc);
            s_refh[i] = acc;
        }
        __syncthreads();
        for (int i = tid; i < kTY * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            const int y = y0 + r, x = x0 + c;
            if (y < A.hd && x < A.wd) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < KP; ++k) acc = fmaf(wr[k], s_refh[(r + k) * kTX + c], acc);
                dst[(int64_t)y * A.wd + x] = acc + s_ref[(r + T::PAD) * T::RW + c + T::PAD];
            }
        }
        return;
    }

    const int c = job - 1;
    float wu[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wu[k] = prm[A.up_off + k];
    float *s_src = s_mem, *s_h = s_mem + T::SH * T::SW;
    {
        const float *src = A.src + (int64_t)b * A.src_stride + (int64_t)c * A.hs * A.ws;
        const int sy0 = y0 / 2 + T::D0, sx0 = x0 / 2 + T::D0;
        constexpr int NU = (T::SH * T::SW + kThreads - 1) / kThreads;
        float lv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = tid + u * kThreads;
            const int r = i / T::SW, cc = i - r * T::SW;
            const int y = clampi(sy0 + r, A.hs - 1), x = clampi(sx0 + cc, A.ws - 1);
            lv[u] = i < T::SH * T::SW ? src[y * A.ws + x] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = tid + u * kThreads;
            if (i < T::SH * T::SW) s_src[i] = A.src_quant ? rintf(A.gain * lv[u]) : lv[u];
        }
    }
    __syncthreads();
    // horizontal: one (even, odd) destination column pair per item, source column x0/2 + q
    for (int i = tid; i < T::SH * (kTX / 2); i += kThreads) {
        const int r = i / (kTX / 2), q = i - r * (kTX / 2);
        const float *p = s_src + r * T::SW + q; // offset D0 at index 0
        float e = 0.f, o = 0.f;
#pragma unroll
        for (int m = 0; m < T::NS; ++m) {
            const float v = p[m];
            const int d = T::D0 + m;
            const int te = T::tap(0, d), to = T::tap(1, d);
            if (te >= 0) e = fmaf(wu[te], v, e);
            if (to >= 0) o = fmaf(wu[to], v, o);
        }
        *reinterpret_cast<float2 *>(s_h + r * kTX + 2 * q) = make_float2(e, o);
    }
    __syncthreads();
    // vertical: destination rows y0 + 2q, y0 + 2q + 1 of column x
    for (int i = tid; i < (kTY / 2) * kTX; i += kThreads) {
        const int q = i / kTX, x = i - q * kTX;
        const float *p = s_h + q * kTX + x;
        float e = 0.f, o = 0.f;
#pragma unroll
        for (int m = 0; m < T::NS; ++m) {
            const float v = p[m * kTX];
            const int d = T::D0 + m;
            const int te = T::tap(0, d), to = T::tap(1, d);
            if (te >= 0) e = fmaf(wu[te], v, e);
            if (to >= 0) o = fmaf(wu[to], v, o);
        }
        const int yd = y0 + 2 * q, xd = x0 + x;
        if (xd < A.wd) {
            float *out = dst + (int64_t)(c + 1) * dplane + (int64_t)yd * A.wd + xd;
            if (yd < A.hd) out[0] = e;
            if (yd + 1 < A.hd) out[A.wd] = o;
        }
    }
}

} // namespace

extern "C" size_t ccmi_ups_workspace_bytes(int n_grids, const int *h, const int *w, int batch)
{
    size_t per = 0;
    for (int k = 1; k <= n_grids - 2; ++k) per += (size_t)(n_grids - k) * h[k] * w[k];
    return per * sizeof(float) * (size_t)(batch > 0 ? batch : 0);
}

namespace {
int launch_level(const LevelArgs &A, int batch, hipStream_t s)
{
    dim3 grid(A.tiles_x * ccmi_div_up(A.hd, kTY), batch);
    if (A.K == 8 && A.Kp == 7)
        hipLaunchKernelGGL((ups_level_fixed<8, 7>), dim3(grid.x, grid.y, A.C + 1), dim3(kThreads), 0, s, A);
    else
        hipLaunchKernelGGL(ups_level_kernel, grid, dim3(kThreads), 0, s, A);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}
} // namespace

int ccmi_fwd::ups_pyramid(const ccmi_ups_args *a, hipStream_t s, LevelArgs *last, bool launch, LevelArgs *prev)
{
    const int L = a->n_grids;
    if (L < 2) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "ups: needs at least 2 latent grids (got %d)", L);
    if (a->ups_k < 4 || a->ups_k % 2 || a->ups_k > kMaxK)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "ups: ups_k must be even in [4, %d] (got %d)", kMaxK, a->ups_k);
    if (a->pre_k < 1 || a->pre_k % 2 == 0 || a->pre_k > kMaxK - 1)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "ups: pre_k must be odd in [1, %d] (got %d)", kMaxK - 1, a->pre_k);
    if (a->n_ups < 1 || a->n_pre < 1) return ccmi_set_error(CCMI_ERR_ARG, "ups: n_ups and n_pre must be >= 1");
    for (int l = 1; l < L; ++l)
        if (a->h[l] != (a->h[l - 1] + 1) / 2 || a->w[l] != (a->w[l - 1] + 1) / 2)
            return ccmi_set_error(CCMI_ERR_ARG, "ups: grid %d is not ceil(half) of grid %d", l, l - 1);
    const size_t need = ccmi_ups_workspace_bytes(L, a->h, a->w, a->batch);
    if (need > 0 && (a->workspace == nullptr || a->workspace_bytes < need))
        return ccmi_set_error(CCMI_ERR_ARG, "ups: workspace of %zu bytes needed", need);

    int off[CCMI_MAX_GRIDS];
    int total = 0;
    for (int l = 0; l < L; ++l) { off[l] = total; total += a->h[l] * a->w[l]; }
    if (a->latent_stride != 0 && a->latent_stride < total) return ccmi_set_error(CCMI_ERR_ARG, "ups: latent_stride < %d", total);

    // workspace layout: stack of level k (1..L-2) for all frames: [batch][L-k][h_k][w_k]
    float *ws_base = static_cast<float *>(a->workspace);
    float *stack_ptr[CCMI_MAX_GRIDS] = {};
    int64_t stack_stride[CCMI_MAX_GRIDS] = {};
    for (int k = 1; k <= L - 2; ++k) {
        stack_ptr[k] = ws_base;
        stack_stride[k] = (int64_t)(L - k) * a->h[k] * a->w[k];
        ws_base += stack_stride[k] * a->batch;
    }

    for (int step = 0; step < L - 1; ++step) {
        const int k = L - 1 - step; // source level
        LevelArgs A{};
        if (k == L - 1) {
            A.src = a->latent + off[k];
            A.src_stride = a->latent_stride;
            A.src_quant = a->quantize;
        } else {
            A.src = stack_ptr[k];
            A.src_stride = stack_stride[k];
            A.src_quant = 0;
        }
        A.C = L - k;
        A.hs = a->h[k];
        A.ws = a->w[k];
        A.ref_src = a->latent + off[k - 1];
        A.ref_stride = a->latent_stride;
        A.ref_quant = a->quantize;
        if (k - 1 == 0) {
            A.dst = a->out; // may be null when the caller fuses the last step
            A.dst_stride = a->out_stride;
        } else {
            A.dst = stack_ptr[k - 1];
            A.dst_stride = stack_stride[k - 1];
        }
        A.hd = a->h[k - 1];
        A.wd = a->w[k - 1];
        A.gain = a->gain;
        A.params = a->params;
        A.pstride = a->param_stride;
        A.K = a->ups_k;
        A.up_off = (step % a->n_ups) * a->ups_k;
        A.Kp = a->pre_k;
        A.pre_off = a->n_ups * a->ups_k + (step % a->n_pre) * a->pre_k;
        A.tiles_x = ccmi_div_up(A.wd, kTX);
        if (step == L - 2) {
            *last = A;
            break;
        }
        if (prev && step == L - 3) { // folded into the caller's fused kernel: not launched
            *prev = A;
            continue;
        }
        if (launch)
            if (int rc = launch_level(A, a->batch, s)) return rc;
    }
    return CCMI_OK;
}

int ccmi_launch_ups_f32(const ccmi_ups_args *a, hipStream_t s)
{
    if (a->out_stride < (int64_t)a->n_grids * a->h[0] * a->w[0])
        return ccmi_set_error(CCMI_ERR_ARG, "ups: out_stride too small");
    LevelArgs last{};
    if (int rc = ups_pyramid(a, s, &last)) return rc;
    return launch_level(last, a->batch, s);
}
