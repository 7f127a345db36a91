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
#include "ccmi_internal.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTY = 16, kTX = 64;
constexpr int kMaxK = 16;                       // max upsampling / refine kernel taps
constexpr int kSrcW = kTX / 2 + kMaxK / 2 + 2;  // source tile row pitch (incl. halo)
constexpr int kRefH = kTY + kMaxK;              // refine rows incl. halo
constexpr int kRefW = kTX + kMaxK;

struct LevelArgs {
    // source stack (level k): C channels of hs x ws; channel c at src + c * hs * ws
    const float *src;
    int64_t src_stride;
    int src_quant; // source is the raw coarsest latent grid -> round(gain * x)
    int C, hs, ws;
    // refine input: raw latent grid of level k-1 (flat latent vector + offset)
    const float *ref_src;
    int64_t ref_stride;
    int ref_quant;
    // destination stack (level k-1): C + 1 channels of hd x wd
    float *dst;
    int64_t dst_stride;
    int hd, wd;
    float gain;
    // kernels, per frame: up taps at params + up_off, refine taps at params + pre_off
    const float *params;
    int64_t pstride;
    int up_off, K;
    int pre_off, Kp;
    int tiles_x;
};

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

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
//   * one staging pass loads the refine input and the source tiles of ALL channels, so a
//     tile costs 2 barriers instead of 3 * (C + 1);
//   * the polyphase loops are unrolled: a thread produces an (even, odd) output pair from
//     K/2 + 1 shared source samples, horizontally and then vertically;
//   * no per-element division: all pitches are compile-time.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxC = CCMI_MAX_GRIDS - 1; // channels of the source stack

template <int K, int KP>
struct UpsTile {
    static constexpr int K2 = K / 2;
    static constexpr int D0 = -((K2 + 1) / 2);      // min source offset over both parities
    static constexpr int NS = K2 + 1;               // source samples shared by an (even, odd) pair
    static constexpr int SH = kTY / 2 + NS - 1;     // source tile rows
    static constexpr int SW = kTX / 2 + NS - 1;     // source tile cols
    static constexpr int PAD = KP / 2;
    static constexpr int RH = kTY + KP - 1, RW = kTX + KP - 1;
    // tap used by parity a at source offset d (or -1)
    static constexpr int tap(int a, int d) { return (a + K2 - 1 - 2 * d >= 0 && a + K2 - 1 - 2 * d < K) ? a + K2 - 1 - 2 * d : -1; }
};

template <int K, int KP>
__global__ __launch_bounds__(kThreads) void ups_level_fixed(LevelArgs A)
{
    using T = UpsTile<K, KP>;
    static_assert(T::NS == K / 2 + 1, "");
    __shared__ float s_ref[T::RH * T::RW];
    __shared__ float s_refh[T::RH * kTX];
    __shared__ float s_src[kMaxC * T::SH * T::SW];
    __shared__ float s_h[kMaxC * T::SH * kTX];

    const int b = blockIdx.y;
    const int y0 = (blockIdx.x / A.tiles_x) * kTY;
    const int x0 = (blockIdx.x % A.tiles_x) * kTX;
    const float *prm = A.params + (int64_t)b * A.pstride;
    float wu[K], wr[KP];
#pragma unroll
    for (int k = 0; k < K; ++k) wu[k] = prm[A.up_off + k];
#pragma unroll
    for (int k = 0; k < KP; ++k) wr[k] = prm[A.pre_off + k];
    float *dst = A.dst + (int64_t)b * A.dst_stride;
    const int64_t dplane = (int64_t)A.hd * A.wd;
    const int tid = threadIdx.x;
    const int C = A.C;

    // ---- stage: refine input (zero padded) and every source channel (replicate clamped) ----
    {
        const float *rs = A.ref_src + (int64_t)b * A.ref_stride;
        for (int i = tid; i < T::RH * T::RW; i += kThreads) {
            const int r = i / T::RW, c = i - r * T::RW;
            const int y = y0 - T::PAD + r, x = x0 - T::PAD + c;
            float v = 0.f;
            if (y >= 0 && y < A.hd && x >= 0 && x < A.wd) {
                v = rs[y * A.wd + x];
                if (A.ref_quant) v = rintf(A.gain * v);
            }
            s_ref[i] = v;
        }
        const float *src = A.src + (int64_t)b * A.src_stride;
        const int64_t splane = (int64_t)A.hs * A.ws;
        const int sy0 = y0 / 2 + T::D0, sx0 = x0 / 2 + T::D0;
        const int n = C * T::SH * T::SW;
        for (int i = tid; i < n; i += kThreads) {
            const int c = i / (T::SH * T::SW), rem = i - c * (T::SH * T::SW);
            const int r = rem / T::SW, cc = rem - r * T::SW;
            const int y = clampi(sy0 + r, A.hs - 1), x = clampi(sx0 + cc, A.ws - 1);
            float v = src[c * splane + y * A.ws + x];
            if (A.src_quant) v = rintf(A.gain * v);
            s_src[i] = v;
        }
    }
    __syncthreads();

    // ---- horizontal passes ----
    for (int i = tid; i < T::RH * kTX; i += kThreads) {
        const int r = i / kTX, c = i - r * kTX;
        const float *p = s_ref + r * T::RW + c;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) acc = fmaf(wr[k], p[k], acc);
        s_refh[i] = acc;
    }
    {
        // one (even, odd) destination column pair per item: source column j = x0/2 + q
        const int n = C * T::SH * (kTX / 2);
        for (int i = tid; i < n; i += kThreads) {
            const int row = i / (kTX / 2), q = i - row * (kTX / 2); // row = c * SH + r
            const float *p = s_src + row * T::SW + q;              // offset D0 at index 0
            float e = 0.f, o = 0.f;
#pragma unroll
            for (int m = 0; m < T::NS; ++m) {
                const float v = p[m];
                const int d = T::D0 + m;
                const int te = T::tap(0, d), to = T::tap(1, d);
                if (te >= 0) e = fmaf(wu[te], v, e);
                if (to >= 0) o = fmaf(wu[to], v, o);
            }
            *reinterpret_cast<float2 *>(s_h + row * kTX + 2 * q) = make_float2(e, o);
        }
    }
    __syncthreads();

    // ---- vertical passes + coalesced stores ----
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
    {
        const int n = C * (kTY / 2) * kTX;
        for (int i = tid; i < n; i += kThreads) {
            const int c = i / ((kTY / 2) * kTX), rem = i - c * ((kTY / 2) * kTX);
            const int q = rem / kTX, x = rem - q * kTX; // destination rows y0 + 2q, y0 + 2q + 1
            const float *p = s_h + (c * T::SH + q) * kTX + x;
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
}

} // namespace

extern "C" size_t ccmi_ups_workspace_bytes(int n_grids, const int *h, const int *w, int batch)
{
    size_t per = 0;
    for (int k = 1; k <= n_grids - 2; ++k) per += (size_t)(n_grids - k) * h[k] * w[k];
    return per * sizeof(float) * (size_t)(batch > 0 ? batch : 0);
}

int ccmi_launch_ups_f32(const ccmi_ups_args *a, hipStream_t s)
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
    if (a->latent_stride < total) return ccmi_set_error(CCMI_ERR_ARG, "ups: latent_stride < %d", total);
    if (a->out_stride < (int64_t)L * a->h[0] * a->w[0]) return ccmi_set_error(CCMI_ERR_ARG, "ups: out_stride too small");

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
            A.dst = a->out;
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
        dim3 grid(A.tiles_x * ccmi_div_up(A.hd, kTY), a->batch);
        if (A.K == 8 && A.Kp == 7 && A.C <= kMaxC)
            hipLaunchKernelGGL((ups_level_fixed<8, 7>), grid, dim3(kThreads), 0, s, A);
        else
            hipLaunchKernelGGL(ups_level_kernel, grid, dim3(kThreads), 0, s, A);
        CCMI_HIP_CHECK(hipGetLastError());
    }
    return CCMI_OK;
}
