// train.hip -- the encoder overfit step on the GPU: training forward, backward, gradient
// clipping and Adam for a batch of independent frames (one network + latents each).
//
// Reference, enc/training/train.py:238-262 (one iteration):
//   frame_encoder.forward (train mode)  coolchic.py:291-479, frame.py:175-183
//     quantize            quantizer.py:16-232   (softround / noise / STE variants)
//     ARM + Laplace rate  arm.py:227-370, coolchic.py:395-424
//     Upsampling          upsampling.py:195-202, 322-335, 476-506 (train = kron-2D form,
//                         mathematically the separable eval form computed here)
//     Synthesis           synthesis.py:69-84, 264-277
//     420 nearest + clamp yuv.py:275-299
//   loss_function          loss.py (MSE + lmbda * rate_bpp)
//   loss.backward(); clip_grad_norm_(params, 0.1); torch.optim.Adam.step()
//
// Kernels, in launch order (all frames of the batch in every launch, grid.y = frame):
//   t_prologue    per-step zeroing + trainable half kernels -> full symmetric kernels (upsampling.py:46-68)
//   t_quant       y_hat = Q(gain * y) and dQ/dy; noise from a counter-based RNG (or given)
//   t_arm<D,NH>   ARM forward + rate + full backward in one pass: 4 x 64 latent tile + causal
//                 halo in LDS; context gradients accumulate in an LDS tile (ds_add) and are
//                 flushed with one global atomic per tile position; weight gradients are
//                 reduced per workgroup through LDS into a partial row (summed by t_colsum)
//   (upsampling forward: the path-A level kernels, keeping every pyramid stack)
//   t_head_fwd / t_sp_fwd   synthesis forward, intermediate 3-channel maps kept
//   t_loss        train-mode output (420 nearest, clamp), MSE and its gradient
//   t_sp_gpre / t_sp_bwd    3x3 layers backward (replicate-padding adjoint as a gather)
//   t_head_bwd    1x1 head backward; weight gradients reduced through LDS
//   t_lvl_bwd     upsampling backward, one launch per pyramid level (refine + transposed conv)
//   t_latgrad_sumsq, t_adam      dL/dy + global grad norm, clipped Adam update
#include <stdlib.h>

#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "fwd_common.h"

using ccmi_fwd::cfloat_ptr;

namespace {

constexpr int kT = 256;
constexpr int kMaxSp = 3;
constexpr int kHeadT = 128;
// Parameter gradients: every workgroup that reduces weight / bias gradients (the ARM, the head,
// the 3x3 layers, the upsampling kernels) adds its partial sums into one of kDwSlots copies of
// the frame's parameter-gradient row (slot = workgroup % kDwSlots), and t_dw_fold sums the
// slots into the gradient row once per step: same-address atomics serialise (≈80 ns each), and
// the persistent kernels' workgroups all flush at once at their end.  The ARM's rate sums take
// the same form (kDwSlots per frame).
constexpr int kDwSlots = 32;
constexpr float kLn2 = 0.6931471805599453f;

// Per-frame geometry and parameter offsets (same for every frame of a batch).
struct Geo {
    int L, N, H, W;
    int h[CCMI_MAX_GRIDS], w[CCMI_MAX_GRIDS], off[CCMI_MAX_GRIDS];
    int d, nh, P_arm;
    int K, n_ups, hu, up_off;
    int Kp, n_pre, hp, pre_off;
    int syn_off, hid, r0, r1, w0, b0, w1, b1, P_head;
    int n_sp, sp_w[kMaxSp], sp_b[kMaxSp], sp_res[kMaxSp], sp_relu[kMaxSp];
    int P, kfull;
};

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

// Sum over the wave, in every lane, without an LDS round trip: DPP within the 16-lane rows
// (xor 1, xor 2, half-row mirror, row mirror), then gfx950's permlane16 / permlane32 swaps
// across them.  (The __shfl_xor butterfly is six ds_bpermute_b32 in a dependent chain.)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum(float v)
{
    v += dpp_mov<0xb1>(v);  // quad_perm [1, 0, 3, 2]: lane ^ 1
    v += dpp_mov<0x4e>(v);  // quad_perm [2, 3, 0, 1]: lane ^ 2
    v += dpp_mov<0x141>(v); // row_half_mirror: the other quad of the half-row
    v += dpp_mov<0x140>(v); // row_mirror: the other half of the row
    const auto h = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(h[0]) + __uint_as_float(h[1]);
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

__device__ __forceinline__ float block_sum(float v, float *red)
{
    v = wave_sum(v);
    const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wid] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

// ------------------------------------------------------------------ parameters
// Per-step prologue in one launch (three launches before: a memset, t_zero_rows, t_expand --
// each a dependent dispatch of ~6 us on the step's critical path, profiles/r5l_train_timeline.txt):
// zero nz floats from z (acc4, the rate and parameter-gradient slots, the ARM's side gradient),
// expand the symmetric upsampling kernels, and count the step in the caller's step counters.
__global__ void t_prologue(float *__restrict__ z, int64_t nz, const float *__restrict__ th, int64_t ps, Geo g,
                           float *__restrict__ kf, int B, int32_t *__restrict__ counters)
{
    if (counters && blockIdx.x == 0)
        for (int i = threadIdx.x; i < B; i += kT) counters[i] += 1; // the caller's per-frame step counts
    const int64_t n = nz + (int64_t)B * g.kfull;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        if (i < nz) {
            z[i] = 0.f;
        } else {
            const int j = (int)(i - nz), b = j / g.kfull, e = j - b * g.kfull;
            const float *p = th + (int64_t)b * ps;
            float v;
            if (e < g.n_ups * g.K) {
                const int u = e / g.K, t = e - u * g.K;
                v = p[g.up_off + u * g.hu + min(t, g.K - 1 - t)];
            } else {
                const int r = e - g.n_ups * g.K, u = r / g.Kp, t = r - u * g.Kp;
                v = p[g.pre_off + u * g.hp + min(t, g.Kp - 1 - t)];
            }
            kf[(int64_t)b * g.kfull + e] = v;
        }
    }
}

// ------------------------------------------------------------------ quantizer
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float unif(uint64_t r) { return ((float)(r >> 40) + 0.5f) * 5.9604644775390625e-08f; }

struct SoftRound {
    float t, inv; // inv = 1 / tanh(1 / (2t))
    __device__ float f(float x) const
    {
        const float fx = floorf(x), d = x - fx - 0.5f;
        return fx + 0.5f * tanhf(d / t) * inv + 0.5f;
    }
    __device__ float df(float x) const
    {
        const float fx = floorf(x), th = tanhf((x - fx - 0.5f) / t);
        return 0.5f * (1.f - th * th) / t * inv;
    }
    // f(x) and df(x) from one tanh (the same expressions as f / df)
    __device__ void fdf(float x, float &y, float &d) const
    {
        const float fx = floorf(x), th = tanhf((x - fx - 0.5f) / t);
        y = fx + 0.5f * th * inv + 0.5f;
        d = 0.5f * (1.f - th * th) / t * inv;
    }
};

// Quantiser constants, uniform over the launch (computed once on the host): softround
// temperature and 1 / tanh(1 / 2t); kumaraswamy a, 1 / a and 1 / b (quantizer.py:60-102)
struct QuantArgs {
    float temp, inv, ka_inv, kb_inv, nprm;
};

QuantArgs quant_args(float temp, float nprm)
{
    QuantArgs q{temp, 0.f, 0.f, 0.f, nprm};
    if (temp > 0.f) q.inv = 1.f / std::tanh(1.f / (2.f * temp));
    if (nprm > 0.f) {
        const float a = nprm, b = (std::exp2(a) * (a - 1.f) + 1.f) / a;
        q.ka_inv = 1.f / a;
        q.kb_inv = 1.f / b;
    }
    return q;
}

__global__ void t_quant(const float *__restrict__ lat, int64_t ls, int N, float gain, int qt, int nz, QuantArgs Q,
                        uint64_t seed, int step, const float *__restrict__ noise_in, float *__restrict__ yq,
                        float *__restrict__ dq, float *__restrict__ gq)
{
    const int b = blockIdx.y, i = blockIdx.x * kT + threadIdx.x;
    if (i >= N) return;
    const int64_t li = (int64_t)b * ls + i, wi = (int64_t)b * N + i;
    const float x = gain * lat[li];
    float n = 0.f;
    if (noise_in) {
        n = noise_in[li];
    } else if (nz != CCMI_NOISE_NONE) {
        const uint64_t r = mix64(seed ^ mix64(((uint64_t)step << 40) ^ ((uint64_t)b << 32) ^ (uint64_t)i));
        const float u1 = unif(r);
        if (nz == CCMI_NOISE_KUMARASWAMY) { // generate_kumaraswamy_noise: (1 - (1 - u)^(1/b))^(1/a) - 1/2
            // powers through v_log_f32 / v_exp_f32 (u1 in (0, 1): both bases in (0, 1]); the
            // draw only has to follow the distribution, parity tests pass their noise in
            const float p = exp2f(__log2f(1.f - u1) * Q.kb_inv);
            n = exp2f(__log2f(1.f - p) * Q.ka_inv) - 0.5f;
        } else { // gaussian: Box-Muller
            const float u2 = unif(mix64(r + 0x632BE59BD9B4E019ull));
            n = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2) * Q.nprm;
        }
    }
    const SoftRound s{Q.temp, Q.inv};
    float y, d;
    switch (qt) {
    case CCMI_Q_NONE: y = x + n; d = 1.f; break;
    case CCMI_Q_SOFTROUND_ALONE: s.fdf(x, y, d); break;
    case CCMI_Q_SOFTROUND: {
        float fx, dx, du;
        s.fdf(x, fx, dx);
        s.fdf(fx + n, y, du);
        d = du * dx;
        break;
    }
    case CCMI_Q_STE: y = rintf(x); d = s.df(x); break;
    case CCMI_Q_TRUE_STE: y = rintf(x); d = 1.f; break;
    default: y = rintf(x); d = 0.f; break; // hardround: torch.round has a zero gradient
    }
    yq[wi] = y;
    if (dq) dq[wi] = gain * d;
    if (gq) gq[wi] = 0.f;
}

// ------------------------------------------------------------------ ARM forward + backward
constexpr int kATX = 64, kATY = 4, kAH = 4;
constexpr int kALW = kATX + 2 * kAH, kALH = kATY + kAH;

struct ArmTiles {
    int n, tiles_x[CCMI_MAX_GRIDS], start[CCMI_MAX_GRIDS + 1];
};

template <int D>
__device__ __forceinline__ void ctx_off(int i, int &dy, int &dx)
{
    constexpr signed char k8[8] = {13, 22, 30, 31, 32, 37, 38, 39};
    constexpr signed char k16[16] = {13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39};
    constexpr signed char k24[24] = {4, 11, 12, 13, 14, 15, 19, 20, 21, 22, 23, 24, 25, 28, 29, 30, 31, 32, 33, 34,
                                     36, 37, 38, 39};
    constexpr signed char k32[32] = {2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 19, 20, 21, 22, 23, 24, 25, 26, 27,
                                     28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39};
    const int k = D == 8 ? k8[i] : D == 16 ? k16[i] : D == 24 ? k24[i] : k32[i];
    dy = k / 9 - 4;
    dx = k % 9 - 4;
}

// The context gradients a position (r, c) of the tile + causal halo receives: the gradient of
// every latent of the tile whose context holds it (context input k of the latent at
// (r - kAH - dy_k, c - kAH - dx_k)), plus the latent's own gradient (column D of its s_g row)
// when (r, c) is a latent of the tile.  s_g: [kATY * kATX][D + 1].  Every term's LDS read is
// issued unconditionally -- a term outside the tile reads s_zero -- so a position's D + 1
// reads are in flight together (as `if (inside) v += s_g[..]` they compiled to D + 1
// exec-mask branches with one LDS round trip each).
// Summation order as before (own value, then k = 0 .. D - 1).
template <int D>
__device__ __forceinline__ float gather_ctx(const float *s_g, const float *s_zero, int r, int c)
{
    const int ly0 = r - kAH, lx0 = c - kAH;
    const int base = (ly0 * kATX + lx0) * (D + 1);
    auto inside = [](int ly, int lx) { return (unsigned)ly < (unsigned)kATY && (unsigned)lx < (unsigned)kATX; };
    float t[D + 1];
    t[D] = *(inside(ly0, lx0) ? s_g + base + D : s_zero);
#pragma unroll
    for (int k = 0; k < D; ++k) {
        int dy, dx;
        ctx_off<D>(k, dy, dx);
        t[k] = *(inside(ly0 - dy, lx0 - dx) ? s_g + base + (-dy * kATX - dx) * (D + 1) + k : s_zero);
    }
    // all reads issued before the first add (the scheduler otherwise sinks each read to its
    // add: one LDS round trip per term again)
    __builtin_amdgcn_sched_barrier(0);
    float v = t[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v += t[k];
    return v;
}

typedef float v4f __attribute__((ext_vector_type(4)));

// Lane exchanges between the four 16-lane rows of a wave on gfx950's permlane swaps (VALU ops,
// no LDS round trip as ds_bpermute / __shfl): v_permlane16_swap exchanges rows 1 <-> 0 and
// 3 <-> 2 of its two operands, v_permlane32_swap lanes 32..63 <-> 0..31.
struct f2 {
    float a, b;
};
__device__ __forceinline__ f2 swap16(float x)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return {__uint_as_float(r[0]), __uint_as_float(r[1])}; // {rows 0, 0, 2, 2}, {rows 1, 1, 3, 3}
}
__device__ __forceinline__ f2 swap32(float x)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return {__uint_as_float(r[0]), __uint_as_float(r[1])}; // {rows 0, 1, 0, 1}, {rows 2, 3, 2, 3}
}
// x + x[lane ^ 16], then + the same at lane ^ 32: the sum over the four rows, in every lane
// (the values and their order are those of two __shfl_xor steps)
__device__ __forceinline__ float sum_rows(float x)
{
    const f2 h = swap16(x);
    const f2 q = swap32(h.a + h.b);
    return q.a + q.b;
}
// bc[g] = row g of x, in every row (as __shfl(x, 16 g + (lane & 15)))
__device__ __forceinline__ void bcast_rows(float x, float (&bc)[4])
{
    const f2 h = swap32(x), lo = swap16(h.a), hi = swap16(h.b);
    bc[0] = lo.a;
    bc[1] = lo.b;
    bc[2] = hi.a;
    bc[3] = hi.b;
}
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: an fmaf chain in another order).
// Lane l supplies A[m = l & 15][k = l >> 4] and B[k = l >> 4][n = l & 15]; accumulator
// register r of lane l is D[m = 4 (l >> 4) + r][n = l & 15].
__device__ __forceinline__ v4f mfma4(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
// v_mfma_f32_4x4x1_16b_f32: sixteen independent 4x4 outer products, block bk = l >> 2.  Lane l
// supplies A[bk][m = l & 3] and B[bk][n = l & 3]; accumulator register r of lane l is
// D[bk][m = r][n = l & 3].  2 passes (8 cycles) against 16x16x4's 8 (32 cycles) at a quarter
// of the MACs -- the same MAC rate, so a product whose M or N is 3-8 wide wastes less of it.
__device__ __forceinline__ v4f mfma4x4(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0); }

// One layer's weight gradient over a wave's 64 rows, on the matrix cores:
// acc[mt][nt] += G^T A, G = [64][R] (pitch R + 1, column R zero), A = [64][D] (pitch D + 1,
// column D zero): a GEMM
// whose K is the latent index, 4 latents per MFMA.
// With B = 1 the same A operand also accumulates the bias gradient sum_k A[m][k] (accb).
template <int R, int D, bool BIAS = true>
__device__ __forceinline__ void mfma_outer(const float *s_g, const float *s_a, v4f (&acc)[(R + 15) / 16][(D + 15) / 16],
                                           v4f (&accb)[(R + 15) / 16])
{
    constexpr int MT = (R + 15) / 16, NT = (D + 15) / 16;
    const int lane = threadIdx.x & 63, ln = lane & 15, lk = lane >> 4;
    // operand columns past R / D read the rows' zero pad column (R, D): no exec-mask branch
    // between the LDS reads and the MFMAs
    int ca[MT], cb[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ca[mt] = 16 * mt + ln < R ? 16 * mt + ln : R;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) cb[nt] = 16 * nt + ln < D ? 16 * nt + ln : D;
    // K = rows in the order r = s + 16 lk: the two 16-lane groups of a 32-lane half read rows 16
    // apart, 16 banks apart for the odd pitches D + 1 / R + 1 (4 s + lk put rows 1 apart:
    // a 2-way conflict per read)
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
        const int r = s + 16 * lk;
        float bv[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bv[nt] = s_a[r * (D + 1) + cb[nt]];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const float av = s_g[r * (R + 1) + ca[mt]];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma4(av, bv[nt], acc[mt][nt]);
#if !defined(CCMI_DIAG_ARM_NOBIAS) // diagnostic builds only (tools/arm_diag.sh): wrong results
            if constexpr (BIAS) accb[mt] = mfma4(av, 1.f, accb[mt]);
#endif
        }
    }
}

// mfma_outer's accumulators stored into a wave's partial [R][D] weight-gradient block and its
// [R] bias in LDS (every element is written), for the workgroup-level reduction of the flush
template <int R, int D>
__device__ __forceinline__ void stage_outer(const v4f (&acc)[(R + 15) / 16][(D + 15) / 16], const v4f (&accb)[(R + 15) / 16],
                                            float *dst, float *dstb)
{
    constexpr int MT = (R + 15) / 16, NT = (D + 15) / 16;
    const int lane = threadIdx.x & 63, ln = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = 16 * mt + 4 * lk + r, n = 16 * nt + ln;
                if (m < R && n < D) dst[m * D + n] = acc[mt][nt][r];
                if (nt == 0 && m < R && ln == 0) dstb[m] = accb[mt][r];
            }
}

// Orders a wave's LDS stores before its own later LDS loads of other lanes' rows: a wave's
// LDS instructions execute in order, so only the compiler must not move them across.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum over the wave of v, added to *dst by lane 0.
__device__ __forceinline__ void wave_add(float v, float *dst)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) atomicAdd(dst, v);
}

// weights of the ARM MLP: wave-uniform scalar loads (the diagnostic build replaces them by
// constants to bound their cost -- wrong results, tools/arm_diag.sh)
#if defined(CCMI_DIAG_ARM_NOWLOAD)
#define ARMW(ptr, idx) (0.001f * (float)((idx) & 7))
#else
#define ARMW(ptr, idx) ((ptr)[idx])
#endif
// Laplace rate of one latent and its gradients (coolchic.py:419-424, arm.py:262-266):
// scale = exp(clamp(ls - 4, -4.6, 5)); P = F(q + 1/2) - F(q - 1/2); bits = -log2(max(P, 2^-16)).
// Returns (through refs) the rate in bits (valid latents) and dL/dq, dL/dmu, dL/dls for the
// per-latent rate weight lam (0 when P < 2^-16: clamp_min blocks the gradient).
__device__ __forceinline__ void arm_rate(float q, float mu, float ls, bool valid, float lam, float &rbits, float &g_q,
                                         float &g_mu, float &g_ls)
// One IEEE division (1 / sig) shared by the four |s| / sig terms and the two gradient terms
// (torch divides each time; the products differ from those quotients by at most an ulp of
// the argument, far inside the gradient tolerances -- the exp / expm1 evaluations themselves
// keep their accurate forms, which the tail cancellation of P = F1 - F2 needs).
{
    const float l4 = ls - 4.f, sig = expf(fminf(fmaxf(l4, -4.6f), 5.0f));
    const float inv = 1.f / sig;
    const float s1 = q + 0.5f - mu, s2 = q - 0.5f - mu;
    const float a1 = fabsf(s1) * inv, a2 = fabsf(s2) * inv;
    const float sg1 = s1 > 0.f ? 1.f : (s1 < 0.f ? -1.f : 0.f), sg2 = s2 > 0.f ? 1.f : (s2 < 0.f ? -1.f : 0.f);
    const float F1 = 0.5f - 0.5f * sg1 * expm1f(-a1), F2 = 0.5f - 0.5f * sg2 * expm1f(-a2);
    const float Pr = F1 - F2;
    g_q = 0.f, g_mu = 0.f, g_ls = 0.f, rbits = 0.f;
    if (valid) {
        rbits = -log2f(fmaxf(Pr, 1.52587890625e-05f));
        if (Pr >= 1.52587890625e-05f) { // clamp_min passes the gradient where P >= 2^-16
            const float dLdP = -lam / (Pr * kLn2);
            // torch autograd of 0.5 - 0.5 sign(s) expm1(-|s|/sig): d/ds = 0.5 sign(s)^2 e / sig,
            // d/dsig = -0.5 sign(s) e |s| / sig^2 = -sign(s) (0.5 e / sig) (|s| / sig)
            const float h1 = 0.5f * expf(-a1) * inv, h2 = 0.5f * expf(-a2) * inv;
            const float Fs1 = sg1 * sg1 * h1, Fs2 = sg2 * sg2 * h2;
            const float Fg1 = -sg1 * h1 * a1, Fg2 = -sg2 * h2 * a2;
            g_q = dLdP * (Fs1 - Fs2);
            g_mu = -g_q;
            const float g_sig = dLdP * (Fg1 - Fg2);
            g_ls = (l4 >= -4.6f && l4 <= 5.0f) ? g_sig * sig : 0.f;
        }
    }
}

// waves / SIMD the VALU ARM's registers are budgeted for (3: <= 168 VGPRs); the dim-24 / 32
// ARMs with 2+ hidden layers hold more per-latent state than that (-DCCMI_TARM_WPE24=2 builds
// the A/B variant with their 256-VGPR budget)
#ifndef CCMI_TARM_WPE24
#define CCMI_TARM_WPE24 3
#endif
constexpr int t_arm_wpe(int d, int nh) { return d >= 24 && nh >= 2 ? CCMI_TARM_WPE24 : 3; }

template <int D, int NH>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(t_arm_wpe(D, NH)))) void t_arm(const float *__restrict__ yq, Geo g, ArmTiles at, const float *__restrict__ th,
                                            int64_t ps, float lam_px, float *__restrict__ gq,
                                            float *__restrict__ gth, int64_t gstride, float *__restrict__ acc4,
                                            const float *__restrict__ grad_rate, float *__restrict__ rate_out)
{
    constexpr int NT = (D + 15) / 16, MT = (D + 15) / 16;
    __shared__ float s_y[kALH][kALW];
    // MFMA staging rows (per wave: gradients s_g, activations s_a), one array so the
    // context-gradient planes can span both once the MFMA stage is over
    __shared__ float s_ga[2 * kT * (D + 1)];
    float *const s_g = s_ga, *const s_a = s_ga + kT * (D + 1);
    __shared__ float s_zero[1]; // what the context gather reads for terms outside the tile
    if (threadIdx.x == 0) s_zero[0] = 0.f; // visible after the tile loop's first barrier

    const int b = blockIdx.y;
    const int w = threadIdx.x >> 6;
    const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
    float *sg = s_g + 64 * w * (D + 1), *sa = s_a + 64 * w * (D + 1); // this wave's rows
    const int cx = threadIdx.x % kATX, cy = threadIdx.x / kATX;
    // weight-gradient accumulators (matrix cores) and bias-gradient sums (VALU), kept over
    // every tile this workgroup visits
    v4f acc_o[1][NT], acc_h[NH > 0 ? NH : 1][MT][NT], accb_o[1], accb_h[NH > 0 ? NH : 1][MT];
    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    accb_o[0] = z4;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc_o[0][nt] = z4;
#pragma unroll
    for (int L = 0; L < (NH > 0 ? NH : 1); ++L)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            accb_h[L][mt] = z4;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc_h[L][mt][nt] = z4;
        }
    float rsum = 0.f;

    // the latent tile (+ causal halo) of the NEXT tile is loaded into registers while this
    // one is processed, so a tile starts without waiting on HBM
    constexpr int kSU = (kALH * kALW + kT - 1) / kT;
    float pre[kSU];
    auto tile_geo = [&](int t, int &l, int &y0, int &x0) {
        l = 0;
#pragma unroll
        for (int k = 1; k < CCMI_MAX_GRIDS; ++k)
            if (k < at.n && t >= at.start[k]) l = k;
        const int lt = t - at.start[l];
        y0 = (lt / at.tiles_x[l]) * kATY;
        x0 = (lt % at.tiles_x[l]) * kATX;
    };
    auto load_tile = [&](int t) {
        int l, y0, x0;
        tile_geo(t, l, y0, x0);
        const int H = g.h[l], W = g.w[l];
        const float *src = yq + (int64_t)b * g.N + g.off[l];
        int tid = threadIdx.x; // opaque: its tile-invariant indices are not hoisted and kept live
        asm volatile("" : "+v"(tid));
#pragma unroll
        for (int u = 0; u < kSU; ++u) {
            const int i = tid + u * kT;
            const int r = i / kALW, c = i - r * kALW;
            const int y = y0 - kAH + r, x = x0 - kAH + c;
            pre[u] = (i < kALH * kALW && y >= 0 && y < H && x >= 0 && x < W) ? src[y * W + x] : 0.f;
        }
    };
    const int n_tiles = at.start[at.n];
    if ((int)blockIdx.x < n_tiles) load_tile(blockIdx.x);

    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        int l, y0, x0;
        tile_geo(t, l, y0, x0);
        const int H = g.h[l], W = g.w[l];
        float *gdst = gq + (int64_t)b * g.N + g.off[l];
        __syncthreads(); // previous tile's LDS readers are done
#pragma unroll
        for (int u = 0; u < kSU; ++u) {
            const int i = threadIdx.x + u * kT;
            if (i < kALH * kALW) (&s_y[0][0])[i] = pre[u];
        }
        if (t + (int)gridDim.x < n_tiles) load_tile(t + gridDim.x);
        __syncthreads();
        const bool valid = (y0 + cy) < H && (x0 + cx) < W;

        float xs[NH + 1][D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            int dy, dx;
            ctx_off<D>(i, dy, dx);
            xs[0][i] = s_y[cy + kAH + dy][cx + kAH + dx];
        }
#pragma unroll
        for (int L = 0; L < NH; ++L) {
            const cfloat_ptr Wl = P + L * (D * D + D);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                float z = ARMW(Wl, D * D + j);
#pragma unroll
                for (int i = 0; i < D; ++i) z = fmaf(ARMW(Wl, j * D + i), xs[L][i], z);
                z += xs[L][j];
                xs[L + 1][j] = fmaxf(z, 0.f);
            }
        }
        const cfloat_ptr Wo = P + NH * (D * D + D);
        float mu = ARMW(Wo, 2 * D), ls = ARMW(Wo, 2 * D + 1);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            mu = fmaf(ARMW(Wo, i), xs[NH][i], mu);
            ls = fmaf(ARMW(Wo, D + i), xs[NH][i], ls);
        }
        const float q = s_y[cy + kAH][cx + kAH];
        float g_q, g_mu, g_ls, rbits;
        {
            const int64_t li = (int64_t)b * g.N + g.off[l] + (int64_t)(y0 + cy) * W + (x0 + cx);
            float lam = lam_px;
            if (valid && grad_rate) {
                lam = grad_rate[li];
                // waited for here: at the use below, past the branch, the compiler's wait is a
                // vmcnt(0) on every path -- also behind the next tile's prefetch loads and the
                // gather atomics when there is no grad_rate (training)
                __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
            }
            arm_rate(q, mu, ls, valid, lam, rbits, g_q, g_mu, g_ls);
            if (valid) {
                rsum += rbits;
                if (rate_out) rate_out[li] = rbits;
            }
        }
        // ---- backward through the MLP; weight gradients on the matrix cores
        float gx[D];
        {
#pragma unroll
            for (int i = 0; i < D; ++i) gx[i] = ARMW(Wo, i) * g_mu + ARMW(Wo, D + i) * g_ls;
            sg[(threadIdx.x & 63) * 3 + 0] = g_mu; // [64][2], pitch 3, column 2 zero
            sg[(threadIdx.x & 63) * 3 + 1] = g_ls;
            sg[(threadIdx.x & 63) * 3 + 2] = 0.f;
#pragma unroll
            for (int i = 0; i < D; ++i) sa[(threadIdx.x & 63) * (D + 1) + i] = xs[NH][i];
            sa[(threadIdx.x & 63) * (D + 1) + D] = 0.f;
            wave_lds_sync(); // each wave stages and reads only its own 64 rows
#if !defined(CCMI_DIAG_ARM_NOOUTER)
            mfma_outer<2, D>(sg, sa, acc_o, accb_o);
#endif
            wave_lds_sync();
        }
#pragma unroll
        for (int L = NH - 1; L >= 0; --L) {
            const cfloat_ptr Wl = P + L * (D * D + D);
            float gz[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                gz[j] = xs[L + 1][j] > 0.f ? gx[j] : 0.f;
                sg[(threadIdx.x & 63) * (D + 1) + j] = gz[j];
            }
            sg[(threadIdx.x & 63) * (D + 1) + D] = 0.f;
#pragma unroll
            for (int i = 0; i < D; ++i) sa[(threadIdx.x & 63) * (D + 1) + i] = xs[L][i];
            sa[(threadIdx.x & 63) * (D + 1) + D] = 0.f;
            wave_lds_sync();
#if !defined(CCMI_DIAG_ARM_NOOUTER)
            mfma_outer<D, D>(sg, sa, acc_h[L], accb_h[L]);
#endif
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < D; ++i) {
                float a = gz[i]; // residual
#pragma unroll
                for (int j = 0; j < D; ++j) a = fmaf(ARMW(Wl, j * D + i), gz[j], a);
                gx[i] = a;
            }
        }
        // ---- context gradients: each latent's D + 1 gradients (contexts, then its own value)
        // go to LDS rows (this wave's own rows of s_g, free after its MFMA stage); every
        // position of the tile + causal halo then GATHERS what the latents whose context holds
        // it send, and adds the sum to HBM with one atomic.  (Scattering with LDS float atomics
        // instead runs at about half a lane per clock on gfx950: 35 % of this kernel; a
        // row-per-wave gather over zero-padded planes measured slower than this form.)
        {
            float *row = sg + (threadIdx.x & 63) * (D + 1);
#pragma unroll
            for (int i = 0; i < D; ++i) row[i] = valid ? gx[i] : 0.f;
            row[D] = valid ? g_q : 0.f;
        }
        __syncthreads();
        // the context of dims 8 / 16 reaches 3 rows up (halo row 0 receives nothing); that of
        // dims 24 / 32 reaches 4 (offsets 4 and 2..5 of ctx_off: dy = -4)
        constexpr int kR0 = D >= 24 ? 0 : 1;
        // a fixed number of atomics per thread (positions past the halo or outside the grid add
        // 0 at a clamped in-grid address): the next tile's staging then waits for its prefetch
        // loads only, not for these atomics; indices from an opaque thread index (not hoisted)
        constexpr int kGN = (kALH - kR0) * kALW, kGI = (kGN + kT - 1) / kT;
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
#pragma unroll
        for (int u = 0; u < kGI; ++u) {
            const int i = tid + u * kT;
            const int r = kR0 + i / kALW, c = i - (r - kR0) * kALW;
            const int y = y0 - kAH + r, x = x0 - kAH + c;
            const float v = gather_ctx<D>(s_g, s_zero, r, c);
            const bool in = i < kGN && y >= 0 && y < H && x >= 0 && x < W;
            atomicAdd(&gdst[min(max(y, 0), H - 1) * W + min(max(x, 0), W - 1)], in ? v : 0.f);
        }
    }
    // ---- flush: the four waves' weight / bias gradients meet in LDS, then one atomic per value
    // per workgroup (see t_arm16's flush)
    static_assert(kT == 4 * 64, "four waves per workgroup");
    constexpr int LS = D * D + D, kRed = NH * LS + 2 * D + 2;
    static_assert(4 * kRed <= 2 * kT * (D + 1), "the partial rows fit s_ga");
    float *red = s_ga + w * kRed;
    __syncthreads(); // last tile's gather reads of s_g are done
    stage_outer<2, D>(acc_o, accb_o, red + NH * LS, red + NH * LS + 2 * D);
#pragma unroll
    for (int L = 0; L < NH; ++L) stage_outer<D, D>(acc_h[L], accb_h[L], red + L * LS, red + L * LS + D * D);
    __syncthreads();
    float *G = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
    for (int e = threadIdx.x; e < kRed; e += kT)
        atomicAdd(&G[e], (s_ga[e] + s_ga[kRed + e]) + (s_ga[2 * kRed + e] + s_ga[3 * kRed + e]));
    wave_add(rsum, &acc4[b * kDwSlots + blockIdx.x % kDwSlots]); // the frame's rate slots
}

// ARM forward + rate + backward for dim_arm = 16 with the MLP on the matrix cores.
// A wave owns one 64-latent row of the 4 x 64 tile, as 4 groups of 16 latents.  Each
// 16 x 16 layer is Z^T = W X^T on v_mfma_f32_16x16x4_f32 (A = W, B = X^T, K = the layer's
// inputs), with the K order permuted so that input k = 4 (lane >> 4) + s: the accumulator
// register r of lane l then holds unit 4 (l >> 4) + r of latent l & 15 -- exactly the B
// operand of the next layer, so activations never leave the registers, and residual, bias
// and ReLU are elementwise on the accumulators.  The weights (W for the forward, W^T for
// the input gradients, the output layer) are loaded from HBM ONCE per workgroup (one frame)
// into LDS and read from there per tile: no per-tile global weight loads (their scalar-load
// waits were 37 % of the VALU kernel, tools/arm_diag.sh NOWLOAD).  The 2-wide output layer and the rate are VALU
// (an M = 2 MFMA would be 8x padding); the rate runs one latent per lane (lane = tile
// column: group g's values sit in the lanes with lane >> 4 == g).  Weight gradients of the
// hidden layers: LDS-staged rows on the matrix cores (mfma_outer, K = latents); biases and
// the output layer's weight gradients: per-lane partial sums over every tile the workgroup
// visits, reduced once at the end.
// waves / SIMD the register allocation targets: 4 (<= 128 VGPRs) for up to two hidden layers --
// the few values it spills are the epilogue's, outside the tile loop -- 3 for three
#ifndef CCMI_ARM16_WAVES
#define CCMI_ARM16_WAVES 4
#endif
constexpr int t_arm16_wpe(int nh) { return nh <= 2 ? CCMI_ARM16_WAVES : 3; }
template <int NH>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(t_arm16_wpe(NH)))) void t_arm16(
    const float *__restrict__ yq, Geo g, ArmTiles at, const float *__restrict__ th, int64_t ps, float lam_px,
    float *__restrict__ gq, float *__restrict__ gth, int64_t gstride, float *__restrict__ acc4,
    const float *__restrict__ grad_rate, float *__restrict__ rate_out)
{
    constexpr int D = 16, LS = D * D + D, NL = NH > 0 ? NH : 1;
    __shared__ float s_y[kALH][kALW];
    __shared__ float s_ga[2 * kT * (D + 1)];
    float *const s_g = s_ga, *const s_a = s_ga + kT * (D + 1);
    __shared__ float s_zero[1]; // what the context gather reads for terms outside the tile
    if (threadIdx.x == 0) s_zero[0] = 0.f; // visible after the tile loop's first barrier
    const int b = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63, ln = lane & 15, lk = lane >> 4;
    const int cy = w, cx = lane; // per-latent phase: this lane's latent in the tile
    const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
    float *sg = s_g + 64 * w * (D + 1), *sa = s_a + 64 * w * (D + 1);

    // the hidden layers' weights and biases in LDS (2.2 KB for two layers: the workgroup's LDS
    // stays <= 40 KB, 4 workgroups per CU), read per tile as the MFMA A operands: held in
    // registers (24 VGPRs) they pushed the kernel past 128 VGPRs into scratch
    __shared__ __attribute__((aligned(16))) float s_w[NL][LS];
    for (int i = threadIdx.x; i < NH * LS; i += kT) s_w[i / LS][i % LS] = P[i];
    const cfloat_ptr Wo = P + NH * LS;
    // the output layer's weights in LDS too, read where used (8 fewer persistent VGPRs)
    __shared__ __attribute__((aligned(16))) float s_wo[2 * D];
    for (int i = threadIdx.x; i < 2 * D; i += kT) s_wo[i] = Wo[i];
    const float bo0 = Wo[2 * D], bo1 = Wo[2 * D + 1];
    // s_y offsets of the context inputs k = 4 lk + s, derived per tile from an opaque lane
    // index (kept across the tile loop they were 4 more persistent VGPRs)
    auto ctx_offsets = [&](int (&coff)[4]) {
        int lko = lk;
        asm volatile("" : "+v"(lko));
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            int o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                int dy, dx;
                ctx_off<D>(4 * q + s, dy, dx);
                o[q] = dy * kALW + dx;
            }
            coff[s] = lko == 0 ? o[0] : lko == 1 ? o[1] : lko == 2 ? o[2] : o[3];
        }
    };

    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    v4f acc_h[NL][1][1], accb_dummy[1];
    float accb[NL][4], accwo0[4], accwo1[4];
#pragma unroll
    for (int L = 0; L < NL; ++L) {
        acc_h[L][0][0] = z4;
#pragma unroll
        for (int r = 0; r < 4; ++r) accb[L][r] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) accwo0[r] = accwo1[r] = 0.f;
    float accbo0 = 0.f, accbo1 = 0.f, rsum = 0.f;

    constexpr int kSU = (kALH * kALW + kT - 1) / kT;
    float pre[kSU];
    auto tile_geo = [&](int t, int &l, int &y0, int &x0) {
        l = 0;
#pragma unroll
        for (int k = 1; k < CCMI_MAX_GRIDS; ++k)
            if (k < at.n && t >= at.start[k]) l = k;
        const int lt = t - at.start[l];
        y0 = (lt / at.tiles_x[l]) * kATY;
        x0 = (lt % at.tiles_x[l]) * kATX;
    };
    auto load_tile = [&](int t) {
        int l, y0, x0;
        tile_geo(t, l, y0, x0);
        const int H = g.h[l], W = g.w[l];
        const float *src = yq + (int64_t)b * g.N + g.off[l];
        // the staging indices from an opaque thread index, re-derived per tile: hoisted, two
        // of them were spilled and their reloads' vmcnt(0) inside this prefetch waited for the
        // previous tile's gather atomics (measured neutral, 232 us either way: r6k)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
#pragma unroll
        for (int u = 0; u < kSU; ++u) {
            const int i = tid + u * kT;
            const int r = i / kALW, c = i - r * kALW;
            const int y = y0 - kAH + r, x = x0 - kAH + c;
            pre[u] = (i < kALH * kALW && y >= 0 && y < H && x >= 0 && x < W) ? src[y * W + x] : 0.f;
        }
    };
    const int n_tiles = at.start[at.n];
    if ((int)blockIdx.x < n_tiles) load_tile(blockIdx.x);

    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        int l, y0, x0;
        tile_geo(t, l, y0, x0);
        const int H = g.h[l], W = g.w[l];
        float *gdst = gq + (int64_t)b * g.N + g.off[l];
        __syncthreads(); // previous tile's LDS readers are done
#pragma unroll
        for (int u = 0; u < kSU; ++u) {
            const int i = threadIdx.x + u * kT;
            if (i < kALH * kALW) (&s_y[0][0])[i] = pre[u];
        }
        if (t + (int)gridDim.x < n_tiles) load_tile(t + gridDim.x);
        __syncthreads();
        const bool valid = (y0 + cy) < H && (x0 + cx) < W;

        // ---- forward: X[L][g][r] = input / activation unit 4 lk + r of latent 16 g + ln.
        // What the backward needs of the hidden activations is kept small: their ReLU masks (as
        // lane masks, SGPRs), and the input of the last hidden
        // layer (X[NH - 1], NH >= 2) staged in this wave's rows of s_a right away, where that
        // layer's weight-gradient MFMAs read it -- 32 fewer live VGPRs across the backward, so
        // the kernel fits 4 waves / SIMD without spills (round 3: 168 VGPRs + 13 spilled, and
        // the spill reloads' vmcnt(0) waited for the previous tile's gradient atomics)
        const float *yrow = &s_y[cy + kAH][kAH + ln];
        int coff[4];
        ctx_offsets(coff);
        float X[NH + 1][4][4];
        bool pos[NL][4][4]; // ReLU masks: lane masks in SGPR pairs, one v_cndmask each in the backward
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
            for (int s = 0; s < 4; ++s) X[0][gg][s] = yrow[16 * gg + coff[s]];
#pragma unroll
        for (int L = 0; L < NH; ++L) {
            // A = W[j = ln][i = 4 lk + s]; bias of unit 4 lk + r
            const v4f WA = *reinterpret_cast<const v4f *>(&s_w[L][ln * D + 4 * lk]);
            const v4f BI = *reinterpret_cast<const v4f *>(&s_w[L][D * D + 4 * lk]);
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                v4f acc = BI;
#pragma unroll
                for (int s = 0; s < 4; ++s) acc = mfma4(WA[s], X[L][gg][s], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    X[L + 1][gg][r] = fmaxf(acc[r] + X[L][gg][r], 0.f);
                    pos[L][gg][r] = X[L + 1][gg][r] > 0.f;
                    if (NH >= 2 && L + 1 == NH - 1) sa[(16 * gg + ln) * (D + 1) + 4 * lk + r] = X[L + 1][gg][r];
                }
            }
        }
        // output layer: partial dot products over this lane's 4 units, summed over the 4
        // lanes of the latent; group g's (mu, ls) kept by the lanes with lk == g
        float mu = 0.f, ls = 0.f;
        v4f WO0 = *reinterpret_cast<const v4f *>(&s_wo[4 * lk]), WO1 = *reinterpret_cast<const v4f *>(&s_wo[D + 4 * lk]);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            float pm = 0.f, pl = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pm = fmaf(WO0[r], X[NH][gg][r], pm);
                pl = fmaf(WO1[r], X[NH][gg][r], pl);
            }
            pm = sum_rows(pm);
            pl = sum_rows(pl);
            if (gg == lk) {
                mu = pm + bo0;
                ls = pl + bo1;
            }
        }
        // ---- rate, one latent per lane
        const float q = s_y[cy + kAH][cx + kAH];
        float g_q, g_mu, g_ls, rbits;
        {
            const int64_t li = (int64_t)b * g.N + g.off[l] + (int64_t)(y0 + cy) * W + (x0 + cx);
            float lam = lam_px;
            if (valid && grad_rate) {
                lam = grad_rate[li];
                // waited for here: at the use below, past the branch, the compiler's wait is a
                // vmcnt(0) on every path -- also behind the next tile's prefetch loads and the
                // gather atomics when there is no grad_rate (training)
                __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
            }
#if defined(CCMI_DIAG_A16_NORATE) // diagnostic builds only (tools/arm_diag.sh): wrong results
            rbits = mu; g_q = ls * lam; g_mu = q * ls; g_ls = mu * q;
#else
            arm_rate(q, mu, ls, valid, lam, rbits, g_q, g_mu, g_ls);
#endif
            if (valid) {
                rsum += rbits;
                if (rate_out) rate_out[li] = rbits;
            }
        }
        accbo0 += g_mu;
        accbo1 += g_ls;
        // ---- backward: output layer (VALU), its weight gradients as per-lane partial sums
        WO0 = *reinterpret_cast<const v4f *>(&s_wo[4 * lk]);
        WO1 = *reinterpret_cast<const v4f *>(&s_wo[D + 4 * lk]);
        float G[4][4], gmb[4], glb[4];
        bcast_rows(g_mu, gmb);
        bcast_rows(g_ls, glb);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const float gm = gmb[gg], gl = glb[gg];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                G[gg][r] = WO0[r] * gm + WO1[r] * gl;
                accwo0[r] = fmaf(gm, X[NH][gg][r], accwo0[r]);
                accwo1[r] = fmaf(gl, X[NH][gg][r], accwo1[r]);
            }
        }
        // hidden layers
#pragma unroll
        for (int L = NH - 1; L >= 0; --L) {
            float gz[4][4];
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    gz[gg][r] = pos[L][gg][r] ? G[gg][r] : 0.f;
                    sg[(16 * gg + ln) * (D + 1) + 4 * lk + r] = gz[gg][r];
                    // layer 0's input is the context, re-read from the tile (not kept live);
                    // the last hidden layer's input was staged by the forward
                    if (L == 0) sa[(16 * gg + ln) * (D + 1) + 4 * lk + r] = yrow[16 * gg + coff[r]];
                    else if (L != NH - 1) sa[(16 * gg + ln) * (D + 1) + 4 * lk + r] = X[L][gg][r];
                }
#pragma unroll
            for (int r = 0; r < 4; ++r) accb[L][r] += (gz[0][r] + gz[1][r]) + (gz[2][r] + gz[3][r]);
            wave_lds_sync(); // each wave stages and reads only its own 64 rows
#if !defined(CCMI_DIAG_A16_NOOUTER)
            mfma_outer<D, D, false>(sg, sa, acc_h[L], accb_dummy);
#endif
            wave_lds_sync();
            // input gradient: W^T gz + gz (residual), K permuted like the forward;
            // A = W^T[i = ln][j = 4 lk + s]
            float WT[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) WT[s] = s_w[L][(4 * lk + s) * D + ln];
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                v4f acc = {gz[gg][0], gz[gg][1], gz[gg][2], gz[gg][3]};
#pragma unroll
                for (int s = 0; s < 4; ++s) acc = mfma4(WT[s], gz[gg][s], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) G[gg][r] = acc[r];
            }
        }
        // ---- context gradients (input k = 4 lk + r of latent 16 g + ln) and the latent's own
        // gradient to this wave's rows of s_g, then the gather of t_arm
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
            for (int r = 0; r < 4; ++r) sg[(16 * gg + ln) * (D + 1) + 4 * lk + r] = G[gg][r];
        sg[lane * (D + 1) + D] = g_q;
        __syncthreads();
        // exactly two atomics per thread (positions past the halo, or outside the grid, add 0 at
        // a clamped in-grid address): with a fixed count after the next tile's prefetch loads,
        // the next tile's staging waits for those loads only (vmcnt(2)), not for these atomics
        static_assert((kALH - 1) * kALW <= 2 * kT, "two gather positions per thread");
        // the positions' tile-invariant indices are re-derived from an opaque copy of the
        // thread index per tile: hoisted out of the tile loop they held ~60 VGPRs
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
#if defined(CCMI_DIAG_A16_NOGATHER)
        if (tid < 0)
#endif
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + u * kT;
            const int r = 1 + i / kALW, c = i - (r - 1) * kALW;
            const int y = y0 - kAH + r, x = x0 - kAH + c;
            const float v = gather_ctx<D>(s_g, s_zero, r, c);
            const bool in = i < (kALH - 1) * kALW && y >= 0 && y < H && x >= 0 && x < W;
            atomicAdd(&gdst[min(max(y, 0), H - 1) * W + min(max(x, 0), W - 1)], in ? v : 0.f);
        }
    }
#if defined(CCMI_DIAG_NOFLUSH) // diagnostic build only (make diag): wrong results -- and with the
    return;                       // accumulators dead, the compiler drops the weight-gradient work too
#endif
    // ---- flush: the four waves' partial sums meet in LDS (s_ga is free after the tile loop) and
    // each value goes out with ONE atomic per workgroup.  (One atomic per value per wave, every
    // workgroup of a frame on the same ~600 addresses, serialised in L2: the kernel's time grew
    // linearly with its grid -- 293 / 460 / 572 / 745 us for 1024 / 2048 / 3072 / 4096
    // workgroups, profiles/r4l_*.)
    static_assert(kT == 4 * 64, "four waves per workgroup");
    constexpr int kRed = NH * LS + 2 * D + 2; // the gradient row's ARM part, Gp layout
    float *red = s_ga + w * kRed;             // this wave's partial row
    __syncthreads();                          // last tile's gather reads of s_g are done
#pragma unroll
    for (int L = 0; L < NH; ++L) {
#pragma unroll
        for (int r = 0; r < 4; ++r) { // dW_L[m = 4 lk + r][n = ln]
            red[L * LS + (4 * lk + r) * D + ln] = acc_h[L][0][0][r];
            float v = accb[L][r];
            for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
            if (ln == 0) red[L * LS + D * D + 4 * lk + r] = v;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float v0 = accwo0[r], v1 = accwo1[r];
        for (int o = 1; o < 16; o <<= 1) {
            v0 += __shfl_xor(v0, o);
            v1 += __shfl_xor(v1, o);
        }
        if (ln == 0) {
            red[NH * LS + 4 * lk + r] = v0;
            red[NH * LS + D + 4 * lk + r] = v1;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        accbo0 += __shfl_xor(accbo0, o);
        accbo1 += __shfl_xor(accbo1, o);
    }
    if (lane == 0) {
        red[NH * LS + 2 * D] = accbo0;
        red[NH * LS + 2 * D + 1] = accbo1;
    }
    __syncthreads();
    float *Gp = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
    for (int e = threadIdx.x; e < kRed; e += kT)
        atomicAdd(&Gp[e], (s_ga[e] + s_ga[kRed + e]) + (s_ga[2 * kRed + e] + s_ga[3 * kRed + e]));
    wave_add(rsum, &acc4[b * kDwSlots + blockIdx.x % kDwSlots]); // the frame's rate slots
}

// Column sums of per-workgroup partial rows: dst[b][col] += sum_r part[b][r][col].
__global__ void t_colsum(const float *__restrict__ part, int nrows, int ncols, float *__restrict__ dst, int64_t dstride)
{
    __shared__ float s[4][64];
    const int b = blockIdx.z, col = blockIdx.x * 64 + threadIdx.x;
    const int r0 = blockIdx.y * 256;
    float acc = 0.f;
    if (col < ncols) {
        const float *p = part + (int64_t)b * nrows * ncols;
        for (int r = r0 + threadIdx.y; r < min(nrows, r0 + 256); r += 4) acc += p[(int64_t)r * ncols + col];
    }
    s[threadIdx.y][threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.y == 0 && col < ncols)
        atomicAdd(&dst[(int64_t)b * dstride + col], s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x]);
}

// ------------------------------------------------------------------ synthesis
// Four pixels per thread (p + u kT of the workgroup's 4 kT, u = 0..3, as two packed pairs):
// each broadcast weight record serves four pixels, a quarter of the one-pixel form's LDS record
// traffic per pixel (that form sat 56 % of its wave cycles in SQ_WAIT_INST_LDS, the two-pixel
// form still 55 %, profiles/r5d_train_pmc.txt).  Record slots 3, 7, 11 stay empty when the
// fields fit without them (the compiler copies a broadcast operand out of the last dword of a
// ds_read_b128 first), as in the path-A fused kernel.
constexpr int kHeadFwdPx = 4 * kT; // pixels per workgroup
template <int CIN>
__global__ __launch_bounds__(kT) void t_head_fwd(const float *__restrict__ dense, Geo g, const float *__restrict__ th,
                                                 int64_t ps, float *__restrict__ z0)
{
    using ccmi_fwd::f2;
    constexpr bool kPad = CIN + 4 <= 12;
    auto hr = [](int f) constexpr { return kPad ? f + f / 3 : f; };
    __shared__ __attribute__((aligned(16))) float s_rec[64][16];
    static_assert(CIN + 4 <= 16, "hidden-unit record");
    const int b = blockIdx.y, hid = g.hid;
    const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
    for (int e = threadIdx.x; e < 64 * 16; e += kT) {
        const int j = e >> 4, f = e & 15;
        float v = 0.f;
        if (j < hid) {
            if (f < CIN) v = P[g.w0 + j * CIN + f];
            else if (f == CIN) v = P[g.b0 + j];
            else if (f <= CIN + 3) v = P[g.w1 + (f - CIN - 1) * hid + j];
        }
        if (f <= CIN + 3) s_rec[j][hr(f)] = v;
    }
    const int64_t npx = (int64_t)g.H * g.W, p0 = (int64_t)blockIdx.x * kHeadFwdPx + threadIdx.x;
    const float *x = dense + (int64_t)b * CIN * npx;
    // pair q = pixels p0 + 2q kT, p0 + (2q + 1) kT (zeros past the frame)
    f2 xv[2][CIN];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int64_t pa = p0 + 2 * q * kT, pb = pa + kT;
#pragma unroll
        for (int i = 0; i < CIN; ++i) xv[q][i] = f2{pa < npx ? x[i * npx + pa] : 0.f, pb < npx ? x[i * npx + pb] : 0.f};
    }
    __syncthreads();
    const f2 lo0 = f2(g.r0 ? 0.f : -INFINITY);
    f2 o[2][3];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int m = 0; m < 3; ++m) o[q][m] = f2(P[g.b1 + m]);
#pragma unroll 4
    for (int j = 0; j < hid; ++j) {
        const float *r = s_rec[j];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            f2 h = f2(r[hr(CIN)]);
#pragma unroll
            for (int i = 0; i < CIN; ++i) h = __builtin_elementwise_fma(f2(r[hr(i)]), xv[q][i], h);
            h = __builtin_elementwise_max(h, lo0);
#pragma unroll
            for (int m = 0; m < 3; ++m) o[q][m] = __builtin_elementwise_fma(f2(r[hr(CIN + 1 + m)]), h, o[q][m]);
        }
    }
    float *z = z0 + (int64_t)b * 3 * npx;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            f2 v = o[q][m];
            if (g.r1) v = __builtin_elementwise_max(v, f2(0.f));
            const int64_t pa = p0 + 2 * q * kT, pb = pa + kT;
            if (pa < npx) z[m * npx + pa] = v.x;
            if (pb < npx) z[m * npx + pb] = v.y;
        }
}

// 3x3, 3 -> 3, replicate padding (synthesis.py:69-84), optional residual / ReLU.  A thread
// computes kSpRows vertically consecutive pixels of one column: the rows it reads overlap, so
// it loads (kSpRows + 2) x 3 neighbours per channel instead of 9 per pixel (one pixel per
// thread issued 27 loads per pixel); same FMA order per pixel.
// LOSS (the last layer of a training step): t_loss's MSE fused in -- the layer's output is
// consumed where it is produced (its gradient graw, the squared errors into the frame's mse
// slots) and stored only when store_out (a ReLU's mask for the backward, or the caller's raw
// output).  1: 444 target; 2: 420 target (chroma at even rows / columns, frame.py:175-183).
constexpr int kSpRows = 4;
template <int LOSS>
__global__ __launch_bounds__(kT) void t_sp_fwd(const float *__restrict__ in, Geo g, const float *__restrict__ th, int64_t ps,
                                               int wo, int bo, int res, int relu, float *__restrict__ out,
                                               const float *__restrict__ tgt, int64_t tstride, float k2,
                                               float *__restrict__ graw, float *__restrict__ mslots, int store_out)
{
    // 1-D grid of (blocks per frame) x frames in XCD-aware order: the row groups above and below,
    // which load 2 of the same rows, run on one L2
    const int per = (((g.H + kSpRows - 1) / kSpRows) * g.W + kT - 1) / kT; // blocks per frame
    const int wt = ccmi_fwd::xcd_order(blockIdx.x, gridDim.x);
    const int b = wt / per;
    const int64_t npx = (int64_t)g.H * g.W;
    const int q = (wt - b * per) * kT + threadIdx.x; // (row group, column); a frame fits 31 bits
    const int gy = q / g.W, px = q - gy * g.W, y0 = gy * kSpRows;
    float se = 0.f;
    if (y0 < g.H) { // (no early return: the fused loss's block reduction needs every thread)
        const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
        const float *x = in + (int64_t)b * 3 * npx;
        int xo[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) xo[d] = clampi(px + d - 1, g.W - 1);
        float v[3][kSpRows + 2][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int r = 0; r < kSpRows + 2; ++r) {
                const float *row = x + i * npx + (int64_t)clampi(y0 + r - 1, g.H - 1) * g.W;
#pragma unroll
                for (int d = 0; d < 3; ++d) v[i][r][d] = row[xo[d]];
            }
        const int64_t pix = (int64_t)y0 * g.W + px;
        float *o = out + (int64_t)b * 3 * npx + pix;
        const int h2 = g.H / 2, w2 = g.W / 2;
        // the fused loss's target values, loaded with the inputs (loaded where used, each was a
        // dependent memory latency per output: 62 % of the wave cycles in WAIT_ANY,
        // profiles/r5zk_train_pmc.txt)
        float tv[LOSS > 0 ? kSpRows : 1][3];
        bool tu[LOSS > 0 ? kSpRows : 1][3];
        if constexpr (LOSS > 0) {
#pragma unroll
            for (int t = 0; t < kSpRows; ++t)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const int y = y0 + t;
                    bool used = y < g.H;
                    int64_t ti = c * npx + (int64_t)y * g.W + px;
                    if (LOSS == 2 && c > 0) {
                        used = used && (y % 2 == 0) && (px % 2 == 0) && (y / 2) < h2 && (px / 2) < w2;
                        ti = npx + (int64_t)(c - 1) * h2 * w2 + (int64_t)(y / 2) * w2 + px / 2;
                    }
                    tu[t][c] = used;
                    tv[t][c] = used ? tgt[(int64_t)b * tstride + ti] : 0.f;
                }
        }
#pragma unroll
        for (int t = 0; t < kSpRows; ++t) {
            if (y0 + t >= g.H) break;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float a = P[bo + c];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 9; ++k) a = fmaf(P[wo + (c * 3 + i) * 9 + k], v[i][t + k / 3][k % 3], a);
                if (res) a += v[c][t + 1][1];
                if (relu) a = fmaxf(a, 0.f);
                const int64_t e = c * npx + (int64_t)t * g.W;
                if (LOSS == 0 || store_out) o[e] = a;
                if constexpr (LOSS > 0) { // t_loss on this pixel, same arithmetic
                    float gv = 0.f;
                    if (tu[t][c]) {
                        const float vc = fminf(fmaxf(a, 0.f), 1.f), d = vc - tv[t][c];
                        se += d * d;
                        gv = (a >= 0.f && a <= 1.f) ? k2 * d : 0.f;
                    }
                    graw[(int64_t)b * 3 * npx + e + pix] = gv;
                }
            }
        }
    }
    if constexpr (LOSS > 0) {
        __shared__ float s_red[8];
        const float sum = block_sum(se, s_red);
        if (threadIdx.x == 0) atomicAdd(&mslots[b * kDwSlots + blockIdx.x % kDwSlots], sum);
    }
}

// Train-mode frame output + MSE (frame.py:175-183, loss.py _compute_mse): gradient of the
// MSE w.r.t. the raw synthesis output; sum of squared errors into acc4[b][0].
// 444: kLossPx pixels per thread and iteration with every load issued first (one pixel per
// iteration left the kernel waiting on memory latency: 82 % of its wave cycles in WAIT_ANY at
// 2 waves / SIMD, profiles/r5l_train_pmc.txt); 420: the chroma planes at even rows / columns.
constexpr int kLossPx = 4;
__global__ __launch_bounds__(kT) void t_loss(const float *__restrict__ raw, Geo g, const float *__restrict__ tgt,
                                             int64_t tstride, int yuv420, float *__restrict__ graw, float *__restrict__ acc4)
{
    __shared__ float s_red[8];
    const int b = blockIdx.y;
    const int64_t npx = (int64_t)g.H * g.W;
    const int h2 = g.H / 2, w2 = g.W / 2;
    const float total = yuv420 ? (float)(npx + 2 * (int64_t)h2 * w2) : (float)(3 * npx);
    const float k2 = 2.f / total;
    float se = 0.f;
    const float *o = raw + (int64_t)b * 3 * npx;
    const float *T = tgt + (int64_t)b * tstride;
    float *go = graw + (int64_t)b * 3 * npx;
    // grid-stride: a few hundred workgroups per frame, so the per-workgroup atomic on the
    // frame's one loss slot stays cheap (one workgroup per 256 pixels serialised ~1,500
    // same-address atomics per frame: 124 us per 8-frame 512x768 iteration)
    if (!yuv420) {
        for (int64_t p0 = (int64_t)blockIdx.x * kT * kLossPx + threadIdx.x; p0 < npx; p0 += (int64_t)gridDim.x * kT * kLossPx) {
            float v[kLossPx][3], t[kLossPx][3];
#pragma unroll
            for (int u = 0; u < kLossPx; ++u) {
                const int64_t p = p0 + u * kT;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    v[u][c] = p < npx ? o[c * npx + p] : 0.f;
                    t[u][c] = p < npx ? T[c * npx + p] : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < kLossPx; ++u) {
                const int64_t p = p0 + u * kT;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float vc = fminf(fmaxf(v[u][c], 0.f), 1.f), d = vc - t[u][c];
                    se += d * d; // 0 past the frame
                    if (p < npx) go[c * npx + p] = (v[u][c] >= 0.f && v[u][c] <= 1.f) ? k2 * d : 0.f;
                }
            }
        }
    } else {
        for (int64_t p = (int64_t)blockIdx.x * kT + threadIdx.x; p < npx; p += (int64_t)gridDim.x * kT) {
            const int py = (int)p / g.W, px = (int)p - py * g.W; // a frame's pixels fit 31 bits
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                bool used = true;
                int64_t ti = c * npx + p;
                if (c > 0) {
                    used = (py % 2 == 0) && (px % 2 == 0) && (py / 2) < h2 && (px / 2) < w2;
                    ti = npx + (int64_t)(c - 1) * h2 * w2 + (int64_t)(py / 2) * w2 + px / 2;
                }
                float gv = 0.f;
                if (used) {
                    const float vv = o[c * npx + p], vc = fminf(fmaxf(vv, 0.f), 1.f), d = vc - T[ti];
                    se += d * d;
                    gv = (vv >= 0.f && vv <= 1.f) ? k2 * d : 0.f;
                }
                go[c * npx + p] = gv;
            }
        }
    }
    const float s = block_sum(se, s_red);
    if (threadIdx.x == 0) atomicAdd(&acc4[b * 4 + 0], s);
}

// workgroups per frame of the per-frame sum reductions (t_loss, t_latgrad_sumsq): each
// workgroup ends in ONE atomic on the frame's accumulator, and same-address atomics serialise
// at ≈80 ns each (256 -> 384 workgroups per frame took t_loss from 29 to 35 us and 256 -> 512
// t_latgrad_sumsq from 29 to 53 us, profiles/r5m_*), so a frame gets at most kSumWGs
// workgroups, each with several batched iterations
constexpr int kSumWGs = 128;
static unsigned sum_blocks(int64_t n, int per_iter)
{
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(kSumWGs, (n + (int64_t)kT * per_iter - 1) / ((int64_t)kT * per_iter)));
}

// g_pre = g_out * relu'(out), in place.
__global__ void t_sp_gpre(float *__restrict__ gout, const float *__restrict__ out, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n && out[i] <= 0.f) gout[i] = 0.f;
}

// 3x3 layer backward on 16 x 64 pixel tiles staged in LDS (grid-stride over the tiles).
//  * X (the layer input) at replicate-clamped coordinates over the tile + 1-pixel ring:
//    dW[c][i][ky][kx] += G[c][q] X[i][clamp(q + (ky-1, kx-1))], accumulated per thread in
//    registers over every tile the workgroup visits, reduced once at the end;
//  * G (the output gradient, times relu'(out) when the layer has a ReLU: the old
//    t_sp_gpre fused in) over the same ring, zero outside the image: the input gradient of
//    an interior pixel p is the plain correlation sum_{c,k} W[c][i][k] G[c][p - d_k]; a
//    pixel on the image border also collects the taps that the replicate padding clamps
//    onto it (one kernel row / column / corner tap per image side it lies on), all within the ring.
// MODE: 1 = input gradient only, 2 = weight / bias gradients only (per-thread VALU sums, 84
// accumulators), 3 = both, the weight gradients on the matrix cores.  Round 4 ran modes 1 and 2
// as two launches: with 84 accumulators per thread the combined VALU kernel sat 71 % of its wave
// cycles in s_waitcnt / barrier waits (SQ_WAIT_ANY).  Mode 3 keeps them in the 4 accumulator
// registers of v_mfma_f32_4x4x1_16b_f32 (+ 3 bias sums), so one launch reads every tile once.
// (Measured and dropped: the input gradient one channel per iteration with 27 scalar weights
// each instead of all 81 at once -- 74 vs 40 us, the scalar-load waits per channel.)
// MODE 7 = MODE 3 over a persistent grid (one resident round of workgroups per frame): the next
// tile's ring (X, and G with the ReLU mask already applied) is loaded into registers while the
// current tile computes, and a workgroup flushes its weight gradients once for all its tiles.
constexpr int kSY = 16, kSX = 64;
template <int MODE>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu((MODE & 7) == 2 || (MODE & 7) == 7 ? 4 : (MODE & 7) == 3 ? 5 : 1))) void t_sp_bwd(const float *__restrict__ gout, const float *__restrict__ outp,
                                               const float *__restrict__ in, Geo g, const float *__restrict__ th,
                                               int64_t ps, int wo, int bo, int res, float *__restrict__ gin,
                                               float *__restrict__ gth, int64_t gstride)
{
    constexpr bool DX = (MODE & 1) != 0, DW = (MODE & 2) != 0, PF = (MODE & 4) != 0;
    // MODE bit 8: the previous layer's ReLU applied to the input gradient written here, where its
    // output (this layer's input X) is staged -- that layer's backward then loads no output planes
    // (a compile-time bit: as a run-time flag the border pass's select spilled ~50 VGPRs)
    constexpr bool mask_in = (MODE & 8) != 0;
    static_assert(!mask_in || DW, "the mask reads the staged X");
    constexpr int RH = kSY + 2, RW = kSX + 2;
    // ring images at row pitch kRP = 67 and plane pitch kPP = 1225 (== 3 and 9 mod 32 banks): the 27
    // taps (i, ky, kx) of one pixel sit on 27 distinct banks (9 i + 3 ky + kx), so the weight-
    // gradient MFMA loop's operand reads are conflict-free (pitches 66 / 1188: ~3-way)
    constexpr int kRP = 67, kPP = 1225;
    static_assert(kRP >= RW && kPP >= RH * kRP, "ring fits its pitches");
    __shared__ float sXf[3 * kPP];
    __shared__ float sGf[3 * kPP];
#define SX(ch, r, q) sXf[(ch) * kPP + (r) * kRP + (q)]
#define SG(ch, r, q) sGf[(ch) * kPP + (r) * kRP + (q)]
    __shared__ float s_red[4][84];
    __shared__ float s_wt[81]; // MODE 3: the layer's weights for the border-tap fold
    const int b = blockIdx.y;
    const int H = g.H, W = g.W;
    const int64_t npx = (int64_t)H * W;
    const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
    const float *Gb = gout + (int64_t)b * 3 * npx;
    const float *Ob = outp ? outp + (int64_t)b * 3 * npx : nullptr;
    const float *Xb = in + (int64_t)b * 3 * npx;
    float *Ib = gin + (int64_t)b * 3 * npx;
    const int tx = (W + kSX - 1) / kSX, ntile = tx * ((H + kSY - 1) / kSY);
    const int c = threadIdx.x & 63, rb = (threadIdx.x >> 6) * 4;
    constexpr bool VW = MODE == 2; // the VALU weight-gradient form
    if constexpr (DX) // visible after the tile loop's first barrier
        for (int e = threadIdx.x; e < 81; e += kT) s_wt[e] = P[wo + e];
    float acc[VW ? 84 : 1];
#pragma unroll
    for (int e = 0; e < (VW ? 84 : 1); ++e) acc[e] = 0.f;
    v4f dacc = {0.f, 0.f, 0.f, 0.f}; // MODE 3: the MFMA blocks
    float bacc[3] = {0.f, 0.f, 0.f};  // MODE 3: bias sums
    // PF: the ring of tile tt in registers: X and the masked G of NU elements per thread
    constexpr int kPU = (RH * RW + kT - 1) / kT;
    float px_[PF ? kPU : 1][3], pg_[PF ? kPU : 1][3], po_[PF ? kPU : 1][3]; // raw: the mask is applied at the LDS store (a select here would wait for the loads)
    auto prefetch = [&](int tt) __attribute__((always_inline)) {
        const int py0 = (tt / tx) * kSY, px0 = (tt % tx) * kSX;
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            const int i = threadIdx.x + u * kT;
            const int r = i / RW, q = i - r * RW;
            const int y = py0 - 1 + r, x = px0 - 1 + q;
            const int64_t cl = (int64_t)clampi(y, H - 1) * W + clampi(x, W - 1);
            const bool inb = y >= 0 && y < H && x >= 0 && x < W, live = i < RH * RW;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                px_[u][ch] = live ? Xb[ch * npx + cl] : 0.f;
                pg_[u][ch] = (live && inb) ? Gb[ch * npx + cl] : 0.f;
                po_[u][ch] = (Ob && live && inb) ? Ob[ch * npx + cl] : 1.f;
            }
        }
    };
    if constexpr (PF)
        if ((int)blockIdx.x < ntile) prefetch(blockIdx.x);
    for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
        const int y0 = (t / tx) * kSY, x0 = (t % tx) * kSX;
        __syncthreads();
        if constexpr (PF) {
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                const int i = threadIdx.x + u * kT;
                if (i >= RH * RW) continue;
                const int r = i / RW, q = i - r * RW;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    SX(ch, r, q) = px_[u][ch];
                    SG(ch, r, q) = po_[u][ch] <= 0.f ? 0.f : pg_[u][ch];
                }
            }
            if (t + (int)gridDim.x < ntile) prefetch(t + gridDim.x); // in flight behind this tile's work
        } else
        // the ring in batches of UN elements per thread: a batch's loads are all in flight
        // before its LDS stores (the input-gradient kernel, with few registers, takes the
        // whole ring in one batch; the weight-gradient kernel two per batch)
        {
        constexpr int NU = (RH * RW + kT - 1) / kT, UN = VW ? 2 : NU;
#pragma unroll
        for (int u0 = 0; u0 < NU; u0 += UN) {
            float xs[UN][3], gs[UN][3], os[UN][3];
            bool inb[UN];
#pragma unroll
            for (int uu = 0; uu < UN; ++uu) {
                const int i = threadIdx.x + (u0 + uu) * kT;
                const int r = i / RW, q = i - r * RW;
                const int y = y0 - 1 + r, x = x0 - 1 + q;
                const int64_t cl = (int64_t)clampi(y, H - 1) * W + clampi(x, W - 1);
                inb[uu] = y >= 0 && y < H && x >= 0 && x < W;
                const bool live = u0 + uu < NU && i < RH * RW;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
#if defined(CCMI_DIAG_SPB_NOLOAD) // diagnostic builds only (tools/spb_diag.sh): wrong results
                    xs[uu][ch] = 0.001f * (float)(cl + ch);
                    gs[uu][ch] = inb[uu] ? 0.002f * (float)(cl - ch) : 0.f;
                    os[uu][ch] = 1.f;
#else
                    xs[uu][ch] = (DW && live) ? Xb[ch * npx + cl] : 0.f;
                    gs[uu][ch] = (live && inb[uu]) ? Gb[ch * npx + cl] : 0.f;
                    os[uu][ch] = (Ob && live && inb[uu]) ? Ob[ch * npx + cl] : 1.f;
#endif
                }
            }
#pragma unroll
            for (int uu = 0; uu < UN; ++uu) {
                const int i = threadIdx.x + (u0 + uu) * kT;
                if (u0 + uu >= NU || i >= RH * RW) continue;
                const int r = i / RW, q = i - r * RW;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    if (DW) SX(ch, r, q) = xs[uu][ch];
                    SG(ch, r, q) = os[uu][ch] <= 0.f ? 0.f : gs[uu][ch];
                }
            }
        }
        }
        __syncthreads();
#if !defined(CCMI_DIAG_SPB_NODW)
        if constexpr ((MODE & 3) == 3) {
            // dW[oc][n = (i, ky, kx)] += sum_q G[oc][q] X[i][q + (ky - 1, kx - 1)] over the wave's 4 x 64
            // pixels: block bk = lane >> 2 < 14 is (column quad nq = bk % 7, pixel stream bk / 7;
            // stream s takes rows rb + 2 s, rb + 2 s + 1), A = G[oc = lane & 3], B = X at tap column
            // n = 4 nq + (lane & 3), one pixel per MFMA.  Row oc = 3, column n = 27 and blocks 14, 15
            // read valid (clamped) LDS and are never flushed.  Every operand address is a lane base +
            // a compile-time offset.
            const int ln4 = threadIdx.x & 3, bk = (threadIdx.x & 63) >> 2;
            const int st = bk >= 7 ? 1 : 0, n = min(4 * (bk - 7 * st) + ln4, 26);
            const int i = n / 9, k = n - 9 * i, ky = k / 3, kx = k - 3 * ky;
            const float *pa = &SG(ln4 < 3 ? ln4 : 0, rb + 2 * st + 1, 1);
            const float *pb = &SX(i, rb + 2 * st + ky, kx);
#pragma unroll 1
            for (int j = 0; j < 2 * kSX; j += 16) { // 16 pixels per iteration (operand reads in flight)
                const int o = (j >= kSX ? kRP - kSX : 0) + j;
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) dacc = mfma4x4(pa[o + cc], pb[o + cc], dacc);
            }
        }
#endif
        const int px = x0 + c;
#pragma unroll 1
        for (int pr = 0; pr < 4; ++pr) {
            const int ry = rb + pr, py = y0 + ry;
            if (py >= H || px >= W) continue;
            // weight / bias gradients at output q = (py, px)
            float gp[3];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) gp[ch] = SG(ch, ry + 1, c + 1);
            if constexpr ((MODE & 3) == 3) {
#pragma unroll
                for (int oc = 0; oc < 3; ++oc) bacc[oc] += gp[oc];
            }
            if constexpr (VW) {
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 9; ++k) {
                        const float xv = SX(i, ry + k / 3, c + k % 3);
#pragma unroll
                        for (int oc = 0; oc < 3; ++oc) acc[(oc * 3 + i) * 9 + k] = fmaf(gp[oc], xv, acc[(oc * 3 + i) * 9 + k]);
                    }
#pragma unroll
                for (int oc = 0; oc < 3; ++oc) acc[81 + oc] += gp[oc];
            }
            if constexpr (!DX) continue;
            // input gradient at p = (py, px): the correlation sum_{oc,k} W[oc][i][k] G[oc][p - d_k]
            // (G is zero outside the image); border pixels get the rest after the row loop
            float gi[3] = {0.f, 0.f, 0.f};
#if !defined(CCMI_DIAG_SPB_NODX)
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int ky = k / 3, kx = k % 3;
#pragma unroll
                for (int oc = 0; oc < 3; ++oc) {
                    const float gq = SG(oc, ry + 2 - ky, c + 2 - kx);
#pragma unroll
                    for (int i = 0; i < 3; ++i) gi[i] = fmaf(P[wo + (oc * 3 + i) * 9 + k], gq, gi[i]);
                }
            }
#endif
            const int64_t pi = (int64_t)py * W + px;
            // mask_in (MODE bit 8): the previous layer's ReLU
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float v = gi[i] + (res ? gp[i] : 0.f);
                Ib[i * npx + pi] = (mask_in && SX(i, ry + 1, c + 1) <= 0.f) ? 0.f : v;
            }
        }
#if !defined(CCMI_DIAG_SPB_NODX) && !defined(CCMI_DIAG_SPB_NOBORDER)
        // What the replicate padding clamps onto a border pixel -- the padded-domain adjoint at the
        // ring positions r with clamp(r) = p: above the top row the kernel's row 0 against G's row
        // py, below the bottom row its row 2, left / right of the image its column 0 / 2 against G's
        // column px, at a corner the one corner tap against G(p); a 1-pixel image side takes both of
        // its edges' terms.  (The qrange enumeration's sums in another order.)  Added after the
        // barrier by one thread per border pixel of a tile that touches the image border -- inside
        // the row loop, a border lane held up its whole wave (profiles/r5ze_*, r5zf_*).  Slots:
        // threads [0, 64) the top row, [64, 128) the bottom row, [128, 144) / [144, 160) the left /
        // right column without those rows; the barrier orders the rows' global writes before these.
        if constexpr (DX) {
            const int rbot = H - 1 - y0, crt = W - 1 - x0; // the image's last row / column in tile coordinates
            const bool etop = y0 == 0, ebot = rbot < kSY, elft = x0 == 0, ergt = crt < kSX;
            if (etop || ebot || elft || ergt) { // workgroup-uniform
                __syncthreads();
                const int t = threadIdx.x;
                int ry = -1, cx = -1;
                if (t < kSX) {
                    if (etop) ry = 0, cx = t;
                } else if (t < 2 * kSX) {
                    if (ebot && !(etop && rbot == 0)) ry = rbot, cx = t - kSX;
                } else if (t < 2 * kSX + kSY) {
                    const int r = t - 2 * kSX;
                    if (elft && y0 + r != 0 && r != rbot) ry = r, cx = 0;
                } else if (t < 2 * kSX + 2 * kSY) {
                    const int r = t - 2 * kSX - kSY;
                    if (ergt && !(elft && crt == 0) && y0 + r != 0 && r != rbot) ry = r, cx = crt;
                }
                const int by = y0 + ry, bx = x0 + cx;
                if (ry >= 0 && by < H && bx < W) {
                    const bool top = by == 0, bot = by == H - 1, lft = bx == 0, rgt = bx == W - 1;
                    float e[3] = {0.f, 0.f, 0.f};
#pragma unroll
                    for (int oc = 0; oc < 3; ++oc) {
                        const float *Wk = s_wt + oc * 27;
                        const float gq = SG(oc, ry + 1, cx + 1);
#pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            const float *Wi = Wk + i * 9; // Wi[3 ky + kx]
#pragma unroll
                            for (int u = 0; u < 3; ++u) {
                                const float wr = (top ? Wi[u] : 0.f) + (bot ? Wi[6 + u] : 0.f);
                                const float wc = (lft ? Wi[3 * u] : 0.f) + (rgt ? Wi[3 * u + 2] : 0.f);
                                e[i] = fmaf(wr, SG(oc, ry + 1, cx + 2 - u), e[i]);
                                e[i] = fmaf(wc, SG(oc, ry + 2 - u, cx + 1), e[i]);
                            }
                            const float wy0 = top ? 1.f : 0.f, wy2 = bot ? 1.f : 0.f;
                            const float wcn = (lft ? wy0 * Wi[0] + wy2 * Wi[6] : 0.f) + (rgt ? wy0 * Wi[2] + wy2 * Wi[8] : 0.f);
                            e[i] = fmaf(wcn, gq, e[i]);
                        }
                    }
                    const int64_t pi = (int64_t)by * W + bx;
#pragma unroll
                    for (int i = 0; i < 3; ++i) // a masked pixel was written 0 and stays 0
                        Ib[i * npx + pi] += (mask_in && SX(i, ry + 1, cx + 1) <= 0.f) ? 0.f : e[i];
                }
            }
        }
#endif
    }
    if constexpr (!DW) return;
    // block reduction of the 84 weight / bias gradients
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if constexpr (VW) {
#pragma unroll
        for (int e = 0; e < 84; ++e) {
            const float v = wave_sum(acc[e]);
            if (lane == 0) s_red[wid][e] = v;
        }
    } else {
        // lane l < 27 and lane l + 28 (the same column quad, the other stream) hold column n = l;
        // register r is row oc = r
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const float v = dacc[r] + __shfl(dacc[r], (lane + 28) & 63);
            if (lane < 27) s_red[wid][r * 27 + lane] = v;
        }
#pragma unroll
        for (int oc = 0; oc < 3; ++oc) {
            const float v = wave_sum(bacc[oc]);
            if (lane == 0) s_red[wid][81 + oc] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < 84) {
        const int e = threadIdx.x;
        const float v = s_red[0][e] + s_red[1][e] + s_red[2][e] + s_red[3][e];
        float *dst = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
        atomicAdd(&dst[e < 81 ? wo + e : bo + (e - 81)], v);
    }
}
#undef SX
#undef SG

// 1x1 head backward.  Per pixel (lane = pixel, VALU): the hidden layer recomputed, g_h and
// g_dense.  The weight gradients are sums over pixels -- GEMMs with K = pixels -- and run on
// the matrix cores (v_mfma_f32_16x16x4_f32, f32 in / f32 accumulate: the same products as
// an fmaf chain, only the summation order differs):
//   dW1[k][j] = sum_px gp[px][k] h[px][j]          (M = k < 3, N = j, one MFMA per 16 j)
//   dW0[j][i] = sum_px gh[px][j] [x[px][i] | 1]    (M = j, N = i <= CIN, column CIN = db0)
// A wave stages its 64 pixels' rows in LDS (pixel-major, pitch kHP: conflict-free writes)
// and feeds 4 pixels per MFMA (K = lane >> 4).  Accumulators live in registers across
// every pixel chunk the workgroup visits (grid-stride) and are flushed once, with one
// atomic per weight per wave.
// diagnostic builds (tools/arm_diag.sh; wrong results, timing only): NOREC replaces the LDS
// weight records by constants, NOHMFMA drops the weight-gradient MFMAs
#if defined(CCMI_DIAG_ARM_NOREC)
#define HEAD_BWD_REC(r, j) const float r[12] = {0.01f, 0.02f, 0.03f, 0.01f, 0.02f, 0.03f, 0.01f, 0.02f, 0.03f, 0.01f, 0.02f, 0.03f}
#else
#define HEAD_BWD_REC(r, j) const float *r = s_rec[j]
#endif
#if defined(CCMI_DIAG_ARM_NOHMFMA)
#define HEAD_MFMA(a, b, c) (c)
#else
#define HEAD_MFMA(a, b, c) mfma4(a, b, c)
#endif
// PAIR (the instantiated form; PAIR = false is the round-1 unit-at-a-time form, measured
// 397 vs 350-383 us per 8-frame iteration): the per-pixel
// work runs over PAIRS of hidden units with packed FMAs -- records interleave the two units'
// weights ({w0[j][i], w0[j+1][i]}, {b0[j], b0[j+1]}, {w1[k][j], w1[k][j+1]}), so every
// packed operand is an aligned register pair -- and the output / g_x sums keep one partial
// per unit parity, added at the end: 26 VALU per unit pair instead of 46.
template <int CIN, int NT, bool PAIR>
__global__ __launch_bounds__(kHeadT) void t_head_bwd(const float *__restrict__ dense, const float *__restrict__ gz0, Geo g,
                                                     const float *__restrict__ th, int64_t ps, float *__restrict__ gdense,
                                                     float *__restrict__ gth, int64_t gstride)
{
    // dynamic LDS, per wave: [64][hp] h, then g_h (pixel-major, hp = 16 NT + 1: conflict-free
    // row writes, columns [hid, 16 NT) zero); [64][kXP] gp | 0, then x | 1 | 0.  The zero
    // columns let every lane read its MFMA operand unconditionally (no exec-mask branches
    // between the LDS reads and the MFMAs).
    extern __shared__ float s_dyn[];
    // odd row pitch: conflict-free row writes (lane * kXP covers the 32 banks once per half),
    // and rows s and s + 16 of the MFMA operand reads land 16 banks apart
    constexpr int kXP = (CIN + 2 > 5 ? CIN + 2 : 5) | 1;
    // hidden unit j: w0[j][0..CIN), b0[j], w1[0..3)[j] -- read back as broadcast ds_read_b128
    // (sized for the 16 NT units of the instantiation: 2.3 KB at NT = 3, where 64 units' worth
    // put the workgroup at exactly 32 KB and five per CU did not fit)
    __shared__ __attribute__((aligned(16))) float s_rec[16 * NT][12];
    static_assert(CIN + 4 <= 12, "hidden-unit record");
    const int b = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int hid = g.hid; // NT = ceil(hid / 16), a template argument: the accumulator tiles
                           // must be compile-time registers
    constexpr int hp = 16 * NT + 1;
    const int64_t npx = (int64_t)g.H * g.W;
    const float *P = th + (int64_t)b * ps;
    // pair records: unit pair jp = units 2jp, 2jp + 1, field f interleaved as [2f + parity]
    constexpr int kPR = 2 * (CIN + 4) <= 24 ? 24 : 32;
    float(*s_rec2)[kPR] = reinterpret_cast<float(*)[kPR]>(&s_rec[0][0]);
    static_assert(8 * NT * kPR <= 16 * NT * 12, "pair records fit in the record area");
    if constexpr (!PAIR) {
        for (int e = t; e < 16 * NT * 12; e += kHeadT) {
            const int j = e / 12, f = e - j * 12;
            float v = 0.f;
            if (j < hid) {
                if (f < CIN) v = P[g.w0 + j * CIN + f];
                else if (f == CIN) v = P[g.b0 + j];
                else if (f <= CIN + 3) v = P[g.w1 + (f - CIN - 1) * hid + j];
            }
            s_rec[j][f] = v;
        }
    } else {
        for (int e = t; e < 8 * NT * kPR; e += kHeadT) {
            const int jp = e / kPR, r = e - jp * kPR, f = r >> 1, j = 2 * jp + (r & 1);
            float v = 0.f;
            if (j < hid) {
                if (f < CIN) v = P[g.w0 + j * CIN + f];
                else if (f == CIN) v = P[g.b0 + j];
                else if (f <= CIN + 3) v = P[g.w1 + (f - CIN - 1) * hid + j];
            }
            s_rec2[jp][r] = v;
        }
    }
    const float bo0 = P[g.b1], bo1 = P[g.b1 + 1], bo2 = P[g.b1 + 2];
    float *sv = s_dyn + w * 64 * (hp + kXP), *sw = sv + 64 * hp;
    const int ln = lane & 15, lk = lane >> 4;
    for (int j = hid; j < 16 * NT; ++j) sv[lane * hp + j] = 0.f; // pad columns of this lane's row
    const int ia = ln < 3 ? ln : 3, ib = ln <= CIN ? ln : CIN + 1; // operand columns (pads read 0)
    v4f a1[NT], a0[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) a1[q] = a0[q] = v4f{0.f, 0.f, 0.f, 0.f};
    float db1[3] = {0.f, 0.f, 0.f};
    __syncthreads(); // s_rec staged
    const int64_t nchunk = (npx + kHeadT - 1) / kHeadT;
    // the next chunk's pixel inputs (x, g_out) are loaded into registers while this one is
    // processed: at 2 waves / SIMD (LDS-bound) the loads' latency was left exposed per chunk
    float nx[CIN], ng[3];
    auto load_chunk = [&](int64_t ch) {
        const int64_t p = ch * kHeadT + t;
        const bool valid = p < npx;
        const float *x = dense + (int64_t)b * CIN * npx + p;
        const float *G = gz0 + (int64_t)b * 3 * npx + p;
#pragma unroll
        for (int i = 0; i < CIN; ++i) nx[i] = valid ? x[i * npx] : 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) ng[k] = valid ? G[k * npx] : 0.f;
    };
    if ((int64_t)blockIdx.x < nchunk) load_chunk(blockIdx.x);
    for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int64_t p = ch * kHeadT + t;
        const bool valid = p < npx;
        float xv[CIN], gp1[3];
#pragma unroll
        for (int i = 0; i < CIN; ++i) xv[i] = nx[i];
#pragma unroll
        for (int k = 0; k < 3; ++k) gp1[k] = ng[k];
        if (ch + gridDim.x < nchunk) load_chunk(ch + gridDim.x);
        // ---- hidden layer (kept in this lane's LDS row) and the output pre-activations
        float o0 = bo0, o1 = bo1, o2 = bo2;
        if constexpr (PAIR) {
            using ccmi_fwd::f2;
            const f2 lo0 = f2(g.r0 ? 0.f : -INFINITY);
            f2 op[3] = {f2(0.f), f2(0.f), f2(0.f)};
#pragma unroll 2
            for (int jp = 0; jp < (hid + 1) / 2; ++jp) {
                const f2 *r = reinterpret_cast<const f2 *>(s_rec2[jp]);
                f2 a = r[CIN];
#pragma unroll
                for (int i = 0; i < CIN; ++i) a = __builtin_elementwise_fma(r[i], f2(xv[i]), a);
                a = __builtin_elementwise_max(a, lo0);
                sv[lane * hp + 2 * jp] = a.x;
                sv[lane * hp + 2 * jp + 1] = a.y;
#pragma unroll
                for (int k = 0; k < 3; ++k) op[k] = __builtin_elementwise_fma(r[CIN + 1 + k], a, op[k]);
            }
            o0 += op[0].x + op[0].y;
            o1 += op[1].x + op[1].y;
            o2 += op[2].x + op[2].y;
        } else {
#pragma unroll 4
            for (int j = 0; j < hid; ++j) {
                HEAD_BWD_REC(r, j);
                float a = r[CIN];
#pragma unroll
                for (int i = 0; i < CIN; ++i) a = fmaf(r[i], xv[i], a);
                if (g.r0) a = fmaxf(a, 0.f);
                sv[lane * hp + j] = a;
                o0 = fmaf(r[CIN + 1], a, o0);
                o1 = fmaf(r[CIN + 2], a, o1);
                o2 = fmaf(r[CIN + 3], a, o2);
            }
        }
        if (g.r1) {
            if (o0 <= 0.f) gp1[0] = 0.f;
            if (o1 <= 0.f) gp1[1] = 0.f;
            if (o2 <= 0.f) gp1[2] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) db1[k] += gp1[k];
        // ---- dW1 += gp^T h (invalid pixels have gp = 0)
#pragma unroll
        for (int k = 0; k < 3; ++k) sw[lane * kXP + k] = gp1[k];
        sw[lane * kXP + 3] = 0.f;
        wave_lds_sync();
        // K = pixels in the order px = s + 16 (lane >> 4): the two 16-lane groups of each
        // 32-lane half read rows 16 apart, i.e. 16 banks apart (pitches hp, kXP odd)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int px = s + 16 * lk;
            const float a = sw[px * kXP + ia];
#pragma unroll
            for (int q = 0; q < NT; ++q) a1[q] = HEAD_MFMA(a, sv[px * hp + 16 * q + ln], a1[q]);
        }
        wave_lds_sync();
        // ---- g_h (replaces h in this lane's row), g_x
        float gxv[CIN];
#pragma unroll
        for (int i = 0; i < CIN; ++i) gxv[i] = 0.f;
        if constexpr (PAIR) {
            using ccmi_fwd::f2;
            f2 gxp[CIN];
#pragma unroll
            for (int i = 0; i < CIN; ++i) gxp[i] = f2(0.f);
#pragma unroll 2
            for (int jp = 0; jp < (hid + 1) / 2; ++jp) {
                const f2 *r = reinterpret_cast<const f2 *>(s_rec2[jp]);
                f2 gh = r[CIN + 1] * f2(gp1[0]);
                gh = __builtin_elementwise_fma(r[CIN + 2], f2(gp1[1]), gh);
                gh = __builtin_elementwise_fma(r[CIN + 3], f2(gp1[2]), gh);
                float *row = sv + lane * hp + 2 * jp;
                if (g.r0) {
                    if (row[0] <= 0.f) gh.x = 0.f;
                    if (row[1] <= 0.f) gh.y = 0.f;
                }
                row[0] = gh.x;
                row[1] = gh.y;
#pragma unroll
                for (int i = 0; i < CIN; ++i) gxp[i] = __builtin_elementwise_fma(r[i], gh, gxp[i]);
            }
#pragma unroll
            for (int i = 0; i < CIN; ++i) gxv[i] = gxp[i].x + gxp[i].y;
        } else {
#pragma unroll 4
            for (int j = 0; j < hid; ++j) {
                HEAD_BWD_REC(r, j);
                float gh = r[CIN + 1] * gp1[0] + r[CIN + 2] * gp1[1] + r[CIN + 3] * gp1[2];
                if (g.r0 && sv[lane * hp + j] <= 0.f) gh = 0.f;
                sv[lane * hp + j] = gh;
#pragma unroll
                for (int i = 0; i < CIN; ++i) gxv[i] = fmaf(r[i], gh, gxv[i]);
            }
        }
        if (valid) {
            float *gd = gdense + (int64_t)b * CIN * npx + p;
#pragma unroll
            for (int i = 0; i < CIN; ++i) gd[i * npx] = gxv[i];
        }
        // ---- dW0 | db0 += g_h^T [x | 1]
#pragma unroll
        for (int i = 0; i < CIN; ++i) sw[lane * kXP + i] = xv[i];
        sw[lane * kXP + CIN] = 1.f;
        sw[lane * kXP + CIN + 1] = 0.f;
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int px = s + 16 * lk;
            const float bb = sw[px * kXP + ib];
#pragma unroll
            for (int q = 0; q < NT; ++q) a0[q] = HEAD_MFMA(sv[px * hp + 16 * q + ln], bb, a0[q]);
        }
        wave_lds_sync();
    }
    // ---- flush: accumulator register r of lane l holds D[m = 4 (l >> 4) + r][n = l & 15].
    // The waves' partial sums meet in LDS (each wave's own rows, free after the chunk loop),
    // then ONE atomic per value per workgroup (one per wave put every workgroup of a frame on
    // the same few hundred addresses -- the t_arm16 flush lesson, profiles/r4l_*)
    // partial row: w0 [hid][CIN] | b0 [hid] | w1 [3][hid] | b1 [3]
    const int nred = hid * (CIN + 4) + 3;
    float *red = s_dyn + w * 64 * (hp + kXP);
    static_assert(64 * (hp + kXP) >= 16 * NT * (CIN + 4) + 3, "a wave's partial row fits its LDS rows");
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NT; ++q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 4 * lk + r;
            if (m < 3) { // dW1[k = m][j]
                const int j = 16 * q + ln;
                if (j < hid) red[hid * (CIN + 1) + m * hid + j] = a1[q][r];
            }
            const int j = 16 * q + m; // dW0[j][i = ln]
            if (j < hid) {
                if (ln < CIN) red[j * CIN + ln] = a0[q][r];
                else if (ln == CIN) red[hid * CIN + j] = a0[q][r];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float v = db1[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) red[hid * (CIN + 4) + k] = v;
    }
    __syncthreads();
    float *Gp = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
    constexpr int kW = kHeadT / 64;
    for (int e = t; e < nred; e += kHeadT) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < kW; ++ww) v += s_dyn[ww * 64 * (hp + kXP) + e];
        const int dst = e < hid * CIN ? g.w0 + e
                        : e < hid * (CIN + 1) ? g.b0 + (e - hid * CIN)
                        : e < hid * (CIN + 4) ? g.w1 + (e - hid * (CIN + 1))
                                              : g.b1 + (e - hid * (CIN + 4));
        atomicAdd(&Gp[dst], v);
    }
}

// Tiled form (the one launched): the hidden layer stays in registers (pairs of units, packed
// FMAs, as the PAIR form), and the LDS that feeds the weight-gradient MFMAs holds ONE 16-unit
// tile at a time next to the pixel fields gp | 0 | x | 1 shared by both MFMA loops: 8.2 KB of
// LDS per wave instead of 14.8 KB (LDS had capped the full-width form at 2.5 waves / SIMD with
// 55 % of its wave cycles in WAIT_ANY; profiles/r4w_train_pmc.txt).  Both are stored
// pixel-minor -- one row of the wave's 64 pixels per unit / field, pitch 68 -- so a lane's
// writes are consecutive across the wave and an MFMA loop reads its operands for four K-steps
// (4 pixels) with one 128-bit read each (the 16 lanes of a read start 4 banks apart).
// Per tile q: h -> dW1 tile (M = k < 3, N = the tile's units) -> g_h (the ReLU mask from the
// registers) -> dW0 tile (M = the tile's units, N = i <= CIN) and this pixel's g_x.
// Both products run on the 4x4x1 sixteen-block MFMA (blocks = pixel streams x unit / column
// quads, the streams summed once at the flush): on 16x16x4 the dW1 tile used 3 of 16 rows and
// the dW0 tile 8 of 16 columns, 1,024 MFMA cycles per tile and wave; now 128 + 256.
// The output layer must be linear (g.r1 == 0, every reference architecture's "X-1-linear-none"):
// then g_out needs no pass over all units first, and a tile's units are computed just in time.
// Register form (the one launched for a linear output layer): no LDS round trip between the
// hidden layer and the matrix cores.  Per 16-pixel block a wave evaluates the hidden layer TWICE
// on v_mfma_f32_16x16x4_f32 (K = the CIN inputs + the constant 1 of the bias, two K-steps), with
// the same operand registers in swapped roles:
//   layout B: Z^T = W0 X, accumulator register r of lane l = unit 16 t + 4 (l >> 4) + r of pixel
//     l & 15 -- g_h in this layout is exactly the A operand of g_x = g_h W0 with the K order
//     permuted (K-step r takes units 16 t + 4 g + r from lane group g), so g_x comes out of the
//     matrix cores with no data movement;
//   layout A: Z = X^T W0^T, register r of lane l = pixel 4 (l >> 4) + r of unit 16 t + (l & 15) --
//     g_h here is the A operand of dW0 = g_h^T [x | 1] with K = the pixels (K-step r takes
//     pixel 4 g + r from lane group g), and dW1 = g_out h^T is 12 VALU FMAs into per-lane
//     partial sums (3 outputs: a matrix core would be 13/16 padding).
// Two hidden-layer evaluations cost 4 MFMA per 16-unit tile; what they replace is the LDS staging
// of every tile (WAIT_INST_LDS 17 % of the tiled form's wave cycles, profiles/r5zk_train_pmc.txt).
template <int CIN, int NT>
__global__ __launch_bounds__(256) void t_head_bwd_m(const float *__restrict__ dense, const float *__restrict__ gz0, Geo g,
                                                    const float *__restrict__ th, int64_t ps, float *__restrict__ gdense,
                                                    float *__restrict__ gth, int64_t gstride)
{
    static_assert(CIN + 1 <= 8, "inputs + bias in two K-steps of 4");
    constexpr int kU = 16 * NT, kRedN = kU * (CIN + 4) + 3;
    __shared__ __attribute__((aligned(16))) float s_w1[3][kU];
    __shared__ float s_red[4][kRedN];
    const int b = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6, i = lane & 15, gq = lane >> 4;
    const int hid = g.hid;
    const int64_t npx = (int64_t)g.H * g.W;
    const cfloat_ptr P = (cfloat_ptr)(size_t)(th + (int64_t)b * ps);
    for (int e = t; e < 3 * kU; e += 256) {
        const int k = e / kU, u = e - k * kU;
        s_w1[k][u] = u < hid ? P[g.w1 + k * hid + u] : 0.f;
    }
    // per-lane constants: aB[tt][s] = W0|b0 [unit 16 tt + i][input 4 s + gq] (A of layout B, B of
    // layout A); bG[tt][r] = W0[unit 16 tt + 4 gq + r][input i] (B of g_x); w1A[tt][k] = W1[k][16 tt + i]
    float aB[NT][2], bG[NT][4], w1A[NT][3];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        const int u = 16 * tt + i;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 4 * s + gq;
            aB[tt][s] = u < hid ? (c < CIN ? P[g.w0 + u * CIN + c] : c == CIN ? P[g.b0 + u] : 0.f) : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ur = 16 * tt + 4 * gq + r;
            bG[tt][r] = (ur < hid && i < CIN) ? P[g.w0 + ur * CIN + i] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) w1A[tt][k] = u < hid ? P[g.w1 + k * hid + u] : 0.f;
    }
    const bool relu = g.r0 != 0;
    v4f dw0[NT];
    float acc1[NT][3], db1[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        dw0[tt] = v4f{0.f, 0.f, 0.f, 0.f};
        acc1[tt][0] = acc1[tt][1] = acc1[tt][2] = 0.f;
    }
    __syncthreads(); // s_w1 staged
    const float *xg = dense + (int64_t)b * CIN * npx;
    const float *gpg = gz0 + (int64_t)b * 3 * npx;
    float *gdb = gdense + (int64_t)b * CIN * npx;
    const int64_t nblk = (npx + 15) >> 4, wstride = (int64_t)gridDim.x * 4;
    for (int64_t blk = (int64_t)blockIdx.x * 4 + w; blk < nblk; blk += wstride) {
        const int64_t p0 = blk << 4, pi = p0 + i, pa = p0 + 4 * gq;
        // X[input 4 s + gq][pixel p0 + i] (0 past the frame, bias input included)
        float xb[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 4 * s + gq;
            xb[s] = pi >= npx ? 0.f : c < CIN ? xg[c * npx + pi] : c == CIN ? 1.f : 0.f;
        }
        float gpT[3], gpA[3][4], xA[4];
#pragma unroll
        for (int k = 0; k < 3; ++k) gpT[k] = pi < npx ? gpg[k * npx + pi] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const bool v = pa + r < npx;
#pragma unroll
            for (int k = 0; k < 3; ++k) gpA[k][r] = v ? gpg[k * npx + pa + r] : 0.f;
            xA[r] = !v ? 0.f : i < CIN ? xg[i * npx + pa + r] : i == CIN ? 1.f : 0.f;
        }
        if (gq == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) db1[k] += gpT[k];
        }
        v4f gx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            v4f zT = mfma4(aB[tt][0], xb[0], v4f{0.f, 0.f, 0.f, 0.f});
            zT = mfma4(aB[tt][1], xb[1], zT);
            v4f zA = mfma4(xb[0], aB[tt][0], v4f{0.f, 0.f, 0.f, 0.f});
            zA = mfma4(xb[1], aB[tt][1], zA);
            // layout B: g_h of units 16 tt + 4 gq + r at pixel i, then g_x += g_h W0
            const v4f wk0 = *reinterpret_cast<const v4f *>(&s_w1[0][16 * tt + 4 * gq]);
            const v4f wk1 = *reinterpret_cast<const v4f *>(&s_w1[1][16 * tt + 4 * gq]);
            const v4f wk2 = *reinterpret_cast<const v4f *>(&s_w1[2][16 * tt + 4 * gq]);
            float ghT[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float sgh = fmaf(wk2[r], gpT[2], fmaf(wk1[r], gpT[1], wk0[r] * gpT[0]));
                ghT[r] = (!relu || zT[r] > 0.f) ? sgh : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) gx = mfma4(ghT[r], bG[tt][r], gx);
            // layout A: h and g_h of unit 16 tt + i at pixels 4 gq + r; dW1 partials, dW0 += g_h^T [x | 1]
            float ghA[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float h = relu ? fmaxf(zA[r], 0.f) : zA[r];
#pragma unroll
                for (int k = 0; k < 3; ++k) acc1[tt][k] = fmaf(gpA[k][r], h, acc1[tt][k]);
                const float sgh = fmaf(w1A[tt][2], gpA[2][r], fmaf(w1A[tt][1], gpA[1][r], w1A[tt][0] * gpA[0][r]));
                ghA[r] = (!relu || zA[r] > 0.f) ? sgh : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) dw0[tt] = mfma4(ghA[r], xA[r], dw0[tt]);
        }
        // g_x: register r of lane l = pixel 4 gq + r, input i
        if (i < CIN) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (pa + r < npx) gdb[i * npx + pa + r] = gx[r];
        }
    }
    // ---- flush: this wave's partial row (w0 [hid][CIN] | b0 [hid] | w1 [3][hid] | b1 [3]), the
    // four waves summed in LDS, one atomic per value per workgroup into its slot row
    float *red = s_red[w];
    const int nred = hid * (CIN + 4) + 3;
    for (int e = lane; e < nred; e += 64) red[e] = 0.f;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int u = 16 * tt + 4 * gq + r; // dW0[u][c = i]
            if (u < hid) {
                if (i < CIN) red[u * CIN + i] = dw0[tt][r];
                else if (i == CIN) red[hid * CIN + u] = dw0[tt][r];
            }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float v = acc1[tt][k];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            const int u = 16 * tt + i;
            if (gq == 0 && u < hid) red[hid * (CIN + 1) + k * hid + u] = v;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float v = wave_sum(db1[k]);
        if (lane == 0) red[hid * (CIN + 4) + k] = v;
    }
    __syncthreads();
    float *Gp = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
    for (int e = t; e < nred; e += 256) {
        const float v = (s_red[0][e] + s_red[1][e]) + (s_red[2][e] + s_red[3][e]);
        const int dst = e < hid * CIN ? g.w0 + e
                        : e < hid * (CIN + 1) ? g.b0 + (e - hid * CIN)
                        : e < hid * (CIN + 4) ? g.w1 + (e - hid * (CIN + 1))
                                              : g.b1 + (e - hid * (CIN + 4));
        atomicAdd(&Gp[dst], v);
    }
}

constexpr int kHbXP = 68;
constexpr int head_bwd_t_wave_floats(int cin) { return (16 + 4 + cin + 1) * kHbXP; }

template <int CIN, int NT>
__global__ __launch_bounds__(kHeadT, 4) void t_head_bwd_t(const float *__restrict__ dense, const float *__restrict__ gz0,
                                                       Geo g, const float *__restrict__ th, int64_t ps,
                                                       float *__restrict__ gdense, float *__restrict__ gth, int64_t gstride)
{
    extern __shared__ float s_dyn[];
    constexpr int kXP = kHbXP;         // row pitch (64 pixels + 4)
    constexpr int kGX = 4;             // first x row
    constexpr int kWF = head_bwd_t_wave_floats(CIN);
    __shared__ __attribute__((aligned(16))) float s_rec[16 * NT][12];
    static_assert(CIN + 4 <= 12, "hidden-unit record");
    constexpr int kPR = 2 * (CIN + 4) <= 24 ? 24 : 32;
    static_assert(8 * NT * kPR <= 16 * NT * 12, "pair records fit in the record area");
    float(*s_rec2)[kPR] = reinterpret_cast<float(*)[kPR]>(&s_rec[0][0]);
    const int b = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int hid = g.hid;
    const int64_t npx = (int64_t)g.H * g.W;
    const float *P = th + (int64_t)b * ps;
    // pair records: unit pair jp = units 2jp, 2jp + 1, field f interleaved as [2f + parity];
    // units >= hid are zero records (h = 0: no contribution anywhere)
    for (int e = t; e < 8 * NT * kPR; e += kHeadT) {
        const int jp = e / kPR, r = e - jp * kPR, f = r >> 1, j = 2 * jp + (r & 1);
        float v = 0.f;
        if (j < hid) {
            if (f < CIN) v = P[g.w0 + j * CIN + f];
            else if (f == CIN) v = P[g.b0 + j];
            else if (f <= CIN + 3) v = P[g.w1 + (f - CIN - 1) * hid + j];
        }
        s_rec2[jp][r] = v;
    }
    // sv: [16 units][64 px] (the tile's h, then its g_h); sw: [field][64 px]
    float *sv = s_dyn + w * kWF, *sw = sv + 16 * kXP;
    const int ln = lane & 15, lk = lane >> 4;
    // weight gradients on v_mfma_f32_4x4x1_16b (mfma4x4), 4x4 blocks bk = lane >> 2:
    //  dW1: block (pixel stream lk, unit quad), A = gp k = lane & 3 (3: the zero row 3),
    //       B = h of unit ln; stream lk covers pixels 16 lk .. 16 lk + 15
    //  dW0: block (pixel stream s0, column quad iq, unit quad), A = g_h of unit ln, B = x | 1
    //       column 4 iq + (lane & 3) (> CIN: the zero row 3); kNQ column quads, 4 / kNQ
    //       streams of kPS pixels each
    constexpr int kNQ = CIN + 1 <= 4 ? 1 : CIN + 1 <= 8 ? 2 : 4, kPS = 16 * kNQ;
    const int iq = lk % kNQ, s0 = lk / kNQ, ic = 4 * iq + (lane & 3);
    const int ia = (lane & 3) < 3 ? (lane & 3) : 3, ib = ic <= CIN ? kGX + ic : 3;
    // constant rows: 0 (row 3), 1 (row kGX + CIN), written once
    sw[3 * kXP + lane] = 0.f;
    sw[(kGX + CIN) * kXP + lane] = 1.f;
    typedef float v4 __attribute__((ext_vector_type(4)));
    v4f a1[NT], a0[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) a1[q] = a0[q] = v4f{0.f, 0.f, 0.f, 0.f};
    float db1[3] = {0.f, 0.f, 0.f};
    __syncthreads(); // records staged
    const int64_t nchunk = (npx + kHeadT - 1) / kHeadT;
    float nx[CIN], ng[3];
    auto load_chunk = [&](int64_t ch) {
        const int64_t p = ch * kHeadT + t;
        const bool valid = p < npx;
        const float *x = dense + (int64_t)b * CIN * npx + p;
        const float *G = gz0 + (int64_t)b * 3 * npx + p;
#pragma unroll
        for (int i = 0; i < CIN; ++i) nx[i] = valid ? x[i * npx] : 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) ng[k] = valid ? G[k * npx] : 0.f;
    };
    using ccmi_fwd::f2;
    const f2 lo0 = f2(g.r0 ? 0.f : -INFINITY);
    if ((int64_t)blockIdx.x < nchunk) load_chunk(blockIdx.x);
    for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int64_t p = ch * kHeadT + t;
        const bool valid = p < npx;
        float xv[CIN], gp1[3];
#pragma unroll
        for (int i = 0; i < CIN; ++i) xv[i] = nx[i];
#pragma unroll
        for (int k = 0; k < 3; ++k) gp1[k] = ng[k];
        if (ch + gridDim.x < nchunk) load_chunk(ch + gridDim.x);
#pragma unroll
        for (int k = 0; k < 3; ++k) db1[k] += gp1[k];
        // ---- this pixel's column: gp, x (invalid pixels: gp = 0, x = 0)
#pragma unroll
        for (int k = 0; k < 3; ++k) sw[k * kXP + lane] = gp1[k];
#pragma unroll
        for (int i = 0; i < CIN; ++i) sw[(kGX + i) * kXP + lane] = xv[i];
        f2 gxp[CIN];
#pragma unroll
        for (int i = 0; i < CIN; ++i) gxp[i] = f2(0.f);
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            // the tile's records through an opaque base: the compiler must not keep them (or the
            // other tiles') loaded across the chunk
            int roff = 0;
            asm volatile("" : "+s"(roff));
            const float(*rec)[kPR] = s_rec2 + 8 * q + roff;
            float *col = sv + lane; // unit u of this pixel at col[u * kXP]
            // ---- the tile's hidden units h (pairs, packed FMAs) -> this lane's row; only the
            // ReLU mask stays in a register (bit 2u + parity)
            uint32_t hmask = 0;
#pragma unroll 2
            for (int u = 0; u < 8; ++u) {
                const f2 *r = reinterpret_cast<const f2 *>(rec[u]);
                f2 a = r[CIN];
#pragma unroll
                for (int i = 0; i < CIN; ++i) a = __builtin_elementwise_fma(r[i], f2(xv[i]), a);
                a = __builtin_elementwise_max(a, lo0);
                col[(2 * u) * kXP] = a.x;
                col[(2 * u + 1) * kXP] = a.y;
                hmask |= ((a.x > 0.f ? 1u : 0u) | (a.y > 0.f ? 2u : 0u)) << (2 * u);
            }
            wave_lds_sync();
            // ---- dW1 tile q += gp^T h, per pixel stream; four MFMAs per pair of 128-bit reads
#pragma unroll
            for (int s = 0; s < 16; s += 4) {
                const v4 av = *reinterpret_cast<const v4 *>(sw + ia * kXP + 16 * lk + s);
                const v4 bv = *reinterpret_cast<const v4 *>(sv + ln * kXP + 16 * lk + s);
#pragma unroll
                for (int e = 0; e < 4; ++e) a1[q] = mfma4x4(av[e], bv[e], a1[q]);
            }
            wave_lds_sync(); // every lane has read the h rows before g_h replaces them
            // ---- g_h of the tile (replaces h in this lane's row) and g_x
            const uint32_t keep = g.r0 ? hmask : 0xFFFFu;
#pragma unroll 2
            for (int u = 0; u < 8; ++u) {
                const f2 *r = reinterpret_cast<const f2 *>(rec[u]);
                f2 gh = r[CIN + 1] * f2(gp1[0]);
                gh = __builtin_elementwise_fma(r[CIN + 2], f2(gp1[1]), gh);
                gh = __builtin_elementwise_fma(r[CIN + 3], f2(gp1[2]), gh);
                gh.x = (keep >> (2 * u)) & 1u ? gh.x : 0.f; // selects, not exec-mask branches
                gh.y = (keep >> (2 * u + 1)) & 1u ? gh.y : 0.f;
                col[(2 * u) * kXP] = gh.x;
                col[(2 * u + 1) * kXP] = gh.y;
#pragma unroll
                for (int i = 0; i < CIN; ++i) gxp[i] = __builtin_elementwise_fma(r[i], gh, gxp[i]);
            }
            wave_lds_sync();
            // ---- dW0 | db0 tile q += g_h^T [x | 1]
#pragma unroll
            for (int s = 0; s < kPS; s += 4) {
                const v4 av = *reinterpret_cast<const v4 *>(sv + ln * kXP + kPS * s0 + s);
                const v4 bv = *reinterpret_cast<const v4 *>(sw + ib * kXP + kPS * s0 + s);
#pragma unroll
                for (int e = 0; e < 4; ++e) a0[q] = mfma4x4(av[e], bv[e], a0[q]);
            }
            wave_lds_sync(); // before the next tile's h (or the next chunk's rows) overwrite these
        }
        if (valid) {
            float *gd = gdense + (int64_t)b * CIN * npx + p;
#pragma unroll
            for (int i = 0; i < CIN; ++i) gd[i * npx] = gxp[i].x + gxp[i].y;
        }
    }
    // ---- flush (t_head_bwd's): the waves' partial rows meet in LDS, one atomic per value
#if defined(CCMI_DIAG_NOFLUSH) // diagnostic build only (make diag): wrong results -- and with the
    return;                       // accumulators dead, the compiler drops the weight-gradient work too
#endif
    const int nred = hid * (CIN + 4) + 3;
    float *red = s_dyn + w * kWF;
    static_assert(kWF >= 16 * NT * (CIN + 4) + 3, "a wave's partial row fits its LDS rows");
    __syncthreads();
    // the pixel streams' partial blocks summed across lanes (16 lanes apart), then register r of
    // lane l holds dW1[k = r][unit 16 q + ln] (l < 16) and dW0[unit 16 q + 4 ((l >> 2) & 3) + r][ic]
    // (l < 16 kNQ)
#pragma unroll
    for (int q = 0; q < NT; ++q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v1 = a1[q][r], v0 = a0[q][r];
            v1 += __shfl_xor(v1, 16);
            v1 += __shfl_xor(v1, 32);
#pragma unroll
            for (int o = 16 * kNQ; o < 64; o <<= 1) v0 += __shfl_xor(v0, o);
            if (r < 3 && lane < 16) { // dW1[k = r][j]
                const int j = 16 * q + ln;
                if (j < hid) red[hid * (CIN + 1) + r * hid + j] = v1;
            }
            const int j = 16 * q + 4 * ((lane >> 2) & 3) + r; // dW0[j][i = ic]
            if (lane < 16 * kNQ && j < hid) {
                if (ic < CIN) red[j * CIN + ic] = v0;
                else if (ic == CIN) red[hid * CIN + j] = v0;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float v = wave_sum(db1[k]);
        if (lane == 0) red[hid * (CIN + 4) + k] = v;
    }
    __syncthreads();
    float *Gp = gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride; // this workgroup's slot row
    constexpr int kW = kHeadT / 64;
    for (int e = t; e < nred; e += kHeadT) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < kW; ++ww) v += s_dyn[ww * kWF + e];
        const int dst = e < hid * CIN ? g.w0 + e
                        : e < hid * (CIN + 1) ? g.b0 + (e - hid * CIN)
                        : e < hid * (CIN + 4) ? g.w1 + (e - hid * (CIN + 1))
                                              : g.b1 + (e - hid * (CIN + 4));
        atomicAdd(&Gp[dst], v);
    }
}

// ------------------------------------------------------------------ upsampling backward
// Polyphase taps of the 2x transposed conv: destination 2j + a reads source clamp(j + d)
// with tap a + K/2 - 1 - 2d (fwd_ups.hip).
struct UpLevel {
    int C, hs, ws, hd, wd, K, d_lo, d_hi, sidx; // sidx: kernel slot (step % n_ups)
};

// Sum of per-thread tap gradients over the workgroup, folded onto the symmetric half
// kernel (upsampling.py:46-68): one atomic per half tap per workgroup.
// (The slot rows: see kDwSlots.)

__global__ void t_dw_fold(const float *__restrict__ slots, int nreg, float *__restrict__ gth, int64_t gstride, int off)
{
    const int b = blockIdx.y, e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nreg) return;
    const float *sl = slots + (int64_t)b * kDwSlots * nreg + e;
    float v = 0.f;
#pragma unroll 8
    for (int k = 0; k < kDwSlots; ++k) v += sl[(int64_t)k * nreg];
    gth[(int64_t)b * gstride + off + e] = v; // the only writer of the parameter gradients
}

template <int K>
__device__ __forceinline__ void reduce_taps(float (&dw)[K], float *__restrict__ dst)
{
    __shared__ float s_r[kT / 64][K];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float v = wave_sum(dw[k]);
        if (lane == 0) s_r[wid][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < K) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < kT / 64; ++i) v += s_r[i][threadIdx.x];
        atomicAdd(&dst[min((int)threadIdx.x, K - 1 - (int)threadIdx.x)], v);
    }
}

// Refine backward of one pyramid level in ONE launch (formerly four
// passes over the level through HBM temporaries): a 16 x 64 tile of the level
// with its KP / 2 halo of X and GY staged in LDS; the horizontal pass U = X * w and the
// vertical adjoint GU = GY (*) w of the tile are formed in LDS, then the latent gradient
// GX += GY + horizontal adjoint of GU and the tap gradients (GY x U, GU x X) of the tile's
// positions.  Per element the same fmaf chains in the same order as the former separate passes
// (a zero-padded tap adds an exact 0).
struct RefBwd {
    const float *GY;
    int64_t gys;
    const float *X;
    int64_t xs;
    int h, w;
    const float *kf;
    int kstride, koff;
    float *GX;
    int64_t gxs;
    float *slots;
    int64_t gstride;
    int hoff, tiles_x;
};
template <int KP>
constexpr int ref_bwd_lds()
{
    return 2 * (16 + KP / 2 * 2) * (64 + KP / 2 * 2) + (16 + KP / 2 * 2) * 64 + 16 * (64 + KP / 2 * 2);
}
// tile bx of the level (blockIdx.x of its own launch, or of the combined t_lvl_bwd)
template <int KP>
__device__ __forceinline__ void ref_bwd_tile(float *pool, int bx, int b, const RefBwd &R)
{
    constexpr int P = KP / 2, TY = 16, TX = 64, SY = TY + 2 * P, SX = TX + 2 * P;
    float(*sx)[SX] = reinterpret_cast<float(*)[SX]>(pool);
    float(*sg)[SX] = reinterpret_cast<float(*)[SX]>(pool + SY * SX);
    float(*su)[TX] = reinterpret_cast<float(*)[TX]>(pool + 2 * SY * SX);
    float(*sgu)[SX] = reinterpret_cast<float(*)[SX]>(pool + 2 * SY * SX + SY * TX);
    const float *GY = R.GY, *X = R.X, *kf = R.kf;
    const int64_t gys = R.gys, xs = R.xs, gxs = R.gxs, gstride = R.gstride;
    const int h = R.h, w = R.w, kstride = R.kstride, koff = R.koff, hoff = R.hoff, tiles_x = R.tiles_x;
    float *GX = R.GX, *slots = R.slots;
    const int tid = threadIdx.x;
    const int ty0 = (bx / tiles_x) * TY, tx0 = (bx % tiles_x) * TX;
    const float *wk = kf + (int64_t)b * kstride + koff;
    float wv[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) wv[k] = wk[k];
    const float *xb = X + (int64_t)b * xs, *gb = GY + (int64_t)b * gys;
    {
        // every load of a thread in flight before its LDS stores
        constexpr int NL = (SY * SX + kT - 1) / kT;
        float vx[NL], vg[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int i = tid + k * kT, r = i / SX, c = i - r * SX, y = ty0 - P + r, x = tx0 - P + c;
            const bool in = i < SY * SX && y >= 0 && y < h && x >= 0 && x < w;
            vx[k] = in ? xb[(int64_t)y * w + x] : 0.f;
            vg[k] = in ? gb[(int64_t)y * w + x] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int i = tid + k * kT;
            if (i < SY * SX) {
                (&sx[0][0])[i] = vx[k];
                (&sg[0][0])[i] = vg[k];
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < SY * TX; i += kT) { // U rows ty0 - P .. ty0 + TY + P - 1
        const int r = i / TX, c = i - r * TX;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) a = fmaf(wv[k], sx[r][c + k], a);
        su[r][c] = a;
    }
    for (int i = tid; i < TY * SX; i += kT) { // GU cols tx0 - P .. tx0 + TX + P - 1
        const int t = i / SX, c = i - t * SX;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) a = fmaf(wv[k], sg[t + 2 * P - k][c], a);
        sgu[t][c] = a;
    }
    __syncthreads();
    float dw[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) dw[k] = 0.f;
    float *gxb = GX + (int64_t)b * gxs;
    for (int i = tid; i < TY * TX; i += kT) {
        const int t = i / TX, c = i - t * TX, y = ty0 + t, x = tx0 + c;
        if (y >= h || x >= w) continue;
        const float gv = sg[t + P][c + P], guv = sgu[t][c + P];
        float a = gv;
#pragma unroll
        for (int k = 0; k < KP; ++k) a = fmaf(wv[k], sgu[t][c - k + 2 * P], a);
        gxb[(int64_t)y * w + x] += a;
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            dw[k] = fmaf(gv, su[t + k][c], dw[k]);
            dw[k] = fmaf(guv, sx[t + P][c + k], dw[k]);
        }
    }
    reduce_taps<KP>(dw, slots + ((int64_t)b * kDwSlots + bx % kDwSlots) * gstride + hoff);
}

template <int KP>
__global__ __launch_bounds__(kT) void t_ref_bwd(RefBwd R)
{
    __shared__ __attribute__((aligned(16))) float pool[ref_bwd_lds<KP>()];
    ref_bwd_tile<KP>(pool, blockIdx.x, blockIdx.y, R);
}

__device__ __forceinline__ int up_tap(int a, int d, int K) { return a + K / 2 - 1 - 2 * d; }

// upsample, horizontal pass: U[c][r][xd] = sum_d w[tap] S[c][r][clamp(xd/2 + d)]
__global__ void t_up_u(const float *__restrict__ S, int64_t ss, UpLevel A, const float *__restrict__ kf, int kstride,
                       int koff, float *__restrict__ U, int64_t us)
{
    const int b = blockIdx.y;
    const int n = A.C * A.hs * A.wd, i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const int cr = i / A.wd, xd = i - cr * A.wd; // cr = c * hs + r
    const float *wk = kf + (int64_t)b * kstride + koff, *src = S + (int64_t)b * ss + cr * A.ws;
    const int j = xd >> 1, a = xd & 1;
    float acc = 0.f;
    for (int d = A.d_lo; d <= A.d_hi; ++d) {
        const int t = up_tap(a, d, A.K);
        if (t >= 0 && t < A.K) acc = fmaf(wk[t], src[clampi(j + d, A.ws - 1)], acc);
    }
    U[(int64_t)b * us + i] = acc;
}

// upsample, vertical adjoint: GU[c][r][xd] = sum over (yd = 2j + a, d) with clamp(j + d) == r
__global__ void t_up_gu(const float *__restrict__ GY, int64_t gys, UpLevel A, const float *__restrict__ kf, int kstride,
                        int koff, float *__restrict__ GU, int64_t us)
{
    const int b = blockIdx.y;
    const int n = A.C * A.hs * A.wd, i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const int cr = i / A.wd, xd = i - cr * A.wd;
    const int c = cr / A.hs, r = cr - c * A.hs;
    const float *wk = kf + (int64_t)b * kstride + koff;
    const float *gy = GY + (int64_t)b * gys + (int64_t)(c + 1) * A.hd * A.wd + xd; // channel c+1 of the dest stack
    const int nj = (A.hd + 1) >> 1;
    float acc = 0.f;
    for (int d = A.d_lo; d <= A.d_hi; ++d) {
        int jlo = r == 0 ? 0 : r - d, jhi = r == A.hs - 1 ? nj - 1 : r - d;
        jlo = max(jlo, 0);
        jhi = min(jhi, nj - 1);
        for (int j = jlo; j <= jhi; ++j) {
            if (clampi(j + d, A.hs - 1) != r) continue;
            for (int a = 0; a < 2; ++a) {
                const int yd = 2 * j + a, t = up_tap(a, d, A.K);
                if (yd < A.hd && t >= 0 && t < A.K) acc = fmaf(wk[t], gy[(int64_t)yd * A.wd], acc);
            }
        }
    }
    GU[(int64_t)b * us + i] = acc;
}

// upsample, horizontal adjoint: GS[c][r][m] (+= into the source gradient)
__global__ void t_up_gs(const float *__restrict__ GU, int64_t us, UpLevel A, const float *__restrict__ kf, int kstride,
                        int koff, float *__restrict__ GS, int64_t gss, int accumulate)
{
    const int b = blockIdx.y;
    const int n = A.C * A.hs * A.ws, i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const int cr = i / A.ws, m = i - cr * A.ws;
    const float *wk = kf + (int64_t)b * kstride + koff;
    const float *gu = GU + (int64_t)b * us + cr * A.wd;
    const int nj = (A.wd + 1) >> 1;
    float acc = 0.f;
    for (int d = A.d_lo; d <= A.d_hi; ++d) {
        int jlo = m == 0 ? 0 : m - d, jhi = m == A.ws - 1 ? nj - 1 : m - d;
        jlo = max(jlo, 0);
        jhi = min(jhi, nj - 1);
        for (int j = jlo; j <= jhi; ++j) {
            if (clampi(j + d, A.ws - 1) != m) continue;
            for (int a = 0; a < 2; ++a) {
                const int xd = 2 * j + a, t = up_tap(a, d, A.K);
                if (xd < A.wd && t >= 0 && t < A.K) acc = fmaf(wk[t], gu[xd], acc);
            }
        }
    }
    float *o = GS + (int64_t)b * gss + i;
    *o = accumulate ? *o + acc : acc;
}

// upsample kernel gradient: vertical taps over destination row pairs (c, j, xd),
// horizontal taps over destination column pairs (c, r, j); taps are compile-time per
// parity: destination 2j + a, source offset d -> tap a + K/2 - 1 - 2d.
template <int K>
__global__ __launch_bounds__(kT) void t_up_dw(const float *__restrict__ GY, int64_t gys, const float *__restrict__ U,
                                              const float *__restrict__ GU, int64_t us, const float *__restrict__ S,
                                              int64_t ss, UpLevel A, float *__restrict__ gth, int64_t gstride, int hoff)
{
    constexpr int K2 = K / 2, DLO = -((K2 + 1) / 2), DHI = K2 / 2;
    const int b = blockIdx.y;
    float dw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dw[k] = 0.f;
    const int njy = (A.hd + 1) >> 1, njx = (A.wd + 1) >> 1;
    const float *gyb = GY + (int64_t)b * gys, *ub = U + (int64_t)b * us, *gub = GU + (int64_t)b * us;
    const float *sb = S + (int64_t)b * ss;
    const int64_t nv = (int64_t)A.C * njy * A.wd;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kT) {
        const int cj = (int)i / A.wd, xd = (int)i - cj * A.wd;
        const int c = cj / njy, j = cj - c * njy;
        const float *gy = gyb + (int64_t)(c + 1) * A.hd * A.wd + xd;
        const float ge = gy[(int64_t)(2 * j) * A.wd];
        const float go = 2 * j + 1 < A.hd ? gy[(int64_t)(2 * j + 1) * A.wd] : 0.f;
        const float *u = ub + (int64_t)c * A.hs * A.wd + xd;
#pragma unroll
        for (int d = DLO; d <= DHI; ++d) {
            const float uv = u[(int64_t)clampi(j + d, A.hs - 1) * A.wd];
            const int te = K2 - 1 - 2 * d, to = K2 - 2 * d;
            if (te >= 0 && te < K) dw[te] = fmaf(ge, uv, dw[te]);
            if (to >= 0 && to < K) dw[to] = fmaf(go, uv, dw[to]);
        }
    }
    const int64_t nh = (int64_t)A.C * A.hs * njx;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < nh; i += (int64_t)gridDim.x * kT) {
        const int cr = (int)i / njx, j = (int)i - cr * njx;
        const float *gu = gub + cr * A.wd;
        const float ge = gu[2 * j];
        const float go = 2 * j + 1 < A.wd ? gu[2 * j + 1] : 0.f;
        const float *src = sb + cr * A.ws;
#pragma unroll
        for (int d = DLO; d <= DHI; ++d) {
            const float sv = src[clampi(j + d, A.ws - 1)];
            const int te = K2 - 1 - 2 * d, to = K2 - 2 * d;
            if (te >= 0 && te < K) dw[te] = fmaf(ge, sv, dw[te]);
            if (to >= 0 && to < K) dw[to] = fmaf(go, sv, dw[to]);
        }
    }
    reduce_taps<K>(dw, gth + ((int64_t)b * kDwSlots + blockIdx.x % kDwSlots) * gstride + hoff);
}

// Upsampling backward of one pyramid step in ONE launch (formerly t_up_u, t_up_gu, t_up_dw
// and t_up_gs with compile-time taps, with the [C][hs][wd] temporaries U and GU through HBM).  A workgroup owns
// source rows [r0, r0 + TR) x destination columns [x0, x0 + TX) of one channel.  It stages
// in LDS the clamped source rows r0 + DLO .. r0 + TR - 1 + DHI (columns m0 + DLO .. m0 + TM - 1
// + DHI, m0 = x0 / 2) and the destination-gradient rows 2 (r0 - DHI) .. 2 (r0 + TR - 1 - DLO) + 1
// with 2 DHI halo columns on each side (zero outside the level), forms
//   U  = horizontal pass of S        rows r0 + DLO .. r0 + TR - 1 + DHI, the tile's columns;
//   GU = vertical adjoint of GY      rows r0 .. r0 + TR - 1, the tile's columns + halo;
// and emits GS (horizontal adjoint of GU) for its TM source columns and the tap-gradient
// partial sums (GY x U, GU x S) of its destination positions.  Border rows / columns take
// the generic clamped-gather loops of t_up_gu / t_up_gs over the staged tiles.
struct UpBwd {
    const float *GY;
    int64_t gys;
    const float *S;
    int64_t ss;
    UpLevel A;
    const float *kf;
    int kstride, koff;
    float *GS;
    int64_t gss;
    int accumulate;
    float *slots;
    int64_t gstride;
    int hoff, tiles_x, tiles_y;
    int batch; // frames (t_lvl_bwd's 1-D grid)
};
template <int K>
constexpr int up_bwd_lds()
{
    constexpr int K2 = K / 2, DW = K2 / 2 + (K2 + 1) / 2, TR = 16, TX = 64, TM = TX / 2;
    return (TR + DW) * (TM + DW) + (TR + DW) * TX + 2 * (TR + DW) * (TX + 2 * DW) + TR * (TX + 2 * DW);
}
template <int K>
__device__ __forceinline__ void up_bwd_tile(float *pool, int bx, int b, const UpBwd &Q)
{
    constexpr int K2 = K / 2, DLO = -((K2 + 1) / 2), DHI = K2 / 2, DW = DHI - DLO;
    constexpr int TR = 16, TX = 64, TM = TX / 2;
    constexpr int SR = TR + DW, SC = TM + DW; // staged source tile
    constexpr int GR = 2 * (TR + DW), GC = TX + 2 * DW; // staged GY tile (GU has GC columns too)
    float(*s_s)[SC] = reinterpret_cast<float(*)[SC]>(pool);
    float(*s_u)[TX] = reinterpret_cast<float(*)[TX]>(pool + SR * SC);
    float(*s_gy)[GC] = reinterpret_cast<float(*)[GC]>(pool + SR * SC + SR * TX);
    float(*s_gu)[GC] = reinterpret_cast<float(*)[GC]>(pool + SR * SC + SR * TX + GR * GC);
    const float *GY = Q.GY, *S = Q.S, *kf = Q.kf;
    const int64_t gys = Q.gys, ss = Q.ss, gss = Q.gss, gstride = Q.gstride;
    const UpLevel A = Q.A;
    const int kstride = Q.kstride, koff = Q.koff, accumulate = Q.accumulate, hoff = Q.hoff;
    const int tiles_x = Q.tiles_x, tiles_y = Q.tiles_y;
    float *GS = Q.GS, *slots = Q.slots;
    const int tid = threadIdx.x;
    const int tile = bx % (tiles_x * tiles_y), c = bx / (tiles_x * tiles_y);
    const int r0 = (tile / tiles_x) * TR, x0 = (tile % tiles_x) * TX, m0 = x0 / 2;
    const int gy0 = 2 * (r0 - DHI), gx0 = x0 - 2 * DHI; // GY / GU tile origin
    const int hs = A.hs, ws = A.ws, hd = A.hd, wd = A.wd;
    const int njy = (hd + 1) >> 1, njx = (wd + 1) >> 1;
    float w[K];
    {
        const float *wk = kf + (int64_t)b * kstride + koff;
#pragma unroll
        for (int t = 0; t < K; ++t) w[t] = wk[t];
    }
    const float *sb = S + (int64_t)b * ss + (int64_t)c * hs * ws;
    const float *gb = GY + (int64_t)b * gys + (int64_t)(c + 1) * hd * wd; // channel c + 1 of the dest stack
    // staging: every load of a thread issued before its LDS stores (a load-store pair per
    // loop iteration paid one memory latency per element)
    {
        constexpr int NS = (SR * SC + kT - 1) / kT, NG = (GR * GC + kT - 1) / kT;
        float vs[NS], vg[NG];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const int i = tid + k * kT, r = i / SC, q = i - r * SC;
            vs[k] = i < SR * SC ? sb[(int64_t)clampi(r0 + DLO + r, hs - 1) * ws + clampi(m0 + DLO + q, ws - 1)] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int i = tid + k * kT, r = i / GC, q = i - r * GC, y = gy0 + r, x = gx0 + q;
            vg[k] = (i < GR * GC && y >= 0 && y < hd && x >= 0 && x < wd) ? gb[(int64_t)y * wd + x] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const int i = tid + k * kT;
            if (i < SR * SC) (&s_s[0][0])[i] = vs[k];
        }
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int i = tid + k * kT;
            if (i < GR * GC) (&s_gy[0][0])[i] = vg[k];
        }
    }
    __syncthreads();
    // U: destination column x0 + q reads source columns m0 + (q >> 1) + d.  A thread takes the
    // column pair (2 j, 2 j + 1), so the tap index of each parity is a compile-time constant (a
    // per-lane parity made every w[t] a select chain over the K registers)
    for (int i = tid; i < SR * TM; i += kT) {
        const int r = i / TM, j = i - r * TM;
        float acc[2] = {0.f, 0.f};
#pragma unroll
        for (int d = DLO; d <= DHI; ++d) {
            const float sv = s_s[r][j + d - DLO];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int t = a + K2 - 1 - 2 * d;
                if (t >= 0 && t < K) acc[a] = fmaf(w[t], sv, acc[a]);
            }
        }
        s_u[r][2 * j] = acc[0];
        s_u[r][2 * j + 1] = acc[1];
    }
    // GU at source row r0 + tr, destination column gx0 + q
    for (int i = tid; i < TR * GC; i += kT) {
        const int tr = i / GC, q = i - tr * GC, r = r0 + tr, x = gx0 + q;
        float acc = 0.f;
        if (r < hs && x >= 0 && x < wd) {
            if (r >= 1 && r <= hs - 2 && r - DHI >= 0 && r - DLO <= njy - 1 && 2 * (r - DLO) + 1 < hd) {
#pragma unroll
                for (int d = DLO; d <= DHI; ++d)
#pragma unroll
                    for (int a = 0; a < 2; ++a) {
                        const int t = a + K2 - 1 - 2 * d;
                        if (t >= 0 && t < K) acc = fmaf(w[t], s_gy[2 * (tr - d + DHI) + a][q], acc);
                    }
            } else {
                for (int d = DLO; d <= DHI; ++d) {
                    int jlo = r == 0 ? 0 : r - d, jhi = r == hs - 1 ? njy - 1 : r - d;
                    jlo = max(jlo, 0);
                    jhi = min(jhi, njy - 1);
                    for (int j = jlo; j <= jhi; ++j) {
                        if (clampi(j + d, hs - 1) != r) continue;
                        for (int a = 0; a < 2; ++a) {
                            const int yd = 2 * j + a, t = up_tap(a, d, K);
                            if (yd < hd && t >= 0 && t < K) acc = fmaf(w[t], s_gy[yd - gy0][q], acc);
                        }
                    }
                }
            }
        }
        s_gu[tr][q] = acc;
    }
    __syncthreads();
    // GS at source row r0 + tr, column m0 + mm
    float *gsb = GS + (int64_t)b * gss + (int64_t)c * hs * ws;
    for (int i = tid; i < TR * TM; i += kT) {
        const int tr = i / TM, mm = i - tr * TM, r = r0 + tr, m = m0 + mm;
        if (r >= hs || m >= ws) continue;
        float acc = 0.f;
        if (m >= 1 && m <= ws - 2 && m - DHI >= 0 && m - DLO <= njx - 1 && 2 * (m - DLO) + 1 < wd) {
#pragma unroll
            for (int d = DLO; d <= DHI; ++d)
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    const int t = a + K2 - 1 - 2 * d;
                    if (t >= 0 && t < K) acc = fmaf(w[t], s_gu[tr][2 * (mm - d + DHI) + a], acc);
                }
        } else {
            for (int d = DLO; d <= DHI; ++d) {
                int jlo = m == 0 ? 0 : m - d, jhi = m == ws - 1 ? njx - 1 : m - d;
                jlo = max(jlo, 0);
                jhi = min(jhi, njx - 1);
                for (int j = jlo; j <= jhi; ++j) {
                    if (clampi(j + d, ws - 1) != m) continue;
                    for (int a = 0; a < 2; ++a) {
                        const int xd = 2 * j + a, t = up_tap(a, d, K);
                        if (xd < wd && t >= 0 && t < K) acc = fmaf(w[t], s_gu[tr][xd - gx0], acc);
                    }
                }
            }
        }
        float *o = gsb + (int64_t)r * ws + m;
        *o = accumulate ? *o + acc : acc;
    }
#if defined(CCMI_DIAG_LVL_NODW)
    return;
#endif
    // tap gradients: vertical use (GY x U at the tile's destination rows), horizontal use
    // (GU x S at the tile's source rows)
    float dw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dw[k] = 0.f;
    // vertical use: destination row ty has parity a = ty & 1 -- with kT a multiple of 2 TX, the
    // parity of a wave's rows (tid >> 6) never changes: a wave-uniform branch into a loop whose
    // tap indices are compile-time constants
    static_assert(kT % (2 * TX) == 0 && TX == 64, "row parity is wave-uniform");
    auto vertical = [&](auto par) {
        constexpr int a = decltype(par)::value;
        for (int i = tid; i < 2 * TR * TX; i += kT) {
            const int ty = i / TX, q = i - ty * TX;
            if (2 * r0 + ty >= hd || x0 + q >= wd) continue;
            const float g = s_gy[ty + 2 * DHI][q + 2 * DHI];
#pragma unroll
            for (int d = DLO; d <= DHI; ++d) {
                const int t = a + K2 - 1 - 2 * d;
                if (t >= 0 && t < K) dw[t] = fmaf(g, s_u[(ty >> 1) + d - DLO][q], dw[t]);
            }
        }
    };
    if (((tid >> 6) & 1) == 0) vertical(std::integral_constant<int, 0>{});
    else vertical(std::integral_constant<int, 1>{});
    // horizontal use: a thread takes the column pair (2 j, 2 j + 1), one per parity
    for (int i = tid; i < TR * TM; i += kT) {
        const int tr = i / TM, j = i - tr * TM;
        if (r0 + tr >= hs) continue;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int q = 2 * j + a;
            if (x0 + q >= wd) continue;
            const float g = s_gu[tr][q + 2 * DHI];
#pragma unroll
            for (int d = DLO; d <= DHI; ++d) {
                const int t = a + K2 - 1 - 2 * d;
                if (t >= 0 && t < K) dw[t] = fmaf(g, s_s[tr - DLO][j + d - DLO], dw[t]);
            }
        }
    }
    reduce_taps<K>(dw, slots + ((int64_t)b * kDwSlots + bx % kDwSlots) * gstride + hoff);
}

// One pyramid step of the upsampling backward in ONE launch: workgroups [0, nref) are tiles
// of the refine backward (latent k-1, channel 0 of the destination gradient), the rest tiles of
// the transposed-conv backward (channels 1..C): the two read disjoint inputs and write
// disjoint outputs, so they run side by side (the coarse levels are a few workgroups each and
// were latency-bound as two launches)
template <int KP, int K>
__global__ __launch_bounds__(kT) void t_lvl_bwd(RefBwd R, UpBwd Q, int nref)
{
    constexpr int n = ref_bwd_lds<KP>() > up_bwd_lds<K>() ? ref_bwd_lds<KP>() : up_bwd_lds<K>();
    __shared__ __attribute__((aligned(16))) float pool[n];
    // 1-D grid of (nref + up tiles) x frames in XCD-aware order (neighbouring tiles share their
    // halos through one L2)
    const int per = gridDim.x / Q.batch, wt = ccmi_fwd::xcd_order(blockIdx.x, gridDim.x);
    const int b = wt / per, bx = wt - b * per;
#if defined(CCMI_DIAG_LVL_NOREF) // diagnostic builds only (tools/arm_diag.sh): wrong results
    if (bx < nref) return;
#endif
#if defined(CCMI_DIAG_LVL_NOUP)
    if (bx >= nref) return;
#endif
    if (bx < nref) ref_bwd_tile<KP>(pool, bx, b, R);
    else up_bwd_tile<K>(pool, bx - nref, b, Q);
}

// ------------------------------------------------------------------ latents, norm, Adam

// dL/dy of the latents (G[0, N) = dL/dyhat * dyhat/dy) and the squared norm of the whole
// gradient row (latents + parameters, clip_grad_norm_) in one pass
__global__ __launch_bounds__(kT) void t_latgrad_sumsq(const float *__restrict__ gq, const float *__restrict__ gq2,
                                                      const float *__restrict__ dq, int N, float *__restrict__ G,
                                                      int64_t n, int64_t gstride, float *__restrict__ acc4)
{
    __shared__ float s_red[8];
    const int b = blockIdx.y;
    float *g = G + (int64_t)b * gstride;
    const float *gqb = gq + (int64_t)b * N, *dqb = dq + (int64_t)b * N;
    const float *gq2b = gq2 ? gq2 + (int64_t)b * N : nullptr; // the ARM's part (side-stream form)
    float s = 0.f;
    // four elements per thread and iteration, every load issued first (one per iteration waited
    // on memory latency, as t_loss did)
    constexpr int U = 4;
    for (int64_t i0 = (int64_t)blockIdx.x * kT * U + threadIdx.x; i0 < n; i0 += (int64_t)gridDim.x * kT * U) {
        float a[U], a2[U], d[U], r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * kT, il = i < N ? i : 0;
            a[u] = gqb[il];
            a2[u] = gq2b ? gq2b[il] : 0.f;
            d[u] = dqb[il];
            r[u] = (i >= N && i < n) ? g[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * kT;
            float v = r[u];
            if (i < N) {
                v = (gq2b ? a2[u] + a[u] : a[u]) * d[u];
                g[i] = v;
            }
            s = fmaf(v, v, s); // 0 past the row
        }
    }
    s = block_sum(s, s_red);
    if (threadIdx.x == 0) atomicAdd(&acc4[b * 4 + 2], s);
}

struct AdamArgs {
    float lr_bc1, inv_sqrt_bc2, beta1, beta2, eps, clip;
    int N, latents_only;
    int64_t n, gstride, ls, ps, ms;
    const float *bc; // optional [B][2] per-frame (lr / bc1, 1 / sqrt(bc2)) (per-frame Adam steps)
    float *loss_out; // optional [B][4]: t_finish's row, written by workgroup (0, b)
    const float *rslots, *mslots;
    float inv_total, lam_px;
};

// per-frame bias corrections when frames carry their own Adam step (a frame whose optimizer
// state was reloaded from its best record, train.py:226-236): computed in double like the
// host path (torch.optim.Adam's bias_correction1/2 are Python floats); step <= 0 freezes
// the frame: its parameters AND its Adam moments stay as they are (marked by a negative
// second entry, which t_adam checks first)
__global__ void t_adam_bc(const int32_t *__restrict__ steps, double lr, double beta1, double beta2, int B,
                          float *__restrict__ bc)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int t = steps[b];
    if (t <= 0) {
        bc[2 * b] = 0.f;
        bc[2 * b + 1] = -1.f;
        return;
    }
    bc[2 * b] = (float)(lr / (1.0 - pow(beta1, (double)t)));
    bc[2 * b + 1] = (float)(1.0 / sqrt(1.0 - pow(beta2, (double)t)));
}

// torch.optim.Adam (_single_tensor_adam, no weight decay / amsgrad) after clip_grad_norm_
// rslots: [B][kDwSlots] rate sums; mslots: [B][kDwSlots] squared-error sums of the loss fused
// into the last t_sp_fwd (zero when t_loss ran: it adds into acc4[b][0])
__device__ __forceinline__ void finish_row(const float *__restrict__ acc4, const float *__restrict__ rslots,
                                           const float *__restrict__ mslots, float inv_total, float lam_px,
                                           float *__restrict__ out, int b)
{
    float rate = 0.f, sq = acc4[b * 4 + 0];
#pragma unroll 8
    for (int k = 0; k < kDwSlots; ++k) {
        rate += rslots[b * kDwSlots + k];
        sq += mslots[b * kDwSlots + k];
    }
    const float mse = sq * inv_total;
    out[b * 4 + 0] = mse + lam_px * rate;
    out[b * 4 + 1] = mse;
    out[b * 4 + 2] = rate;
    out[b * 4 + 3] = sqrtf(acc4[b * 4 + 2]);
}
__global__ void t_adam(const float *__restrict__ G, float *__restrict__ lat, float *__restrict__ th, float *__restrict__ m,
                       float *__restrict__ v, const float *__restrict__ acc4, AdamArgs A)
{
    const int b = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (A.loss_out && i == 0) finish_row(acc4, A.rslots, A.mslots, A.inv_total, A.lam_px, A.loss_out, b); // (t_finish folded in)
    if (i >= A.n || (A.latents_only && i >= A.N)) return;
    if (A.bc && A.bc[2 * b + 1] < 0.f) return; // frozen frame (adam_steps <= 0)
    float coef = 1.f;
    if (A.clip > 0.f) coef = fminf(A.clip / (sqrtf(acc4[b * 4 + 2]) + 1e-6f), 1.f);
    const float g = G[(int64_t)b * A.gstride + i] * coef;
    const int64_t mi = (int64_t)b * A.ms + i;
    const float mm = A.beta1 * m[mi] + (1.f - A.beta1) * g;
    const float vv = A.beta2 * v[mi] + (1.f - A.beta2) * g * g;
    m[mi] = mm;
    v[mi] = vv;
    const float lr_bc1 = A.bc ? A.bc[2 * b] : A.lr_bc1, inv_sqrt_bc2 = A.bc ? A.bc[2 * b + 1] : A.inv_sqrt_bc2;
    const float denom = sqrtf(vv) * inv_sqrt_bc2 + A.eps;
    float *p = i < A.N ? lat + (int64_t)b * A.ls + i : th + (int64_t)b * A.ps + (i - A.N);
    *p -= lr_bc1 * mm / denom;
}

__global__ void t_finish(const float *__restrict__ acc4, const float *__restrict__ rslots, const float *__restrict__ mslots,
                         float inv_total, float lam_px, float *__restrict__ out, int B)
{
    const int b = threadIdx.x;
    if (b < B) finish_row(acc4, rslots, mslots, inv_total, lam_px, out, b);
}

// ------------------------------------------------------------------ host planning
size_t align256(size_t v) { return (v + 255) / 256 * 256; }

// CCMI_ARM_OVERLAP = k > 0: the ARM forward + backward runs on a side stream, concurrently with
// the synthesis / upsampling forward and backward, with at most k workgroups per CU (its latent
// gradients in their own buffer, summed by t_latgrad_sumsq).  k = 1: the latency-bound ARM
// fills what the chain's kernels leave of each CU (8-frame 512x768 step 1.112 / 1.117 ->
// 1.049 / 1.050 ms; k = 2: 1.067 / 1.072, k = 3: 1.084 / 1.076; profiles/r4ah_*).  With the
// full resident grid (round 4, earlier) it took every CU's LDS and the chain queued behind it.
#ifndef CCMI_ARM_OVERLAP
#define CCMI_ARM_OVERLAP 1
#endif
// the compile-time default, or the environment's CCMI_ARM_OVERLAP (0 .. 3) read once per process
// (0 runs the ARM in line: kernel traces where every kernel runs alone)
static int arm_overlap()
{
    static const int v = [] {
        const char *e = getenv("CCMI_ARM_OVERLAP");
        if (e && e[0] >= '0' && e[0] <= '3' && !e[1]) return e[0] - '0';
        return (int)CCMI_ARM_OVERLAP;
    }();
    return v;
}
struct Plan {
    Geo g;
    ArmTiles at;
    int B, nblk_arm;
    // workspace offsets (bytes)
    size_t gq_arm = 0; // the ARM's latent gradients when it runs on the side stream (CCMI_ARM_OVERLAP)
    size_t yq, dq, gq, kf, stacks, stacks_bytes, dense, z[kMaxSp + 1], graw, gbuf[2], gdense, gstack, tmpU, tmpG, G,
        acc4, bc, rslots, mslots, slots, total;
    int64_t gstack_off[CCMI_MAX_GRIDS]; // per level k (1..L-2) inside gstack, elements per frame
    int64_t gstack_per, stack_per, tmp_per;
};

int make_plan(const ccmi_train_args *a, Plan &pl)
{
    Geo &g = pl.g;
    g = Geo{};
    const int L = a->n_grids;
    if (a->batch < 1) return ccmi_set_error(CCMI_ERR_ARG, "train: batch must be >= 1");
    if (L < 2 || L > CCMI_MAX_GRIDS) return ccmi_set_error(CCMI_ERR_ARG, "train: n_grids %d", L);
    g.L = L;
    int off = 0;
    for (int l = 0; l < L; ++l) {
        g.h[l] = a->h[l];
        g.w[l] = a->w[l];
        if (g.h[l] < 1 || g.w[l] < 1) return ccmi_set_error(CCMI_ERR_ARG, "train: grid %d is %dx%d", l, g.h[l], g.w[l]);
        if (l > 0 && (g.h[l] != (g.h[l - 1] + 1) / 2 || g.w[l] != (g.w[l - 1] + 1) / 2))
            return ccmi_set_error(CCMI_ERR_ARG, "train: grid %d is not ceil(half) of grid %d", l, l - 1);
        g.off[l] = off;
        off += g.h[l] * g.w[l];
    }
    g.N = off;
    g.H = g.h[0];
    g.W = g.w[0];
    if (a->latent_stride < g.N) return ccmi_set_error(CCMI_ERR_ARG, "train: latent_stride < %d", g.N);
    g.d = a->dim_arm;
    g.nh = a->n_hidden;
    if ((g.d != 8 && g.d != 16 && g.d != 24 && g.d != 32) || g.nh < 0 || g.nh > 3)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "train: ARM dim %d with %d hidden layers", g.d, g.nh);
    g.P_arm = g.nh * (g.d * g.d + g.d) + 2 * g.d + 2;
    g.K = a->ups_k;
    g.n_ups = a->n_ups;
    g.Kp = a->pre_k;
    g.n_pre = a->n_pre;
    if ((g.K != 4 && g.K != 6 && g.K != 8) || (g.Kp != 1 && g.Kp != 3 && g.Kp != 5 && g.Kp != 7 && g.Kp != 9) ||
        g.n_ups < 1 || g.n_pre < 1)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "train: upsampling kernels %d / %d", g.K, g.Kp);
    g.hu = (g.K + 1) / 2;
    g.hp = (g.Kp + 1) / 2;
    g.up_off = g.P_arm;
    g.pre_off = g.up_off + g.n_ups * g.hu;
    g.syn_off = g.pre_off + g.n_pre * g.hp;
    g.kfull = g.n_ups * g.K + g.n_pre * g.Kp;
    // synthesis: 1x1 (C -> hid) + 1x1 (hid -> 3), then <= 3 3x3 layers 3 -> 3
    const int ns = a->n_syn_layers;
    if (ns < 2 || ns > 2 + kMaxSp) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "train: %d synthesis layers", ns);
    const ccmi_syn_layer *S = a->syn;
    if (S[0].ks != 1 || S[1].ks != 1 || S[0].residual || S[1].residual || S[1].n_out != 3 || S[0].n_out < 1 ||
        S[0].n_out > 64)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "train: synthesis head must be 1x1 (C -> <=64) then 1x1 (-> 3)");
    g.hid = S[0].n_out;
    g.r0 = S[0].relu;
    g.r1 = S[1].relu;
    int p = g.syn_off;
    g.w0 = p;
    p += g.hid * L;
    g.b0 = p;
    p += g.hid;
    g.w1 = p;
    p += 3 * g.hid;
    g.b1 = p;
    p += 3;
    g.P_head = p - g.syn_off;
    g.n_sp = ns - 2;
    for (int i = 0; i < g.n_sp; ++i) {
        const ccmi_syn_layer &l = S[2 + i];
        if (l.ks != 3 || l.n_out != 3) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "train: layer %d must be 3x3, 3 -> 3", 2 + i);
        g.sp_w[i] = p;
        p += 81;
        g.sp_b[i] = p;
        p += 3;
        g.sp_res[i] = l.residual;
        g.sp_relu[i] = l.relu;
    }
    g.P = p;
    if (a->param_stride < g.P) return ccmi_set_error(CCMI_ERR_ARG, "train: param_stride < %d", g.P);

    pl.B = a->batch;
    ArmTiles &at = pl.at;
    at = ArmTiles{};
    at.n = L;
    int tiles = 0;
    for (int l = 0; l < L; ++l) {
        at.tiles_x[l] = ccmi_div_up(g.w[l], kATX);
        at.start[l] = tiles;
        tiles += at.tiles_x[l] * ccmi_div_up(g.h[l], kATY);
    }
    at.start[L] = tiles;
    pl.nblk_arm = tiles;
    const int64_t npx = (int64_t)g.H * g.W;

    // buffers
    const size_t B = (size_t)pl.B;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += align256(bytes); return r; };
    pl.yq = take(4 * B * g.N);
    pl.dq = take(4 * B * g.N);
    pl.gq = take(4 * B * g.N);
    pl.kf = take(4 * B * g.kfull);
    pl.stack_per = 0;
    for (int k = 1; k <= L - 2; ++k) pl.stack_per += (int64_t)(L - k) * g.h[k] * g.w[k];
    pl.stacks_bytes = 4 * B * (size_t)pl.stack_per;
    pl.stacks = take(pl.stacks_bytes + 4);
    pl.dense = take(4 * B * L * npx);
    for (int i = 0; i <= g.n_sp; ++i) pl.z[i] = take(4 * B * 3 * npx);
    pl.graw = take(4 * B * 3 * npx);
    pl.gbuf[0] = take(4 * B * 3 * npx);
    pl.gbuf[1] = take(4 * B * 3 * npx);
    pl.gdense = take(4 * B * L * npx);
    pl.gstack_per = pl.stack_per;
    {
        int64_t so = 0;
        for (int k = 1; k <= L - 2; ++k) {
            pl.gstack_off[k] = so;
            so += (int64_t)(L - k) * g.h[k] * g.w[k];
        }
    }
    pl.gstack = take(4 * B * pl.gstack_per + 4);
    int64_t tmax = 0;
    for (int k = 1; k <= L - 1; ++k) {
        tmax = std::max(tmax, (int64_t)(L - k) * g.h[k] * g.w[k - 1]); // upsample temps: C x hs x wd
        tmax = std::max(tmax, (int64_t)g.h[k - 1] * g.w[k - 1]);       // refine temps: hd x wd
    }
    pl.tmp_per = tmax;
    pl.tmpU = take(4 * B * tmax);
    pl.tmpG = take(4 * B * tmax);
    pl.G = take(4 * B * ((size_t)g.N + g.P));
    pl.acc4 = take(4 * B * 4);
    pl.bc = take(4 * B * 2);
    pl.rslots = take(4 * B * kDwSlots);
    pl.mslots = take(4 * B * kDwSlots); // the fused loss's squared-error sums
    // every parameter's gradient through kDwSlots slot rows per frame (one row per workgroup
    // residue), folded into the gradient row by t_dw_fold (kDwSlots)
    pl.slots = take(4 * B * kDwSlots * (size_t)g.P);
    if (arm_overlap()) pl.gq_arm = take(4 * B * g.N); // after acc4: zeroed with it
    pl.total = o;
    return CCMI_OK;
}

// Workgroups of `fn` that fit on the device at once (occupancy x CUs): the grid of the
// persistent (grid-stride) training kernels is ONE resident round.  A second round only adds
// workgroups, and each workgroup's flush costs one atomic per value on addresses every
// workgroup of the frame shares (t_arm16: 227 us with one round of 1024 workgroups, 232 us
// with 2048, after the flush reduction; before it 293 vs 460 us, profiles/r4l_*, r4m_*).
static int resident_wgs(const void *fn, int threads, size_t lds, int max_per_cu)
{
    static std::mutex mu;
    static std::map<std::tuple<const void *, size_t, int, int>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(fn, lds, dev, max_per_cu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, lds) != hipSuccess || per < 1) per = 1;
    return cache[key] = std::min(per, max_per_cu) * cus;
}

// the 1x1 head backward in the register form (t_head_bwd_m, opt-in: CCMI_HEAD_BWD_REGS=1) or the
// LDS-tiled form (t_head_bwd_t, the default).  The register form is bit-for-bit a different
// summation but passes every gradient test; it measured 273 us per launch against the tiled
// form's 190 us (step 0.842 -> 0.910 ms, profiles/r6h_head_bwd_regs_ab.txt): its 36 16x16x4
// MFMAs per 16 pixels are half padding (N = 8 of 16 inputs for g_x and dW0), and at 180 VGPRs it
// runs 2 waves / SIMD with no prefetch of the next block's 25 small loads.
// (read per call, like CCMI_SP_BWD_PF below, so a test can select either form within one
// process: a getenv per launch against a ~1 ms step)
static bool head_bwd_regs()
{
    const char *e = getenv("CCMI_HEAD_BWD_REGS");
    return e && *e == '1';
}

// the 3x3 backward as a persistent prefetching grid (t_sp_bwd<7>) or one tile per workgroup
// (t_sp_bwd<3>); CCMI_SP_BWD_PF=0 selects the latter (A/B)
static bool sp_bwd_persistent()
{
    const char *e = getenv("CCMI_SP_BWD_PF");
    return !(e && *e == '0');
}

// grid of a persistent kernel over `units` work units per frame, B frames
static dim3 resident_grid(const void *fn, int threads, size_t lds, int64_t units, int B, int max_per_cu = 1 << 20)
{
    const int64_t per_frame = std::max<int64_t>(1, resident_wgs(fn, threads, lds, max_per_cu) / B);
    return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(units, per_frame)), (unsigned)B);
}

template <int D>
int launch_arm_d(int nh, int64_t nblk, int B, int cap, hipStream_t s, const float *yq, const Geo &g, const ArmTiles &at, const float *th,
                 int64_t ps, float lam_px, float *gq, float *gth, int64_t gstride, float *acc4, const float *grate,
                 float *rate_out)
{
    if constexpr (D == 16) {
        // the matrix-core ARM (t_arm16): its MFMA chains replace the scalar weight loads of
        // the VALU kernel's tile loop (606 -> 499 us per 8-frame iteration)
        {
            switch (nh) {
            case 0: hipLaunchKernelGGL((t_arm16<0>), resident_grid((const void *)t_arm16<0>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
            case 1: hipLaunchKernelGGL((t_arm16<1>), resident_grid((const void *)t_arm16<1>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
            case 2: hipLaunchKernelGGL((t_arm16<2>), resident_grid((const void *)t_arm16<2>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
            default: hipLaunchKernelGGL((t_arm16<3>), resident_grid((const void *)t_arm16<3>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
            }
            return CCMI_OK;
        }
    }
    switch (nh) {
    case 0: hipLaunchKernelGGL((t_arm<D, 0>), resident_grid((const void *)t_arm<D, 0>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
    case 1: hipLaunchKernelGGL((t_arm<D, 1>), resident_grid((const void *)t_arm<D, 1>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
    case 2: hipLaunchKernelGGL((t_arm<D, 2>), resident_grid((const void *)t_arm<D, 2>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
    default: hipLaunchKernelGGL((t_arm<D, 3>), resident_grid((const void *)t_arm<D, 3>, kT, 0, nblk, B, cap), dim3(kT), 0, s, yq, g, at, th, ps, lam_px, gq, gth, gstride, acc4, grate, rate_out); break;
    }
    return CCMI_OK;
}

template <int CIN>
void launch_head(bool bwd, dim3 grid, hipStream_t s, const float *dense, const float *gz0, const Geo &g, const float *th,
                 int64_t ps, float *z0_or_gdense, float *gth, int64_t gstride)
{
    if (!bwd) {
        const unsigned nwg = (unsigned)(((int64_t)g.H * g.W + kHeadFwdPx - 1) / kHeadFwdPx);
        hipLaunchKernelGGL((t_head_fwd<CIN>), dim3(nwg, grid.y), dim3(kT), 0, s, dense, g, th, ps, z0_or_gdense);
    }
    else {
        // the tiled form for a linear output layer (every reference architecture); the full-width
        // form otherwise (and in -DCCMI_HEAD_BWD_FULL A/B builds)
#if defined(CCMI_HEAD_BWD_FULL)
        const bool tiled = false;
#else
        const bool tiled = !g.r1;
#endif
        constexpr int kXP = (CIN + 2 > 5 ? CIN + 2 : 5) | 1; // t_head_bwd's per-wave LDS rows
        const size_t lds = tiled ? sizeof(float) * (kHeadT / 64) * head_bwd_t_wave_floats(CIN)
                                 : sizeof(float) * (kHeadT / 64) * 64 * (16 * ((g.hid + 15) / 16) + 1 + kXP);
        // one resident round over the pixel chunks (full-width form LDS-bound: 5 workgroups per CU
        // at 32,000 B each, 276 us; at exactly 32 KB the query also allowed 5, but they did not all
        // fit: 399 us against 286 us capped at 4; profiles/r4n_*, r4o_*, r4y_*)
        const int64_t nchunk = ((int64_t)g.H * g.W + kHeadT - 1) / kHeadT;
#define CCMI_HB(N)                                                                                                     \
    if (tiled && head_bwd_regs() && CIN + 1 <= 8)                                                                      \
        hipLaunchKernelGGL((t_head_bwd_m<(CIN + 1 <= 8 ? CIN : 7), N>),                                               \
                           resident_grid((const void *)t_head_bwd_m<(CIN + 1 <= 8 ? CIN : 7), N>, 256, 0,                \
                                         ((int64_t)g.H * g.W + 63) / 64, (int)grid.y),                                  \
                           dim3(256), 0, s, dense, gz0, g, th, ps, z0_or_gdense, gth, gstride);                         \
    else if (tiled)                                                                                                    \
        hipLaunchKernelGGL((t_head_bwd_t<CIN, N>), resident_grid((const void *)t_head_bwd_t<CIN, N>, kHeadT, lds, nchunk, (int)grid.y), \
                           dim3(kHeadT), lds, s, dense, gz0, g, th, ps, z0_or_gdense, gth, gstride);                    \
    else                                                                                                               \
        hipLaunchKernelGGL((t_head_bwd<CIN, N, true>), resident_grid((const void *)t_head_bwd<CIN, N, true>, kHeadT, lds, nchunk, (int)grid.y), \
                           dim3(kHeadT), lds, s, dense, gz0, g, th, ps, z0_or_gdense, gth, gstride)
        switch ((g.hid + 15) / 16) {
        case 1: CCMI_HB(1); break;
        case 2: CCMI_HB(2); break;
        case 3: CCMI_HB(3); break;
        default: CCMI_HB(4); break;
        }
#undef CCMI_HB
    }
}

void head_dispatch(int cin, bool bwd, dim3 grid, hipStream_t s, const float *dense, const float *gz0, const Geo &g,
                   const float *th, int64_t ps, float *o, float *gth, int64_t gstride)
{
    switch (cin) {
    case 2: launch_head<2>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    case 3: launch_head<3>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    case 4: launch_head<4>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    case 5: launch_head<5>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    case 6: launch_head<6>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    case 7: launch_head<7>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    default: launch_head<8>(bwd, grid, s, dense, gz0, g, th, ps, o, gth, gstride); break;
    }
}

dim3 grid1(int64_t n, int B) { return dim3((unsigned)((n + kT - 1) / kT), (unsigned)B); }
// workgroups for a grid-stride reduction over n items: enough to fill the chip with a
// batch of frames, few enough that the per-workgroup atomics stay cheap
unsigned red_blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + kT - 1) / kT, 64)); }
// kernel-gradient reductions spread over kDwSlots addresses: one item per thread (the
// loops are latency-bound -- their inputs were just written by other XCDs, so every load
// goes past the local L2 -- and a thread's items run one after another)
unsigned dw_blocks(int64_t n, int per_thread = 1)
{
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per_thread * kT - 1) / (per_thread * kT), 4096));
}

} // namespace

extern "C" int ccmi_quantize_f32(const float *x, int64_t n, int quantizer, float temperature, const float *noise,
                                 float *y, float *dy, void *stream)
{
    if (!x || !y || n < 0) return ccmi_set_error(CCMI_ERR_ARG, "quantize: null argument");
    if (n > INT32_MAX - kT) return ccmi_set_error(CCMI_ERR_ARG, "quantize: n > 2^31 - %d", kT); // int thread indices
    if (quantizer < CCMI_Q_NONE || quantizer > CCMI_Q_TRUE_STE) return ccmi_set_error(CCMI_ERR_ARG, "quantize: type %d", quantizer);
    if ((quantizer == CCMI_Q_SOFTROUND || quantizer == CCMI_Q_SOFTROUND_ALONE || quantizer == CCMI_Q_STE) &&
        !(temperature > 0.f))
        return ccmi_set_error(CCMI_ERR_ARG, "quantize: soft-round temperature must be > 0");
    if (n == 0) return CCMI_OK;
    // noise comes as a tensor (or none): the counter-based generator is not used here
    hipLaunchKernelGGL(t_quant, grid1(n, 1), dim3(kT), 0, static_cast<hipStream_t>(stream), x, (int64_t)n, (int)n, 1.f,
                       quantizer, (int)CCMI_NOISE_NONE, quant_args(temperature, 1.f), (uint64_t)0, 0, noise, y, dy,
                       (float *)nullptr);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

extern "C" size_t ccmi_train_param_count(const ccmi_train_args *a)
{
    if (!a) return 0;
    ccmi_train_args t = *a;
    t.latent_stride = 1 << 30;
    t.param_stride = 1 << 30;
    t.batch = 1;
    Plan pl;
    if (make_plan(&t, pl)) return 0;
    return (size_t)pl.g.P;
}

extern "C" size_t ccmi_train_workspace_bytes(const ccmi_train_args *a)
{
    if (!a) return 0;
    Plan pl;
    if (make_plan(a, pl)) return 0;
    return pl.total;
}

// The ARM's side stream (CCMI_ARM_OVERLAP): leased from the process-wide pool for one call
// (ccmi_api.cpp; st[0], events ev[0] fork and ev[1] join).  SideJoin orders the side stream
// back into the caller's stream on EVERY exit after the fork: the explicit waits (forward-only
// return, before t_latgrad_sumsq) and, through its destructor, every error return in between,
// so no ARM kernel can still be writing gq_arm / acc4 / Gth / rate_out once the call returned.
struct SideJoin {
    hipStream_t s = nullptr, side = nullptr;
    hipEvent_t ev = nullptr;
    bool recorded = false, pending = false;
    void record()
    {
        if (pending && !recorded) recorded = hipEventRecord(ev, side) == hipSuccess;
    }
    hipError_t wait()
    {
        if (!pending) return hipSuccess;
        record();
        pending = false;
        return recorded ? hipStreamWaitEvent(s, ev, 0) : hipStreamSynchronize(side);
    }
    ~SideJoin() { (void)wait(); }
};

#if defined(CCMI_DIAG_SIDE_SPIN)
// Diagnostic build only (make spin): ~5 ms of spinning queued on the side stream before the
// ARM, so a consumer that reads the ARM's outputs without the join sees stale data every time.
__global__ void t_diag_spin(uint64_t ticks)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime(); // 100 MHz constant clock
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
#endif

extern "C" int ccmi_train_step(const ccmi_train_args *a, void *stream)
{
    if (!a || !a->latent || !a->params || !a->target) return ccmi_set_error(CCMI_ERR_ARG, "train: null argument");
    Plan pl;
    if (int rc = make_plan(a, pl)) return rc;
    if (!a->workspace || a->workspace_bytes < pl.total)
        return ccmi_set_error(CCMI_ERR_ARG, "train: workspace of %zu bytes needed", pl.total);
    if (a->update && (!a->adam_m || !a->adam_v || (a->step < 1 && !a->adam_steps)))
        return ccmi_set_error(CCMI_ERR_ARG, "train: Adam state and step >= 1 needed to update");
    if ((a->quantizer == CCMI_Q_SOFTROUND || a->quantizer == CCMI_Q_SOFTROUND_ALONE || a->quantizer == CCMI_Q_STE) &&
        !(a->temperature > 0.f))
        return ccmi_set_error(CCMI_ERR_ARG, "train: soft-round temperature must be > 0");
    if (a->noise == CCMI_NOISE_KUMARASWAMY && !(a->noise_param > 0.f))
        return ccmi_set_error(CCMI_ERR_ARG, "train: kumaraswamy parameter must be > 0");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const Geo &g = pl.g;
    const int B = pl.B;
    uint8_t *ws = static_cast<uint8_t *>(a->workspace);
    auto F = [&](size_t off) { return reinterpret_cast<float *>(ws + off); };
    float *yq = F(pl.yq), *dq = F(pl.dq), *gq = F(pl.gq), *kf = F(pl.kf), *dense = F(pl.dense), *graw = F(pl.graw);
    float *gd = F(pl.gdense), *gst = F(pl.gstack), *U = F(pl.tmpU), *GU = F(pl.tmpG), *acc4 = F(pl.acc4);
    const int64_t GS = (int64_t)g.N + g.P; // gradient row per frame: latents then parameters
    float *G = a->grad_out ? a->grad_out : F(pl.G);
    float *Gth = G + g.N;
    const int64_t npx = (int64_t)g.H * g.W;
    const float lam_px = a->lmbda / (float)npx;

    // the parameter gradients' slot rows ([B][kDwSlots][P], see make_plan) and the rate slots
    float *slots = F(pl.slots), *rslots = F(pl.rslots);
    float *uslots = slots + g.up_off; // the upsampling kernels' columns (their offsets are relative to up_off)
    {
        // acc4 .. the end of the workspace plan (rate and parameter-gradient slots, the ARM's side
        // gradient) zeroed and the symmetric kernels expanded, in one launch; the gradient rows
        // need no zeroing: t_latgrad_sumsq writes their latent part and t_dw_fold their parameters
        const int64_t nz = (int64_t)(pl.total - pl.acc4) / (int64_t)sizeof(float);
        const int64_t n = nz + (int64_t)B * g.kfull;
        const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ccmi_div_up(n, 4 * kT), 2048));
        hipLaunchKernelGGL(t_prologue, dim3(nb), dim3(kT), 0, s, acc4, nz, a->params, a->param_stride, g, kf, B,
                           a->update ? a->step_counters : nullptr);
    }

    // ---- forward
    hipLaunchKernelGGL(t_quant, grid1(g.N, B), dim3(kT), 0, s, a->latent, a->latent_stride, g.N, a->gain, a->quantizer,
                       a->noise, quant_args(a->temperature, a->noise_param), (uint64_t)a->seed, a->step, a->noise_in, yq,
                       dq, gq);
    StreamSetLease lease; // declared before the join: released after it
    SideJoin join;
    bool side = false;
    {
        // persistent over the latent tiles: one resident round of workgroups for the batch (or,
        // with CCMI_ARM_OVERLAP, at most that many per CU, on the side stream)
        hipStream_t sa = s;
        float *gqa = gq;
        int cap = 1 << 20;
        if (arm_overlap() > 0) {
            lease.set = ccmi_streamset_acquire(1, 2, false);
            if (!lease.set) return CCMI_ERR_HIP;
            CCMI_HIP_CHECK(hipEventRecord(lease.set->ev[0], s));
            CCMI_HIP_CHECK(hipStreamWaitEvent(lease.set->st[0], lease.set->ev[0], 0));
            side = true;
            sa = lease.set->st[0];
            join.s = s;
            join.side = sa;
            join.ev = lease.set->ev[1];
            join.pending = true; // from here on every return joins
            gqa = F(pl.gq_arm);
            cap = arm_overlap();
#if defined(CCMI_DIAG_SIDE_SPIN)
            hipLaunchKernelGGL(t_diag_spin, dim3(1), dim3(64), 0, sa, (uint64_t)500000);
#endif
        }
        switch (g.d) {
        case 8: launch_arm_d<8>(g.nh, pl.nblk_arm, B, cap, sa, yq, g, pl.at, a->params, a->param_stride, lam_px, gqa, slots, g.P, rslots, a->grad_rate, a->rate_out); break;
        case 16: launch_arm_d<16>(g.nh, pl.nblk_arm, B, cap, sa, yq, g, pl.at, a->params, a->param_stride, lam_px, gqa, slots, g.P, rslots, a->grad_rate, a->rate_out); break;
        case 24: launch_arm_d<24>(g.nh, pl.nblk_arm, B, cap, sa, yq, g, pl.at, a->params, a->param_stride, lam_px, gqa, slots, g.P, rslots, a->grad_rate, a->rate_out); break;
        default: launch_arm_d<32>(g.nh, pl.nblk_arm, B, cap, sa, yq, g, pl.at, a->params, a->param_stride, lam_px, gqa, slots, g.P, rslots, a->grad_rate, a->rate_out); break;
        }
        CCMI_HIP_CHECK(hipGetLastError());
        join.record();
    }
    {
        ccmi_ups_args u{};
        u.latent = yq;
        u.latent_stride = g.N;
        u.n_grids = g.L;
        for (int l = 0; l < g.L; ++l) {
            u.h[l] = g.h[l];
            u.w[l] = g.w[l];
        }
        u.gain = 1.f;
        u.quantize = 0;
        u.ups_k = g.K;
        u.n_ups = g.n_ups;
        u.pre_k = g.Kp;
        u.n_pre = g.n_pre;
        u.params = kf;
        u.param_stride = g.kfull;
        u.out = dense;
        u.out_stride = (int64_t)g.L * npx;
        u.workspace = F(pl.stacks);
        u.workspace_bytes = pl.stacks_bytes + 4;
        u.batch = B;
        if (int rc = ccmi_launch_ups_f32(&u, s)) return rc; // joined by ~SideJoin
    }
    head_dispatch(g.L, false, dim3((unsigned)((npx + 2 * kT - 1) / (2 * kT)), (unsigned)B), s, dense, nullptr, g, a->params,
                  a->param_stride, F(pl.z[0]), nullptr, 0); // two pixels per thread
    // the training step's MSE fused into the last 3x3 layer (no separate t_loss pass over the
    // synthesis output); the output itself is stored only when something reads it
    const bool fuse_loss = !a->forward_only && !a->grad_raw && g.n_sp > 0;
    for (int i = 0; i < g.n_sp; ++i) {
        const bool fl = fuse_loss && i == g.n_sp - 1;
        const int store = !fl || a->raw_out || g.sp_relu[i];
        const dim3 grid(grid1((int64_t)ccmi_div_up(g.H, kSpRows) * g.W, 1).x * B);
        const float total = a->yuv420 ? (float)(npx + 2 * (int64_t)(g.H / 2) * (g.W / 2)) : (float)(3 * npx);
        auto launch = [&](auto LOSS) {
            hipLaunchKernelGGL((t_sp_fwd<decltype(LOSS)::value>), grid, dim3(kT), 0, s, F(pl.z[i]), g, a->params, a->param_stride,
                               g.sp_w[i], g.sp_b[i], g.sp_res[i], g.sp_relu[i], F(pl.z[i + 1]), a->target, a->target_stride,
                               2.f / total, graw, F(pl.mslots), store);
        };
        if (!fl) launch(std::integral_constant<int, 0>{});
        else if (a->yuv420) launch(std::integral_constant<int, 2>{});
        else launch(std::integral_constant<int, 1>{});
    }
    if (a->raw_out)
        CCMI_HIP_CHECK(hipMemcpyAsync(a->raw_out, F(pl.z[g.n_sp]), sizeof(float) * 3 * npx * B, hipMemcpyDeviceToDevice, s));
    if (a->forward_only) {
        // the ARM's rate (rate_out, the rate sums in acc4) comes from the side stream
        CCMI_HIP_CHECK(join.wait());
        if (a->loss_out) {
            // with a real target (target_stride > 0) the loss row holds the built-in MSE too;
            // otherwise (autograd: the loss lives in torch) MSE reads 0 and loss = lmbda-rate
            if (a->target && a->target_stride > 0)
                hipLaunchKernelGGL(t_loss, dim3(sum_blocks(npx, kLossPx), B), dim3(kT), 0, s, F(pl.z[g.n_sp]), g,
                                   a->target, a->target_stride, a->yuv420, graw, acc4);
            const float total = a->yuv420 ? (float)(npx + 2 * (int64_t)(g.H / 2) * (g.W / 2)) : (float)(3 * npx);
            hipLaunchKernelGGL(t_finish, dim3(1), dim3(std::max(64, B)), 0, s, acc4, F(pl.rslots), F(pl.mslots), 1.f / total, lam_px, a->loss_out, B);
        }
        CCMI_HIP_CHECK(hipGetLastError());
        return CCMI_OK;
    }
    if (a->grad_raw) // the caller's d loss / d raw output (autograd); no built-in MSE term
        CCMI_HIP_CHECK(hipMemcpyAsync(graw, a->grad_raw, sizeof(float) * 3 * npx * B, hipMemcpyDeviceToDevice, s));
    else if (!fuse_loss)
        hipLaunchKernelGGL(t_loss, dim3(sum_blocks(npx, kLossPx), B), dim3(kT), 0, s, F(pl.z[g.n_sp]), g, a->target, a->target_stride,
                           a->yuv420, graw, acc4);

    // ---- synthesis backward
    float *gcur = graw;
    for (int i = g.n_sp - 1; i >= 0; --i) {
        float *gin = F(pl.gbuf[i & 1]);
        const int ntile = ccmi_div_up(g.W, kSX) * ccmi_div_up(g.H, kSY);
        // weight gradients: grid-stride over <= 1024 / B workgroups per frame (measured fastest
        // against 32 .. 512 per frame)
        const unsigned nb = (unsigned)std::max(1, std::min(ntile, 1024 / B));
        // a ReLU layer's mask comes from its output planes only for the last layer (its output
        // gradient is the loss's); for the others the next layer's backward applied it (mask_in)
        const float *outp = g.sp_relu[i] && i == g.n_sp - 1 ? F(pl.z[i + 1]) : nullptr;
        const int mask_in = i >= 1 && g.sp_relu[i - 1];
#if defined(CCMI_SP_BWD_SPLIT) // A/B builds: the round-4 pair of launches
        {
            const float *outp = g.sp_relu[i] ? F(pl.z[i + 1]) : nullptr; // no mask bit: MODE 1 stages no X
            // input gradient: one tile per workgroup; weight gradients: grid-stride as before
            hipLaunchKernelGGL(t_sp_bwd<1>, dim3((unsigned)ntile, B), dim3(kT), 0, s, gcur, outp, F(pl.z[i]), g, a->params,
                               a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
            hipLaunchKernelGGL(t_sp_bwd<2>, dim3(nb, B), dim3(kT), 0, s, gcur, outp, F(pl.z[i]), g, a->params,
                               a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
        }
#else
        (void)nb;
        // both halves, one tile per workgroup: each tile's X / G / out read once
        if (sp_bwd_persistent() && mask_in)
            hipLaunchKernelGGL(t_sp_bwd<15>, resident_grid((const void *)t_sp_bwd<15>, kT, 0, ntile, B), dim3(kT), 0, s, gcur,
                               outp, F(pl.z[i]), g, a->params, a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
        else if (sp_bwd_persistent())
            hipLaunchKernelGGL(t_sp_bwd<7>, resident_grid((const void *)t_sp_bwd<7>, kT, 0, ntile, B), dim3(kT), 0, s, gcur,
                               outp, F(pl.z[i]), g, a->params, a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
        else if (mask_in)
            hipLaunchKernelGGL(t_sp_bwd<11>, dim3((unsigned)ntile, B), dim3(kT), 0, s, gcur, outp, F(pl.z[i]), g, a->params,
                               a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
        else
            hipLaunchKernelGGL(t_sp_bwd<3>, dim3((unsigned)ntile, B), dim3(kT), 0, s, gcur, outp, F(pl.z[i]), g, a->params,
                               a->param_stride, g.sp_w[i], g.sp_b[i], g.sp_res[i], gin, slots, g.P);
#endif
        gcur = gin;
    }
    {
        // grid-stride over pixel chunks: one resident round of workgroups (set by launch_head)
        head_dispatch(g.L, true, dim3(1, B), s, dense, gcur, g, a->params, a->param_stride, gd, slots, g.P);
    }

    // ---- upsampling backward, finest level first (step L-2 .. 0)
    const int K2 = g.K / 2;
    for (int step = g.L - 2; step >= 0; --step) {
        const int k = g.L - 1 - step; // source level; destination level k-1
        const int hd = g.h[k - 1], wd = g.w[k - 1];
        const int C = g.L - k;
        const float *GY = (k - 1 == 0) ? gd : gst + pl.gstack_off[k - 1];
        const int64_t gys = (k - 1 == 0) ? (int64_t)g.L * npx : pl.gstack_per;
        // refine of y_hat(k-1): channel 0 of the destination stack (tiles 16 x 64)
        const int rtx = ccmi_div_up(wd, 64), nref = rtx * ccmi_div_up(hd, 16);
        const RefBwd R{GY, gys, yq + g.off[k - 1], (int64_t)g.N, hd, wd, kf, g.kfull,
                       g.n_ups * g.K + (step % g.n_pre) * g.Kp, gq + g.off[k - 1], (int64_t)g.N, uslots, (int64_t)g.P,
                       g.pre_off + (step % g.n_pre) * g.hp - g.up_off, rtx};
        // transposed-conv upsampling of the source stack: channels 1..C
        {
            UpLevel A{C, g.h[k], g.w[k], hd, wd, g.K, -((K2 + 1) / 2), K2 / 2, step % g.n_ups};
            const float *S = (k == g.L - 1) ? yq + g.off[k] : F(pl.stacks) + 0;
            int64_t ss = (k == g.L - 1) ? (int64_t)g.N : 0;
            if (k != g.L - 1) {
                // stacks laid out by ccmi_launch_ups_f32: level k at sum_{k'<k} (L-k') h w, [batch][...]
                int64_t so = 0;
                for (int kk = 1; kk < k; ++kk) so += (int64_t)(g.L - kk) * g.h[kk] * g.w[kk] * B;
                S = F(pl.stacks) + so;
                ss = (int64_t)(g.L - k) * g.h[k] * g.w[k];
            }
            const int koff = A.sidx * g.K;
            const int hoff = g.up_off + A.sidx * g.hu;
            float *GSd = (k == g.L - 1) ? gq + g.off[k] : gst + pl.gstack_off[k];
            const int64_t gss = (k == g.L - 1) ? (int64_t)g.N : pl.gstack_per;
            if (g.K == 8 && A.d_lo == -2 && A.d_hi == 2) {
                // the whole step, refine and transposed conv, in one launch (t_lvl_bwd)
                const int tx = ccmi_div_up(wd, 64), ty = ccmi_div_up(A.hs, 16);
                const UpBwd Q{GY, gys, S, ss, A, kf, g.kfull, koff, GSd, gss, k == g.L - 1 ? 1 : 0, uslots, (int64_t)g.P,
                              hoff - g.up_off, tx, ty, B};
                const dim3 grid((unsigned)((nref + tx * ty * C) * B));
                switch (g.Kp) {
                case 1: hipLaunchKernelGGL((t_lvl_bwd<1, 8>), grid, dim3(kT), 0, s, R, Q, nref); break;
                case 3: hipLaunchKernelGGL((t_lvl_bwd<3, 8>), grid, dim3(kT), 0, s, R, Q, nref); break;
                case 5: hipLaunchKernelGGL((t_lvl_bwd<5, 8>), grid, dim3(kT), 0, s, R, Q, nref); break;
                case 7: hipLaunchKernelGGL((t_lvl_bwd<7, 8>), grid, dim3(kT), 0, s, R, Q, nref); break;
                default: hipLaunchKernelGGL((t_lvl_bwd<9, 8>), grid, dim3(kT), 0, s, R, Q, nref); break;
                }
                continue;
            }
            const dim3 rgr((unsigned)nref, B);
            switch (g.Kp) {
            case 1: hipLaunchKernelGGL(t_ref_bwd<1>, rgr, dim3(kT), 0, s, R); break;
            case 3: hipLaunchKernelGGL(t_ref_bwd<3>, rgr, dim3(kT), 0, s, R); break;
            case 5: hipLaunchKernelGGL(t_ref_bwd<5>, rgr, dim3(kT), 0, s, R); break;
            case 7: hipLaunchKernelGGL(t_ref_bwd<7>, rgr, dim3(kT), 0, s, R); break;
            default: hipLaunchKernelGGL(t_ref_bwd<9>, rgr, dim3(kT), 0, s, R); break;
            }
            const int64_t nu = (int64_t)C * A.hs * wd;
            hipLaunchKernelGGL(t_up_u, grid1(nu, B), dim3(kT), 0, s, S, ss, A, kf, g.kfull, koff, U, pl.tmp_per);
            hipLaunchKernelGGL(t_up_gu, grid1(nu, B), dim3(kT), 0, s, GY, gys, A, kf, g.kfull, koff, GU, pl.tmp_per);
            const dim3 gr(dw_blocks((int64_t)C * hd * wd, 8), B); // measured: 8 items per thread beat 1 here
            switch (g.K) {
            case 4: hipLaunchKernelGGL(t_up_dw<4>, gr, dim3(kT), 0, s, GY, gys, U, GU, pl.tmp_per, S, ss, A, uslots, (int64_t)g.P, hoff - g.up_off); break;
            case 6: hipLaunchKernelGGL(t_up_dw<6>, gr, dim3(kT), 0, s, GY, gys, U, GU, pl.tmp_per, S, ss, A, uslots, (int64_t)g.P, hoff - g.up_off); break;
            default: hipLaunchKernelGGL(t_up_dw<8>, gr, dim3(kT), 0, s, GY, gys, U, GU, pl.tmp_per, S, ss, A, uslots, (int64_t)g.P, hoff - g.up_off); break;
            }
            hipLaunchKernelGGL(t_up_gs, grid1((int64_t)C * A.hs * A.ws, B), dim3(kT), 0, s, GU, pl.tmp_per, A, kf, g.kfull,
                               koff, GSd, gss, k == g.L - 1 ? 1 : 0);
        }
    }
    CCMI_HIP_CHECK(hipGetLastError());


    // ---- latent gradients, norm, Adam
    const unsigned nls = sum_blocks(GS, 4);
    CCMI_HIP_CHECK(join.wait());
    // every parameter gradient (the ARM's from the side stream too) from its slot rows
    hipLaunchKernelGGL(t_dw_fold, dim3((unsigned)ccmi_div_up(g.P, 64), B), dim3(64), 0, s, slots, g.P, Gth, GS, 0);
    hipLaunchKernelGGL(t_latgrad_sumsq, dim3(nls, B), dim3(kT), 0, s, gq, side ? F(pl.gq_arm) : nullptr, dq, g.N, G, GS,
                       GS, acc4);
    const float total = a->yuv420 ? (float)(npx + 2 * (int64_t)(g.H / 2) * (g.W / 2)) : (float)(3 * npx);
    if (a->loss_out && !a->update)
        hipLaunchKernelGGL(t_finish, dim3(1), dim3(std::max(64, B)), 0, s, acc4, F(pl.rslots), F(pl.mslots), 1.f / total, lam_px, a->loss_out, B);
    if (a->update) {
        const double bc1 = 1.0 - std::pow((double)a->beta1, a->step), bc2 = 1.0 - std::pow((double)a->beta2, a->step);
        AdamArgs A{(float)(a->lr / bc1), (float)(1.0 / std::sqrt(bc2)), a->beta1, a->beta2, a->eps, a->clip, g.N,
                   a->update == 2 ? 1 : 0, GS, GS,
                   a->latent_stride, a->param_stride, (int64_t)a->latent_stride + a->param_stride, nullptr,
                   a->loss_out, F(pl.rslots), F(pl.mslots), 1.f / total, lam_px};
        if (a->adam_steps) {
            A.bc = F(pl.bc);
            hipLaunchKernelGGL(t_adam_bc, dim3((unsigned)ccmi_div_up(B, 64)), dim3(64), 0, s, a->adam_steps, (double)a->lr,
                               (double)a->beta1, (double)a->beta2, B, F(pl.bc));
        }
        hipLaunchKernelGGL(t_adam, grid1(GS, B), dim3(kT), 0, s, G, a->latent, a->params, a->adam_m, a->adam_v, acc4, A);
    }
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}
