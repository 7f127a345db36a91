// dec_kernels.hip -- path B: HIP kernels of the bit-exact fixed-point .cool decoder.
//
// Compiled with -fwrapv: every accumulation is int32 with two's-complement wrap,
// every right shift of a sum is the reference's truncation toward zero
// (s < 0 ? -((-s) >> p) : s >> p) unless the reference rounds.
//
//  dec_arm_kernel   one wavefront per latent-layer CABAC stream (arm_cpu.cpp:18-106,
//                   cc-bac.h:3-253): raster-order serial decode.  The CABAC state is
//                   wave-uniform (scalar registers); lane o < d owns MLP neuron o; the
//                   4 causal rows live in an LDS ring; same-row contexts come from
//                   registers, so the only per-latent LDS traffic is the above-row
//                   gather.  Many streams (7 per frame x frames) run concurrently.
//  dec_ups_level    one launch per pyramid level (ups_refine_cpu.hpp:11-79,
//                   ups_upsample_cpu.hpp:12-91): integer refine + 2x polyphase upsample
//                   with the reference's per-pass truncations, LDS-tiled.
//  dec_syn_fused    1x1+1x1 fused head (synfused_cpu.hpp:17-109 semantics) + 3x3 layers
//                   (syn_cpu.hpp / synlb_cpu.hpp) with replicate padding, one launch.
//  dec_syn_layer    generic per-layer integer conv (any ks / widths).
//  dec_output       444 -> 420/444 8/10-bit or PPM payload (ccdecapi.cpp:59-240).
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "ccmi_cabac.h"
#include "dec_internal.h"

namespace ccmi {
namespace {

// ------------------------------------------------------------------ context table
struct CtxPack {
    uint32_t v[17 * 50 * 2];
};
constexpr uint8_t k_ctx_bytes[17 * 50 * 5] = {
#include "ccmi_ctx_table.inc"
};
constexpr CtxPack make_ctx_pack()
{
    CtxPack p{};
    for (int i = 0; i < 17 * 50; ++i) {
        const uint8_t *s = &k_ctx_bytes[i * 5];
        p.v[2 * i] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
        p.v[2 * i + 1] = s[4];
    }
    return p;
}
__constant__ CtxPack c_ctx = make_ctx_pack();

__device__ __forceinline__ int32_t tshift(int32_t s, int p) { return s < 0 ? -((-s) >> p) : s >> p; }
__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

// ------------------------------------------------------------------ device byte source
// The stream is read through a constant-address-space pointer so that the wave-uniform
// word loads become scalar (SMEM) loads; the next word is prefetched one word ahead.
typedef const __attribute__((address_space(4))) uint32_t *const_u32_ptr;

struct DevBytes {
    const_u32_ptr p;
    uint32_t nwords, pos, wi, cur, nxt;
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return i < nwords ? p[i] : 0u; }
    __device__ __forceinline__ void init(const uint32_t *base, uint32_t nbytes)
    {
        p = (const_u32_ptr)(size_t)base;
        nwords = (nbytes + 3u) >> 2;
        pos = 0;
        wi = 0;
        cur = ld(0);
        nxt = ld(1);
    }
    __device__ __forceinline__ uint32_t next()
    {
        const uint32_t b = (cur >> ((pos & 3u) * 8u)) & 0xFFu;
        ++pos;
        if ((pos & 3u) == 0) {
            cur = nxt;
            ++wi;
            nxt = ld(wi + 1);
        }
        return b;
    }
};

// Sum of v over each DPP row of 16 lanes; the result is valid in lane 15 of the row.
__device__ __forceinline__ int row_sum16(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true); // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true); // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true); // row_shr:8
    return v;
}

// Context pixel (dy, dx) of context index i (cc-frame-decoder.cpp:111-154 order).
template <int D>
__device__ __forceinline__ void ctx_dydx(int i, int &dy, int &dx)
{
    // flattened 9x9 mask index k -> (k/9 - 4, k%9 - 4); same neighbourhoods as the C stride tables
    constexpr signed char k8[8] = {13, 22, 30, 31, 32, 37, 38, 39};
    constexpr signed char k16[16] = {13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39};
    constexpr signed char k24[24] = {4, 11, 12, 13, 14, 15, 19, 20, 21, 22, 23, 24, 25, 28, 29, 30, 31, 32, 33, 34,
                                     36, 37, 38, 39};
    constexpr signed char k32[32] = {2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 19, 20, 21, 22, 23, 24, 25, 26, 27,
                                     28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39};
    int k = 40;
    if (i < D) k = D == 8 ? k8[i] : D == 16 ? k16[i] : D == 24 ? k24[i] : k32[i];
    dy = k / 9 - 4;
    dx = k % 9 - 4;
}

constexpr int kRing = 5;   // rows y-4 .. y
constexpr int kRingS = 4;  // speculative kernel (D <= 16: contexts reach row y-3): rows y-3 .. y
constexpr int kPad = 8;    // zero columns either side of a ring row (speculative groups read x+3+4)

// int32 multiply with two's-complement wrap; the 24-bit form (v_mad_i32_i24, full rate)
// is exact whenever both operands fit in 24 signed bits.
template <bool F24>
__device__ __forceinline__ int32_t imul(int32_t a, int32_t b)
{
    if constexpr (F24) return __mul24(a, b);
    else return (int32_t)((uint32_t)a * (uint32_t)b);
}

// OR of CCMI_ARM_FLAG_* bits into the stream's status word (one lane; a vector global atomic)
__device__ __forceinline__ void put_status(const ArmStreamDesc &S, uint32_t bits)
{
    if (bits && S.status) __hip_atomic_fetch_or(S.status, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One residual hidden layer, lane o = neuron o: (b + 256 a_o + sum_i W[o][i] a_i), ReLU, round >> 8.
template <int D, bool F24>
__device__ __forceinline__ int32_t arm_hidden(const int32_t (&W)[D], int32_t bias, int32_t a)
{
    int32_t acc = bias + a * 256;
#pragma unroll
    for (int i = 0; i < D; ++i) acc += imul<F24>(W[i], __builtin_amdgcn_readlane(a, i));
    return acc < 0 ? 0 : (acc + 128) >> 8;
}

#if defined(CCMI_ARM_STAMPS)
// Diagnostic build only (make stamps): per-stream cycle totals of the decode segments.
#define STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define ACC(k, a, b) st_acc[k] += (b) - (a)
#else
#define STAMP(var)
#define ACC(k, a, b)
#endif

template <int D, int NH>
__global__ __launch_bounds__(64) void dec_arm_kernel(const ArmStreamDesc *__restrict__ streams, int pitch)
{
#if defined(CCMI_ARM_STAMPS)
    uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    extern __shared__ int32_t smem[];
    int32_t *ring = smem;                                              // kRing x pitch
    uint8_t *bmap = reinterpret_cast<uint8_t *>(smem + kRing * pitch); // block sig/flat map

    const ArmStreamDesc S = streams[blockIdx.x];
    const int lane = threadIdx.x;
    const int h = S.h, w = S.w;
    // weights fit in 24 signed bits (host check): hidden layers >= 2 and the output layer
    // then use 24-bit multiplies (their inputs are ReLU-rounded sums, < 2^23 by construction)
    const bool w24 = (S.flags & 1) != 0;

#if defined(CCMI_ARM_STAMPS)
    const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#endif
    for (int i = lane; i < kRing * pitch; i += 64) ring[i] = 0;

    // ---- weights: lane owns neuron o = lane % D (lanes >= D duplicate, masked in sums)
    const int o = lane % D;
    int32_t Wh[NH > 0 ? NH : 1][D], Bh[NH > 0 ? NH : 1];
#pragma unroll
    for (int l = 0; l < NH; ++l) {
        const int32_t *base = S.weights + l * (D * D + D);
#pragma unroll
        for (int i = 0; i < D; ++i) Wh[l][i] = base[o * D + i];
        Bh[l] = base[D * D + o];
    }
    const int32_t *ob = S.weights + NH * (D * D + D);
    const int32_t Wo0 = lane < D ? ob[o] : 0, Wo1 = lane < D ? ob[D + o] : 0;
    const int32_t bo0 = __builtin_amdgcn_readfirstlane(ob[2 * D]);
    const int32_t bo1 = __builtin_amdgcn_readfirstlane(ob[2 * D + 1]);

    // ---- CABAC start + block significance / flat maps (BACContext::set_layer, cc-bac.h:24-130)
    Cabac<DevBytes> cab;
    cab.src.init(S.bytes, S.nbytes);
    cab.start();
    const int updated = S.sig_blk < 0;
    const int blk = S.sig_blk < 0 ? -S.sig_blk : S.sig_blk;
    int shift = 0;
    while ((1 << shift) < blk) ++shift;
    const int mask = (1 << shift) - 1;
    int nby = 1, nbx = 1;
    if (blk > 0) {
        nby = (h + blk - 1) >> shift;
        nbx = (w + blk - 1) >> shift;
    }
    const int nblk = nby * nbx;
    for (int i = lane; i < nblk; i += 64) bmap[i] = 1; // bit0 sig, bit1 flat
    __syncthreads();
    if (nblk > 1) {
        if (cab.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const uint32_t b = updated ? cab.bin_adaptive(m) : cab.ep();
                if (lane == 0) bmap[i] = (uint8_t)b;
            }
        }
        __syncthreads();
        if (cab.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const int sig = __builtin_amdgcn_readfirstlane((int)bmap[i]);
                if (sig) {
                    const uint32_t f = updated ? cab.bin_adaptive(m) : cab.ep();
                    if (lane == 0) bmap[i] = (uint8_t)(sig | (f << 1));
                }
            }
        }
    }
    __syncthreads();

#if defined(CCMI_ARM_STAMPS)
    st_acc[5] = __builtin_amdgcn_s_memtime() - t_begin; // setup incl. block maps
    const uint64_t t_loop = __builtin_amdgcn_s_memtime();
#endif
    // ---- context geometry of this lane (context index = o)
    int cdy, cdx;
    ctx_dydx<D>(o, cdy, cdx);
    const bool same_row = cdy == 0;
    int big = 0; // uniform: a decoded |latent| >= 2^15 was seen -> contexts may exceed 24 bits

    for (int y = 0; y < h; ++y) {
        int32_t *row = ring + (y % kRing) * pitch + kPad;
        const int32_t *up = ring + ((y + kRing - 1) % kRing) * pitch + kPad;
        const int32_t *crow = ring + ((y + cdy + kRing) % kRing) * pitch + kPad + cdx;
        int32_t r1 = 0, r2 = 0, r3 = 0, r4 = 0; // decoded values at x-1 .. x-4 (this row)
        const int brow = blk > 0 ? (y >> shift) * nbx : 0;
        int bm = 1;
        for (int x = 0; x < w; ++x) {
            int32_t v;
            if (blk > 0 && (x & mask) == 0) bm = __builtin_amdgcn_readfirstlane((int)bmap[brow + (x >> shift)]);
            if (!(bm & 1)) {
                v = 0;
            } else if ((bm & 2) && (x & mask)) {
                v = r1;
            } else if ((bm & 2) && (y & mask)) {
                v = __builtin_amdgcn_readfirstlane(up[x]);
            } else {
                STAMP(t0);
                const int32_t al = crow[x]; // same-row lanes read a stale slot, replaced below
                const int32_t rs = cdx == -1 ? r1 : cdx == -2 ? r2 : cdx == -3 ? r3 : r4;
                int32_t a = same_row ? rs : al;
                const bool f1 = w24 && !big; // contexts (latent << 8) fit in 24 bits
#pragma unroll
                for (int l = 0; l < NH; ++l) {
                    if (l == 0) a = f1 ? arm_hidden<D, true>(Wh[0], Bh[0], a) : arm_hidden<D, false>(Wh[0], Bh[0], a);
                    else a = w24 ? arm_hidden<D, true>(Wh[l], Bh[l], a) : arm_hidden<D, false>(Wh[l], Bh[l], a);
                }
                STAMP(t1);
                const bool fo = NH > 0 ? w24 : f1;
                const int32_t p0 = fo ? imul<true>(Wo0, a) : imul<false>(Wo0, a);
                const int32_t p1 = fo ? imul<true>(Wo1, a) : imul<false>(Wo1, a);
                int32_t s0 = row_sum16(p0), s1 = row_sum16(p1);
                int32_t m0 = __builtin_amdgcn_readlane(s0, 15), m1 = __builtin_amdgcn_readlane(s1, 15);
                if (D > 16) {
                    m0 += __builtin_amdgcn_readlane(s0, 31);
                    m1 += __builtin_amdgcn_readlane(s1, 31);
                }
                m0 += bo0;
                m1 += bo1;
                STAMP(t2);
                const int32_t mu = m0 < 0 ? -((-m0 + 128) >> 8) : (m0 + 128) >> 8;
                const int32_t ls = m1 < 0 ? -((-m1 + 128) >> 8) : (m1 + 128) >> 8;
                // get_val_mu_indicies (cc-contexts.h:20-48)
                const int32_t mr = mu >= 0 ? ((mu + 128) >> 8) << 8 : -(((-mu + 128) >> 8) << 8);
                int32_t mi = (mu - mr) * 16;
                mi = (mi >= 0 ? (mi + 128) >> 8 : -((-mi + 128) >> 8)) + 8;
                const int32_t lsp = ls + 256;
                int32_t si = lsp < 0 ? 0 : (lsp * 5 + 128) >> 8;
                si = si > 49 ? 49 : si;
                const uint32_t ci = (uint32_t)(mi * 50 + si) * 2u;
                const uint32_t st = c_ctx.v[ci], stp = c_ctx.v[ci + 1];
#if defined(CCMI_ARM_STAMPS)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
                STAMP(t3);
                // decode_single (cc-bac.h:192-231): static contexts
                int32_t val = 0;
                if (cab.bin_static(st & 0xFF)) {
                    if (!cab.bin_static((st >> 8) & 0xFF)) val = 1;
                    else if (!cab.bin_static((st >> 16) & 0xFF)) val = 2;
                    else if (!cab.bin_static(st >> 24)) val = 3;
                    else val = cab.expgolomb(0) + 4;
                    if (cab.bin_static(stp)) val = -val;
                }
                STAMP(t4);
                ACC(0, t0, t1);
                ACC(1, t1, t2);
                ACC(2, t2, t3);
                ACC(3, t3, t4);
#if defined(CCMI_ARM_STAMPS)
                st_acc[4] += 1;
#endif
                const int32_t q = (mr >> 8) + val;
                big |= (q >= 32768 || q <= -32768);
                v = (int32_t)((uint32_t)q << kArmPrec);
            }
            r4 = r3;
            r3 = r2;
            r2 = r1;
            r1 = v;
            if (lane == 0) row[x] = v;
        }
        __syncthreads();
        int32_t *dst = S.out + (int64_t)y * w;
        for (int x = lane; x < w; x += 64) dst[x] = row[x];
        __syncthreads();
    }
    if (lane == 0) put_status(S, (big ? CCMI_ARM_FLAG_BIG : 0u) | (w24 ? 0u : CCMI_ARM_FLAG_W32));
#if defined(CCMI_ARM_STAMPS)
    st_acc[6] = __builtin_amdgcn_s_memtime() - t_loop; // whole latent loop
    if (lane == 0 && S.dbg)
        for (int k = 0; k < 8; ++k) S.dbg[k] = st_acc[k];
#endif
}

// ------------------------------------------------------------------ speculative ARM decode (d <= 16)
// Same stream semantics as dec_arm_kernel, restructured for latency.  The wave's four
// DPP rows (16 lanes each) evaluate the ARM for four consecutive latents x .. x+3 at
// once: row g assumes the latents x .. x+g-1 (not decoded yet) are 0, the most likely
// value.  The CABAC then decodes x, x+1, ... in order and stops at the first latent
// whose decoded value is not 0: every later row was computed from a wrong guess and is
// discarded; all rows up to and including that latent were exact.  Neuron o of row g
// sits in lane 16g + o; the matrix-vector products broadcast a_i inside each row with
// DPP row_newbcast (no SGPR round trip), fused by the compiler into v_mul_i32_i24_dpp.
// The 17 x 50 context table is staged in LDS (one ds_read_b64 per latent instead of a
// scalar load that misses the constant cache).
template <bool F24, int... I>
__device__ __forceinline__ int32_t row_dot(const int32_t (&W)[16], int32_t a, std::integer_sequence<int, I...>)
{
    int32_t acc = 0;
    ((acc += imul<F24>(W[I], __builtin_amdgcn_update_dpp(0, a, 0x150 + I, 0xF, 0xF, false))), ...);
    return acc;
}

template <int D, bool F24>
__device__ __forceinline__ int32_t arm_hidden_rows(const int32_t (&W)[16], int32_t bias, int32_t a)
{
    const int32_t acc = bias + a * 256 + row_dot<F24>(W, a, std::make_integer_sequence<int, D>{});
    return acc < 0 ? 0 : (acc + 128) >> 8;
}

constexpr int kSpec = 4; // latents evaluated per ARM pass (one per DPP row)

template <int D, int NH>
__global__ __launch_bounds__(64) void dec_arm_spec_kernel(const ArmStreamDesc *__restrict__ streams, int pitch)
{
    static_assert(D <= 16, "one neuron per lane of a DPP row");
#if defined(CCMI_ARM_STAMPS)
    // [0] ARM pass (ctx + MLP + output sums)  [1] index + table  [2] CABAC  [3] ARM passes
    // [4] coded latents  [5] setup  [6] latent loop
    uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ int32_t smem[];
    uint32_t *ctab = reinterpret_cast<uint32_t *>(smem);               // 17 x 50 x 2
    int32_t *ring = smem + 17 * 50 * 2;                                 // kRingS x pitch
    uint8_t *bmap = reinterpret_cast<uint8_t *>(ring + kRingS * pitch); // block sig/flat map

    const ArmStreamDesc S = streams[blockIdx.x];
    const int lane = threadIdx.x;
    const int grp = lane >> 4, o = lane & 15;
    const bool live = o < D;
    const int h = S.h, w = S.w;
    const bool w24 = (S.flags & 1) != 0;

    // context table with every static-context index already turned into its model state
    // (Model::init + state(), done once here instead of per bin)
    for (int i = lane; i < 17 * 50 * 2; i += 64) {
        const uint32_t v = c_ctx.v[i];
        uint32_t o = 0;
        for (int k = 0; k < 4; ++k) {
            Model m;
            m.init((int)((v >> (8 * k)) & 0xFF));
            o |= m.state() << (8 * k);
        }
        ctab[i] = (i & 1) ? (o & 0xFF) : o;
    }
    for (int i = lane; i < kRingS * pitch; i += 64) ring[i] = 0;

    int32_t Wh[NH > 0 ? NH : 1][16], Bh[NH > 0 ? NH : 1];
#pragma unroll
    for (int l = 0; l < NH; ++l) {
        const int32_t *base = S.weights + l * (D * D + D);
#pragma unroll
        for (int i = 0; i < 16; ++i) Wh[l][i] = (live && i < D) ? base[o * D + i] : 0;
        Bh[l] = live ? base[D * D + o] : 0;
    }
    const int32_t *ob = S.weights + NH * (D * D + D);
    const int32_t Wo0 = live ? ob[o] : 0, Wo1 = live ? ob[D + o] : 0;
    const int32_t bo0 = __builtin_amdgcn_readfirstlane(ob[2 * D]);
    const int32_t bo1 = __builtin_amdgcn_readfirstlane(ob[2 * D + 1]);

    // ---- CABAC start + block significance / flat maps (BACContext::set_layer, cc-bac.h:24-130)
    Cabac<DevBytes> cab;
    cab.src.init(S.bytes, S.nbytes);
    cab.start();
    const int updated = S.sig_blk < 0;
    const int blk = S.sig_blk < 0 ? -S.sig_blk : S.sig_blk;
    int shift = 0;
    while ((1 << shift) < blk) ++shift;
    const int mask = (1 << shift) - 1;
    int nby = 1, nbx = 1;
    if (blk > 0) {
        nby = (h + blk - 1) >> shift;
        nbx = (w + blk - 1) >> shift;
    }
    const int nblk = nby * nbx;
    for (int i = lane; i < nblk; i += 64) bmap[i] = 1; // bit0 sig, bit1 flat
    __syncthreads();
    if (nblk > 1) {
        if (cab.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const uint32_t b = updated ? cab.bin_adaptive(m) : cab.ep();
                if (lane == 0) bmap[i] = (uint8_t)b;
            }
        }
        __syncthreads();
        if (cab.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const int sig = __builtin_amdgcn_readfirstlane((int)bmap[i]);
                if (sig) {
                    const uint32_t f = updated ? cab.bin_adaptive(m) : cab.ep();
                    if (lane == 0) bmap[i] = (uint8_t)(sig | (f << 1));
                }
            }
        }
    }
    __syncthreads();

    int cdy, cdx;
    ctx_dydx<D>(o, cdy, cdx);
    const bool same_row = cdy == 0;
    int big = 0;
#if defined(CCMI_ARM_STAMPS)
    st_acc[5] = __builtin_amdgcn_s_memtime() - t_begin;
    const uint64_t t_loop = __builtin_amdgcn_s_memtime();
#endif

    for (int y = 0; y < h; ++y) {
        int32_t *row = ring + (y % kRingS) * pitch + kPad;
        const int32_t *up = ring + ((y + kRingS - 1) % kRingS) * pitch + kPad;
        const int32_t *crow = ring + ((y + cdy + kRingS) % kRingS) * pitch + kPad + cdx + grp;
        int32_t r1 = 0, r2 = 0, r3 = 0, r4 = 0; // decoded values at x-1 .. x-4 (this row)
        const int brow = blk > 0 ? (y >> shift) * nbx : 0;
        auto push = [&](int32_t v, int x) {
            r4 = r3;
            r3 = r2;
            r2 = r1;
            r1 = v;
            if (lane == 0) row[x] = v;
        };
        // n (>= 1) uncoded columns [x, x+n) written by the lanes in parallel; the last four
        // values are re-read into r1..r4 (they are uniform)
        auto fill = [&](int x, int n, int kind /*0 zero, 1 = r1, 2 = up*/) {
            const int32_t c1 = r1;
            for (int i = lane; i < n; i += 64) row[x + i] = kind == 0 ? 0 : kind == 1 ? c1 : up[x + i];
            if (kind == 2) {
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
                auto at = [&](int j) { return __builtin_amdgcn_readfirstlane(row[j]); };
                r4 = n >= 4 ? at(x + n - 4) : n == 3 ? r1 : n == 2 ? r2 : r3;
                r3 = n >= 3 ? at(x + n - 3) : n == 2 ? r1 : r2;
                r2 = n >= 2 ? at(x + n - 2) : r1;
                r1 = at(x + n - 1);
            } else {
                const int32_t v = kind == 0 ? 0 : c1;
                r4 = n >= 4 ? v : n == 3 ? r1 : n == 2 ? r2 : r3;
                r3 = n >= 3 ? v : n == 2 ? r1 : r2;
                r2 = n >= 2 ? v : r1;
                r1 = v;
            }
        };
        int bm = 1, bend = 0; // flags of the current block and its end column
        // above-row context of the next pass, prefetched from LDS before the CABAC of the
        // current one: the next pass starts at x + nd (nd = 1..4 latents decoded)
        int pf_x = -1;
        int32_t pf_a = 0;
        for (int x = 0; x < w;) {
            int L;
            if (blk > 0) {
                if (x >= bend) {
                    bm = __builtin_amdgcn_readfirstlane((int)bmap[brow + (x >> shift)]);
                    bend = min((x | mask) + 1, w);
                }
                if (!(bm & 1)) {
                    fill(x, bend - x, 0);
                    x = bend;
                    continue;
                }
                if (bm & 2) {
                    if (y & mask) {
                        fill(x, bend - x, 2);
                        x = bend;
                        continue;
                    }
                    if (x & mask) {
                        fill(x, bend - x, 1);
                        x = bend;
                        continue;
                    }
                    L = 1; // the coded corner of a flat block
                } else {
                    L = min(kSpec, bend - x);
                }
            } else {
                L = min(kSpec, w - x);
            }
            STAMP(t0);

            // context of lane (g, o): latent x+g, neighbour (cdy, cdx); same-row neighbours
            // at or right of x are the speculative zeros
            const int k = -(grp + cdx); // same row: distance back from x (1..4), <= 0 -> guess
            const int32_t rs = k == 1 ? r1 : k == 2 ? r2 : k == 3 ? r3 : k == 4 ? r4 : 0;
            int32_t a = same_row ? rs : (x == pf_x ? pf_a : crow[x]);
            const bool f1 = w24 && !big;
#pragma unroll
            for (int l = 0; l < NH; ++l) {
                if (l == 0) a = f1 ? arm_hidden_rows<D, true>(Wh[0], Bh[0], a) : arm_hidden_rows<D, false>(Wh[0], Bh[0], a);
                else a = w24 ? arm_hidden_rows<D, true>(Wh[l], Bh[l], a) : arm_hidden_rows<D, false>(Wh[l], Bh[l], a);
            }
            const bool fo = NH > 0 ? w24 : f1;
            const int32_t m_0 = row_sum16(fo ? imul<true>(Wo0, a) : imul<false>(Wo0, a)) + bo0;
            const int32_t m_1 = row_sum16(fo ? imul<true>(Wo1, a) : imul<false>(Wo1, a)) + bo1;
#if defined(CCMI_ARM_STAMPS)
            __builtin_amdgcn_s_waitcnt(0);
#endif
            STAMP(t1);
            // mu / scale -> context-table entry, in every lane at once (lane 16g+15 holds
            // row g's sums; the other lanes compute harmless in-range garbage)
            const int32_t mu = m_0 < 0 ? -((-m_0 + 128) >> 8) : (m_0 + 128) >> 8;
            const int32_t ls = m_1 < 0 ? -((-m_1 + 128) >> 8) : (m_1 + 128) >> 8;
            // get_val_mu_indicies (cc-contexts.h:20-48)
            const int32_t mr = mu >= 0 ? ((mu + 128) >> 8) << 8 : -(((-mu + 128) >> 8) << 8);
            int32_t mi = (mu - mr) * 16;
            mi = (mi >= 0 ? (mi + 128) >> 8 : -((-mi + 128) >> 8)) + 8;
            const int32_t lsp = ls + 256;
            int32_t si = lsp < 0 ? 0 : (lsp * 5 + 128) >> 8;
            si = si > 49 ? 49 : si;
            const uint2 e = *reinterpret_cast<const uint2 *>(ctab + (uint32_t)(mi * 50 + si) * 2u);
            const int32_t mq = mr >> 8;
            const int32_t pf1 = crow[x + 1], pf2 = crow[x + 2], pf3 = crow[x + 3], pf4 = crow[x + 4];
            STAMP(t2);
            // decode_single (cc-bac.h:192-231), in order, until the first non-zero latent
            int nd = 0;
#pragma unroll 1
            for (int j = 0; j < L; ++j) {
                const int src_lane = 16 * j + 15;
                const uint32_t st = __builtin_amdgcn_readlane(e.x, src_lane);
                const uint32_t stp = __builtin_amdgcn_readlane(e.y, src_lane);
                int32_t val = 0;
                if (cab.bin_state(st & 0xFF)) {
                    if (!cab.bin_state((st >> 8) & 0xFF)) val = 1;
                    else if (!cab.bin_state((st >> 16) & 0xFF)) val = 2;
                    else if (!cab.bin_state(st >> 24)) val = 3;
                    else val = cab.expgolomb(0) + 4;
                    if (cab.bin_state(stp)) val = -val;
                }
                const int32_t q = __builtin_amdgcn_readlane(mq, src_lane) + val;
                big |= (q >= 32768 || q <= -32768);
                push((int32_t)((uint32_t)q << kArmPrec), x + j);
                ++nd;
                if (q != 0) break;
            }
            STAMP(t3);
            ACC(0, t0, t1);
            ACC(1, t1, t2);
            ACC(2, t2, t3);
#if defined(CCMI_ARM_STAMPS)
            st_acc[3] += 1;
            st_acc[4] += nd;
#endif
            x += nd;
            pf_x = x;
            pf_a = nd == 1 ? pf1 : nd == 2 ? pf2 : nd == 3 ? pf3 : pf4;
        }
        __syncthreads();
        int32_t *dst = S.out + (int64_t)y * w;
        for (int x = lane; x < w; x += 64) dst[x] = row[x];
        __syncthreads();
    }
    if (lane == 0) put_status(S, (big ? CCMI_ARM_FLAG_BIG : 0u) | (w24 ? 0u : CCMI_ARM_FLAG_W32));
#if defined(CCMI_ARM_STAMPS)
    st_acc[6] = __builtin_amdgcn_s_memtime() - t_loop;
    if (lane == 0 && S.dbg)
        for (int k = 0; k < 8; ++k) S.dbg[k] = st_acc[k];
#endif
}

// ------------------------------------------------------------------ chain kernel support
constexpr int kDS = 3; // same-row contexts (0, -3), (0, -2), (0, -1): the last three context indices

// Byte source of the chain kernel: the stream's words come through wave-uniform VECTOR
// loads issued one word ahead (the scalar-load reader's fetch is counted in lgkmcnt with
// the LDS reads, so every LDS wait of a pass also waited for it).  Word indices clamp to the
// zero padding after the stream (>= 64 bytes, dec_host.cpp), which reads as zeros.
struct DevBytesV {
    typedef const __attribute__((address_space(1))) uint32_t *gptr; // global, not flat: vmcnt only
    gptr p;
    uint32_t lim, pos, wi, cur;
    int32_t vnext; // word wi + 1, in a VGPR (possibly still in flight)
    __device__ __forceinline__ int32_t fetch(uint32_t i) const
    {
        int vi = (int)(i < lim ? i : lim);
        asm volatile("" : "+v"(vi)); // a vector load
        return (int32_t)p[vi];
    }
    __device__ __forceinline__ void init(const uint32_t *base, uint32_t nbytes)
    {
        p = (gptr)(size_t)base;
        lim = ((nbytes + 3u) >> 2) + 8u;
        pos = 0;
        wi = 0;
        cur = (uint32_t)__builtin_amdgcn_readfirstlane(fetch(0));
        vnext = fetch(1);
    }
    __device__ __forceinline__ uint32_t next()
    {
        const uint32_t b = (cur >> ((pos & 3u) * 8u)) & 0xFFu;
        ++pos;
        if ((pos & 3u) == 0) {
            cur = (uint32_t)__builtin_amdgcn_readfirstlane(vnext);
            ++wi;
            vnext = fetch(wi + 1);
        }
        return b;
    }
};

// ------------------------------------------------------------------ chain kernel (d <= 16, >= 1 hidden layer)
// The serial decode chain of one latent-layer stream, built around what one wavefront can
// issue (one instruction per ~4 cycles, SALU and VALU alike): every instruction on the chain
// is one the decode needs.  Speculation as in round 3 (DPP row g evaluates latent x + g,
// its undecoded same-row neighbours guessed equal to the latent above) with:
//  * layer 0 in GUESS-ERROR form: the chunk precompute folds the above-row contexts AND the
//    guessed same-row contexts (the latents above, up[x - 3 .. x - 1]) into one sum per latent
//    and neuron, preG; a pass adds C1 e1 + C2 e2 + C3 e3, where e_j = (decoded - guessed value)
//    of latent x - j (wave-uniform, SGPR) and C_j the per-lane constant weight of that context
//    for the lane's row (0 when the row guessed it).  Exact: int32 sums wrap identically in any
//    order (-fwrapv) and the reference rounds once per layer (arm_cpu.cpp:65-80);
//  * coded RUNS: the block map is turned into runs of coded latents once per run (lanes read
//    the block flags, one ballot), so a pass's only control flow is its CABAC;
//  * the next pass's inputs read ahead at constant LDS offsets: the preG ring (two 64-latent
//    chunks) mirrors its first 8 entries after its end, so latents x + 1 .. x + 7 never wrap;
//  * decoded values collected in a VGPR (v_writelane) and stored 60 at a time;
//  * the CABAC state left-aligned (range << 23, value << 16): the renormalisation shift of
//    both outcomes is one s_flbit of the new range; the five static bin codes of a context
//    (4 unary bins + sign, 6 bits each) in one LDS word;
//  * the multiply forms (24-bit / 32-bit) as instantiations of the pass loop, switched at a
//    pass boundary when a decoded latent leaves the 24-bit range.
constexpr int kPreRing = 256; // four 64-latent chunks of preG (ring slot = chunk sequence number & 3)
constexpr int kPreMir = 8;    // ring entries [0, 8) mirrored at [256, 264)
constexpr uint32_t kQ24 = 16383; // |q| <= kQ24 keeps contexts and guess errors inside 24 signed bits

// 6-bit code of a static context's model state st: bit 5 the MPS, bits 0..4 the LPS class
// ((st or its complement) >> 2; TDecBinCABAC::decodeBin's LPS-range index)
__host__ __device__ constexpr uint32_t code6(uint32_t st)
{
    return ((st >> 7) << 5) | ((((st >> 7) ? st ^ 0xFFu : st) & 0xFFu) >> 2);
}

struct Cab6 {
    DevBytesV src;
    uint32_t R, V; // TDecBinCABAC's m_uiRange << 23 and m_uiValue << 16
    int32_t bn;    // bits_needed
    __device__ __forceinline__ void from(const Cabac<DevBytesV> &c)
    {
        src = c.src;
        R = c.range << 23;
        V = c.value << 16;
        bn = c.bits_needed;
    }
    __device__ __forceinline__ void to(Cabac<DevBytesV> &c) const
    {
        c.src = src;
        c.range = R >> 23;
        c.value = V >> 16;
        c.bits_needed = bn;
    }
};

// One bin of a static context, k-th 6-bit code of the word st (TDecBinCABAC::decodeBin):
// LPS iff value >= (range - lps) << 7; after either outcome the new range is renormalised to
// [256, 511) by one left shift of clz(range << 23) (1 or 0 after an MPS, clz(lps) - 23 after an
// LPS, = the reference's renorm table for lps in [4, 236]).
template <int K>
__device__ __forceinline__ uint32_t bin6(Cab6 &c, uint32_t st)
{
    const uint32_t q5 = (st >> (6 * K)) & 31u, mps = (st >> (6 * K + 5)) & 1u;
    uint32_t R = c.R, V = c.V, t, lps, rm, nb, lp;
    asm("s_lshr_b32 %[t], %[R], 28\n\t"
        "s_mul_i32 %[t], %[t], %[q5]\n\t"
        "s_lshr_b32 %[t], %[t], 1\n\t"
        "s_add_u32 %[t], %[t], 4\n\t"
        "s_lshl_b32 %[lps], %[t], 23\n\t"
        "s_sub_u32 %[rm], %[R], %[lps]\n\t"
        "s_cmp_ge_u32 %[V], %[rm]\n\t"
        "s_cselect_b32 %[R], %[lps], %[rm]\n\t"
        "s_cselect_b32 %[t], %[rm], 0\n\t"
        "s_cselect_b32 %[lp], 1, 0\n\t"
        "s_sub_u32 %[V], %[V], %[t]\n\t"
        "s_flbit_i32_b32 %[nb], %[R]\n\t"
        "s_lshl_b32 %[R], %[R], %[nb]\n\t"
        "s_lshl_b32 %[V], %[V], %[nb]"
        : [R] "+s"(R), [V] "+s"(V), [t] "=&s"(t), [lps] "=&s"(lps), [rm] "=&s"(rm), [nb] "=&s"(nb), [lp] "=&s"(lp)
        : [q5] "s"(q5)
        : "scc");
    c.R = R;
    c.V = V;
    c.bn += (int32_t)nb;
    if (__builtin_expect(c.bn >= 0, 0)) { // the byte refill off the fall-through path
        c.V += c.src.next() << (c.bn + 16);
        c.bn -= 8;
    }
    return lp ^ mps;
}

// decode_single (cc-bac.h:192-231) with the static codes of one context
__device__ __forceinline__ int32_t decode_val(Cab6 &c, uint32_t st)
{
    int32_t val = 0;
    if (bin6<0>(c, st)) {
        if (!bin6<1>(c, st)) val = 1;
        else if (!bin6<2>(c, st)) val = 2;
        else if (!bin6<3>(c, st)) val = 3;
        else {
            Cabac<DevBytesV> t;
            c.to(t);
            val = t.expgolomb(0) + 4;
            c.from(t);
        }
        if (bin6<4>(c, st)) val = -val;
    }
    return val;
}

// ReLU + rounding of a hidden layer, arm_cpu.cpp:76-81 as written (a sum within 127 of INT_MAX
// wraps negative there too)
// v_writelane_b32 (no clang builtin in this toolchain: the LLVM intrinsic by its asm label)
extern "C" __device__ int32_t ccmi_writelane(int32_t v, int32_t lane, int32_t old) __asm("llvm.amdgcn.writelane.i32");

__device__ __forceinline__ int32_t relu_rnd8(int32_t acc) { return acc < 0 ? 0 : (acc + 128) >> 8; }

template <int D, int NH>
__global__ __launch_bounds__(128) void dec_arm_chain_kernel(const ArmStreamDesc *__restrict__ streams, int pitch)
{
    static_assert(D <= 16 && D > kDS && NH >= 1, "one neuron per lane of a DPP row, >= 1 hidden layer");
    constexpr int DA = D - kDS; // above-row contexts
#if defined(CCMI_ARM_STAMPS)
    // chain wave: [0] ARM + index (to the table read)  [1] table wait  [2] CABAC  [3] passes
    // [4] coded latents  [5] setup  [6] latent loop  [7] waits for the helper's preG
    // [8] run starts (fills, block scan)  [9] row copy-out  [10] runs  [11] after the CABAC
    // helper wave (lanes 12..15 of the dump): [12] busy (chunk precompute)  [13] chunks computed
    // [14] chunks skipped (no coded latent)  [15] waiting
    uint32_t st_v = 0;
#define LACC(k, d) st_v += (lane == (k)) ? (uint32_t)(d) : 0u
#define CSTAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
    const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#else
#define LACC(k, d)
#define CSTAMP(var)
#endif
    extern __shared__ int32_t smem[];
    int32_t *ctl = smem;                                                // [0] ready seq [1] chain seq [2] done
    uint32_t *ctab = reinterpret_cast<uint32_t *>(smem + 4);            // 17 x 50 packed bin codes
    int32_t *w0s = smem + 4 + 17 * 50 + 2;                              // [16][16] layer-0 weights, [16] biases (16 B aligned)
    int32_t *pre = w0s + 16 * 16 + 16;                                  // [kPreRing + kPreMir][16] preG
    int32_t *ring = pre + (kPreRing + kPreMir) * 16;                    // kRingS x pitch
    uint8_t *bmap = reinterpret_cast<uint8_t *>(ring + kRingS * pitch); // block sig/flat map

    const ArmStreamDesc S = streams[blockIdx.x];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const int grp = lane >> 4, o = lane & 15;
    const bool live = o < D;
    const int h = S.h, w = S.w;
    const bool w24 = (S.flags & 1) != 0;
    const int nch = (w + 63) >> 6; // 64-latent chunks per row

    for (int i = tid; i < 17 * 50; i += 128) {
        const uint32_t v = c_ctx.v[2 * i], vs = c_ctx.v[2 * i + 1];
        uint32_t e = 0;
        for (int k = 0; k < 4; ++k) {
            Model m;
            m.init((int)((v >> (8 * k)) & 0xFF));
            e |= code6(m.state()) << (6 * k);
        }
        Model m;
        m.init((int)(vs & 0xFF));
        ctab[i] = e | (code6(m.state()) << 24);
    }
    for (int i = tid; i < kRingS * pitch; i += 128) ring[i] = 0;
    for (int i = tid; i < 16 * 16 + 16; i += 128) {
        const int r = i >> 4, cc = i & 15;
        w0s[i] = i < 256 ? (r < D && cc < D ? S.weights[r * D + cc] : 0) : (cc < D ? S.weights[D * D + cc] : 0);
    }
    if (tid < 4) ctl[tid] = 0;

    // ---- CABAC start + block significance / flat maps (BACContext::set_layer, cc-bac.h:24-130);
    // both waves run it (the map is written by thread 0), the chain wave keeps the CABAC state
    Cabac<DevBytesV> cab0;
    cab0.src.init(S.bytes, S.nbytes);
    cab0.start();
    const int updated = S.sig_blk < 0;
    const int blk = S.sig_blk < 0 ? -S.sig_blk : S.sig_blk;
    int shift = 0;
    while ((1 << shift) < blk) ++shift;
    const int mask = (1 << shift) - 1;
    int nby = 1, nbx = 1;
    if (blk > 0) {
        nby = (h + blk - 1) >> shift;
        nbx = (w + blk - 1) >> shift;
    }
    const int nblk = nby * nbx;
    for (int i = tid; i < nblk; i += 128) bmap[i] = 1; // bit0 sig, bit1 flat
    __syncthreads();
    if (nblk > 1) {
        if (cab0.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const uint32_t b = updated ? cab0.bin_adaptive(m) : cab0.ep();
                if (tid == 0) bmap[i] = (uint8_t)b;
            }
        }
        __syncthreads();
        if (cab0.ep()) {
            Model m;
            m.init(65);
            for (int i = 0; i < nblk; ++i) {
                const int sig = __builtin_amdgcn_readfirstlane((int)bmap[i]);
                if (sig) {
                    const uint32_t f = updated ? cab0.bin_adaptive(m) : cab0.ep();
                    if (tid == 0) bmap[i] = (uint8_t)(sig | (f << 1));
                }
            }
        }
    }
    __syncthreads();
    auto lds_order = []() __attribute__((always_inline)) { // this wave's LDS stores before its later loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // the two waves' hand-off words: a workgroup-scope release store publishes everything the
    // wave wrote before it (every lane's stores: lds_order() first), an acquire load orders the
    // reader's later LDS loads (the preG slots, the ring rows) behind the word it saw
    auto ctl_get = [ctl](int k) __attribute__((always_inline)) {
        return __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    auto ctl_put = [ctl, tid](int k, int32_t v) __attribute__((always_inline)) {
        if ((tid & 63) == 0) __hip_atomic_store(ctl + k, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    const int spin_cap = S.spin_cap;

    if (wid == 1) {
        // ================= helper wave: preG of every chunk with a coded latent, in (row, chunk)
        // order, into ring slot seq & 3 (4 slots + the mirror of slot 0's first 8 entries), as
        // soon as (a) the chain wave has left the chunk that held the slot (chain seq >= seq - 3)
        // and (b) the row above is final under the chunk's contexts (done >= its last column)
        const int dmax = blk > 0 ? 0 : 1; // no block map: every latent coded
        int seq = 0;
        uint32_t hbits = 0;
        for (int y = 0; y < h; ++y) {
            const int brow = blk > 0 ? (y >> shift) * nbx : 0;
            for (int c = 0; c < nch; ++c, ++seq) {
                CSTAMP(tw0);
                // is any latent of [64 c, 64 c + 64) coded (the ARM evaluated there)?
                bool coded = dmax != 0;
                if (!coded) {
                    const int b0 = (c * 64) >> shift, b1 = (min(c * 64 + 64, w) - 1) >> shift;
                    const int bb = b0 + lane;
                    const int f = bb <= b1 ? (int)bmap[brow + bb] : 0;
                    // sig and not flat: every latent; sig and flat: the corner, in the block's first row
                    coded = __ballot(bb <= b1 && (f == 1 || (f == 3 && !(y & mask)))) != 0;
                }
                const int need = y == 0 ? 0 : (y - 1) * w + min(c * 64 + 66, w);
                // bounded, so that a lost hand-off ends in a wave that retires and a status word
                // the host turns into an error (CCMI_ARM_FLAG_TIMEOUT), never in a hang
                bool ok = false;
                for (int spin = 0; spin < spin_cap; ++spin) {
                    if (ctl_get(1) >= seq - 3 && ctl_get(2) >= need) {
                        ok = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (!ok) hbits |= CCMI_ARM_FLAG_TIMEOUT;
                CSTAMP(tw1);
                LACC(15, tw1 - tw0);
                if (coded) {
                    const int slot = seq & 3;
                    const int xx = min(c * 64 + lane, w - 1); // lanes past the row end: a copy nobody reads
                    const int32_t *up = ring + ((y + 3) & 3) * pitch + kPad;
                    int32_t ctx[D];
#pragma unroll
                    for (int i = 0; i < DA; ++i) {
                        int dy, dx;
                        ctx_dydx<D>(i, dy, dx);
                        ctx[i] = ring[((y + dy) & 3) * pitch + kPad + xx + dx];
                    }
#pragma unroll
                    for (int j = 0; j < kDS; ++j) ctx[DA + j] = up[xx - kDS + j]; // the guesses
                    // 24-bit products when the weights and every context fit (|v| < 2^22)
                    bool small = w24;
#pragma unroll
                    for (int i = 0; i < D; ++i) small = small && (uint32_t)(ctx[i] + (1 << 22)) < (1u << 23);
                    const bool f24 = __ballot(!small) == 0;
                    if (!f24) hbits |= CCMI_ARM_FLAG_PRE32;
                    int32_t *dst = pre + (slot * 64 + lane) * 16;
                    int32_t *mir = pre + (kPreRing + lane) * 16;
                    auto sums = [&](auto F24) __attribute__((always_inline)) {
                        constexpr bool fz = decltype(F24)::value;
#pragma unroll
                        for (int n = 0; n < 16; n += 4) {
                            int32_t acc[4];
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const int nn = n + q;
                                if (nn >= D) {
                                    acc[q] = 0;
                                    continue;
                                }
                                int32_t a = w0s[256 + nn] + ctx[nn] * 256; // bias + own residual
                                const int4 *wr = reinterpret_cast<const int4 *>(w0s + 16 * nn);
#pragma unroll
                                for (int i4 = 0; i4 < (D + 3) / 4; ++i4) {
                                    const int4 wv = wr[i4];
                                    const int32_t wk[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                                    for (int k = 0; k < 4; ++k)
                                        if (4 * i4 + k < D) a += imul<fz>(wk[k], ctx[4 * i4 + k]);
                                }
                                acc[q] = a;
                            }
                            const int4 v4{acc[0], acc[1], acc[2], acc[3]};
                            *reinterpret_cast<int4 *>(dst + n) = v4;
                            if (slot == 0 && lane < kPreMir) *reinterpret_cast<int4 *>(mir + n) = v4;
                        }
                    };
                    if (f24) sums(std::true_type{});
                    else sums(std::false_type{});
                    LACC(13, 1);
                } else {
                    LACC(14, 1);
                }
                lds_order();
                ctl_put(0, seq + 1);
                CSTAMP(tw2);
                LACC(12, tw2 - tw1);
            }
        }
        if (lane == 0) put_status(S, hbits);
#if defined(CCMI_ARM_STAMPS)
        if (lane >= 12 && lane < 16 && S.dbg) S.dbg[lane] = st_v;
#endif
        return;
    }

    // ================= chain wave
    // guess-error coefficients: latent x - j is a decoded (not guessed) neighbour of row g's
    // latent x + g iff g + j <= 3, at context dx = -(g + j), index DA + 3 - (g + j); the weight
    // carries the neuron's own residual when that index is its own
    int32_t C1, C2, C3;
    {
        int32_t Ws[kDS];
#pragma unroll
        for (int j = 0; j < kDS; ++j) Ws[j] = live ? S.weights[o * D + DA + j] + (o == DA + j ? 256 : 0) : 0;
        C1 = grp == 0 ? Ws[2] : grp == 1 ? Ws[1] : grp == 2 ? Ws[0] : 0;
        C2 = grp == 0 ? Ws[1] : grp == 1 ? Ws[0] : 0;
        C3 = grp == 0 ? Ws[0] : 0;
    }
    int32_t Wh[NH][16], Bh[NH];
#pragma unroll
    for (int l = 1; l < NH; ++l) {
        const int32_t *base = S.weights + l * (D * D + D);
#pragma unroll
        for (int i = 0; i < 16; ++i) Wh[l][i] = (live && i < D) ? base[o * D + i] : 0;
        Bh[l] = live ? base[D * D + o] : 0;
    }
    const int32_t *ob = S.weights + NH * (D * D + D);
    const int32_t Wo0 = live ? ob[o] : 0, Wo1 = live ? ob[D + o] : 0;
    // the output biases ride in neuron 0's product (the row sums add them once)
    const int32_t Bo0 = o == 0 ? ob[2 * D] : 0, Bo1 = o == 0 ? ob[2 * D + 1] : 0;
    Cab6 cab;
    cab.from(cab0);

    // 24-bit guard: max over the decoded q of (q + kQ24) as unsigned, < 2 kQ24 + 1 while every
    // |q| <= kQ24 (contexts < 2^22, guess errors < 2^23)
    uint32_t qspan = 0;
    // 0: 24-bit layer 0 + 24-bit hidden / output layers; 1: 32-bit layer 0; 2: all 32-bit
    int mode = w24 ? 0 : 2;
    uint32_t cbits = 0;
#if defined(CCMI_ARM_STAMPS)
    LACC(5, __builtin_amdgcn_s_memtime() - t_begin);
    const uint64_t t_loop = __builtin_amdgcn_s_memtime();
#endif

    for (int y = 0; y < h; ++y) {
        int32_t *row = ring + (y & 3) * pitch + kPad;
        const int32_t *up = ring + ((y + 3) & 3) * pitch + kPad;
        const int brow = blk > 0 ? (y >> shift) * nbx : 0;
        const int rseq = y * nch;            // chunk sequence number of (y, 0)
        const int rring = (rseq * 64) & 255; // preG ring index of latent (y, 0); latent x at (rring + x) & 255
        int pre_lim = 0;         // a pass at x needs x + 8 <= pre_lim (INT_MAX once the row is covered)
        int32_t vrow = 0;        // lane i < x - xb: decoded value of latent xb + i, not stored yet
        int xb = 0;
        int32_t e1 = 0, e2 = 0, e3 = 0; // guess errors of latents x - 1, x - 2, x - 3
        int32_t pfa = 0;         // preG of this lane's latent x + grp, neuron o
        int32_t upv = 0;         // lane i < 8: up[x - ub + i]
        int ub = 0;
        int x = 0;

        // stores the collected values and publishes the row's progress (the helper's
        // chunks of row y + 1 read this row)
        auto flush = [&]() __attribute__((always_inline)) {
            if (lane < x - xb) row[xb + lane] = vrow;
            xb = x;
            lds_order();
            ctl_put(2, y * w + x);
        };
        // preG for latents up to x + 7: publish the chain's chunk (frees the slots before it) and
        // wait for the helper
        auto wait_pre = [&]() __attribute__((always_inline)) {
            CSTAMP(tq0);
            const int need = (min(x + 8, w) - 1) >> 6;
            ctl_put(1, rseq + (x >> 6));
            bool ok = false;
            for (int spin = 0; spin < spin_cap; ++spin) { // bounded, as the helper's wait
                if (ctl_get(0) > rseq + need) {
                    ok = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) cbits |= CCMI_ARM_FLAG_TIMEOUT;
            pre_lim = (need + 1) * 64 >= w ? 0x7FFFFFFF : (need + 1) * 64;
            CSTAMP(tq1);
            LACC(7, tq1 - tq0);
        };

        // one mode's pass loop over the current run [x, cend): returns at the run end, when the
        // next pass needs preG not waited for yet or a flush of vrow, or when the 24-bit guard
        // trips (mode 0 only); one compare per pass against the bound of all three
        auto passes = [&](int cend, auto F1, auto FW) __attribute__((always_inline)) {
            constexpr bool f1 = decltype(F1)::value, fw = decltype(FW)::value;
            const int stop = min(min(cend, pre_lim - 7), xb + 61);
            while (x < stop) {
                CSTAMP(t0);
                // ---- ARM of latents x .. x + 3 (row g = latent x + g)
                int32_t a = relu_rnd8(pfa + imul<f1>(C1, e1) + imul<f1>(C2, e2) + imul<f1>(C3, e3));
#pragma unroll
                for (int l = 1; l < NH; ++l)
                    a = relu_rnd8(Bh[l] + a * 256 + row_dot<fw>(Wh[l], a, std::make_integer_sequence<int, D>{}));
                const int32_t m0 = row_sum16(imul<fw>(Wo0, a) + Bo0), m1 = row_sum16(imul<fw>(Wo1, a) + Bo1);
                // ---- mu / scale -> context-table entry (lane 16 g + 15 holds row g's sums).  The
                // reference's symmetric rounding m < 0 ? -((-m + 128) >> 8) : (m + 128) >> 8 equals
                // (m + 128 + (m >> 31)) >> 8 (|m| < 2^31 - 128), get_val_mu_indicies cc-contexts.h:20-48
                auto rnd8 = [](int32_t m) __attribute__((always_inline)) { return (m + 128 + (m >> 31)) >> 8; };
                const int32_t mu = rnd8(m0), ls = rnd8(m1);
                const int32_t mr = (mu + 128 + (mu >> 31)) & ~255; // rnd8(mu) << 8
                const int32_t mi = rnd8((mu - mr) * 16) + 8;       // [0, 16]
                const int32_t si = min(max((ls * 5 + 1408) >> 8, 0), 49);
                const uint32_t ent = ctab[__mul24(mi, 50) + si];
                const int32_t mq = mr >> 8;
                // ---- the next pass's inputs, read ahead (it starts at x + nd, nd = 1 .. 4)
                const int32_t *pp = pre + (((rring + x) & (kPreRing - 1)) + grp) * 16 + o;
                const int32_t nx0 = pp[16], nx1 = pp[32], nx2 = pp[48], nx3 = pp[64];
                const int32_t upn = up[x + (lane & 7)];
                CSTAMP(t1);
#if defined(CCMI_ARM_STAMPS)
                __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): the table entry
#endif
                CSTAMP(t2);
                // ---- CABAC, in order, until a latent differs from its guess or the run ends
                const int lim = min(cend - x, 4);
                int nd = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t st = (uint32_t)__builtin_amdgcn_readlane((int)ent, 16 * j + 15);
                    const int32_t q = __builtin_amdgcn_readlane(mq, 16 * j + 15) + decode_val(cab, st);
                    const int32_t g = __builtin_amdgcn_readlane(upv, ub + j);
                    if (f1) qspan = max(qspan, (uint32_t)(q + (int32_t)kQ24));
                    const int32_t v = (int32_t)((uint32_t)q << kArmPrec);
                    vrow = ccmi_writelane(v, x - xb + j, vrow);
                    e3 = e2;
                    e2 = e1;
                    e1 = v - g;
                    pfa = j == 0 ? nx0 : j == 1 ? nx1 : j == 2 ? nx2 : nx3;
                    nd = j + 1;
                    if (e1 != 0 || j + 1 >= lim) break;
                }
                CSTAMP(t3);
                x += nd;
                ub = nd;
                upv = upn;
                CSTAMP(t4);
                LACC(0, t1 - t0);
                LACC(1, t2 - t1);
                LACC(2, t3 - t2);
                LACC(3, 1);
                LACC(4, nd);
                LACC(11, t4 - t3);
                if (f1 && qspan > 2 * kQ24) return;
            }
        };

        while (x < w) {
            CSTAMP(tr0);
            // ---- the run of coded latents starting at x (uncoded blocks before it filled)
            int cend = w;
            if (blk > 0) {
                const int bx = x >> shift;
                const int bm = __builtin_amdgcn_readfirstlane((int)bmap[brow + bx]);
                const int bend = min((x | mask) + 1, w);
                const bool flat = (bm & 2) != 0;
                if (!(bm & 1) || (flat && ((y & mask) || (x & mask)))) {
                    // zero block, flat block below its first row (copy of the row above), or the
                    // rest of a flat block's first row (copy of its decoded corner)
                    flush();
                    const int kind = !(bm & 1) ? 0 : (y & mask) ? 2 : 1;
                    const int32_t c1 = kind == 1 ? __builtin_amdgcn_readfirstlane(row[x - 1]) : 0;
                    for (int i = lane; i < bend - x; i += 64) row[x + i] = kind == 0 ? 0 : kind == 1 ? c1 : up[x + i];
                    x = bend;
                    xb = x;
                    flush(); // nothing to store: publishes the filled block
                    LACC(8, __builtin_amdgcn_s_memtime() - tr0);
                    continue;
                }
                if (flat) {
                    cend = x + 1; // the coded corner of a flat block
                } else {
                    // consecutive coded, non-flat blocks: the first other block ends the run
                    int b = bx + 1;
                    while (b < nbx) {
                        const int bb = b + lane;
                        const int f = bb < nbx ? (int)bmap[brow + bb] : 0;
                        const uint64_t stop = __ballot(bb < nbx && f != 1);
                        if (stop) {
                            b += __builtin_ctzll(stop);
                            break;
                        }
                        b += 64;
                    }
                    cend = min(b << shift, w);
                }
            }
            // run start: guess errors of latents x - 1 .. x - 3 from the stored row (fills)
            flush();
            {
                const int32_t d = lane < kDS ? row[x - 1 - lane] - up[x - 1 - lane] : 0;
                e1 = __builtin_amdgcn_readlane(d, 0);
                e2 = __builtin_amdgcn_readlane(d, 1);
                e3 = __builtin_amdgcn_readlane(d, 2);
            }
            if (x + 8 > pre_lim) wait_pre();
            pfa = pre[(((rring + x) & (kPreRing - 1)) + grp) * 16 + o];
            upv = up[x + (lane & 7)];
            ub = 0;
            LACC(8, __builtin_amdgcn_s_memtime() - tr0);
            LACC(10, 1);
            while (x < cend) {
                if (x + 8 > pre_lim) wait_pre();
                if (x - xb > 60) flush();
                if (mode == 0) {
                    passes(cend, std::true_type{}, std::true_type{});
                    if (qspan > 2 * kQ24) mode = 1;
                } else if (mode == 1) {
                    passes(cend, std::false_type{}, std::true_type{});
                } else {
                    passes(cend, std::false_type{}, std::false_type{});
                }
            }
        }
        CSTAMP(tw0);
        flush(); // done = (y + 1) w: the whole row is final
        // the chain is past every chunk of this row: without this, rows with no coded run (no
        // wait_pre) left the helper waiting for slots forever (the decode's last rows, uncoded)
        ctl_put(1, (y + 1) * nch);
        int32_t *dst = S.out + (int64_t)y * w;
        for (int i = lane; i < w; i += 64) dst[i] = row[i];
        LACC(9, __builtin_amdgcn_s_memtime() - tw0);
    }
    if (lane == 0) put_status(S, cbits | (mode == 1 ? CCMI_ARM_FLAG_Q32 : 0u) | (w24 ? 0u : CCMI_ARM_FLAG_W32));
#if defined(CCMI_ARM_STAMPS)
    LACC(6, __builtin_amdgcn_s_memtime() - t_loop);
    if (lane < 12 && S.dbg) S.dbg[lane] = st_v;
#endif
#undef LACC
#undef CSTAMP
}

// ------------------------------------------------------------------ upsampling (integer)
constexpr int kThreads = 256;
constexpr int kTY = 16, kTX = 64;
constexpr int kMaxKs = 16;

struct DecLevel {
    const int32_t *src;      // level-k stack (or the raw coarsest latent plane)
    int C, hs, ws, src_prec;
    const int32_t *ref;      // latent plane of level k-1 (ARM precision)
    int32_t *dst;            // level k-1 stack: C + 1 channels
    int hd, wd;
    const int32_t *kup;      // ksx2 taps
    int ksx2;
    const int32_t *kpre;     // ks taps
    int ks;
    int tiles_x;
};

__device__ __forceinline__ void ups_level_body(const DecLevel &A, int32_t *s_in, int32_t *s_tmp);

__global__ __launch_bounds__(kThreads) void dec_ups_level(DecLevel A)
{
    __shared__ int32_t s_in[(kTY + kMaxKs) * (kTX + kMaxKs)];
    __shared__ int32_t s_tmp[(kTY + kMaxKs) * kTX];
    ups_level_body(A, s_in, s_tmp);
}

// frames of a batch (identical geometry): blockIdx.y = frame
__global__ __launch_bounds__(kThreads) void dec_ups_level_batch(const DecLevel *__restrict__ As)
{
    __shared__ int32_t s_in[(kTY + kMaxKs) * (kTX + kMaxKs)];
    __shared__ int32_t s_tmp[(kTY + kMaxKs) * kTX];
    const DecLevel A = As[blockIdx.y];
    ups_level_body(A, s_in, s_tmp);
}

__device__ __forceinline__ void ups_level_body(const DecLevel &A, int32_t *s_in, int32_t *s_tmp)
{
    const int y0 = (blockIdx.x / A.tiles_x) * kTY;
    const int x0 = (blockIdx.x % A.tiles_x) * kTX;
    const int tid = threadIdx.x;
    const int64_t dplane = (int64_t)A.hd * A.wd;

    // refine (ups_refine_cpu.hpp): zero padding, two passes with truncation, residual
    {
        const int pad = A.ks / 2;
        const int rh = kTY + 2 * pad, rw = kTX + 2 * pad, pitch = kTX + kMaxKs;
        for (int i = tid; i < rh * rw; i += kThreads) {
            const int r = i / rw, c = i - r * rw;
            const int y = y0 - pad + r, x = x0 - pad + c;
            s_in[r * pitch + c] = (y >= 0 && y < A.hd && x >= 0 && x < A.wd) ? A.ref[y * A.wd + x] : 0;
        }
        __syncthreads();
        for (int i = tid; i < rh * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            const int y = y0 - pad + r;
            int32_t acc = 0;
            for (int k = 0; k < A.ks; ++k) acc += s_in[r * pitch + c + k] * A.kpre[k];
            // rows outside the plane are the zero padding of the vertical pass
            s_tmp[r * kTX + c] = (y >= 0 && y < A.hd) ? tshift(acc, kArmPrec) : 0;
        }
        __syncthreads();
        for (int i = tid; i < kTY * kTX; i += kThreads) {
            const int r = i / kTX, c = i - r * kTX;
            const int y = y0 + r, x = x0 + c;
            if (y < A.hd && x < A.wd) {
                int32_t acc = 0;
                for (int k = 0; k < A.ks; ++k) acc += s_tmp[(r + k) * kTX + c] * A.kpre[k];
                acc += (int32_t)((uint32_t)s_in[(r + pad) * pitch + c + pad] << (kUpsPrec - kArmPrec) << kUpsPrec);
                A.dst[(int64_t)y * A.wd + x] = tshift(acc, kUpsPrec);
            }
        }
        __syncthreads();
    }

    // 2x upsample of every source channel (ups_upsample_cpu.hpp): replicate padding,
    // horizontal pass >> src_prec into tmp (2*ws wide), vertical pass >> 12.
    const int ks = A.ksx2 / 2, pad = ks / 2;
    const int sy0 = y0 / 2 - pad, sx0 = x0 / 2 - pad;
    const int sh = kTY / 2 + ks, sw = kTX / 2 + ks, pitch = kTX / 2 + kMaxKs;
    for (int c = 0; c < A.C; ++c) {
        const int32_t *sp = A.src + (int64_t)c * A.hs * A.ws;
        for (int i = tid; i < sh * sw; i += kThreads) {
            const int r = i / sw, cc = i - r * sw;
            s_in[r * pitch + cc] = sp[clampi(sy0 + r, A.hs - 1) * A.ws + clampi(sx0 + cc, A.ws - 1)];
        }
        __syncthreads();
        for (int i = tid; i < sh * kTX; i += kThreads) {
            const int r = i / kTX, cc = i - r * kTX;
            const int X = x0 + cc, xs = X >> 1, ph = X & 1;
            int32_t acc = 0;
            for (int k = 0; k < ks; ++k) acc += s_in[r * pitch + (xs - pad + ph + k - sx0)] * A.kup[2 * k + ph];
            s_tmp[r * kTX + cc] = tshift(acc, A.src_prec);
        }
        __syncthreads();
        for (int i = tid; i < kTY * kTX; i += kThreads) {
            const int r = i / kTX, cc = i - r * kTX;
            const int Y = y0 + r, X = x0 + cc;
            if (Y < A.hd && X < A.wd) {
                const int ys = Y >> 1, ph = Y & 1;
                int32_t acc = 0;
                for (int k = 0; k < ks; ++k) acc += s_tmp[(ys - pad + ph + k - sy0) * kTX + cc] * A.kup[2 * k + ph];
                A.dst[(int64_t)(c + 1) * dplane + (int64_t)Y * A.wd + X] = tshift(acc, kUpsPrec);
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ synthesis (integer)
constexpr int kRW = 64, kRH = 32, kRegion = kRW * kRH;
constexpr int kMaxSp = 3;

struct DecSynFused {
    const int32_t *in;
    int cin, H, W;
    int hid;                // fused head width (always ReLU), output linear (synfused semantics)
    const int32_t *w0, *b0, *w1, *b1;
    int n_sp;
    const int32_t *wsp[kMaxSp], *bsp[kMaxSp];
    int res[kMaxSp], relu[kMaxSp];
    int32_t *out;
    int tiles_x;
    int f24; // DecSynArgs::f24
};

template <int CIN, int CMID, bool F24>
__device__ __forceinline__ void syn_fused_body(const DecSynFused &A, int32_t (*s_buf)[CMID][kRegion]);

template <int CIN, int CMID>
__global__ __launch_bounds__(kThreads) void dec_syn_fused(DecSynFused A)
{
    __shared__ __attribute__((aligned(16))) int32_t s_buf[2][CMID][kRegion];
    if (A.f24) syn_fused_body<CIN, CMID, true>(A, s_buf);
    else syn_fused_body<CIN, CMID, false>(A, s_buf);
}

template <int CIN, int CMID>
__global__ __launch_bounds__(kThreads) void dec_syn_fused_batch(const DecSynFused *__restrict__ As)
{
    __shared__ __attribute__((aligned(16))) int32_t s_buf[2][CMID][kRegion];
    // by reference: the frame's argument record is read with scalar loads where it is used (a
    // by-value copy with runtime-indexed layer arrays lived in scratch, 160 bytes per lane)
    const DecSynFused &A = As[blockIdx.y];
    if (A.f24) syn_fused_body<CIN, CMID, true>(A, s_buf);
    else syn_fused_body<CIN, CMID, false>(A, s_buf);
}

template <int CIN, int CMID, bool F24>
__device__ __forceinline__ void syn_fused_body(const DecSynFused &A, int32_t (*s_buf)[CMID][kRegion])
{
    const int halo = A.n_sp;
    const int TX = kRW - 2 * halo, TY = kRH - 2 * halo;
    const int y0 = (blockIdx.x / A.tiles_x) * TY, x0 = (blockIdx.x % A.tiles_x) * TX;
    const int oy = y0 - halo, ox = x0 - halo;
    const int64_t plane = (int64_t)A.H * A.W;
    const int c = threadIdx.x & (kRW - 1), r0 = threadIdx.x >> 6;
    const int gx = ox + c, cxg = clampi(gx, A.W - 1);

    // the head's weight records (w0[j][0..CIN), b0[j], w1[0..CMID)[j]; 12 ints) in the second
    // ping-pong buffer, which the first 3x3 layer writes only after its barrier: read back as
    // three broadcast ds_read_b128 per hidden unit, issued ahead of use (scalar weight loads
    // per unit made every unit wait for its own s_load round trip)
    static_assert(CIN + 1 + CMID <= 12, "head record");
    int32_t *s_rec = &s_buf[1][0][0];
    const int hid = A.hid;
    const bool recs = hid * 12 <= CMID * kRegion;
    if (recs) {
        for (int i = threadIdx.x; i < hid * 12; i += kThreads) {
            const int j = i / 12, f = i - j * 12;
            int32_t v = 0;
            if (f < CIN) v = A.w0[j * CIN + f];
            else if (f == CIN) v = A.b0[j];
            else if (f < CIN + 1 + CMID) v = A.w1[(f - CIN - 1) * hid + j];
            s_rec[i] = v;
        }
        __syncthreads();
    }
    auto store_head = [&](int r, const int32_t (&o)[CMID]) {
        const int gy = oy + r;
#pragma unroll
        for (int m = 0; m < CMID; ++m) {
            const int32_t v = tshift(o[m], kSynPrec);
            if (halo == 0) {
                if (gy < A.H && gx < A.W) A.out[m * plane + (int64_t)gy * A.W + gx] = v;
            } else {
                s_buf[0][m][r * kRW + c] = v;
            }
        }
    };
    if (recs) {
        // two rows (r, r + 4) per pass over the records
        typedef int i4v __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(3))) i4v *lds_i4;
        lds_i4 rb = (lds_i4)s_rec;
        for (int r = r0; r < kRH; r += 8) {
            int32_t x[2][CIN], o[2][CMID];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int64_t pix = (int64_t)clampi(oy + r + 4 * p, A.H - 1) * A.W + cxg;
#pragma unroll
                for (int k = 0; k < CIN; ++k) x[p][k] = A.in[k * plane + pix];
#pragma unroll
                for (int m = 0; m < CMID; ++m) o[p][m] = A.b1[m];
            }
#pragma unroll 2
            for (int j = 0; j < hid; ++j) {
                const i4v q0 = rb[3 * j], q1 = rb[3 * j + 1], q2 = rb[3 * j + 2];
                const int32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    int32_t acc = w[CIN];
#pragma unroll
                    for (int k = 0; k < CIN; ++k) acc += imul<F24>(x[p][k], w[k]);
                    acc = acc < 0 ? 0 : acc >> kSynPrec;
#pragma unroll
                    for (int m = 0; m < CMID; ++m) o[p][m] += imul<F24>(acc, w[CIN + 1 + m]);
                }
            }
            store_head(r, o[0]);
            store_head(r + 4, o[1]);
        }
    } else {
        for (int r = r0; r < kRH; r += 4) {
            const int64_t pix = (int64_t)clampi(oy + r, A.H - 1) * A.W + cxg;
            int32_t x[CIN];
#pragma unroll
            for (int k = 0; k < CIN; ++k) x[k] = A.in[k * plane + pix];
            int32_t o[CMID];
#pragma unroll
            for (int m = 0; m < CMID; ++m) o[m] = A.b1[m];
            for (int j = 0; j < hid; ++j) {
                int32_t acc = A.b0[j];
#pragma unroll
                for (int k = 0; k < CIN; ++k) acc += imul<F24>(x[k], A.w0[j * CIN + k]);
                acc = acc < 0 ? 0 : acc >> kSynPrec;
#pragma unroll
                for (int m = 0; m < CMID; ++m) o[m] += imul<F24>(acc, A.w1[m * hid + j]);
            }
            store_head(r, o);
        }
    }
    if (halo == 0) return;

    int cur = 0;
    for (int s = 0; s < A.n_sp; ++s) {
        __syncthreads();
        const int t = s + 1;
        const bool last = s == A.n_sp - 1;
        const int32_t *wt = A.wsp[s], *bs = A.bsp[s];
        const bool col_ok = c >= t && c < kRW - t;
        int lx[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) lx[d] = clampi(cxg + d - 1, A.W - 1) - ox;
        for (int r = r0 + t; r < kRH - t; r += 4) {
            const int gy = oy + r;
            if (!col_ok || (last && (gy >= A.H || gx >= A.W))) continue;
            const int cyg = clampi(gy, A.H - 1);
            int ly[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) ly[d] = (clampi(cyg + d - 1, A.H - 1) - oy) * kRW;
            int32_t nb[CMID][3][3];
#pragma unroll
            for (int k = 0; k < CMID; ++k)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) nb[k][dy][dx] = s_buf[cur][k][ly[dy] + lx[dx]];
#pragma unroll
            for (int m = 0; m < CMID; ++m) {
                int32_t acc = bs[m];
                if (A.res[s]) acc += (int32_t)((uint32_t)nb[m][1][1] << kSynPrec);
#pragma unroll
                for (int k = 0; k < CMID; ++k)
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) acc += imul<F24>(nb[k][dy][dx], wt[((m * CMID + k) * 3 + dy) * 3 + dx]);
                const int32_t v = acc < 0 ? (A.relu[s] ? 0 : -((-acc) >> kSynPrec)) : acc >> kSynPrec;
                if (last)
                    A.out[m * plane + (int64_t)gy * A.W + gx] = v;
                else
                    s_buf[cur ^ 1][m][r * kRW + c] = v;
            }
        }
        cur ^= 1;
    }
}

// generic integer conv layer (syn_cpu.hpp semantics, out-of-place, replicate padding).
// fused_hidden > 0: this launch is the fused 1x1 pair with that hidden width.
__global__ __launch_bounds__(kThreads) void dec_syn_layer(const int32_t *__restrict__ in, int cin, int H, int W,
                                                          const int32_t *__restrict__ wt,
                                                          const int32_t *__restrict__ bs, int nout, int ks,
                                                          int residual, int relu, int32_t *__restrict__ out)
{
    const int64_t plane = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= plane) return;
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    const int pad = ks / 2;
    for (int m = 0; m < nout; ++m) {
        int32_t acc = bs[m];
        if (residual) acc += (int32_t)((uint32_t)in[m * plane + p] << kSynPrec);
        for (int k = 0; k < cin; ++k)
            for (int dy = 0; dy < ks; ++dy) {
                const int yy = clampi(y + dy - pad, H - 1);
                for (int dx = 0; dx < ks; ++dx)
                    acc += in[k * plane + (int64_t)yy * W + clampi(x + dx - pad, W - 1)] *
                           wt[((m * cin + k) * ks + dy) * ks + dx];
            }
        out[m * plane + p] = acc < 0 ? (relu ? 0 : -((-acc) >> kSynPrec)) : acc >> kSynPrec;
    }
}

__global__ __launch_bounds__(kThreads) void dec_syn_fused_generic(const int32_t *__restrict__ in, int cin, int64_t plane,
                                                                  const int32_t *__restrict__ w0,
                                                                  const int32_t *__restrict__ b0, int hid,
                                                                  const int32_t *__restrict__ w1,
                                                                  const int32_t *__restrict__ b1, int nout,
                                                                  int32_t *__restrict__ out)
{
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= plane) return;
    for (int m = 0; m < nout; ++m) {
        int32_t o = b1[m];
        for (int j = 0; j < hid; ++j) {
            int32_t acc = b0[j];
            for (int k = 0; k < cin; ++k) acc += in[k * plane + p] * w0[j * cin + k];
            acc = acc < 0 ? 0 : acc >> kSynPrec;
            o += acc * w1[m * hid + j];
        }
        out[m * plane + p] = tshift(o, kSynPrec);
    }
}

__global__ __launch_bounds__(kThreads) void dec_blend_kernel(int32_t *acc, const int32_t *x, int64_t n, int32_t b_acc,
                                                             int32_t b_x, int first)
{
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    auto cl = [](int32_t v) { return v < 0 ? 0 : (v > (1 << kSynPrec) ? (1 << kSynPrec) : v); };
    const int32_t x0 = cl(x[i]);
    if (first) acc[i] = (cl(acc[i]) * b_acc + x0 * b_x) >> kSynPrec;
    else acc[i] = acc[i] + ((x0 * b_x) >> kSynPrec);
}

// ------------------------------------------------------------------ output bytes
struct DecOut {
    const int32_t *syn;
    int H, W, maxv, kind, bps;
    uint8_t *dst;
};

__device__ __forceinline__ void output_body(const int32_t *__restrict__ syn, int H, int W, int maxv, int kind, int bps,
                                            uint8_t *__restrict__ dst);

__global__ __launch_bounds__(kThreads) void dec_output_kernel(const int32_t *__restrict__ syn, int H, int W, int maxv,
                                                              int kind, int bps, uint8_t *__restrict__ dst)
{
    output_body(syn, H, W, maxv, kind, bps, dst);
}

__global__ __launch_bounds__(kThreads) void dec_output_batch(const DecOut *__restrict__ Os)
{
    const DecOut O = Os[blockIdx.y];
    output_body(O.syn, O.H, O.W, O.maxv, O.kind, O.bps, O.dst);
}

__device__ __forceinline__ void output_body(const int32_t *__restrict__ syn, int H, int W, int maxv, int kind, int bps,
                                            uint8_t *__restrict__ dst)
{
    const int64_t plane = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= plane) return;
    auto smp = [maxv](int32_t v) {
        int32_t s = (v * maxv + (1 << (kSynPrec - 1))) >> kSynPrec;
        return s < 0 ? 0 : (s > maxv ? maxv : s);
    };
    auto put = [&](int64_t idx, int32_t s, bool big_endian) {
        if (bps == 1) dst[idx] = (uint8_t)s;
        else if (big_endian) { dst[2 * idx] = (uint8_t)(s >> 8); dst[2 * idx + 1] = (uint8_t)s; }
        else { dst[2 * idx] = (uint8_t)s; dst[2 * idx + 1] = (uint8_t)(s >> 8); }
    };
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    if (kind == 2) { // PPM: interleaved RGB, 16-bit big endian
        for (int c = 0; c < 3; ++c) put(3 * p + c, smp(syn[c * plane + p]), true);
        return;
    }
    put(p, smp(syn[p]), false);
    if (kind == 1) {
        put(plane + p, smp(syn[plane + p]), false);
        put(2 * plane + p, smp(syn[2 * plane + p]), false);
    } else if (!(y & 1) && !(x & 1) && (y >> 1) < H / 2 && (x >> 1) < W / 2) {
        const int64_t cp = (int64_t)(H / 2) * (W / 2), ci = (int64_t)(y >> 1) * (W / 2) + (x >> 1);
        put(plane + ci, smp(syn[plane + p]), false);
        put(plane + cp + ci, smp(syn[2 * plane + p]), false);
    }
}

} // namespace

// ------------------------------------------------------------------ launchers
int launch_dec_arm(const ArmStreamDesc *d_streams, int n_streams, int max_w, int max_blocks, int d, int nh,
                         hipStream_t s)
{
    const int pitch = max_w + 2 * kPad;
    const size_t lds = sizeof(int32_t) * kRing * pitch + ((size_t)max_blocks + 16);
    // the speculative kernel keeps one ring row fewer (its contexts reach row y-3 only):
    // 5 streams (waves) per CU instead of 4 at 720p
    const size_t lds_spec = sizeof(int32_t) * kRingS * pitch + ((size_t)max_blocks + 16) + sizeof(uint32_t) * 17 * 50 * 2;
    // the one-latent-per-pass kernel below stays for wider ARMs and is what a
    // -DCCMI_DIAG_NOSPEC build runs for every stream (A/B measurements)
#if defined(CCMI_DIAG_NOSPEC)
    constexpr bool spec_off = true;
#else
    constexpr bool spec_off = false;
#endif
    // the chain kernel: packed context table, layer-0 weights, the preG ring (+ mirror), ring
    const size_t lds_lat = sizeof(int32_t) * (4 + 17 * 50 + 2 + 16 * 16 + 16 + (kPreRing + kPreMir) * 16 + kRingS * pitch) +
                           ((size_t)max_blocks + 16);
    if (!spec_off && d <= 16 && d > kDS && nh >= 1 && lds_lat <= 160 * 1024) {
#define CCMI_ARM_LAT(DD, NN)                                                                                    \
        if (d == DD && nh == NN) {                                                                              \
            hipLaunchKernelGGL((dec_arm_chain_kernel<DD, NN>), dim3(n_streams), dim3(128), lds_lat, s, d_streams, pitch); \
            CCMI_HIP_CHECK(hipGetLastError());                                                                  \
            return CCMI_OK;                                                                                     \
        }
        CCMI_ARM_LAT(8, 1) CCMI_ARM_LAT(8, 2) CCMI_ARM_LAT(8, 3) CCMI_ARM_LAT(8, 4)
        CCMI_ARM_LAT(16, 1) CCMI_ARM_LAT(16, 2) CCMI_ARM_LAT(16, 3) CCMI_ARM_LAT(16, 4)
#undef CCMI_ARM_LAT
    }
    if (!spec_off && d <= 16 && lds_spec <= 160 * 1024) {
#define CCMI_ARM_SPEC(DD, NN)                                                                                   \
        if (d == DD && nh == NN) {                                                                              \
            hipLaunchKernelGGL((dec_arm_spec_kernel<DD, NN>), dim3(n_streams), dim3(64), lds_spec, s, d_streams, pitch); \
            CCMI_HIP_CHECK(hipGetLastError());                                                                  \
            return CCMI_OK;                                                                                     \
        }
        CCMI_ARM_SPEC(8, 0) CCMI_ARM_SPEC(8, 1) CCMI_ARM_SPEC(8, 2) CCMI_ARM_SPEC(8, 3) CCMI_ARM_SPEC(8, 4)
        CCMI_ARM_SPEC(16, 0) CCMI_ARM_SPEC(16, 1) CCMI_ARM_SPEC(16, 2) CCMI_ARM_SPEC(16, 3) CCMI_ARM_SPEC(16, 4)
#undef CCMI_ARM_SPEC
    }
    if (lds > 160 * 1024) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "dec: latent width %d too large for LDS ring", max_w);
#define CCMI_ARM_CASE(DD, NN)                                                                                   \
    if (d == DD && nh == NN) {                                                                                  \
        hipLaunchKernelGGL((dec_arm_kernel<DD, NN>), dim3(n_streams), dim3(64), lds, s, d_streams, pitch);      \
        CCMI_HIP_CHECK(hipGetLastError());                                                                      \
        return CCMI_OK;                                                                                         \
    }
#define CCMI_ARM_D(DD) CCMI_ARM_CASE(DD, 0) CCMI_ARM_CASE(DD, 1) CCMI_ARM_CASE(DD, 2) CCMI_ARM_CASE(DD, 3) CCMI_ARM_CASE(DD, 4)
    CCMI_ARM_D(8)
    CCMI_ARM_D(16)
    CCMI_ARM_D(24)
    CCMI_ARM_D(32)
#undef CCMI_ARM_D
#undef CCMI_ARM_CASE
    return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "dec: ARM with d=%d, %d hidden layers not supported", d, nh);
}

size_t dec_ups_workspace_elems(const int *lh, const int *lw, int L)
{
    size_t n = 0;
    for (int k = 1; k <= L - 2; ++k) n += (size_t)(L - k) * lh[k] * lw[k];
    return n;
}

static bool ups_ks_ok(const DecUpsArgs &a)
{
    return a.ups_ks >= 2 && a.ups_ks <= kMaxKs && a.pre_ks >= 1 && a.pre_ks <= kMaxKs - 1;
}

// kernel arguments of every pyramid step of one frame (coarsest first); returns the step count
static int make_levels(const DecUpsArgs &a, DecLevel *lv)
{
    const int L = a.n_layers;
    int32_t *stack[CCMI_MAX_GRIDS] = {};
    int32_t *ws = a.workspace;
    for (int k = 1; k <= L - 2; ++k) {
        stack[k] = ws;
        ws += (size_t)(L - k) * a.lh[k] * a.lw[k];
    }
    for (int step = 0; step < L - 1; ++step) {
        const int k = L - 1 - step;
        DecLevel &A = lv[step];
        A = DecLevel{};
        A.src = k == L - 1 ? a.lat + a.off[k] : stack[k];
        A.C = L - k;
        A.hs = a.lh[k];
        A.ws = a.lw[k];
        A.src_prec = k == L - 1 ? kArmPrec : kUpsPrec;
        A.ref = a.lat + a.off[k - 1];
        A.dst = k - 1 == 0 ? a.out : stack[k - 1];
        A.hd = a.lh[k - 1];
        A.wd = a.lw[k - 1];
        // reference indices: ups layer (L-2-target)%n_ups, preconcat (L-2-layer)%n_pre; target = layer = k-1
        A.kup = a.kernels + ((L - 2 - (k - 1)) % a.n_ups) * a.ups_ks;
        A.ksx2 = a.ups_ks;
        A.kpre = a.kernels + a.n_ups * a.ups_ks + ((L - 2 - (k - 1)) % a.n_pre) * a.pre_ks;
        A.ks = a.pre_ks;
        A.tiles_x = ccmi_div_up(A.wd, kTX);
    }
    return L > 1 ? L - 1 : 0;
}

int launch_dec_ups(const DecUpsArgs &a, hipStream_t s)
{
    if (!ups_ks_ok(a))
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "dec: upsampling kernel sizes %d/%d", a.ups_ks, a.pre_ks);
    DecLevel lv[CCMI_MAX_GRIDS];
    const int steps = make_levels(a, lv);
    for (int step = 0; step < steps; ++step) {
        const DecLevel &A = lv[step];
        hipLaunchKernelGGL(dec_ups_level, dim3(A.tiles_x * ccmi_div_up(A.hd, kTY)), dim3(kThreads), 0, s, A);
        CCMI_HIP_CHECK(hipGetLastError());
    }
    return CCMI_OK;
}

static int syn_maxc(const DecSynArgs &a)
{
    int m = a.c_in;
    for (int l = 0; l < a.n_layers; ++l) m = a.layers[l].n_out > m ? a.layers[l].n_out : m;
    return m;
}

static bool syn_fast(const DecSynArgs &a, int *cmid)
{
    if (a.n_layers < 2 || a.layers[0].ks != 1 || a.layers[1].ks != 1) return false;
    if (a.c_in < 1 || a.c_in > 8) return false;
    const int cm = a.layers[1].n_out;
    if (cm != 3) return false;
    if (a.n_layers - 2 > kMaxSp) return false;
    for (int l = 2; l < a.n_layers; ++l)
        if (a.layers[l].ks != 3 || a.layers[l].n_out != cm) return false;
    *cmid = cm;
    return true;
}

size_t dec_syn_workspace_elems(const DecSynArgs &a)
{
    int cm;
    if (syn_fast(a, &cm)) return 0;
    return 2 * (size_t)syn_maxc(a) * a.h * a.w;
}

int launch_dec_syn(const DecSynArgs &a, hipStream_t s)
{
    // weight offsets (per layer W then b)
    const int32_t *wp[CCMI_MAX_SYN_LAYERS], *bp[CCMI_MAX_SYN_LAYERS];
    int cin_of[CCMI_MAX_SYN_LAYERS];
    {
        const int32_t *q = a.params;
        int c = a.c_in;
        for (int l = 0; l < a.n_layers; ++l) {
            cin_of[l] = c;
            wp[l] = q;
            q += (size_t)a.layers[l].n_out * c * a.layers[l].ks * a.layers[l].ks;
            bp[l] = q;
            q += a.layers[l].n_out;
            c = a.layers[l].n_out;
        }
    }
    int cm;
    if (syn_fast(a, &cm)) {
        DecSynFused F{};
        F.in = a.in;
        F.cin = a.c_in;
        F.H = a.h;
        F.W = a.w;
        F.hid = a.layers[0].n_out;
        F.w0 = wp[0];
        F.b0 = bp[0];
        F.w1 = wp[1];
        F.b1 = bp[1];
        F.n_sp = a.n_layers - 2;
        for (int i = 0; i < F.n_sp; ++i) {
            F.wsp[i] = wp[2 + i];
            F.bsp[i] = bp[2 + i];
            F.res[i] = a.layers[2 + i].residual;
            F.relu[i] = a.layers[2 + i].relu;
        }
        F.out = a.out;
        F.f24 = a.f24;
        const int halo = F.n_sp;
        F.tiles_x = ccmi_div_up(a.w, kRW - 2 * halo);
        dim3 grid(F.tiles_x * ccmi_div_up(a.h, kRH - 2 * halo));
        switch (a.c_in) {
        case 1: hipLaunchKernelGGL((dec_syn_fused<1, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 2: hipLaunchKernelGGL((dec_syn_fused<2, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 3: hipLaunchKernelGGL((dec_syn_fused<3, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 4: hipLaunchKernelGGL((dec_syn_fused<4, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 5: hipLaunchKernelGGL((dec_syn_fused<5, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 6: hipLaunchKernelGGL((dec_syn_fused<6, 3>), grid, dim3(kThreads), 0, s, F); break;
        case 7: hipLaunchKernelGGL((dec_syn_fused<7, 3>), grid, dim3(kThreads), 0, s, F); break;
        default: hipLaunchKernelGGL((dec_syn_fused<8, 3>), grid, dim3(kThreads), 0, s, F); break;
        }
        CCMI_HIP_CHECK(hipGetLastError());
        return CCMI_OK;
    }
    // generic: the reference fuses the first two layers whenever both are 1x1 (can_fuse)
    const int64_t plane = (int64_t)a.h * a.w;
    const int maxc = syn_maxc(a);
    int32_t *bufs[2] = {a.workspace, a.workspace + (size_t)maxc * plane};
    const int32_t *src = a.in;
    dim3 grid((unsigned)((plane + kThreads - 1) / kThreads));
    int l = 0, k = 0;
    while (l < a.n_layers) {
        const bool fused = l == 0 && a.n_layers >= 2 && a.layers[0].ks == 1 && a.layers[1].ks == 1;
        const int last_layer = fused ? 1 : l;
        int32_t *dst = last_layer == a.n_layers - 1 ? a.out : bufs[k & 1];
        if (fused) {
            hipLaunchKernelGGL(dec_syn_fused_generic, grid, dim3(kThreads), 0, s, src, cin_of[0], plane, wp[0], bp[0],
                               a.layers[0].n_out, wp[1], bp[1], a.layers[1].n_out, dst);
        } else {
            const SynLayerDesc &L = a.layers[l];
            hipLaunchKernelGGL(dec_syn_layer, grid, dim3(kThreads), 0, s, src, cin_of[l], a.h, a.w, wp[l], bp[l],
                               L.n_out, L.ks, L.residual, L.relu, dst);
        }
        CCMI_HIP_CHECK(hipGetLastError());
        src = dst;
        l = last_layer + 1;
        ++k;
    }
    return CCMI_OK;
}

int launch_dec_blend(int32_t *acc, const int32_t *x, int64_t n, int32_t b_acc, int32_t b_x, int first, hipStream_t s)
{
    hipLaunchKernelGGL(dec_blend_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, acc, x,
                       n, b_acc, b_x, first);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

int launch_dec_output(const int32_t *syn, int h, int w, int bitdepth, int kind, uint8_t *dst, hipStream_t s)
{
    const int64_t plane = (int64_t)h * w;
    hipLaunchKernelGGL(dec_output_kernel, dim3((unsigned)((plane + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                       syn, h, w, (1 << bitdepth) - 1, kind, bitdepth <= 8 ? 1 : 2, dst);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

// ------------------------------------------------------------------ batched decoder tail
// fused-synthesis kernel arguments of one frame (syn_fast architectures only); the same
// weight walk as launch_dec_syn
static DecSynFused make_syn_fused(const DecSynArgs &a)
{
    const int32_t *wp[CCMI_MAX_SYN_LAYERS], *bp[CCMI_MAX_SYN_LAYERS];
    const int32_t *q = a.params;
    int c = a.c_in;
    for (int l = 0; l < a.n_layers; ++l) {
        wp[l] = q;
        q += (size_t)a.layers[l].n_out * c * a.layers[l].ks * a.layers[l].ks;
        bp[l] = q;
        q += a.layers[l].n_out;
        c = a.layers[l].n_out;
    }
    DecSynFused F{};
    F.in = a.in;
    F.cin = a.c_in;
    F.H = a.h;
    F.W = a.w;
    F.hid = a.layers[0].n_out;
    F.w0 = wp[0];
    F.b0 = bp[0];
    F.w1 = wp[1];
    F.b1 = bp[1];
    F.n_sp = a.n_layers - 2;
    for (int i = 0; i < F.n_sp; ++i) {
        F.wsp[i] = wp[2 + i];
        F.bsp[i] = bp[2 + i];
        F.res[i] = a.layers[2 + i].residual;
        F.relu[i] = a.layers[2 + i].relu;
    }
    F.out = a.out;
    F.f24 = a.f24;
    F.tiles_x = ccmi_div_up(a.w, kRW - 2 * F.n_sp);
    return F;
}

bool dec_tail_batchable(const DecTailFrame &f)
{
    int cm;
    return f.ups.n_layers >= 2 && ups_ks_ok(f.ups) && f.syn.c_in == f.ups.n_layers && syn_fast(f.syn, &cm);
}

// launch geometry only: the grids depend on the plane sizes, the synthesis halo and the
// synthesis input width (template); everything else is per-frame table data
bool dec_tail_same_group(const DecTailFrame &a, const DecTailFrame &b)
{
    if (a.ups.n_layers != b.ups.n_layers) return false;
    for (int l = 0; l < a.ups.n_layers; ++l)
        if (a.ups.lh[l] != b.ups.lh[l] || a.ups.lw[l] != b.ups.lw[l]) return false;
    return a.syn.n_layers == b.syn.n_layers && a.syn.c_in == b.syn.c_in && a.syn.h == b.syn.h && a.syn.w == b.syn.w;
}

static size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// table of a group of n frames: [step][frame] DecLevel, [frame] DecSynFused, [frame] DecOut
size_t dec_tail_table_bytes(int n_layers, int n)
{
    const size_t steps = n_layers > 1 ? (size_t)(n_layers - 1) : 0;
    return al16(sizeof(DecLevel) * steps * n) + al16(sizeof(DecSynFused) * (size_t)n) + al16(sizeof(DecOut) * (size_t)n);
}

void dec_tail_fill(const DecTailFrame *const *fr, int n, void *host_tab)
{
    const int steps = fr[0]->ups.n_layers - 1;
    uint8_t *p = static_cast<uint8_t *>(host_tab);
    DecLevel *lv = reinterpret_cast<DecLevel *>(p);
    DecSynFused *sf = reinterpret_cast<DecSynFused *>(p + al16(sizeof(DecLevel) * (size_t)steps * n));
    DecOut *oo = reinterpret_cast<DecOut *>(reinterpret_cast<uint8_t *>(sf) + al16(sizeof(DecSynFused) * (size_t)n));
    for (int i = 0; i < n; ++i) {
        DecLevel tmp[CCMI_MAX_GRIDS];
        make_levels(fr[i]->ups, tmp);
        for (int st = 0; st < steps; ++st) lv[(size_t)st * n + i] = tmp[st];
        sf[i] = make_syn_fused(fr[i]->syn);
        const DecSynArgs &sa = fr[i]->syn;
        const int bd = fr[i]->bitdepth;
        oo[i] = DecOut{sa.out, sa.h, sa.w, (1 << bd) - 1, fr[i]->kind, bd <= 8 ? 1 : 2, fr[i]->dst};
    }
}

int launch_dec_tail_batch(const DecTailFrame &f0, int n, const void *dev_tab, hipStream_t s)
{
    if (n < 1 || n > 65535) return ccmi_set_error(CCMI_ERR_ARG, "dec: tail batch of %d frames", n);
    const int L = f0.ups.n_layers, steps = L - 1;
    const uint8_t *p = static_cast<const uint8_t *>(dev_tab);
    const DecLevel *lv = reinterpret_cast<const DecLevel *>(p);
    const DecSynFused *sf = reinterpret_cast<const DecSynFused *>(p + al16(sizeof(DecLevel) * (size_t)steps * n));
    const DecOut *oo =
        reinterpret_cast<const DecOut *>(reinterpret_cast<const uint8_t *>(sf) + al16(sizeof(DecSynFused) * (size_t)n));
    for (int st = 0; st < steps; ++st) {
        const int k = L - 1 - st;
        const int hd = f0.ups.lh[k - 1], wd = f0.ups.lw[k - 1];
        const dim3 grid(ccmi_div_up(wd, kTX) * ccmi_div_up(hd, kTY), n);
        hipLaunchKernelGGL(dec_ups_level_batch, grid, dim3(kThreads), 0, s, lv + (size_t)st * n);
        CCMI_HIP_CHECK(hipGetLastError());
    }
    const int halo = f0.syn.n_layers - 2;
    const dim3 sg(ccmi_div_up(f0.syn.w, kRW - 2 * halo) * ccmi_div_up(f0.syn.h, kRH - 2 * halo), n);
    switch (f0.syn.c_in) {
    case 1: hipLaunchKernelGGL((dec_syn_fused_batch<1, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 2: hipLaunchKernelGGL((dec_syn_fused_batch<2, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 3: hipLaunchKernelGGL((dec_syn_fused_batch<3, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 4: hipLaunchKernelGGL((dec_syn_fused_batch<4, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 5: hipLaunchKernelGGL((dec_syn_fused_batch<5, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 6: hipLaunchKernelGGL((dec_syn_fused_batch<6, 3>), sg, dim3(kThreads), 0, s, sf); break;
    case 7: hipLaunchKernelGGL((dec_syn_fused_batch<7, 3>), sg, dim3(kThreads), 0, s, sf); break;
    default: hipLaunchKernelGGL((dec_syn_fused_batch<8, 3>), sg, dim3(kThreads), 0, s, sf); break;
    }
    CCMI_HIP_CHECK(hipGetLastError());
    const int64_t plane = (int64_t)f0.syn.h * f0.syn.w;
    hipLaunchKernelGGL(dec_output_batch, dim3((unsigned)((plane + kThreads - 1) / kThreads), n), dim3(kThreads), 0, s,
                       oo);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}

} // namespace ccmi
