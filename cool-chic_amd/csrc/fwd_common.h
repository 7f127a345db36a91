// fwd_common.h -- path A pieces shared by the per-stage kernels (fwd_ups.hip,
// fwd_syn.hip) and the fused decode kernel (fwd_fused.hip).  Internal.
#pragma once

#include "ccmi_internal.h"

namespace ccmi_fwd {

typedef float f2 __attribute__((ext_vector_type(2)));
// Weights are read through a constant-address-space pointer: the loads are wave-uniform
// and the buffer is never written by the kernel, so they become scalar (SMEM) loads even
// after the kernel's own global stores (which would otherwise force vector loads).
typedef const __attribute__((address_space(4))) float *cfloat_ptr;

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

// XCD-aware workgroup order for a 1-D grid of n workgroups: the dispatcher deals workgroups
// round-robin over the 8 XCDs (block i and i + 8 share one, MI355X_MICROARCH.md "Workgroup
// dispatch"), so block i is given work item xcd_order(i, n), which hands each XCD a contiguous
// run of items: neighbouring tiles, which re-read each other's halos, then meet in one L2.
// A bijection of [0, n) for any n.
__device__ __forceinline__ int xcd_order(int i, int n)
{
    const int per = (n + 7) >> 3, rem = n & 7, xcd = i & 7;
    return (rem == 0 ? xcd * per : xcd * per - max(0, xcd - rem)) + (i >> 3);
}

// ---------------------------------------------------------------- synthesis plan
constexpr int kMaxIn = 8;    // fused path: max synthesis input channels
constexpr int kMaxMid = 4;   // fused path: max channels through the 3x3 layers
constexpr int kMaxSp = 3;    // fused path: max number of 3x3 layers
constexpr int kMaxHid = 64;  // fused path: max hidden width of the 1x1 head (presets: <= 48)

struct SpLayer {
    int w_off, b_off; // offsets in the frame's parameter block
    int residual, relu;
};

struct FusedArgs {
    const float *in;
    int64_t in_stride;
    int cin, H, W;
    int n_head;          // 1 or 2 1x1 layers
    int hid;             // hidden width of a 2-layer head
    int head_mfma;       // 2-layer head on the f32 MFMA form (fwd_syn.hip, CCMI_HEAD_MFMA)
    int head_generic;    // never the unrolled 48-wide head (CCMI_HEAD_GENERIC, a test form)
    int ntiles;          // windows per frame (the fused kernel's 1-D grid is ntiles x batch)
    int w0_off, b0_off, relu0;
    int w1_off, b1_off, relu1;
    int n_sp;            // 3x3 layers after the head
    SpLayer sp[kMaxSp];
    const float *params;
    int64_t pstride;
    float *out;
    int64_t out_stride;
    int tiles_x;
    float qmax;          // > 0: write the post-processed frame (2^bitdepth - 1)
    int yuv420;
};

struct Plan {
    bool fused;
    int hid, cmid;
    FusedArgs fa;
};

// Offsets of each layer's weights / biases in a frame's parameter block.
void layer_offsets(const ccmi_syn_args *a, int *w_off, int *b_off, int *cin_of, int64_t *total);
// Fills P for architectures the fused synthesis kernel handles (1x1 head of <= 2 layers,
// then <= 3 same-width 3x3 layers of 3 or 4 channels); false otherwise.
bool make_plan(const ccmi_syn_args *a, Plan *P);

// ---------------------------------------------------------------- upsampling level
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

// Polyphase geometry of a K-tap 2x transposed conv with a KP-tap refine, for a
// destination tile of TY x TX.
template <int K, int KP, int TY, int TX>
struct UpsTile {
    static constexpr int K2 = K / 2;
    static constexpr int D0 = -((K2 + 1) / 2);      // min source offset over both parities
    static constexpr int NS = K2 + 1;               // source samples shared by an (even, odd) pair
    static constexpr int SH = TY / 2 + NS - 1;      // source tile rows
    static constexpr int SW = TX / 2 + NS - 1;      // source tile cols
    static constexpr int PAD = KP / 2;
    static constexpr int RH = TY + KP - 1, RW = TX + KP - 1;
    // tap used by parity a at source offset d (or -1)
    static constexpr int tap(int a, int d) { return (a + K2 - 1 - 2 * d >= 0 && a + K2 - 1 - 2 * d < K) ? a + K2 - 1 - 2 * d : -1; }
};

// Validates the ups arguments and (launch = true) runs pyramid steps 0 .. L-3 (every step
// but the last, which produces the full-resolution stack); fills *last with the arguments
// of the final step (source level 1 -> level 0).  prev (fold): step L-3 (level 2 -> 1) is not
// launched either, its arguments go to *prev for a kernel that evaluates it in place.
// Returns CCMI_OK or an error code.
int ups_pyramid(const ccmi_ups_args *a, hipStream_t s, LevelArgs *last, bool launch = true, LevelArgs *prev = nullptr);

} // namespace ccmi_fwd
