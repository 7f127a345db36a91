// fwd_syn.hip -- path A synthesis (Synthesis.forward), float32, plus frame post-processing.
//
// Reference: coolchic/enc/component/core/synthesis.py
//   SynthesisConv2d.forward :69-84  -- replicate pad (ks-1)/2, conv2d + bias, (+ x if residual)
//   Synthesis.forward      :264-277 -- layers in sequence, ReLU / identity after each.
// Post-processing: FrameEncoder.forward eval branch, coolchic/enc/component/frame.py:175-183,
//   convert_444_to_420 coolchic/enc/io/format/yuv.py:275-299 (nearest = even rows / cols).
//
// Fast path (every architecture made of a 1x1 "MLP" head followed by 3x3 layers with
// <= 4 channels -- all the reference presets: hop, mop, lop, ...): ONE fused kernel per
// launch.  A workgroup owns a 32 x 64 pixel window.  Pass 0 evaluates the per-pixel MLP
// (c_in -> hid -> c_mid, weights wave-uniform in SGPRs) on the whole window (output tile
// plus a halo of one pixel per 3x3 layer) and keeps its c_mid outputs in LDS; each 3x3 layer then shrinks
// the region by one pixel, ping-ponging between two LDS images; the last layer writes
// to HBM.  Replicate padding is reproduced by evaluating halo pixels at the clamped
// image coordinate (a pointwise head commutes with clamping; a 3x3 layer reads its
// input at clamp(clamp(g) + d)).  HBM traffic: c_in planes read once (+ halo), c_out
// planes written once.
//
// Any other architecture runs the generic per-layer kernel (one launch per layer,
// ping-pong through the caller's workspace).
#include "ccmi_internal.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxIn = 8;   // fused path: max synthesis input channels
constexpr int kMaxMid = 4;  // fused path: max channels through the 3x3 layers
constexpr int kMaxSp = 3;   // fused path: max number of 3x3 layers

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
    int w0_off, b0_off, relu0;
    int w1_off, b1_off, relu1;
    int n_sp;            // 3x3 layers after the head
    SpLayer sp[kMaxSp];
    const float *params;
    int64_t pstride;
    float *out;
    int64_t out_stride;
    int tiles_x;
};

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

typedef float f2 __attribute__((ext_vector_type(2)));
// Weights are read through a constant-address-space pointer: the loads are wave-uniform
// and the buffer is never written by the kernel, so they become scalar (SMEM) loads even
// after the kernel's own global stores (which would otherwise force vector loads).
typedef const __attribute__((address_space(4))) float *cfloat_ptr;

// Fused head + 3x3 tail.  The workgroup's working region is a fixed 32 x 64 window
// (2048 pixels, 512 threads, 4 per thread): the output tile is the window minus a halo
// of one pixel per 3x3 layer.  All stages share the window's coordinate frame (pitch
// 64); stage t is valid on rows/cols [t, 32-t) x [t, 64-t).  Thread (c = tid & 63,
// g = tid >> 6) owns column c of the 4 consecutive rows 4g .. 4g+3 in every stage.
//  * head: packed fp32 (v_pk_fma_f32) over pixel pairs, wave-uniform weights from
//    SGPRs, hidden activations consumed as they are produced (never stored);
//  * 3x3 layers: the thread slides a 3-row register window down its 4 rows, so a
//    pixel costs 3*CMID LDS reads instead of 9*CMID.  Window row i maps to image row
//    clamp(oy + i) (replicate padding); rows whose image row lies outside the image
//    or outside the stage's valid band are computed but never read or stored, which
//    keeps control flow uniform.
constexpr int kFThreads = 512;
constexpr int kRW = 64, kRH = 32;
constexpr int kPlane = kRW * (kRH + 2); // LDS plane: window rows -1 .. kRH (guard rows)
constexpr int kRowsPerThread = kRH / (kFThreads / kRW); // 4

template <int CIN, int CMID>
__global__ __launch_bounds__(kFThreads) void syn_fused_kernel(FusedArgs A)
{
    constexpr int NR = kRowsPerThread;
    constexpr int NW = CMID * CMID * 9 + CMID; // weights + biases of one 3x3 layer
    __shared__ float s_buf[2][CMID][kPlane];
    // 3x3 weights staged in LDS: read back as broadcast ds_read_b128 into VGPRs (the
    // 81+ weights of a layer do not fit the SGPR budget next to the head's state)
    __shared__ __attribute__((aligned(16))) float s_w[kMaxSp][(NW + 3) & ~3];

    const int b = blockIdx.y;
    const int halo = A.n_sp;
    const int TX = kRW - 2 * halo, TY = kRH - 2 * halo;
    const int y0 = (blockIdx.x / A.tiles_x) * TY;
    const int x0 = (blockIdx.x % A.tiles_x) * TX;
    const int oy = y0 - halo, ox = x0 - halo; // global coords of window (0,0)
    const cfloat_ptr prm = (cfloat_ptr)(size_t)(A.params + (int64_t)b * A.pstride);
    const float *in = A.in + (int64_t)b * A.in_stride;
    float *out = A.out + (int64_t)b * A.out_stride;
    const int64_t plane = (int64_t)A.H * A.W;
    const int c = threadIdx.x & (kRW - 1);
    const int rb = (threadIdx.x >> 6) * NR; // first window row of this thread
    const int gx = ox + c;
    const int cxg = clampi(gx, A.W - 1);

    for (int i = threadIdx.x; i < A.n_sp * NW; i += kFThreads) {
        const int l = i / NW, j = i - l * NW;
        s_w[l][j] = prm[A.sp[l].w_off + j]; // biases follow the weights in the block
    }

    // ------------------------ pass 0: per-pixel 1x1 head ------------------------
    {
        const cfloat_ptr w0 = prm + A.w0_off, b0 = prm + A.b0_off;
        const cfloat_ptr w1 = prm + A.w1_off, b1 = prm + A.b1_off;
        float x[NR][CIN];
        float o[NR][CMID];
#pragma unroll
        for (int p = 0; p < NR; ++p) {
            const int64_t pix = (int64_t)clampi(oy + rb + p, A.H - 1) * A.W + cxg;
#pragma unroll
            for (int k = 0; k < CIN; ++k) x[p][k] = in[k * plane + pix];
        }
        if (A.n_head == 2) {
            const int hid = A.hid;
            // fmaxf(acc, lo0) is the optional ReLU without a per-element select
            const f2 lo0 = f2(A.relu0 ? 0.f : -INFINITY);
            f2 xp[NR / 2][CIN], op[NR / 2][CMID];
#pragma unroll
            for (int q = 0; q < NR / 2; ++q) {
#pragma unroll
                for (int k = 0; k < CIN; ++k) xp[q][k] = f2{x[2 * q][k], x[2 * q + 1][k]};
#pragma unroll
                for (int m = 0; m < CMID; ++m) op[q][m] = f2(0.f);
            }
#pragma unroll 2
            for (int j = 0; j < hid; ++j) {
                const cfloat_ptr wj = w0 + j * CIN;
                const f2 bj = f2(b0[j]);
                f2 wm[CMID];
#pragma unroll
                for (int m = 0; m < CMID; ++m) wm[m] = f2(w1[m * hid + j]);
#pragma unroll
                for (int q = 0; q < NR / 2; ++q) {
                    f2 acc = bj;
#pragma unroll
                    for (int k = 0; k < CIN; ++k) acc = __builtin_elementwise_fma(f2(wj[k]), xp[q][k], acc);
                    acc = __builtin_elementwise_max(acc, lo0);
#pragma unroll
                    for (int m = 0; m < CMID; ++m) op[q][m] = __builtin_elementwise_fma(wm[m], acc, op[q][m]);
                }
            }
            const float lo1 = A.relu1 ? 0.f : -INFINITY;
#pragma unroll
            for (int q = 0; q < NR / 2; ++q)
#pragma unroll
                for (int m = 0; m < CMID; ++m) {
                    o[2 * q][m] = fmaxf(op[q][m].x + b1[m], lo1);
                    o[2 * q + 1][m] = fmaxf(op[q][m].y + b1[m], lo1);
                }
        } else {
            const float lo0 = A.relu0 ? 0.f : -INFINITY;
#pragma unroll
            for (int m = 0; m < CMID; ++m) {
                const float bm = b0[m];
#pragma unroll
                for (int p = 0; p < NR; ++p) {
                    float acc = bm;
#pragma unroll
                    for (int k = 0; k < CIN; ++k) acc = fmaf(w0[m * CIN + k], x[p][k], acc);
                    o[p][m] = fmaxf(acc, lo0);
                }
            }
        }
        if (halo == 0) {
#pragma unroll
            for (int p = 0; p < NR; ++p) {
                const int gy = oy + rb + p;
                if (gy < A.H && gx < A.W)
#pragma unroll
                    for (int m = 0; m < CMID; ++m) out[m * plane + (int64_t)gy * A.W + gx] = o[p][m];
            }
            return;
        }
#pragma unroll
        for (int p = 0; p < NR; ++p)
#pragma unroll
            for (int m = 0; m < CMID; ++m) s_buf[0][m][(rb + p + 1) * kRW + c] = o[p][m];
    }

    // ------------------------ 3x3 layers, replicate padding ------------------------
    // Every LDS image is kept "pre-clamped" along rows: a window row outside the image
    // holds the value of the nearest image row wherever it can be read.  The head computes
    // all window rows at clamped coordinates; a 3x3 layer stores its in-image rows and the
    // edge rows again one row further out (the only out-of-image rows an in-image output
    // reads).  So the vertical neighbours of window row r are simply rows r-1, r+1, and a
    // thread reads row pairs {r, r+1} straight into packed registers.  Columns are lanes:
    // the horizontal neighbours use clamped columns lx[].
    int lx[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) lx[d] = clampi(cxg + d - 1, A.W - 1) - ox;
    const bool col_in = gx < A.W;
    int cur = 0;
    for (int s = 0; s < A.n_sp; ++s) {
        __syncthreads();
        const int t = s + 1;
        const bool last = s == A.n_sp - 1;
        const float *wt = s_w[s];
        const float *bs = s_w[s] + CMID * CMID * 9;
        const float lo = A.sp[s].relu ? 0.f : -INFINITY;
        const float rsd = A.sp[s].residual ? 1.f : 0.f;
        // plane row of window row (rb - 1) in this thread's column
        const float *src = &s_buf[cur][0][0] + rb * kRW + c;
#pragma unroll
        for (int q = 0; q < NR / 2; ++q) {
            // output rows rb + 2q, rb + 2q + 1 read window rows rb + 2q - 1 .. rb + 2q + 2
            f2 P[3][CMID][3]; // P[dy] = {row rb+2q-1+dy, row rb+2q+dy}
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int k = 0; k < CMID; ++k)
#pragma unroll
                    for (int d = 0; d < 3; ++d) {
                        const float *e = src + k * kPlane + (2 * q + dy) * kRW + (lx[d] - c);
                        P[dy][k][d] = f2{e[0], e[kRW]};
                    }
            f2 acc[CMID];
#pragma unroll
            for (int m = 0; m < CMID; ++m) {
                // one output channel's weights in flight at a time (bounds VGPR use)
                __builtin_amdgcn_sched_barrier(0);
                acc[m] = f2(bs[m]);
#pragma unroll
                for (int k = 0; k < CMID; ++k)
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx)
                            acc[m] = __builtin_elementwise_fma(f2(wt[((m * CMID + k) * 3 + dy) * 3 + dx]),
                                                               P[dy][k][dx], acc[m]);
                // residual: the input at the centre
                acc[m] = __builtin_elementwise_max(__builtin_elementwise_fma(f2(rsd), P[1][m][1], acc[m]), f2(lo));
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = rb + 2 * q + h, gy = oy + r;
                if (last) {
                    if (r >= t && r < kRH - t && c >= t && c < kRW - t && gy < A.H && col_in)
#pragma unroll
                        for (int m = 0; m < CMID; ++m) out[m * plane + (int64_t)gy * A.W + gx] = h ? acc[m].y : acc[m].x;
                } else if (gy >= 0 && gy < A.H) {
                    float *dst = &s_buf[cur ^ 1][0][0] + (r + 1) * kRW + c;
#pragma unroll
                    for (int m = 0; m < CMID; ++m) {
                        const float v = h ? acc[m].y : acc[m].x;
                        dst[m * kPlane] = v;
                        if (gy == 0) dst[m * kPlane - kRW] = v;     // replicate above the image
                        if (gy == A.H - 1) dst[m * kPlane + kRW] = v; // and below it
                    }
                }
            }
        }
        cur ^= 1;
    }
}

// Generic layer: any ks (odd), any channel counts; replicate padding.
__global__ __launch_bounds__(kThreads) void syn_layer_kernel(const float *__restrict__ in, int64_t in_stride, int cin,
                                                             int H, int W, const float *__restrict__ params,
                                                             int64_t pstride, int w_off, int b_off, int nout, int ks,
                                                             int residual, int relu, float *__restrict__ out,
                                                             int64_t out_stride)
{
    const int b = blockIdx.y;
    const int64_t plane = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= plane) return;
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    const float *src = in + (int64_t)b * in_stride;
    float *dst = out + (int64_t)b * out_stride;
    const float *wt = params + (int64_t)b * pstride + w_off;
    const float *bs = params + (int64_t)b * pstride + b_off;
    const int pad = ks / 2;
    for (int m = 0; m < nout; ++m) {
        float acc = 0.f;
        for (int k = 0; k < cin; ++k)
            for (int dy = 0; dy < ks; ++dy) {
                const int yy = clampi(y + dy - pad, H - 1);
                for (int dx = 0; dx < ks; ++dx) {
                    const int xx = clampi(x + dx - pad, W - 1);
                    acc = fmaf(wt[((m * cin + k) * ks + dy) * ks + dx], src[k * plane + (int64_t)yy * W + xx], acc);
                }
            }
        float v = acc + bs[m];
        if (residual) v += src[m * plane + p];
        if (relu) v = fmaxf(v, 0.f);
        dst[m * plane + p] = v;
    }
}

__global__ __launch_bounds__(kThreads) void post_kernel(const float *__restrict__ in, int64_t in_stride, int H, int W,
                                                        float qmax, int yuv420, float *__restrict__ out,
                                                        int64_t out_stride)
{
    const int b = blockIdx.y;
    const int64_t plane = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= plane) return;
    const float *src = in + (int64_t)b * in_stride;
    float *dst = out + (int64_t)b * out_stride;
    auto q = [qmax](float v) { return fminf(fmaxf(rintf(v * qmax) / qmax, 0.f), 1.f); };
    dst[p] = q(src[p]);
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    if (!yuv420) {
        dst[plane + p] = q(src[plane + p]);
        dst[2 * plane + p] = q(src[2 * plane + p]);
    } else if (!(y & 1) && !(x & 1) && y / 2 < H / 2 && x / 2 < W / 2) {
        const int64_t cp = (int64_t)(H / 2) * (W / 2);
        const int64_t ci = (int64_t)(y / 2) * (W / 2) + x / 2;
        dst[plane + ci] = q(src[plane + p]);
        dst[plane + cp + ci] = q(src[2 * plane + p]);
    }
}

struct Plan {
    bool fused;
    int hid, cmid;
    FusedArgs fa;
};

// Offsets of each layer's weights / biases in a frame's parameter block.
void layer_offsets(const ccmi_syn_args *a, int *w_off, int *b_off, int *cin_of, int64_t *total)
{
    int64_t o = 0;
    int c = a->c_in;
    for (int l = 0; l < a->n_layers; ++l) {
        const ccmi_syn_layer &L = a->layers[l];
        cin_of[l] = c;
        w_off[l] = (int)o;
        o += (int64_t)L.n_out * c * L.ks * L.ks;
        b_off[l] = (int)o;
        o += L.n_out;
        c = L.n_out;
    }
    *total = o;
}

bool make_plan(const ccmi_syn_args *a, Plan *P)
{
    int w_off[CCMI_MAX_SYN_LAYERS], b_off[CCMI_MAX_SYN_LAYERS], cin_of[CCMI_MAX_SYN_LAYERS];
    int64_t tot;
    layer_offsets(a, w_off, b_off, cin_of, &tot);
    P->fused = false;
    const ccmi_syn_layer *L = a->layers;
    int n_head = 0;
    while (n_head < a->n_layers && n_head < 2 && L[n_head].ks == 1 && !L[n_head].residual) n_head++;
    if (n_head == 0 || a->c_in > kMaxIn) return false;
    const int cmid = L[n_head - 1].n_out;
    if (cmid < 1 || cmid > kMaxMid) return false;
    int hid = n_head == 2 ? L[0].n_out : 0;
    const int n_sp = a->n_layers - n_head;
    if (n_sp > kMaxSp) return false;
    for (int l = n_head; l < a->n_layers; ++l)
        if (L[l].ks != 3 || L[l].n_out != cmid) return false;
    if (cmid != 3 && cmid != 4) return false; // instantiated shapes
    FusedArgs &f = P->fa;
    f = FusedArgs{};
    f.cin = a->c_in;
    f.H = a->h;
    f.W = a->w;
    f.n_head = n_head;
    f.hid = hid;
    f.w0_off = w_off[0];
    f.b0_off = b_off[0];
    f.relu0 = L[0].relu;
    if (n_head == 2) {
        f.w1_off = w_off[1];
        f.b1_off = b_off[1];
        f.relu1 = L[1].relu;
    }
    f.n_sp = n_sp;
    for (int s = 0; s < n_sp; ++s) {
        f.sp[s].w_off = w_off[n_head + s];
        f.sp[s].b_off = b_off[n_head + s];
        f.sp[s].residual = L[n_head + s].residual;
        f.sp[s].relu = L[n_head + s].relu;
    }
    P->fused = true;
    P->hid = hid;
    P->cmid = cmid;
    return true;
}

template <int CMID>
void launch_fused(dim3 grid, hipStream_t s, const FusedArgs &fa)
{
    switch (fa.cin) {
    case 1: hipLaunchKernelGGL((syn_fused_kernel<1, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 2: hipLaunchKernelGGL((syn_fused_kernel<2, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 3: hipLaunchKernelGGL((syn_fused_kernel<3, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 4: hipLaunchKernelGGL((syn_fused_kernel<4, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 5: hipLaunchKernelGGL((syn_fused_kernel<5, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 6: hipLaunchKernelGGL((syn_fused_kernel<6, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 7: hipLaunchKernelGGL((syn_fused_kernel<7, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    case 8: hipLaunchKernelGGL((syn_fused_kernel<8, CMID>), grid, dim3(kFThreads), 0, s, fa); break;
    }
}

} // namespace

extern "C" size_t ccmi_syn_workspace_bytes(const ccmi_syn_args *a)
{
    Plan P;
    if (make_plan(a, &P)) return 0;
    int maxc = a->c_in;
    for (int l = 0; l < a->n_layers; ++l) maxc = a->layers[l].n_out > maxc ? a->layers[l].n_out : maxc;
    return 2 * sizeof(float) * (size_t)maxc * a->h * a->w * (size_t)(a->batch > 0 ? a->batch : 0);
}

int ccmi_launch_syn_f32(const ccmi_syn_args *a, hipStream_t s)
{
    if (a->n_layers < 1 || a->n_layers > CCMI_MAX_SYN_LAYERS)
        return ccmi_set_error(CCMI_ERR_ARG, "syn: n_layers must be in [1, %d]", CCMI_MAX_SYN_LAYERS);
    int c = a->c_in;
    for (int l = 0; l < a->n_layers; ++l) {
        const ccmi_syn_layer &L = a->layers[l];
        if (L.n_out < 1 || L.ks < 1 || L.ks % 2 == 0)
            return ccmi_set_error(CCMI_ERR_ARG, "syn: layer %d has n_out=%d ks=%d (ks must be odd)", l, L.n_out, L.ks);
        if (L.residual && L.n_out != c)
            return ccmi_set_error(CCMI_ERR_ARG, "syn: residual layer %d needs n_out == n_in", l);
        c = L.n_out;
    }
    Plan P;
    if (make_plan(a, &P)) {
        P.fa.in = a->in;
        P.fa.in_stride = a->in_stride;
        P.fa.params = a->params;
        P.fa.pstride = a->param_stride;
        P.fa.out = a->out;
        P.fa.out_stride = a->out_stride;
        const int halo = P.fa.n_sp;
        P.fa.tiles_x = ccmi_div_up(a->w, kRW - 2 * halo);
        dim3 grid(P.fa.tiles_x * ccmi_div_up(a->h, kRH - 2 * halo), a->batch);
        if (P.cmid == 3) launch_fused<3>(grid, s, P.fa);
        else launch_fused<4>(grid, s, P.fa);
        CCMI_HIP_CHECK(hipGetLastError());
        return CCMI_OK;
    }
    // generic path
    const size_t need = ccmi_syn_workspace_bytes(a);
    if (a->workspace == nullptr || a->workspace_bytes < need)
        return ccmi_set_error(CCMI_ERR_ARG, "syn: workspace of %zu bytes needed for this architecture", need);
    int w_off[CCMI_MAX_SYN_LAYERS], b_off[CCMI_MAX_SYN_LAYERS], cin_of[CCMI_MAX_SYN_LAYERS];
    int64_t tot;
    layer_offsets(a, w_off, b_off, cin_of, &tot);
    int maxc = a->c_in;
    for (int l = 0; l < a->n_layers; ++l) maxc = a->layers[l].n_out > maxc ? a->layers[l].n_out : maxc;
    const int64_t buf_stride = (int64_t)maxc * a->h * a->w;
    float *bufs[2] = {static_cast<float *>(a->workspace), static_cast<float *>(a->workspace) + buf_stride * a->batch};
    const float *src = a->in;
    int64_t src_stride = a->in_stride;
    const int64_t plane = (int64_t)a->h * a->w;
    dim3 grid((unsigned)((plane + kThreads - 1) / kThreads), a->batch);
    for (int l = 0; l < a->n_layers; ++l) {
        const bool last = l == a->n_layers - 1;
        float *dst = last ? a->out : bufs[l & 1];
        const int64_t dst_stride = last ? a->out_stride : buf_stride;
        const ccmi_syn_layer &L = a->layers[l];
        hipLaunchKernelGGL(syn_layer_kernel, grid, dim3(kThreads), 0, s, src, src_stride, cin_of[l], a->h, a->w,
                           a->params, a->param_stride, w_off[l], b_off[l], L.n_out, L.ks, L.residual, L.relu, dst,
                           dst_stride);
        CCMI_HIP_CHECK(hipGetLastError());
        src = dst;
        src_stride = dst_stride;
    }
    return CCMI_OK;
}

int ccmi_launch_post_f32(const ccmi_post_args *a, hipStream_t s)
{
    if (a->bitdepth < 1 || a->bitdepth > 16) return ccmi_set_error(CCMI_ERR_ARG, "post: bitdepth %d", a->bitdepth);
    const int64_t plane = (int64_t)a->h * a->w;
    dim3 grid((unsigned)((plane + kThreads - 1) / kThreads), a->batch);
    hipLaunchKernelGGL(post_kernel, grid, dim3(kThreads), 0, s, a->in, a->in_stride, a->h, a->w,
                       (float)((1 << a->bitdepth) - 1), a->yuv420, a->out, a->out_stride);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}
