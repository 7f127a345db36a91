// dec_internal.h -- path B (fixed-point .cool decoder) shared definitions.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "ccmi_internal.h"

namespace ccmi {

constexpr int kArmPrec = 8;  // ARM_PRECISION   (coolchic/cpp/common.h:26)
constexpr int kUpsPrec = 12; // UPS_PRECISION   (common.h:29)
constexpr int kSynPrec = 12; // SYN_*_PRECISION (common.h:31-34)

struct SynLayerDesc {
    int n_out, ks, residual, relu;
};

// One intra frame of a .cool stream, parsed and with its networks decoded to the
// fixed-point integers the kernels use (host side).
struct FrameHost {
    // GOP header (cc-bitstream.cpp:58-84)
    int h = 0, w = 0, bitdepth = 8, frame_data_type = 0, intra_period = 0;
    // frame header (cc-bitstream.cpp:140-234)
    int dim_arm = 0, n_hidden = 0;
    int n_ups = 0, ups_ks = 0, n_pre = 0, pre_ks = 0;
    int n_branches = 1;
    std::vector<SynLayerDesc> layers;
    int sig_blk = 0;
    int n_layers = 0;
    int lh[CCMI_MAX_GRIDS] = {}, lw[CCMI_MAX_GRIDS] = {};
    const uint8_t *lat_bytes[CCMI_MAX_GRIDS] = {};
    uint32_t lat_n[CCMI_MAX_GRIDS] = {};
    // network substreams (arm w / b, ups w, syn w / b) and their q-step records (qw, qb, sw,
    // sb, nw, nb for arm / ups / syn), kept by the header parse for decode_frame_weights
    const uint8_t *wbytes[5] = {};
    int lqi[3][6] = {};
    // decoded networks
    std::vector<int32_t> arm;   // per hidden layer: W[d][d] (out, in) then b[d]; then Wout[2][d], bout[2]
    std::vector<int32_t> ups;   // n_ups kernels of ups_ks taps, then n_pre kernels of pre_ks taps (mirrored)
    std::vector<int32_t> syn;   // per branch, per layer: W[n_out][n_in][ks][ks] then b[n_out]
    std::vector<int32_t> blend; // n_branches values when n_branches > 1
    bool fusable_head() const { return layers.size() >= 2 && layers[0].ks == 1 && layers[1].ks == 1; }
};

// Parses the GOP + first frame of `bs` and decodes its weights.  Returns CCMI_OK or an
// error code (message set).  Pointers in `f` alias `bs`.
int parse_and_decode_frame(const uint8_t *bs, size_t n, FrameHost &f);
// The two halves: headers only (geometry, architecture, substream sizes; the weight arrays
// sized, not filled) -- enough to plan memory and output sizes -- then the CABAC decode of
// the network weights.
int parse_frame_header(const uint8_t *bs, size_t n, FrameHost &f);
int decode_frame_weights(FrameHost &f);

// Descriptor of one latent-layer CABAC stream for the ARM decode kernel.
struct ArmStreamDesc {
    const uint32_t *bytes; // device, zero-padded to a multiple of 16 bytes
    uint32_t nbytes;
    int h, w, sig_blk;
    int d, nh;
    int flags;              // bit 0: every ARM weight fits in 24 signed bits
    const int32_t *weights; // device copy of FrameHost::arm
    int32_t *out;           // device h*w plane, value << kArmPrec
    uint64_t *dbg;          // diagnostic builds only (CCMI_ARM_STAMPS): 8 counters per stream
    uint32_t *status;       // device word, zeroed by the host: CCMI_ARM_FLAG_* bits OR-ed in by the kernel
    int spin_cap;           // chain kernel: polls per wait before it gives up and flags CCMI_ARM_FLAG_TIMEOUT
};

// One launch for n_streams streams sharing (d, nh); max_w / max_blocks size the LDS
// ring and the block map.
int launch_dec_arm(const ArmStreamDesc *d_streams, int n_streams, int max_w, int max_blocks, int d, int nh,
                   hipStream_t s);

// Upsampling of one frame: latent planes (int32, flat) -> [L][H][W] at UPS precision.
struct DecUpsArgs {
    const int32_t *lat; // flat: grid l at off[l]
    int n_layers;
    int lh[CCMI_MAX_GRIDS], lw[CCMI_MAX_GRIDS], off[CCMI_MAX_GRIDS];
    const int32_t *kernels; // device copy of FrameHost::ups
    int ups_ks, n_ups, pre_ks, n_pre;
    int32_t *workspace;     // stacks of levels 1..L-2
    int32_t *out;           // [L][H][W]
};
size_t dec_ups_workspace_elems(const int *lh, const int *lw, int L);
int launch_dec_ups(const DecUpsArgs &a, hipStream_t s);

// Synthesis of one frame (single branch): [C][H][W] at 12-bit -> [C_out][H][W].
struct DecSynArgs {
    const int32_t *in;
    int c_in, h, w;
    int n_layers;
    SynLayerDesc layers[CCMI_MAX_SYN_LAYERS];
    const int32_t *params; // per layer W then b (one branch)
    int32_t *out;
    int32_t *workspace;    // generic path ping-pong, 2 * maxc * h * w
    // every weight fits 24 signed bits (host-checked): the fused kernel multiplies with
    // v_mul_i32_i24 (full rate) instead of v_mul_lo_u32 (quarter rate).  The activations
    // always fit: each is an int32 shifted right by UPS_/SYN_ precision 12 (|v| <= 2^19), and
    // a 24x24-bit product's low 32 bits equal the int32 product's.
    int f24 = 0;
};
size_t dec_syn_workspace_elems(const DecSynArgs &a);
int launch_dec_syn(const DecSynArgs &a, hipStream_t s);

// Multi-branch blend (synblend_cpu.hpp): first: acc = (clamp(acc)*b0 + clamp(x)*b1) >> 12,
// later: acc += (clamp(x) * bk) >> 12; 3 planes.
int launch_dec_blend(int32_t *acc, const int32_t *x, int64_t n, int32_t b_acc, int32_t b_x, int first,
                     hipStream_t s);

// Output conversion (ccdecapi.cpp:59-240): syn output (12-bit) -> file bytes.
// kind: 0 yuv420, 1 yuv444, 2 ppm payload (interleaved RGB).  bps = 1 or 2 bytes/sample.
int launch_dec_output(const int32_t *syn, int h, int w, int bitdepth, int kind, uint8_t *dst, hipStream_t s);

// Batched decoder tail: frames with the same geometry and a fused-synthesis architecture
// (single branch) share one launch per pyramid step, one synthesis and one output launch
// (grid.y = frame) instead of ~8 launches per frame.  The per-frame argument tables live
// in device memory: dec_tail_table_bytes() sizes them, dec_tail_fill() writes them on the
// host (device pointers inside), the caller uploads them, launch_dec_tail_batch() runs.
struct DecTailFrame {
    DecUpsArgs ups;
    DecSynArgs syn;
    int bitdepth, kind;
    uint8_t *dst;
};
bool dec_tail_batchable(const DecTailFrame &f);
bool dec_tail_same_group(const DecTailFrame &a, const DecTailFrame &b);
size_t dec_tail_table_bytes(int n_layers, int n);
void dec_tail_fill(const DecTailFrame *const *fr, int n, void *host_tab);
int launch_dec_tail_batch(const DecTailFrame &f0, int n, const void *dev_tab, hipStream_t s);

} // namespace ccmi
