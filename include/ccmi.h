/*
 * ccmi.h -- C ABI of libccmi, the MI355X (gfx950) implementation of Cool-chic's
 * per-image decode / forward hot path.
 *
 * Every entry point takes plain pointers and sizes (no C++ or torch types), is
 * reentrant (no globals; per-call state only) and never calls exit(): errors are
 * returned as a CCMI_ERR_* code with a message in ccmi_last_error() (thread-local).
 * Device pointers are caller-owned; kernels are enqueued on the caller's stream
 * (a hipStream_t passed as void*, e.g. torch.cuda.current_stream().cuda_stream).
 *
 * Two forms of the hot path, mirroring the reference:
 *   A. float forward  (coolchic/enc/component/coolchic.py:291-479): ARM probability
 *      model + rate, upsampling, synthesis, frame post-processing;
 *   B. fixed-point .cool bitstream decoder (coolchic/cpp/): CABAC + integer ARM,
 *      integer upsampling, integer synthesis, bit-exact with the reference C decoder.
 */
#ifndef CCMI_H
#define CCMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCMI_OK 0
#define CCMI_ERR_ARG 1         /* invalid argument / shape */
#define CCMI_ERR_HIP 2         /* HIP runtime error (no device, launch failure, ...) */
#define CCMI_ERR_UNSUPPORTED 3 /* architecture or stream feature not implemented */
#define CCMI_ERR_BITSTREAM 4   /* malformed .cool bitstream */
#define CCMI_ERR_IO 5          /* file open / read / write failure */

#define CCMI_MAX_GRIDS_PUBLIC 8
#define CCMI_MAX_SYN_LAYERS 16

/* Thread-local message for the last failing call on this thread. */
const char *ccmi_last_error(void);
/* ABI version (major*100 + minor). */
int ccmi_version(void);
/* Number of visible HIP devices (0 when none; never fails). */
int ccmi_device_count(void);

/* ------------------------------------------------------------------------- */
/* Path A: float forward, batched over independent frames of the same size and */
/* architecture.  Each frame has its own parameters (Cool-chic overfits one     */
/* network per image).  Latents of one frame are the flat concatenation of its  */
/* grids, grid l being h[l] x w[l] (coolchic.py:360-363).                        */
/* ------------------------------------------------------------------------- */

/* ARM: causal context gather + MLP + Laplace rate for every latent.
 * Replaces _get_neighbor (arm.py:308-352), Arm.forward (arm.py:227-268) and the
 * rate of CoolChicEncoder.forward (coolchic.py:395-424).
 * params per frame, float32: for each hidden layer l < n_hidden: W_l [d][d] (out,in)
 * then b_l [d]; then W_out [2][d], b_out [2]  (= arm.mlp state_dict order). */
typedef struct ccmi_arm_args {
    const float *latent;    /* [batch][latent_stride], N = sum h[l]*w[l] used; stride 0: shared */
    int64_t latent_stride;
    int n_grids;
    int h[CCMI_MAX_GRIDS_PUBLIC];
    int w[CCMI_MAX_GRIDS_PUBLIC];
    float gain;             /* encoder gain (coolchic.py:91) */
    int quantize;           /* 1: y = round(gain * latent) (eval quantizer); 0: latent used as is */
    int dim_arm;            /* 8, 16, 24 or 32 */
    int n_hidden;           /* 0..4 */
    const float *params;
    int64_t param_stride;
    float *mu;              /* optional outputs [batch][out_stride] (NULL to skip) */
    float *scale;
    float *log_scale;
    float *rate;            /* bits per latent, optional */
    int64_t out_stride;
    int batch;
} ccmi_arm_args;
int ccmi_arm_forward_f32(const ccmi_arm_args *args, void *stream);

/* Standalone pieces of the ARM for API parity with the reference modules (the fused
 * ccmi_arm_forward_f32 is what CoolChicEncoder.forward uses):
 *  ccmi_arm_context_f32: _get_neighbor (arm.py:308-352), grids [batch][h][w] -> [batch][h*w][dim_arm]
 *  ccmi_arm_mlp_f32:     Arm.forward (arm.py:227-268) on given contexts [m][dim_arm] -> mu, scale,
 *                        log_scale [m] (any may be NULL); params as in ccmi_arm_args (one model). */
int ccmi_arm_context_f32(const float *grid, int batch, int h, int w, int dim_arm, float *out, void *stream);
int ccmi_arm_mlp_f32(const float *ctx, int64_t m, int dim_arm, int n_hidden, const float *params, float *mu,
                     float *scale, float *log_scale, void *stream);

/* Upsampling: Upsampling.forward in eval mode (upsampling.py:476-506, separable
 * paths :205-209 and :337-353).  params per frame, float32: n_ups kernels of ups_k
 * taps (full symmetric kernels, conv_transpose2ds[i]), then n_pre kernels of
 * pre_k taps (conv2ds[i]).  out: [batch][n_grids][H][W] with H,W = h[0],w[0]. */
typedef struct ccmi_ups_args {
    const float *latent;
    int64_t latent_stride;
    int n_grids;
    int h[CCMI_MAX_GRIDS_PUBLIC];
    int w[CCMI_MAX_GRIDS_PUBLIC];
    float gain;
    int quantize;
    int ups_k;              /* even, >= 4 */
    int n_ups;
    int pre_k;              /* odd */
    int n_pre;
    const float *params;
    int64_t param_stride;
    float *out;
    int64_t out_stride;
    void *workspace;        /* device scratch of ccmi_ups_workspace_bytes() */
    size_t workspace_bytes;
    int batch;
} ccmi_ups_args;
size_t ccmi_ups_workspace_bytes(int n_grids, const int *h, const int *w, int batch);
int ccmi_ups_forward_f32(const ccmi_ups_args *args, void *stream);

/* Synthesis: Synthesis.forward (synthesis.py:264-277, SynthesisConv2d :69-84):
 * conv layers with replicate padding, optional residual, optional ReLU.
 * params per frame, float32, per layer: W [n_out][c_in][ks][ks] then b [n_out]. */
typedef struct ccmi_syn_layer {
    int n_out;
    int ks;
    int residual;
    int relu;
} ccmi_syn_layer;

typedef struct ccmi_syn_args {
    const float *in;        /* [batch][c_in][h][w] */
    int64_t in_stride;
    int c_in;
    int h;
    int w;
    int n_layers;
    ccmi_syn_layer layers[CCMI_MAX_SYN_LAYERS];
    const float *params;
    int64_t param_stride;
    float *out;             /* [batch][n_out_last][h][w] */
    int64_t out_stride;
    void *workspace;        /* ccmi_syn_workspace_bytes(); may be NULL for fused architectures */
    size_t workspace_bytes;
    int batch;
} ccmi_syn_args;
size_t ccmi_syn_workspace_bytes(const ccmi_syn_args *args);
int ccmi_syn_forward_f32(const ccmi_syn_args *args, void *stream);

/* Frame post-processing of FrameEncoder.forward in eval mode (frame.py:175-183):
 * x -> clamp(round(x * (2^bitdepth-1)) / (2^bitdepth-1), 0, 1), optionally 444->420
 * nearest (yuv.py:275-299).  out420: Y [h][w] then U, V [h/2][w/2] per frame;
 * out444: [3][h][w] per frame. */
typedef struct ccmi_post_args {
    const float *in;        /* [batch][3][h][w] raw synthesis output */
    int64_t in_stride;
    int h;
    int w;
    int bitdepth;
    int yuv420;
    float *out;
    int64_t out_stride;
    int batch;
} ccmi_post_args;
int ccmi_post_f32(const ccmi_post_args *args, void *stream);

/* Fused decode tail: Upsampling.forward -> Synthesis.forward -> post-processing of
 * FrameEncoder.forward (eval) as ONE pass that never materialises the [n_grids][H][W]
 * upsampled stack nor the raw synthesis output (the composition of
 * ccmi_ups_forward_f32, ccmi_syn_forward_f32 and ccmi_post_f32, the decoder's path:
 * coolchic.py:395-437 then frame.py:175-183).  ups.out and syn.in are ignored;
 * syn.c_in must equal ups.n_grids and syn.h/w equal ups.h[0]/w[0]; ups.workspace as for
 * ccmi_ups_forward_f32.  bitdepth > 0: out receives the post-processed frame (layout
 * of ccmi_post_f32); bitdepth == 0: out receives the raw synthesis output.
 * CCMI_ERR_UNSUPPORTED when the architecture has no fused kernel (ups_k != 8,
 * pre_k != 7, or a synthesis outside the fused plan): run the three stages instead. */
typedef struct ccmi_decode_args {
    ccmi_ups_args ups;
    ccmi_syn_args syn;
    int bitdepth;
    int yuv420;
    float *out;
    int64_t out_stride;
    int stages;             /* 0 = all; bit 0: upsampling pyramid down to level 1 (into
                               ups.workspace), bit 1: the fused full-resolution kernel --
                               lets a caller time the two apart.  bit 3 (opt-in, the 7-grid
                               48-wide-head decoders): the fused kernel also evaluates the
                               level-2 -> 1 step and the pyramid stops at level 2 (same values
                               bit for bit; measured slower) */
    int head;               /* synthesis 1x1 head arithmetic, CCMI_HEAD_*: both are fp32 (the
                               MFMA form's products are exact f32 fmas, summed in another
                               order); MFMA needs 7 inputs, 48 hidden units and >= 1 3x3 layer
                               and falls back to VALU otherwise; GENERIC is a test form: the
                               runtime-width VALU head without the unrolled 48-wide kernel's
                               scaled ReLU (bitwise equal to VALU while every hidden
                               pre-activation h has 2^-94 <= |h| <= 2^32 or h <= 0) */
} ccmi_decode_args;
enum { CCMI_HEAD_DEFAULT = 0, CCMI_HEAD_VALU = 1, CCMI_HEAD_MFMA = 2, CCMI_HEAD_GENERIC = 3 };
int ccmi_decode_forward_f32(const ccmi_decode_args *args, void *stream);

/* ------------------------------------------------------------------------- */
/* Path B: fixed-point .cool decoder, bit-exact with coolchic/cpp.             */
/* ------------------------------------------------------------------------- */

/* Same contract as the reference pybind cc_decode_cpu(in, out, bitdepth, chroma,
 * verbosity) (ccdecapi_cpu.cpp:20-30, ccdecapi.cpp:673-857): 0 on success, 1 on
 * failure; bitdepth/chroma 0 = take from the header; output format by extension
 * (.yuv -> planar 420/444, otherwise PPM).  Runs on HIP device `device`. */
int ccmi_decode_file(const char *in_path, const char *out_path, int out_bitdepth,
                     int out_chroma, int verbosity, int device);

/* Throughput entry point: decode n independent in-memory .cool streams (intra
 * frames) in one batched launch sequence.  out[i] receives the same bytes the
 * reference writes for stream i (YUV if as_yuv, else PPM), out_caps[i] its
 * capacity; out_sizes[i] (optional) the byte count written.  Host buffers. */
int ccmi_decode_batch(const uint8_t *const *streams, const size_t *lens, int n,
                      uint8_t *const *out, const size_t *out_caps, size_t *out_sizes,
                      int out_bitdepth, int out_chroma, int as_yuv, void *stream);

/* Device-side stage times (ms, HIP events on the decode stream) of this thread's last
 * successful ccmi_decode_batch / ccmi_decode_file: [0] upload of streams + weights,
 * [1] ARM + CABAC latent decode, [2] upsampling + synthesis + output conversion,
 * [3] download of the decoded bytes. */
int ccmi_decode_last_timing(float *ms4);

/* What the latent decode of this thread's last ccmi_decode_* call did, per stream: flags[i]
 * ORs the CCMI_ARM_FLAG_* bits of stream i's latent grids (*n = streams reported, at most
 * cap).  TIMEOUT is an error (the call itself returned CCMI_ERR_HIP and discarded the
 * output); the other bits say which integer multiply forms ran, i.e. which paths a stream
 * exercised (the reference's int32 ARM, arm_cpu.cpp:65-95, has one form).  The chain kernel's
 * wait limit is 2^24 polls, or the environment's CCMI_DEC_SPIN_CAP (a test hook: 0 makes
 * every wait give up at once). */
#define CCMI_ARM_FLAG_TIMEOUT 1u  /* a two-wave synchronisation wait gave up: decode invalid */
#define CCMI_ARM_FLAG_Q32 2u      /* chain kernel: a |q| > 16383 switched layer 0 to 32-bit products */
#define CCMI_ARM_FLAG_W32 4u      /* an ARM weight >= 2^23: every layer in 32-bit products */
#define CCMI_ARM_FLAG_PRE32 8u    /* chain helper wave: a chunk's contexts left 22 bits (32-bit sums) */
#define CCMI_ARM_FLAG_BIG 16u     /* spec / one-latent kernels: a |q| >= 2^15, layer 0 in 32-bit */
int ccmi_decode_last_arm_flags(uint32_t *flags, int cap, int *n);

/* The integer latents of one intra stream (ARM + CABAC decode on the GPU; values, not
 * shifted), grids flattened in order: out needs sum_l h_l * w_l int32 (host buffer). */
int ccmi_decode_latents(const uint8_t *stream, size_t len, int32_t *out, size_t cap, void *stream_handle);

/* Row reductions for batched evaluation (quantize_model search, validation):
 * mode 0: out[b] = sum_i a[b][i];  mode 1: out[b] = sum_i (a[b][i] - t[b][i])^2, t_stride
 * 0 = one target for every row.  Accumulated in double.  Device pointers. */
int ccmi_row_reduce_f32(const float *a, int64_t a_stride, const float *t, int64_t t_stride, int64_t len, int batch,
                        int mode, double *out, void *stream);

/* ccmi_decode_batch with a caller-owned device workspace (no allocation inside):
 * ccmi_decode_batch_workspace_bytes() parses the streams' headers and returns the size the
 * same arguments need; the workspace must be 256-byte aligned.  ccmi_decode_batch_plan()
 * returns both the workspace size and every stream's output size (out_sizes[n]) from one
 * header-only pass (no CABAC, no GPU work).  Output buffers in pinned host memory make the
 * downloads real DMA copies that overlap the rest of the batch. */
int ccmi_decode_batch_workspace_bytes(const uint8_t *const *streams, const size_t *lens, int n,
                                      int out_bitdepth, int out_chroma, int as_yuv, size_t *bytes);
int ccmi_decode_batch_plan(const uint8_t *const *streams, const size_t *lens, int n, int out_bitdepth,
                           int out_chroma, int as_yuv, size_t *out_sizes, size_t *workspace_bytes);
int ccmi_decode_batch_ws(const uint8_t *const *streams, const size_t *lens, int n,
                         uint8_t *const *out, const size_t *out_caps, size_t *out_sizes,
                         int out_bitdepth, int out_chroma, int as_yuv, void *workspace,
                         size_t workspace_bytes, void *stream);

/* Network weights of a stream's intra frame as the decoder's fixed-point integers
 * (cc-frame-decoder.cpp:201-353, read_arm / read_ups / read_syn):
 *   arm: per hidden layer W[d][d] (out, in) then b[d]; then W_out[2][d], b_out[2]
 *        (ARM_PRECISION 8; the reference stores W transposed for its loop, :240-246);
 *   ups: n_ups full kernels of ups_k taps, then n_pre of pre_k taps (UPS_PRECISION 12,
 *        half kernels mirrored, decode_upsweights_qi :188-199);
 *   syn: per branch, per layer W[n_out][n_in][k][k] then b[n_out] (SYN precision 12).
 * counts[3] receives the three lengths; NULL buffers only query them. Host buffers. */
int ccmi_decode_weights_i32(const uint8_t *stream, size_t len, int32_t *arm, size_t arm_cap,
                            int32_t *ups, size_t ups_cap, int32_t *syn, size_t syn_cap, size_t *counts);

/* Integer upsampling (run_ups, cc-frame-decoder.cpp:572-679; ups_refine_cpu.hpp:11-79,
 * ups_upsample_cpu.hpp:12-91): latent grids (value << 8, flat in grid order) -> the
 * [n_grids][h0][w0] synthesis input at precision 12.  Device pointers. */
typedef struct ccmi_ups_i32_args {
    const int32_t *latent;  /* sum_l h[l] w[l] int32, grid l after grids 0..l-1 */
    int n_grids;
    int h[CCMI_MAX_GRIDS_PUBLIC];
    int w[CCMI_MAX_GRIDS_PUBLIC];
    const int32_t *kernels; /* the ups array of ccmi_decode_weights_i32 */
    int ups_k, n_ups, pre_k, n_pre;
    int32_t *out;           /* n_grids * h[0] * w[0] int32 */
    void *workspace;        /* ccmi_ups_workspace_bytes_i32() */
    size_t workspace_bytes;
} ccmi_ups_i32_args;
size_t ccmi_ups_workspace_bytes_i32(int n_grids, const int *h, const int *w);
int ccmi_ups_forward_i32(const ccmi_ups_i32_args *args, void *stream);

/* Integer synthesis of one branch (run_syn_branch, cc-frame-decoder.cpp:773-1042;
 * synfused_cpu.hpp:17-109, synlb_cpu.hpp:22-124, syn_cpu.hpp:21-112): [c_in][h][w] at
 * precision 12 -> [n_out][h][w].  Device pointers. */
typedef struct ccmi_syn_i32_args {
    const int32_t *in;
    int c_in, h, w;
    int n_layers;
    ccmi_syn_layer layers[CCMI_MAX_SYN_LAYERS];
    const int32_t *params;  /* one branch of the syn array of ccmi_decode_weights_i32 */
    int32_t *out;
    void *workspace;        /* ccmi_syn_workspace_bytes_i32(); 0 bytes for fused architectures */
    size_t workspace_bytes;
} ccmi_syn_i32_args;
size_t ccmi_syn_workspace_bytes_i32(const ccmi_syn_i32_args *args);
int ccmi_syn_forward_i32(const ccmi_syn_i32_args *args, void *stream);

/* Byte size of the decoded output of one stream (header parse only). */
int ccmi_decode_output_size(const uint8_t *stream, size_t len, int out_bitdepth,
                            int out_chroma, int as_yuv, size_t *size);

/* ------------------------------------------------------------------------- */
/* Path B writer: .cool encoder (the inverse of the decoder above).           */
/* ------------------------------------------------------------------------- */

/* Network parameter slots, in bitstream order (header.py:352-375, encode.py:364-390). */
enum { CCMI_NN_ARM_W = 0, CCMI_NN_ARM_B, CCMI_NN_UPS_W, CCMI_NN_UPS_B, CCMI_NN_SYN_W, CCMI_NN_SYN_B, CCMI_NN_SLOTS };

/* Everything a .cool intra frame carries besides its latent substreams: the GOP header
 * (header.py:72-117), the frame header (header.py:236-392) and the quantised network
 * integers (the values cc_code_wb_bac codes, encode.py:255-352).  Filled by
 * ccmi_cool_parse, consumed by ccmi_encode_frame. */
typedef struct ccmi_cool_desc {
    int h, w;                  /* image size */
    int bitdepth;              /* 8..16 */
    int frame_data_type;       /* 0 rgb, 1 yuv420, 2 yuv444 */
    int intra_period, p_period;
    int display_index;
    int dim_arm, n_hidden_arm;
    int n_ups, ups_k, n_pre, pre_k;
    int n_branches;
    int n_syn_layers;
    int syn_out[16], syn_ks[16];
    int syn_type[16];          /* raw byte: mode index * 16 + non-linearity index */
    int flow_gain;
    int ac_max_val_nn, ac_max_val_latent;
    int hls_sig_blksize;       /* signed: < 0 = adaptive block flags */
    int q_step_index[6];       /* CCMI_NN_* slots; -1 = slot absent (255 in the stream) */
    int expgol_count[6];       /* Exp-Golomb counts; ccmi_encode_frame: -1 = search 0..12 */
    int n_bytes_nn[6];         /* output of parse / encode */
    int n_grids;               /* latent resolutions (one 2D grid each) */
    int n_bytes_latent[8];     /* output of parse / encode */
    const int32_t *nn[6];      /* quantised integers per slot (host) */
    int nn_len[6];
} ccmi_cool_desc;

/* Parse the GOP + frame header of an intra .cool stream and decode its network
 * integers into nn_buf (nn_cap int32 slots; desc->nn[] point into it).  Host only. */
int ccmi_cool_parse(const uint8_t *stream, size_t len, ccmi_cool_desc *desc, int32_t *nn_buf, size_t nn_cap);

/* cc_code_wb_bac (ccencapi.cpp:97-177): Exp-Golomb(count) magnitudes + EP signs, one
 * CABAC substream.  use_count < 0 searches counts 0..12 for the fewest bytes (first
 * wins ties).  *len = bytes written (or needed, with CCMI_ERR_ARG, when cap is short). */
int ccmi_code_wb(const int32_t *x, int n, int use_count, uint8_t *out, size_t cap, size_t *len, int *count_used);

/* cc_decode_wb::decode_wb_continue (ccencapi.cpp:412-454) without hidden state: decode
 * n_runs consecutive runs of run_len[r] integers, run r with Exp-Golomb count
 * run_count[r], from one network substream; out receives sum(run_len) integers. */
int ccmi_decode_wb(const uint8_t *stream, size_t len, int n_runs, const int *run_len, const int *run_count, int32_t *out);

/* cc_code_latent_layer_bac (ccencapi.cpp:179-410): one latent grid, raster order, with
 * per-latent mu / log_scale in ARM fixed point (x256, the decoder's integers).  Host. */
int ccmi_code_latent_layer(const int32_t *x, const int32_t *mu, const int32_t *log_scale, int h, int w,
                           int hls_sig_blksize, uint8_t *out, size_t cap, size_t *len);

/* Integer ARM over every latent of every grid, fully parallel (the encoder side knows
 * all latents): the decoder's fixed-point arithmetic (arm_cpu.cpp:18-106 = ArmInt
 * pure_int, armint.py:80-261).  latent: int32 values [n] (grids flattened in order);
 * params: the decoder's integers, per hidden layer W[d][d] (out, in) then b[d], then
 * W_out[2][d], b_out[2].  mu / log_scale: int32 [n] (x256).  Device pointers. */
typedef struct ccmi_arm_i32_args {
    const int32_t *latent;
    int n_grids;
    int h[8], w[8];
    int dim_arm, n_hidden;
    const int32_t *params;
    int32_t *mu, *log_scale;
} ccmi_arm_i32_args;
int ccmi_arm_forward_i32(const ccmi_arm_i32_args *args, void *stream);

/* Write a whole .cool stream (GOP header, frame header, network substreams, latent
 * substreams; encode.py:113-623) for integer latents latent_dev (device, int32, grids
 * flattened).  ARM contexts run on the GPU (ccmi_arm_forward_i32); the CABAC substreams
 * are coded on host threads.  Fills desc->expgol_count / n_bytes_nn / n_bytes_latent.
 * *len = bytes written (or needed, with CCMI_ERR_ARG, when cap is short). */
int ccmi_encode_frame(ccmi_cool_desc *desc, const int32_t *latent_dev, uint8_t *out, size_t cap, size_t *len,
                      void *stream);

/* ------------------------------------------------------------------------- */
/* Encoder overfit step: training forward + backward + clip + Adam, on the GPU  */
/* ------------------------------------------------------------------------- */

/* Quantizer / noise selectors (quantizer.py:104-232). */
enum { CCMI_Q_NONE = 0, CCMI_Q_SOFTROUND_ALONE, CCMI_Q_SOFTROUND, CCMI_Q_HARDROUND, CCMI_Q_STE, CCMI_Q_TRUE_STE };
enum { CCMI_NOISE_NONE = 0, CCMI_NOISE_KUMARASWAMY, CCMI_NOISE_GAUSSIAN };

/* One optimisation step of enc/training/train.py:238-262 for `batch` independent frames
 * of the same size and architecture (each its own latents, networks and Adam state):
 *   quantize (quantizer.py) -> ARM + Laplace rate -> upsampling -> synthesis ->
 *   FrameEncoder train-mode output (frame.py:175-183: 420 nearest, clamp) ->
 *   loss = MSE + lmbda * rate_bits / (H*W) (loss.py) -> backward -> clip_grad_norm_(clip)
 *   -> Adam (torch.optim.Adam).
 * params per frame (float32): ARM (as ccmi_arm_args), then the trainable HALF kernels of
 * the n_ups upsampling filters ((ups_k+1)/2 taps each, upsampling.py:46-68), then the
 * n_pre refine filters ((pre_k+1)/2 each), then the synthesis (as ccmi_syn_args).
 * Supported synthesis: a 1x1 head of 2 non-residual layers (C -> hid <= 64 -> 3), then
 * 0..3 3x3 layers 3 -> 3 (replicate padding).  Adam moments: [batch][latent_stride +
 * param_stride], each row N latents then P parameters.  grad_out rows: [N + P], same
 * order.  target: 444 [3][H][W] or 420 Y[H][W], U, V[H/2][W/2]. */
typedef struct ccmi_train_args {
    int batch;
    int n_grids;
    int h[CCMI_MAX_GRIDS_PUBLIC];
    int w[CCMI_MAX_GRIDS_PUBLIC];
    int dim_arm, n_hidden;
    int ups_k, n_ups, pre_k, n_pre;
    int n_syn_layers;
    ccmi_syn_layer syn[CCMI_MAX_SYN_LAYERS];
    float gain;
    float *latent;          /* [batch][latent_stride], updated in place */
    int64_t latent_stride;
    float *params;          /* [batch][param_stride], updated in place */
    int64_t param_stride;
    float *adam_m, *adam_v; /* [batch][latent_stride + param_stride] */
    const float *target;    /* [batch][target_stride] */
    int64_t target_stride;
    int yuv420;
    int quantizer, noise;   /* CCMI_Q_*, CCMI_NOISE_* */
    float temperature, noise_param, lmbda;
    float lr, beta1, beta2, eps, clip;  /* clip <= 0: no gradient clipping */
    int step;               /* Adam step t >= 1 (bias correction) */
    uint64_t seed;          /* noise: counter-based RNG keyed by (seed, step, frame, index) */
    const float *noise_in;  /* optional [batch][latent_stride]: additive noise used as is */
    float *grad_out;        /* optional [batch][N + P]: raw gradients (before clipping) */
    float *loss_out;        /* optional [batch][4]: loss, mse, rate_bits, grad_norm (forward_only:
                               grad_norm 0; mse 0 unless a target is given, target_stride > 0) */
    int update;             /* 0: loss and gradients only; 1: Adam on everything; 2: Adam on the
                               latents only (optimized_module ["latent"]; the norm still covers all) */
    void *workspace;        /* ccmi_train_workspace_bytes() */
    size_t workspace_bytes;
    /* autograd use (torch.autograd.Function around the train-mode forward): */
    int forward_only;       /* 1: run the training forward only and write raw_out / rate_out */
    float *raw_out;         /* optional [batch][3][H][W]: raw synthesis output of the forward */
    float *rate_out;        /* optional [batch][N]: per-latent rate (bits) of the forward */
    const float *grad_raw;  /* optional [batch][3][H][W]: d loss / d raw output, used instead of
                               the built-in MSE term (whose value then reads 0 in loss_out) */
    const float *grad_rate; /* optional [batch][N]: d loss / d rate per latent, used instead of
                               the built-in lmbda / (H W) */
    const int32_t *adam_steps; /* optional device [batch]: each frame's own Adam step (overrides
                               `step`; a frame whose optimizer state was reloaded from its best
                               record, train.py:226-236); a step <= 0 leaves that frame unchanged:
                               neither its parameters nor its Adam moments are written */
    int32_t *step_counters; /* optional device [batch]: +1 per frame at the start of an update
                               step (the caller's per-frame step counts kept on the device without
                               a launch of its own; may alias adam_steps, which then reads the
                               incremented value) */
} ccmi_train_args;
size_t ccmi_train_param_count(const ccmi_train_args *args);
size_t ccmi_train_workspace_bytes(const ccmi_train_args *args);
int ccmi_train_step(const ccmi_train_args *args, void *stream);

/* quantize (quantizer.py:116-232) of n values x (already multiplied by the encoder gain):
 * y = Q(x) and dy = dQ/dx as the reference's autograd sees it (softround derivative for
 * "ste", 1 for "true_ste" and "none", 0 for "hardround"); noise: optional [n] additive
 * noise (the reference draws it with torch.rand_like / randn_like).  Device pointers. */
int ccmi_quantize_f32(const float *x, int64_t n, int quantizer, float temperature, const float *noise, float *y,
                      float *dy, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CCMI_H */
