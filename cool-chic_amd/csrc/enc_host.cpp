// enc_host.cpp -- path B writer: the .cool encoder side (host C++ + the GPU integer ARM).
//
// Reference (what each piece reproduces byte for byte):
//   ccmi_code_wb            cc_code_wb_bac            ccencapi.cpp:97-177
//   ccmi_code_latent_layer  cc_code_latent_layer_bac  ccencapi.cpp:179-410 (code_val :62-93)
//   GOP / frame headers     write_gop_header / write_frame_header  header.py:72-117, :236-392
//   ccmi_encode_frame       encode_frame              encode.py:221-623 (substream order
//                           :580-623: header, arm/ups/syn weight+bias, latent grids)
//   ccmi_cool_parse         read_gop_header / read_frame_header cc-bitstream.cpp:58-275 and the
//                           raw Exp-Golomb integers of decode_weights_qi cc-frame-decoder.cpp:157-178
// Unlike the reference (which exit()s), every failure returns a CCMI_ERR_* code.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "dec_internal.h"
#include "enc_cabac.h"

namespace ccmi {

namespace {

constexpr uint8_t k_ctx_idx[17 * 50 * 5] = {
#include "ccmi_ctx_table.inc"
};

// get_val_mu_indicies (cc-contexts.h:20-48): mu rounded to an integer, mu sub-index, sig index.
void mu_sig_index(int32_t mu, int32_t ls, int32_t &mu_round, int &mi, int &si)
{
    const int32_t mr = mu >= 0 ? ((mu + 128) >> 8) << 8 : -(((-mu + 128) >> 8) << 8);
    int32_t m = (mu - mr) * 16;
    m = m >= 0 ? (m + 128) >> 8 : -((-m + 128) >> 8);
    mi = m + 8;
    const int32_t l = ls + 256;
    int s = l < 0 ? 0 : (l * 5 + 128) >> 8;
    si = s > 49 ? 49 : s;
    mu_round = mr >> 8;
}

// code_val (ccencapi.cpp:62-93): gt0..gt3 flags against static contexts, EG0 escape, sign.
void code_val(CabacEnc &c, const uint8_t *ctx, int32_t v)
{
    const uint32_t a = (uint32_t)(v < 0 ? -(int64_t)v : v);
    if (a == 0) {
        c.bin_static(ctx[0], 0);
        return;
    }
    c.bin_static(ctx[0], 1);
    if (a <= 1) {
        c.bin_static(ctx[1], 0);
    } else {
        c.bin_static(ctx[1], 1);
        if (a <= 2) {
            c.bin_static(ctx[2], 0);
        } else {
            c.bin_static(ctx[2], 1);
            if (a <= 3) {
                c.bin_static(ctx[3], 0);
            } else {
                c.bin_static(ctx[3], 1);
                c.expgolomb(a - 4, 0);
            }
        }
    }
    c.bin_static(ctx[4], v < 0 ? 1 : 0);
}

std::vector<uint8_t> code_wb(const int32_t *x, int n, int count)
{
    CabacEnc c;
    c.start();
    for (int i = 0; i < n; ++i) {
        const uint32_t a = (uint32_t)(x[i] < 0 ? -(int64_t)x[i] : x[i]);
        c.expgolomb(a, (uint32_t)count);
        if (x[i] != 0) c.ep(x[i] < 0 ? 1 : 0);
    }
    std::vector<uint8_t> out = c.close();
    if (!c.ok) out.clear();
    return out;
}

// Best count for a weight vector (the reference's search over 0..12, first wins ties).
bool code_wb_best(const int32_t *x, int n, int use_count, std::vector<uint8_t> &best, int &best_count)
{
    const int lo = use_count >= 0 ? use_count : 0, hi = use_count >= 0 ? use_count : 12;
    best_count = -1;
    for (int k = lo; k <= hi; ++k) {
        std::vector<uint8_t> b = code_wb(x, n, k);
        if (b.empty()) continue; // Exp-Golomb overflow at this count
        if (best_count < 0 || b.size() < best.size()) {
            best = std::move(b);
            best_count = k;
        }
    }
    return best_count >= 0;
}

bool code_latent_layer(const int32_t *xs, const int32_t *mus, const int32_t *lss, int h, int w, int blk_signed,
                       std::vector<uint8_t> &out)
{
    const bool update = blk_signed < 0;
    const int blk = blk_signed < 0 ? -blk_signed : blk_signed;
    int shift = 0;
    while ((1 << shift) < blk) ++shift;
    int nby = 1, nbx = 1;
    if (blk != 0) {
        nby = (h + blk - 1) / blk;
        nbx = (w + blk - 1) / blk;
    }
    const int nblk = nby * nbx;
    std::vector<uint8_t> flat(nblk, 0);
    CabacEnc c;
    c.start();
    if (nblk > 1) {
        int n_zero = 0, n_flat = 0;
        for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
                const int32_t first = xs[(size_t)by * blk * w + (size_t)bx * blk];
                bool s = false, f = true;
                for (int y = by * blk; y < (by + 1) * blk && y < h; ++y)
                    for (int x = bx * blk; x < (bx + 1) * blk && x < w; ++x) {
                        const int32_t v = xs[(size_t)y * w + x];
                        s = s || v != 0;
                        f = f && v == first;
                    }
                flat[by * nbx + bx] = f;
                if (!s) ++n_zero;
                else if (f) ++n_flat;
            }
        // block significance is never signalled any more (ccencapi.cpp:260-268): every block
        // is significant and zero blocks count as flat
        c.ep(0);
        n_flat += n_zero;
        if (n_flat <= nblk / 20) {
            c.ep(0);
            std::fill(flat.begin(), flat.end(), 0);
        } else {
            c.ep(1);
            Model m;
            m.init(65); // PROBA_50_STATE (cc-contexts.h:18)
            for (int i = 0; i < nblk; ++i) {
                if (update) c.bin_adaptive(m, flat[i]);
                else c.ep(flat[i]);
            }
        }
    }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            if (blk > 0 && flat[(y >> shift) * nbx + (x >> shift)] && ((y % blk) != 0 || (x % blk) != 0)) continue;
            const size_t i = (size_t)y * w + x;
            int32_t mr;
            int mi, si;
            mu_sig_index(mus[i], lss[i], mr, mi, si);
            code_val(c, &k_ctx_idx[(mi * 50 + si) * 5], (int32_t)((uint32_t)xs[i] - (uint32_t)mr));
        }
    out = c.close();
    return c.ok;
}

int copy_out(const std::vector<uint8_t> &b, uint8_t *out, size_t cap, size_t *len)
{
    if (len) *len = b.size();
    if (!out || cap < b.size()) return ccmi_set_error(CCMI_ERR_ARG, "output buffer of %zu bytes, need %zu", cap, b.size());
    if (!b.empty()) memcpy(out, b.data(), b.size());
    return CCMI_OK;
}

// ---- headers
struct Reader {
    const uint8_t *p;
    size_t n, pos;
    bool err;
    int u(int nb)
    {
        if (pos + (size_t)nb > n) {
            err = true;
            return 0;
        }
        int v = 0;
        for (int i = 0; i < nb; ++i) v = (v << 8) | p[pos++];
        return v;
    }
};

void put(std::vector<uint8_t> &o, uint32_t v, int nb)
{
    for (int i = nb - 1; i >= 0; --i) o.push_back((uint8_t)(v >> (8 * i)));
}

bool slot_has_extras(const ccmi_cool_desc &d, int k) { return (k & 1) == 0 || d.q_step_index[k] >= 0; }

// Number of integers per network slot for the architecture in `d` (read_arm / read_ups /
// read_syn, cc-frame-decoder.cpp:201-353).
void slot_lengths(const ccmi_cool_desc &d, int len[CCMI_NN_SLOTS])
{
    const int a = d.dim_arm;
    len[CCMI_NN_ARM_W] = d.n_hidden_arm * a * a + 2 * a;
    len[CCMI_NN_ARM_B] = d.n_hidden_arm * a + 2;
    len[CCMI_NN_UPS_W] = d.n_ups * ((d.ups_k + 1) / 2) + d.n_pre * ((d.pre_k + 1) / 2);
    len[CCMI_NN_UPS_B] = 0;
    int nw = d.n_branches > 1 ? d.n_branches : 0, nb = 0, c = d.n_grids;
    for (int l = 0; l < d.n_syn_layers; ++l) {
        nw += d.n_branches * c * d.syn_ks[l] * d.syn_ks[l] * d.syn_out[l];
        nb += d.n_branches * d.syn_out[l];
        c = d.syn_out[l];
    }
    len[CCMI_NN_SYN_W] = nw;
    len[CCMI_NN_SYN_B] = nb;
}

int check_desc(const ccmi_cool_desc &d)
{
    if (d.h < 1 || d.w < 1 || d.h > 65535 || d.w > 65535) return ccmi_set_error(CCMI_ERR_ARG, "encode: image size %dx%d", d.h, d.w);
    if (d.bitdepth < 8 || d.bitdepth > 16 || d.frame_data_type < 0 || d.frame_data_type > 2)
        return ccmi_set_error(CCMI_ERR_ARG, "encode: bitdepth %d / frame type %d", d.bitdepth, d.frame_data_type);
    if (d.intra_period != 0) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "encode: inter frames are outside this path");
    if (d.dim_arm != 8 && d.dim_arm != 16 && d.dim_arm != 24 && d.dim_arm != 32)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "encode: dim_arm %d", d.dim_arm);
    if (d.n_hidden_arm < 0 || d.n_hidden_arm > 4) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "encode: %d ARM hidden layers", d.n_hidden_arm);
    if (d.n_grids < 2 || d.n_grids > CCMI_MAX_GRIDS) return ccmi_set_error(CCMI_ERR_ARG, "encode: %d latent grids", d.n_grids);
    if (d.n_syn_layers < 1 || d.n_syn_layers > 16 || d.n_branches < 1 || d.n_branches > 8)
        return ccmi_set_error(CCMI_ERR_ARG, "encode: synthesis with %d layers / %d branches", d.n_syn_layers, d.n_branches);
    if (d.q_step_index[CCMI_NN_ARM_B] < 0 || d.q_step_index[CCMI_NN_ARM_W] < 0 || d.q_step_index[CCMI_NN_ARM_W] > 8 ||
        d.q_step_index[CCMI_NN_ARM_B] > 16)
        return ccmi_set_error(CCMI_ERR_ARG, "encode: ARM q-step indices %d/%d", d.q_step_index[0], d.q_step_index[1]);
    if (d.hls_sig_blksize < -128 || d.hls_sig_blksize > 127) return ccmi_set_error(CCMI_ERR_ARG, "encode: hls_sig_blksize");
    int len[CCMI_NN_SLOTS];
    slot_lengths(d, len);
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) {
        if (!slot_has_extras(d, k)) continue;
        if (d.nn_len[k] != len[k]) return ccmi_set_error(CCMI_ERR_ARG, "encode: network slot %d has %d integers, architecture needs %d", k, d.nn_len[k], len[k]);
        if (len[k] > 0 && !d.nn[k]) return ccmi_set_error(CCMI_ERR_ARG, "encode: network slot %d is NULL", k);
    }
    return CCMI_OK;
}

std::vector<uint8_t> gop_header(const ccmi_cool_desc &d)
{
    std::vector<uint8_t> o;
    put(o, 9, 2);
    put(o, (uint32_t)d.h, 2);
    put(o, (uint32_t)d.w, 2);
    put(o, (uint32_t)((d.bitdepth - 8) * 16 + d.frame_data_type), 1);
    put(o, (uint32_t)d.intra_period, 1);
    put(o, (uint32_t)d.p_period, 1);
    return o;
}

std::vector<uint8_t> frame_header(const ccmi_cool_desc &d)
{
    std::vector<uint8_t> o;
    put(o, 0, 2); // patched below
    put(o, (uint32_t)d.display_index, 1);
    put(o, (uint32_t)((d.dim_arm / 8) * 16 + d.n_hidden_arm), 1);
    put(o, (uint32_t)((d.n_ups << 4) | d.ups_k), 1);
    put(o, (uint32_t)((d.n_pre << 4) | d.pre_k), 1);
    put(o, (uint32_t)d.n_branches, 1);
    put(o, (uint32_t)d.n_syn_layers, 1);
    for (int l = 0; l < d.n_syn_layers; ++l) {
        put(o, (uint32_t)d.syn_out[l], 1);
        put(o, (uint32_t)d.syn_ks[l], 1);
        put(o, (uint32_t)d.syn_type[l], 1);
    }
    put(o, (uint32_t)d.flow_gain, 1);
    put(o, (uint32_t)d.ac_max_val_nn, 2);
    put(o, (uint32_t)d.ac_max_val_latent, 2);
    put(o, (uint32_t)(uint8_t)(int8_t)d.hls_sig_blksize, 1);
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) put(o, d.q_step_index[k] < 0 ? 255u : (uint32_t)d.q_step_index[k], 1);
    for (int k = 0; k < CCMI_NN_SLOTS; ++k)
        if (slot_has_extras(d, k)) put(o, (uint32_t)d.expgol_count[k], 1);
    for (int k = 0; k < CCMI_NN_SLOTS; ++k)
        if (slot_has_extras(d, k)) put(o, (uint32_t)d.n_bytes_nn[k], 2);
    put(o, (uint32_t)d.n_grids, 1);
    put(o, (uint32_t)d.n_grids, 1); // one 2D grid per resolution
    for (int l = 0; l < d.n_grids; ++l) put(o, 1, 1);
    for (int l = 0; l < d.n_grids; ++l) put(o, (uint32_t)d.n_bytes_latent[l], 3);
    o[0] = (uint8_t)(o.size() >> 8);
    o[1] = (uint8_t)o.size();
    return o;
}

} // namespace

// Decoder-side ARM integers from the coded ones (read_arm, cc-frame-decoder.cpp:201-258):
// per hidden layer W then b, then W_out, b_out; weights << q_w, biases << q_b.
void arm_params_from_coded(const ccmi_cool_desc &d, std::vector<int32_t> &out)
{
    const int a = d.dim_arm, sw = d.q_step_index[CCMI_NN_ARM_W], sb = d.q_step_index[CCMI_NN_ARM_B];
    out.assign((size_t)d.n_hidden_arm * (a * a + a) + 2 * a + 2, 0);
    const int32_t *W = d.nn[CCMI_NN_ARM_W], *B = d.nn[CCMI_NN_ARM_B];
    size_t p = 0;
    for (int l = 0; l <= d.n_hidden_arm; ++l) {
        const int nout = l < d.n_hidden_arm ? a : 2;
        for (int i = 0; i < nout * a; ++i) out[p++] = (int32_t)((uint32_t)*W++ << sw);
        for (int i = 0; i < nout; ++i) out[p++] = (int32_t)((uint32_t)*B++ << sb);
    }
}

int launch_arm_i32(const ccmi_arm_i32_args &a, hipStream_t s);

} // namespace ccmi

using namespace ccmi;

extern "C" int ccmi_code_wb(const int32_t *x, int n, int use_count, uint8_t *out, size_t cap, size_t *len,
                            int *count_used)
{
    if ((!x && n > 0) || n < 0 || use_count > 30) return ccmi_set_error(CCMI_ERR_ARG, "code_wb: bad argument");
    std::vector<uint8_t> best;
    int k;
    if (!code_wb_best(x, n, use_count, best, k)) return ccmi_set_error(CCMI_ERR_ARG, "code_wb: Exp-Golomb code longer than 32 bins");
    if (count_used) *count_used = k;
    return copy_out(best, out, cap, len);
}

extern "C" int ccmi_decode_wb(const uint8_t *bs, size_t n, int n_runs, const int *run_len, const int *run_count,
                              int32_t *out)
{
    if (!bs || n_runs < 0 || (n_runs > 0 && (!run_len || !run_count || !out))) return ccmi_set_error(CCMI_ERR_ARG, "decode_wb: bad argument");
    Cabac<HostBytes> c;
    c.src = HostBytes{bs, (uint32_t)n, 0};
    c.start();
    for (int r = 0; r < n_runs; ++r) {
        if (run_len[r] < 0 || run_count[r] < 0 || run_count[r] > 30) return ccmi_set_error(CCMI_ERR_ARG, "decode_wb: run %d", r);
        for (int i = 0; i < run_len[r]; ++i) {
            int32_t v = c.expgolomb(run_count[r]);
            if (v != 0 && c.ep()) v = -v;
            *out++ = v;
        }
    }
    return CCMI_OK;
}

extern "C" int ccmi_code_latent_layer(const int32_t *x, const int32_t *mu, const int32_t *log_scale, int h, int w,
                                      int hls_sig_blksize, uint8_t *out, size_t cap, size_t *len)
{
    if (!x || !mu || !log_scale || h < 1 || w < 1) return ccmi_set_error(CCMI_ERR_ARG, "code_latent_layer: bad argument");
    std::vector<uint8_t> b;
    if (!code_latent_layer(x, mu, log_scale, h, w, hls_sig_blksize, b))
        return ccmi_set_error(CCMI_ERR_ARG, "code_latent_layer: latent too large for Exp-Golomb coding");
    return copy_out(b, out, cap, len);
}

extern "C" int ccmi_cool_parse(const uint8_t *bs, size_t n, ccmi_cool_desc *d, int32_t *nn_buf, size_t nn_cap)
{
    if (!bs || !d) return ccmi_set_error(CCMI_ERR_ARG, "cool_parse: null argument");
    memset(d, 0, sizeof *d);
    Reader r{bs, n, 0, false};
    r.u(2);
    d->h = r.u(2);
    d->w = r.u(2);
    int raw = r.u(1);
    d->bitdepth = (raw >> 4) + 8;
    d->frame_data_type = raw & 0xF;
    d->intra_period = r.u(1);
    d->p_period = r.u(1);
    if (r.err) return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: truncated GOP header");
    if (d->intra_period != 0) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "cool_parse: inter frames are outside this path");
    const size_t fh_start = r.pos;
    const int fh_bytes = r.u(2);
    d->display_index = r.u(1);
    raw = r.u(1);
    d->dim_arm = 8 * (raw >> 4);
    d->n_hidden_arm = raw & 0xF;
    raw = r.u(1);
    d->n_ups = raw >> 4;
    d->ups_k = raw & 0xF;
    raw = r.u(1);
    d->n_pre = raw >> 4;
    d->pre_k = raw & 0xF;
    d->n_branches = r.u(1);
    d->n_syn_layers = r.u(1);
    if (r.err || d->n_syn_layers < 1 || d->n_syn_layers > 16) return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: synthesis layer count");
    for (int l = 0; l < d->n_syn_layers; ++l) {
        d->syn_out[l] = r.u(1);
        d->syn_ks[l] = r.u(1);
        d->syn_type[l] = r.u(1);
    }
    d->flow_gain = r.u(1);
    d->ac_max_val_nn = r.u(2);
    d->ac_max_val_latent = r.u(2);
    d->hls_sig_blksize = (signed char)r.u(1);
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) {
        d->q_step_index[k] = r.u(1);
        if ((k & 1) && d->q_step_index[k] == 255) d->q_step_index[k] = -1;
    }
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) d->expgol_count[k] = slot_has_extras(*d, k) ? r.u(1) : -1;
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) d->n_bytes_nn[k] = slot_has_extras(*d, k) ? r.u(2) : 0;
    d->n_grids = r.u(1);
    const int n2d = r.u(1);
    if (r.err || d->n_grids < 2 || d->n_grids > CCMI_MAX_GRIDS || n2d != d->n_grids)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: latent grid counts %d/%d", d->n_grids, n2d);
    for (int l = 0; l < d->n_grids; ++l)
        if (r.u(1) != 1) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "cool_parse: only 1 feature per latent resolution");
    for (int l = 0; l < d->n_grids; ++l) d->n_bytes_latent[l] = r.u(3);
    if (r.err || r.pos - fh_start != (size_t)fh_bytes)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: frame header size %d, parsed %zu", fh_bytes, r.pos - fh_start);

    int len[CCMI_NN_SLOTS];
    slot_lengths(*d, len);
    size_t need = 0;
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) need += (size_t)len[k];
    if (!nn_buf || nn_cap < need) return ccmi_set_error(CCMI_ERR_ARG, "cool_parse: network buffer of %zu ints, need %zu", nn_cap, need);
    size_t pos = r.pos;
    int32_t *q = nn_buf;
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) {
        const size_t nb = (size_t)d->n_bytes_nn[k];
        if (pos + nb > n) return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: truncated network substream %d", k);
        d->nn[k] = q;
        d->nn_len[k] = slot_has_extras(*d, k) ? len[k] : 0;
        Cabac<HostBytes> c;
        c.src = HostBytes{bs + pos, (uint32_t)nb, 0};
        c.start();
        for (int i = 0; i < d->nn_len[k]; ++i) {
            int32_t v = c.expgolomb(d->expgol_count[k]);
            if (v != 0 && c.ep()) v = -v;
            *q++ = v;
        }
        pos += nb;
    }
    for (int l = 0; l < d->n_grids; ++l) pos += (size_t)d->n_bytes_latent[l];
    if (pos > n) return ccmi_set_error(CCMI_ERR_BITSTREAM, "cool_parse: truncated latent substreams");
    return CCMI_OK;
}

extern "C" int ccmi_encode_frame(ccmi_cool_desc *d, const int32_t *latent_dev, uint8_t *out, size_t cap, size_t *len,
                                 void *stream)
{
    if (!d || !latent_dev) return ccmi_set_error(CCMI_ERR_ARG, "encode_frame: null argument");
    if (int rc = check_desc(*d)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);

    // ---- latent grid geometry (each halves, rounding up: coolchic.py:101-110)
    int lh[CCMI_MAX_GRIDS], lw[CCMI_MAX_GRIDS];
    size_t off[CCMI_MAX_GRIDS + 1];
    off[0] = 0;
    for (int l = 0, hh = d->h, ww = d->w; l < d->n_grids; ++l, hh = (hh + 1) / 2, ww = (ww + 1) / 2) {
        lh[l] = hh;
        lw[l] = ww;
        off[l + 1] = off[l] + (size_t)hh * ww;
    }
    const size_t N = off[d->n_grids];

    // ---- ARM contexts on the GPU: mu / log_scale of every latent at once
    std::vector<int32_t> arm;
    arm_params_from_coded(*d, arm);
    int32_t *dev = nullptr;
    const size_t arm_bytes = (arm.size() * 4 + 255) / 256 * 256;
    CCMI_HIP_CHECK(hipMalloc(&dev, arm_bytes + 2 * N * 4));
    struct Free {
        int32_t *p;
        ~Free() { if (p) (void)hipFree(p); }
    } guard{dev};
    int32_t *d_arm = dev, *d_mu = dev + arm_bytes / 4, *d_ls = d_mu + N;
    CCMI_HIP_CHECK(hipMemcpyAsync(d_arm, arm.data(), arm.size() * 4, hipMemcpyHostToDevice, s));
    ccmi_arm_i32_args a{};
    a.latent = latent_dev;
    a.n_grids = d->n_grids;
    for (int l = 0; l < d->n_grids; ++l) {
        a.h[l] = lh[l];
        a.w[l] = lw[l];
    }
    a.dim_arm = d->dim_arm;
    a.n_hidden = d->n_hidden_arm;
    a.params = d_arm;
    a.mu = d_mu;
    a.log_scale = d_ls;
    if (int rc = launch_arm_i32(a, s)) return rc;
    std::vector<int32_t> xs(N), mu(N), ls(N);
    CCMI_HIP_CHECK(hipMemcpyAsync(xs.data(), latent_dev, N * 4, hipMemcpyDeviceToHost, s));
    CCMI_HIP_CHECK(hipMemcpyAsync(mu.data(), d_mu, N * 4, hipMemcpyDeviceToHost, s));
    CCMI_HIP_CHECK(hipMemcpyAsync(ls.data(), d_ls, N * 4, hipMemcpyDeviceToHost, s));

    // ---- network substreams (host, while the ARM runs)
    std::vector<uint8_t> nn_bytes[CCMI_NN_SLOTS];
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) {
        if (!slot_has_extras(*d, k) || d->nn_len[k] == 0) {
            d->n_bytes_nn[k] = 0;
            if (slot_has_extras(*d, k) && d->expgol_count[k] < 0) d->expgol_count[k] = 0;
            continue;
        }
        int used;
        if (!code_wb_best(d->nn[k], d->nn_len[k], d->expgol_count[k], nn_bytes[k], used))
            return ccmi_set_error(CCMI_ERR_ARG, "encode_frame: network slot %d does not fit Exp-Golomb coding", k);
        d->expgol_count[k] = used;
        d->n_bytes_nn[k] = (int)nn_bytes[k].size();
        if (nn_bytes[k].size() > 65535) return ccmi_set_error(CCMI_ERR_ARG, "encode_frame: network slot %d needs %zu bytes", k, nn_bytes[k].size());
    }
    CCMI_HIP_CHECK(hipStreamSynchronize(s));

    // ---- latent substreams: one host thread per grid (independent CABAC streams)
    std::vector<uint8_t> lat_bytes[CCMI_MAX_GRIDS];
    bool ok[CCMI_MAX_GRIDS];
    {
        std::vector<std::thread> th;
        for (int l = 0; l < d->n_grids; ++l) {
            th.emplace_back([&, l] {
                const int32_t *x = xs.data() + off[l];
                bool any = false;
                for (size_t i = 0; i < (size_t)lh[l] * lw[l] && !any; ++i) any = x[i] != 0;
                ok[l] = true;
                if (any) // an all-zero grid is sent as an empty substream (encode.py:530-538)
                    ok[l] = code_latent_layer(x, mu.data() + off[l], ls.data() + off[l], lh[l], lw[l], d->hls_sig_blksize,
                                              lat_bytes[l]);
            });
        }
        for (auto &t : th) t.join();
    }
    for (int l = 0; l < d->n_grids; ++l) {
        if (!ok[l]) return ccmi_set_error(CCMI_ERR_ARG, "encode_frame: latent grid %d too large for Exp-Golomb coding", l);
        if (lat_bytes[l].size() > 0xFFFFFF) return ccmi_set_error(CCMI_ERR_ARG, "encode_frame: latent grid %d needs %zu bytes", l, lat_bytes[l].size());
        d->n_bytes_latent[l] = (int)lat_bytes[l].size();
    }

    // ---- assemble: GOP header, frame header, networks, latents (encode.py:580-623)
    std::vector<uint8_t> o = gop_header(*d);
    const std::vector<uint8_t> fh = frame_header(*d);
    o.insert(o.end(), fh.begin(), fh.end());
    for (int k = 0; k < CCMI_NN_SLOTS; ++k) o.insert(o.end(), nn_bytes[k].begin(), nn_bytes[k].end());
    for (int l = 0; l < d->n_grids; ++l) o.insert(o.end(), lat_bytes[l].begin(), lat_bytes[l].end());
    return copy_out(o, out, cap, len);
}

extern "C" int ccmi_arm_forward_i32(const ccmi_arm_i32_args *a, void *stream)
{
    if (!a || !a->latent || !a->params || !a->mu || !a->log_scale) return ccmi_set_error(CCMI_ERR_ARG, "arm_i32: null argument");
    if (a->n_grids < 1 || a->n_grids > CCMI_MAX_GRIDS) return ccmi_set_error(CCMI_ERR_ARG, "arm_i32: n_grids %d", a->n_grids);
    for (int l = 0; l < a->n_grids; ++l)
        if (a->h[l] < 1 || a->w[l] < 1) return ccmi_set_error(CCMI_ERR_ARG, "arm_i32: grid %d is %dx%d", l, a->h[l], a->w[l]);
    if (a->n_hidden < 0 || a->n_hidden > 4) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "arm_i32: %d hidden layers", a->n_hidden);
    return launch_arm_i32(*a, static_cast<hipStream_t>(stream));
}
