// dec_host.cpp -- path B host side: .cool parsing, network weight decoding (CABAC
// Exp-Golomb, tiny), device memory planning and the decode C-ABI entry points.
//
// Reference: cc-bitstream.cpp:58-275 (headers, chunking), cc-frame-decoder.cpp:157-353
// (read_arm / read_ups / read_syn and the Q_STEP_*_SHIFT tables :28-108), ccdecapi.cpp
// :673-857 (cc_decode_* driver, output formats).  All latent-layer decoding, upsampling,
// synthesis and output conversion run on the GPU (dec_kernels.hip).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "ccmi_cabac.h"
#include "dec_internal.h"

namespace ccmi {

namespace {

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
    const uint8_t *take(int nb)
    {
        if (nb < 0 || pos + (size_t)nb > n) {
            err = true;
            return nullptr;
        }
        const uint8_t *q = p + pos;
        pos += (size_t)nb;
        return q;
    }
};

struct Lqi {
    int qw, qb, sw, sb, nw, nb;
};

// Exp-Golomb magnitude + EP sign, then << (precision - q_step_shift)  (decode_weights_qi)
bool read_weights(Cabac<HostBytes> &c, int k, int n, int shift, int prec, int32_t *dst)
{
    if (prec < shift) return false;
    for (int i = 0; i < n; ++i) {
        int32_t v = c.expgolomb(k);
        if (v != 0 && c.ep()) v = -v;
        dst[i] = (int32_t)((uint32_t)v << (prec - shift));
    }
    return true;
}

Cabac<HostBytes> cabac_on(const uint8_t *p, int n)
{
    Cabac<HostBytes> c;
    c.src = HostBytes{p, (uint32_t)(n > 0 ? n : 0), 0};
    c.start();
    return c;
}

} // namespace

int parse_frame_header(const uint8_t *bs, size_t n, FrameHost &f)
{
    Reader r{bs, n, 0, false};
    r.u(2);
    f.h = r.u(2);
    f.w = r.u(2);
    int raw = r.u(1);
    f.bitdepth = (raw >> 4) + 8;
    f.frame_data_type = raw & 0xF;
    f.intra_period = r.u(1);
    r.u(1); // p_period
    if (r.err || f.h < 1 || f.w < 1) return ccmi_set_error(CCMI_ERR_BITSTREAM, "truncated GOP header");
    if (f.intra_period != 0)
        return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "inter (P/B) frames are outside the decoded hot path");
    r.u(2); // frame header size
    r.u(1); // display index
    raw = r.u(1);
    f.dim_arm = 8 * (raw >> 4);
    f.n_hidden = raw & 0xF;
    raw = r.u(1);
    f.n_ups = raw >> 4;
    f.ups_ks = raw & 0xF;
    raw = r.u(1);
    f.n_pre = raw >> 4;
    f.pre_ks = raw & 0xF;
    f.n_branches = r.u(1);
    const int n_syn = r.u(1);
    if (r.err || n_syn < 1 || n_syn > CCMI_MAX_SYN_LAYERS)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "bad synthesis layer count %d", n_syn);
    f.layers.resize(n_syn);
    for (auto &L : f.layers) {
        L.n_out = r.u(1);
        L.ks = r.u(1);
        raw = r.u(1);
        L.residual = (raw >> 4) != 0;
        L.relu = (raw & 0xF) != 0;
    }
    r.u(1); // flow gain
    r.u(2); // ac_max_val_nn
    r.u(2); // ac_max_val_latent
    f.sig_blk = (signed char)r.u(1);
    Lqi arm{}, ups{}, syn{};
    Lqi *q[3] = {&arm, &ups, &syn};
    static_assert(sizeof(Lqi) == sizeof(f.lqi[0]), "Lqi layout");
    for (auto *x : q) {
        x->qw = r.u(1);
        x->qb = r.u(1);
        if (x->qb == 255) x->qb = -1;
    }
    for (auto *x : q) {
        x->sw = r.u(1);
        x->sb = x->qb < 0 ? -1 : r.u(1);
    }
    for (auto *x : q) {
        x->nw = r.u(2);
        x->nb = x->qb < 0 ? -1 : r.u(2);
    }
    f.n_layers = r.u(1);
    const int n_grid = r.u(1);
    if (r.err || f.n_layers < 2 || f.n_layers > CCMI_MAX_GRIDS || n_grid != f.n_layers)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "bad latent layer count %d/%d", f.n_layers, n_grid);
    for (int i = 0; i < f.n_layers; ++i)
        if (r.u(1) != 1) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "only 1 feature per latent resolution");
    for (int i = 0; i < f.n_layers; ++i) f.lat_n[i] = (uint32_t)r.u(3);
    if (r.err) return ccmi_set_error(CCMI_ERR_BITSTREAM, "truncated frame header");
    f.wbytes[0] = r.take(arm.nw);
    f.wbytes[1] = r.take(arm.nb < 0 ? 0 : arm.nb);
    f.wbytes[2] = r.take(ups.nw);
    r.take(ups.nb < 0 ? 0 : ups.nb);
    f.wbytes[3] = r.take(syn.nw);
    f.wbytes[4] = r.take(syn.nb < 0 ? 0 : syn.nb);
    for (int i = 0; i < f.n_layers; ++i) f.lat_bytes[i] = r.take((int)f.lat_n[i]);
    if (r.err) return ccmi_set_error(CCMI_ERR_BITSTREAM, "truncated stream (payload shorter than the header says)");
    for (int l = 0, hh = f.h, ww = f.w; l < f.n_layers; ++l, hh = (hh + 1) / 2, ww = (ww + 1) / 2) {
        f.lh[l] = hh;
        f.lw[l] = ww;
    }
    for (int i = 0; i < 3; ++i) memcpy(f.lqi[i], q[i], sizeof(Lqi));
    const int d = f.dim_arm;
    if (d != 8 && d != 16 && d != 24 && d != 32) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "dim_arm %d", d);
    if (f.n_hidden > 4) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "%d ARM hidden layers", f.n_hidden);
    if (arm.qw > 8 || arm.qb < 0 || arm.qb > 16) return ccmi_set_error(CCMI_ERR_BITSTREAM, "ARM q-step index");
    if (ups.qw > 12 || f.n_ups < 1 || f.n_pre < 1 || f.ups_ks < 2 || f.pre_ks < 1)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "upsampling header");
    if (syn.qw > 12 || syn.qb < 0 || syn.qb > 24 || f.n_branches < 1 || f.n_branches > 8)
        return ccmi_set_error(CCMI_ERR_BITSTREAM, "synthesis header");
    size_t per_branch = 0;
    {
        int c = f.n_layers;
        for (auto &L : f.layers) {
            if (L.n_out < 1 || L.ks < 1 || (L.ks & 1) == 0) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "syn layer ks %d", L.ks);
            per_branch += (size_t)L.n_out * c * L.ks * L.ks + L.n_out;
            c = L.n_out;
        }
    }
    if (f.layers.back().n_out < 3) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "synthesis must output >= 3 planes");
    f.arm.assign((size_t)f.n_hidden * (d * d + d) + 2 * d + 2, 0);
    f.ups.assign((size_t)f.n_ups * f.ups_ks + (size_t)f.n_pre * f.pre_ks, 0);
    f.syn.assign(per_branch * f.n_branches, 0);
    if (f.n_branches > 1) f.blend.assign(f.n_branches, 0);
    return CCMI_OK;
}

int decode_frame_weights(FrameHost &f)
{
    Lqi arm{}, ups{}, syn{};
    memcpy(&arm, f.lqi[0], sizeof(Lqi));
    memcpy(&ups, f.lqi[1], sizeof(Lqi));
    memcpy(&syn, f.lqi[2], sizeof(Lqi));
    const uint8_t *arm_w = f.wbytes[0], *arm_b = f.wbytes[1], *ups_w = f.wbytes[2], *syn_w = f.wbytes[3],
                  *syn_b = f.wbytes[4];
    // ---- ARM (read_arm, cc-frame-decoder.cpp:201-258)
    const int d = f.dim_arm;
    {
        auto cw = cabac_on(arm_w, arm.nw), cb = cabac_on(arm_b, arm.nb);
        const int ws = 8 - arm.qw, bsh = 16 - arm.qb;
        int32_t *p = f.arm.data();
        for (int l = 0; l < f.n_hidden; ++l, p += d * d + d)
            if (!read_weights(cw, arm.sw, d * d, ws, kArmPrec, p) || !read_weights(cb, arm.sb, d, bsh, 2 * kArmPrec, p + d * d))
                return ccmi_set_error(CCMI_ERR_BITSTREAM, "ARM weights");
        if (!read_weights(cw, arm.sw, 2 * d, ws, kArmPrec, p) || !read_weights(cb, arm.sb, 2, bsh, 2 * kArmPrec, p + 2 * d))
            return ccmi_set_error(CCMI_ERR_BITSTREAM, "ARM weights");
    }
    // ---- upsampling (read_ups :261-300): half kernels mirrored (decode_upsweights_qi)
    {
        auto cw = cabac_on(ups_w, ups.nw);
        int32_t *p = f.ups.data();
        auto sym = [&](int ks) {
            const int nw = (ks + 1) / 2;
            if (!read_weights(cw, ups.sw, nw, 12 - ups.qw, kUpsPrec, p)) return false;
            for (int i = 0; i < nw / 2 * 2; ++i) p[ks - 1 - i] = p[i];
            p += ks;
            return true;
        };
        for (int l = 0; l < f.n_ups; ++l)
            if (!sym(f.ups_ks)) return ccmi_set_error(CCMI_ERR_BITSTREAM, "upsampling weights");
        for (int l = 0; l < f.n_pre; ++l)
            if (!sym(f.pre_ks)) return ccmi_set_error(CCMI_ERR_BITSTREAM, "upsampling weights");
    }
    // ---- synthesis (read_syn :302-353)
    {
        auto cw = cabac_on(syn_w, syn.nw), cb = cabac_on(syn_b, syn.nb);
        const int ws = 12 - syn.qw, bsh = 24 - syn.qb;
        if (f.n_branches > 1) {
            if (!read_weights(cw, syn.sw, f.n_branches, ws, kSynPrec, f.blend.data()))
                return ccmi_set_error(CCMI_ERR_BITSTREAM, "blend weights");
        }
        int32_t *p = f.syn.data();
        for (int b = 0; b < f.n_branches; ++b) {
            int c = f.n_layers;
            for (auto &L : f.layers) {
                const int nw = c * L.ks * L.ks * L.n_out;
                if (!read_weights(cw, syn.sw, nw, ws, kSynPrec, p) || !read_weights(cb, syn.sb, L.n_out, bsh, 2 * kSynPrec, p + nw))
                    return ccmi_set_error(CCMI_ERR_BITSTREAM, "synthesis weights");
                p += nw + L.n_out;
                c = L.n_out;
            }
        }
    }
    return CCMI_OK;
}

int parse_and_decode_frame(const uint8_t *bs, size_t n, FrameHost &f)
{
    if (int rc = parse_frame_header(bs, n, f)) return rc;
    return decode_frame_weights(f);
}


} // namespace ccmi

using namespace ccmi;

namespace {

enum OutKind { kYuv420 = 0, kYuv444 = 1, kPpm = 2 };

struct OutFmt {
    int kind, bitdepth;
    size_t payload, header;
    char hdr[48];
};

int out_format(const FrameHost &f, int out_bitdepth, int out_chroma, int as_yuv, OutFmt &o)
{
    o.bitdepth = out_bitdepth ? out_bitdepth : f.bitdepth;
    const int chroma = out_chroma ? out_chroma : (f.frame_data_type == 1 ? 420 : 444);
    const size_t bps = o.bitdepth <= 8 ? 1 : 2;
    const size_t npx = (size_t)f.h * f.w;
    o.header = 0;
    if (as_yuv) {
        if (o.bitdepth != 8 && o.bitdepth != 10)
            return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "YUV output bitdepth must be 8 or 10 (got %d)", o.bitdepth);
        o.kind = chroma == 420 ? kYuv420 : kYuv444;
        o.payload = bps * (o.kind == kYuv420 ? npx + 2 * (size_t)(f.h / 2) * (f.w / 2) : 3 * npx);
    } else {
        if (o.bitdepth < 1 || o.bitdepth > 16) return ccmi_set_error(CCMI_ERR_ARG, "PPM bitdepth %d", o.bitdepth);
        o.kind = kPpm;
        o.header = (size_t)snprintf(o.hdr, sizeof o.hdr, "P6\n%d %d\n%d\n", f.w, f.h, (1 << o.bitdepth) - 1);
        o.payload = bps * 3 * npx;
    }
    return CCMI_OK;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct DevPlan {
    size_t bytes_off[CCMI_MAX_GRIDS];
    size_t arm_off, ups_off, syn_off, lat_off, ws_off, dense_off, synout_off, synws_off, out_off;
    size_t lat_elems, ws_elems, dense_elems, synout_elems, synws_elems;
};

thread_local float g_last_ms[4] = {0, 0, 0, 0};
thread_local std::vector<uint32_t> g_last_flags; // per stream: OR of its grids' CCMI_ARM_FLAG_* bits

// polls per two-wave wait of the chain kernel before it gives up (ArmStreamDesc::spin_cap)
int arm_spin_cap()
{
    const char *e = getenv("CCMI_DEC_SPIN_CAP");
    if (!e || !*e) return 1 << 24;
    const long v = strtol(e, nullptr, 10);
    return v < 0 ? 0 : v > (1L << 30) ? (1 << 30) : (int)v;
}

struct EventSet {
    hipEvent_t e[5] = {};
    bool ok = true;
    EventSet()
    {
        for (auto &x : e)
            if (hipEventCreate(&x) != hipSuccess) ok = false;
    }
    ~EventSet()
    {
        for (auto &x : e)
            if (x) (void)hipEventDestroy(x);
    }
    void rec(int i, hipStream_t s)
    {
        if (ok) (void)hipEventRecord(e[i], s);
    }
};

// every synthesis weight (not the biases) of every branch fits 24 signed bits: the fused
// integer synthesis then multiplies with v_mul_i32_i24 (DecSynArgs::f24)
bool syn_weights_fit24(const FrameHost &f)
{
    const size_t per_branch = f.syn.size() / (size_t)std::max(1, f.n_branches);
    for (int b = 0; b < f.n_branches; ++b) {
        size_t q = per_branch * (size_t)b;
        int c = f.n_layers;
        for (const SynLayerDesc &L : f.layers) {
            const size_t nw = (size_t)L.n_out * c * L.ks * L.ks;
            if (q + nw > f.syn.size()) return false;
            for (size_t i = 0; i < nw; ++i) {
                const int32_t v = f.syn[q + i];
                if (v < -(1 << 23) || v >= (1 << 23)) return false;
            }
            q += nw + (size_t)L.n_out;
            c = L.n_out;
        }
    }
    return true;
}

// CABAC decode of every frame's network weights: host threads over the frames (each
// stream's weights are an independent few-hundred-symbol decode, ~50-100 us)
int decode_weights_all(std::vector<FrameHost> &fr)
{
    const int n = (int)fr.size();
    const int T = n >= 32 ? std::max(1, std::min({8, n / 16, (int)std::thread::hardware_concurrency()})) : 1;
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    auto work = [&](int t) {
        for (int i = t; i < n; i += T)
            if ((rc[i] = decode_frame_weights(fr[i])) != CCMI_OK) msg[i] = ccmi_last_error();
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
    }
    for (int i = 0; i < n; ++i)
        if (rc[i]) return ccmi_set_error(rc[i], "stream %d: %s", i, msg[i].c_str());
    return CCMI_OK;
}

// ws / ws_bytes: caller-owned device workspace (NULL: one hipMalloc per call); need: when
// not NULL, only the workspace size is computed (headers parsed, nothing decoded or launched).
int decode_many(const uint8_t *const *streams, const size_t *lens, int n, uint8_t *const *outs, const size_t *caps,
                size_t *sizes, int out_bitdepth, int out_chroma, int as_yuv, hipStream_t s,
                int32_t *const *lat_out = nullptr, void *ws = nullptr, size_t ws_bytes = 0, size_t *need = nullptr)
{
    if (n < 1) return ccmi_set_error(CCMI_ERR_ARG, "decode: no streams");
    std::vector<FrameHost> fr(n);
    std::vector<OutFmt> of(n);
    for (int i = 0; i < n; ++i) {
        if (!streams[i]) return ccmi_set_error(CCMI_ERR_ARG, "decode: stream %d is NULL", i);
        if (int rc = parse_frame_header(streams[i], lens[i], fr[i])) {
            std::string m = ccmi_last_error();
            return ccmi_set_error(rc, "stream %d: %s", i, m.c_str());
        }
        if (int rc = out_format(fr[i], out_bitdepth, out_chroma, as_yuv, of[i])) return rc;
        if (outs && caps && caps[i] < of[i].header + of[i].payload)
            return ccmi_set_error(CCMI_ERR_ARG, "stream %d: output buffer of %zu bytes, need %zu", i, caps[i],
                                  of[i].header + of[i].payload);
        if (sizes) sizes[i] = of[i].header + of[i].payload;
    }

    // ---- plan one device allocation: constant part (bytes + weights, uploaded) then scratch
    std::vector<DevPlan> pl(n);
    size_t cst = 0;
    for (int i = 0; i < n; ++i) {
        FrameHost &f = fr[i];
        DevPlan &p = pl[i];
        for (int l = 0; l < f.n_layers; ++l) {
            p.bytes_off[l] = cst;
            cst += align_up(f.lat_n[l] + 64, 256);
        }
        p.arm_off = cst;
        cst += align_up(f.arm.size() * 4, 256);
        p.ups_off = cst;
        cst += align_up(f.ups.size() * 4, 256);
        p.syn_off = cst;
        cst += align_up(f.syn.size() * 4, 256);
    }
    size_t tot = align_up(cst, 4096);
    for (int i = 0; i < n; ++i) {
        FrameHost &f = fr[i];
        DevPlan &p = pl[i];
        p.lat_elems = 0;
        for (int l = 0; l < f.n_layers; ++l) p.lat_elems += (size_t)f.lh[l] * f.lw[l];
        p.ws_elems = dec_ups_workspace_elems(f.lh, f.lw, f.n_layers);
        p.dense_elems = (size_t)f.n_layers * f.h * f.w;
        p.synout_elems = (size_t)f.layers.back().n_out * f.h * f.w * f.n_branches;
        DecSynArgs sa{};
        sa.c_in = f.n_layers;
        sa.h = f.h;
        sa.w = f.w;
        sa.n_layers = (int)f.layers.size();
        for (int l = 0; l < sa.n_layers; ++l) sa.layers[l] = f.layers[l];
        p.synws_elems = dec_syn_workspace_elems(sa);
        p.lat_off = tot;
        tot += align_up(p.lat_elems * 4, 256);
        p.ws_off = tot;
        tot += align_up(p.ws_elems * 4 + 4, 256);
        p.dense_off = tot;
        tot += align_up(p.dense_elems * 4, 256);
        p.synout_off = tot;
        tot += align_up(p.synout_elems * 4, 256);
        p.synws_off = tot;
        tot += align_up(p.synws_elems * 4 + 4, 256);
        p.out_off = tot;
        tot += align_up(of[i].payload, 256);
    }
    const size_t desc_off = tot;
    tot += align_up(sizeof(ArmStreamDesc) * (size_t)n * CCMI_MAX_GRIDS, 256);
    // batched-tail argument tables: bounded by one single-frame table per frame
    size_t tail_cap = 0;
    for (int i = 0; i < n; ++i) tail_cap += dec_tail_table_bytes(fr[i].n_layers, 1);
    const size_t tail_off = tot;
    tot += align_up(tail_cap, 256);
    // one status word per (frame, latent grid) for the ARM kernels' CCMI_ARM_FLAG_* bits
    const size_t status_off = tot;
    const size_t n_status = (size_t)n * CCMI_MAX_GRIDS;
    tot += align_up(4 * n_status, 256);
#if defined(CCMI_ARM_STAMPS)
    const size_t dbg_off = tot;
    tot += align_up(16 * 8 * (size_t)n * CCMI_MAX_GRIDS, 256);
    size_t all_count = 0;
#endif

    if (need) {
        *need = tot;
        return CCMI_OK;
    }
    if (int rc = decode_weights_all(fr)) return rc;
    std::vector<uint8_t> host(cst, 0);
    for (int i = 0; i < n; ++i) {
        FrameHost &f = fr[i];
        DevPlan &p = pl[i];
        for (int l = 0; l < f.n_layers; ++l)
            if (f.lat_n[l]) memcpy(&host[p.bytes_off[l]], f.lat_bytes[l], f.lat_n[l]);
        memcpy(&host[p.arm_off], f.arm.data(), f.arm.size() * 4);
        memcpy(&host[p.ups_off], f.ups.data(), f.ups.size() * 4);
        memcpy(&host[p.syn_off], f.syn.data(), f.syn.size() * 4);
    }

    uint8_t *dev = static_cast<uint8_t *>(ws);
    if (dev) {
        if (ws_bytes < tot) return ccmi_set_error(CCMI_ERR_ARG, "decode: workspace of %zu bytes, need %zu", ws_bytes, tot);
        if (reinterpret_cast<uintptr_t>(dev) % 256)
            return ccmi_set_error(CCMI_ERR_ARG, "decode: workspace must be 256-byte aligned");
    } else {
        CCMI_HIP_CHECK(hipMalloc(&dev, tot));
    }
    struct Free {
        uint8_t *p;
        ~Free() { if (p) (void)hipFree(p); }
    } guard{ws ? nullptr : dev};
    EventSet ev;
    ev.rec(0, s);
    CCMI_HIP_CHECK(hipMemcpyAsync(dev, host.data(), cst, hipMemcpyHostToDevice, s));
    uint32_t *status = reinterpret_cast<uint32_t *>(dev + status_off);
    CCMI_HIP_CHECK(hipMemsetAsync(status, 0, 4 * n_status, s));
    const int spin_cap = arm_spin_cap();

    // ---- frames in K chunks by decode cost (coded bytes of their latent layers), cheapest
    // first.  Each chunk's ARM launch and decoder tail run on a stream of their own, so the
    // tails of the early chunks overlap the long ARM chains of the later ones: a batch's ARM
    // stage is the slowest layer-0 chain, and most CUs sit idle once the short streams are done.
    // K = 2: the caller's stream and one more (GPU_MAX_HW_QUEUES is 4 per process; streams
    // beyond the hardware queues share one and serialise)
#ifndef CCMI_DEC_CHUNKS
#define CCMI_DEC_CHUNKS 2
#endif
    const int K = n >= 64 ? CCMI_DEC_CHUNKS : 1;
    std::vector<int> chunk_of(n, 0);
    if (K > 1) {
        std::vector<int> order(n);
        std::vector<size_t> cost(n, 0);
        for (int i = 0; i < n; ++i) {
            order[i] = i;
            for (int l = 0; l < fr[i].n_layers; ++l) cost[i] += fr[i].lat_n[l];
        }
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] < cost[b]; });
        for (int r = 0; r < n; ++r) chunk_of[order[r]] = (int)((int64_t)r * K / n);
    }

    // ---- ARM + CABAC: every non-empty latent layer of every frame, one launch per (chunk, d, nh)
    std::vector<ArmStreamDesc> desc;
    struct Key { int chunk, d, nh; };
    std::vector<std::pair<Key, std::vector<ArmStreamDesc>>> groups;
    int max_w = 0, max_blocks = 1;
    for (int i = 0; i < n; ++i) {
        FrameHost &f = fr[i];
        DevPlan &p = pl[i];
        int32_t *lat = reinterpret_cast<int32_t *>(dev + p.lat_off);
        for (int l = 0; l < f.n_layers; ++l) {
            int32_t *plane = lat;
            lat += (size_t)f.lh[l] * f.lw[l];
            if (f.lat_n[l] == 0) { // zero layer (cc-frame-decoder.cpp:479-484)
                CCMI_HIP_CHECK(hipMemsetAsync(plane, 0, (size_t)f.lh[l] * f.lw[l] * 4, s));
                continue;
            }
            ArmStreamDesc a{};
            a.bytes = reinterpret_cast<const uint32_t *>(dev + p.bytes_off[l]);
            a.nbytes = f.lat_n[l];
            a.h = f.lh[l];
            a.w = f.lw[l];
            a.sig_blk = f.sig_blk;
            a.d = f.dim_arm;
            a.nh = f.n_hidden;
            a.weights = reinterpret_cast<const int32_t *>(dev + p.arm_off);
            a.flags = 1;
            a.dbg = nullptr;
            a.status = status + (size_t)i * CCMI_MAX_GRIDS + l;
            a.spin_cap = spin_cap;
#if defined(CCMI_ARM_STAMPS)
            a.dbg = reinterpret_cast<uint64_t *>(dev + dbg_off) + 16 * (desc.size() + all_count++);
#endif
            for (size_t k = 0; k < f.arm.size(); ++k) {
                // biases sit between weight blocks; checking them too is conservative
                if (f.arm[k] >= (1 << 23) || f.arm[k] < -(1 << 23)) a.flags = 0;
            }
            a.out = plane;
            max_w = std::max(max_w, a.w);
            const int blk = std::abs(a.sig_blk);
            if (blk > 0) {
                int sh = 0;
                while ((1 << sh) < blk) ++sh;
                max_blocks = std::max(max_blocks, ((a.h + blk - 1) >> sh) * ((a.w + blk - 1) >> sh));
            }
            auto it = std::find_if(groups.begin(), groups.end(), [&](auto &g) {
                return g.first.chunk == chunk_of[i] && g.first.d == a.d && g.first.nh == a.nh;
            });
            if (it == groups.end()) {
                groups.push_back({Key{chunk_of[i], a.d, a.nh}, {}});
                it = groups.end() - 1;
            }
            it->second.push_back(a);
        }
    }

    std::vector<ArmStreamDesc> all;
    std::stable_sort(groups.begin(), groups.end(), [](const auto &x, const auto &y) { return x.first.chunk < y.first.chunk; });
    for (auto &g : groups) {
        // longest streams first: they bound the launch
        std::stable_sort(g.second.begin(), g.second.end(),
                         [](const ArmStreamDesc &x, const ArmStreamDesc &y) { return x.h * x.w > y.h * y.w; });
        all.insert(all.end(), g.second.begin(), g.second.end());
    }
    if (!all.empty())
        CCMI_HIP_CHECK(hipMemcpyAsync(dev + desc_off, all.data(), all.size() * sizeof(ArmStreamDesc),
                                      hipMemcpyHostToDevice, s));

    // ---- decoder tail arguments; frames of one geometry with a fused synthesis (single
    // branch) share one launch per stage
    std::vector<DecTailFrame> tail(n);
    for (int i = 0; i < n; ++i) {
        FrameHost &f = fr[i];
        DevPlan &p = pl[i];
        DecTailFrame &t = tail[i];
        DecUpsArgs &ua = t.ups;
        ua = DecUpsArgs{};
        ua.lat = reinterpret_cast<const int32_t *>(dev + p.lat_off);
        ua.n_layers = f.n_layers;
        int off = 0;
        for (int l = 0; l < f.n_layers; ++l) {
            ua.lh[l] = f.lh[l];
            ua.lw[l] = f.lw[l];
            ua.off[l] = off;
            off += f.lh[l] * f.lw[l];
        }
        ua.kernels = reinterpret_cast<const int32_t *>(dev + p.ups_off);
        ua.ups_ks = f.ups_ks;
        ua.n_ups = f.n_ups;
        ua.pre_ks = f.pre_ks;
        ua.n_pre = f.n_pre;
        ua.workspace = reinterpret_cast<int32_t *>(dev + p.ws_off);
        ua.out = reinterpret_cast<int32_t *>(dev + p.dense_off);
        DecSynArgs &sa = t.syn;
        sa = DecSynArgs{};
        sa.in = ua.out;
        sa.c_in = f.n_layers;
        sa.h = f.h;
        sa.w = f.w;
        sa.n_layers = (int)f.layers.size();
        for (int l = 0; l < sa.n_layers; ++l) sa.layers[l] = f.layers[l];
        sa.params = reinterpret_cast<const int32_t *>(dev + p.syn_off);
        sa.out = reinterpret_cast<int32_t *>(dev + p.synout_off);
        sa.workspace = reinterpret_cast<int32_t *>(dev + p.synws_off);
        sa.f24 = syn_weights_fit24(f) ? 1 : 0;
        t.bitdepth = of[i].bitdepth;
        t.kind = of[i].kind;
        t.dst = dev + p.out_off;
    }
    // frames of one geometry share one launch per tail stage (960 class-E frames: 134 ms
    // against 264 ms with per-frame launches)
    std::vector<std::vector<int>> tgroups;
    std::vector<char> batched(n, 0);
    for (int i = 0; i < n; ++i) {
        if (fr[i].n_branches != 1 || !dec_tail_batchable(tail[i])) continue;
        auto it = std::find_if(tgroups.begin(), tgroups.end(), [&](const std::vector<int> &g) {
            return g.size() < 65535 && chunk_of[g[0]] == chunk_of[i] && dec_tail_same_group(tail[g[0]], tail[i]);
        });
        if (it == tgroups.end()) {
            tgroups.emplace_back();
            it = tgroups.end() - 1;
        }
        it->push_back(i);
        batched[i] = 1;
    }
    std::vector<size_t> tg_off(tgroups.size());
    std::vector<uint8_t> tab(tail_cap > 0 ? tail_cap : 1);
    size_t tpos = 0;
    for (size_t g = 0; g < tgroups.size(); ++g) {
        std::vector<const DecTailFrame *> ptr;
        for (int i : tgroups[g]) ptr.push_back(&tail[i]);
        tg_off[g] = tpos;
        dec_tail_fill(ptr.data(), (int)ptr.size(), tab.data() + tpos);
        tpos += dec_tail_table_bytes(tail[tgroups[g][0]].ups.n_layers, (int)ptr.size());
    }
    if (tpos) CCMI_HIP_CHECK(hipMemcpyAsync(dev + tail_off, tab.data(), tpos, hipMemcpyHostToDevice, s));
    ev.rec(1, s);
    // one chunk's ARM launches, then its decoder tail (batched groups, then the rest per frame)
    auto launch_chunk = [&](int c, hipStream_t cs, hipEvent_t arm_done) -> int {
        size_t dp = 0;
        for (auto &g : groups) {
            if (g.first.chunk == c) {
                const ArmStreamDesc *dd = reinterpret_cast<const ArmStreamDesc *>(dev + desc_off) + dp;
                if (int rc = launch_dec_arm(dd, (int)g.second.size(), max_w, max_blocks, g.first.d, g.first.nh, cs))
                    return rc;
            }
            dp += g.second.size();
        }
        if (arm_done) CCMI_HIP_CHECK(hipEventRecord(arm_done, cs));
        for (size_t g = 0; g < tgroups.size(); ++g)
            if (chunk_of[tgroups[g][0]] == c)
                if (int rc = launch_dec_tail_batch(tail[tgroups[g][0]], (int)tgroups[g].size(), dev + tail_off + tg_off[g], cs))
                    return rc;
        for (int i = 0; i < n; ++i) {
            if (batched[i] || chunk_of[i] != c) continue;
            FrameHost &f = fr[i];
            DevPlan &p = pl[i];
            if (int rc = launch_dec_ups(tail[i].ups, cs)) return rc;

            const int nout = f.layers.back().n_out;
            const int64_t plane = (int64_t)f.h * f.w;
            size_t per_branch = f.syn.size() / f.n_branches;
            int32_t *synout = reinterpret_cast<int32_t *>(dev + p.synout_off);
            for (int b = 0; b < f.n_branches; ++b) {
                DecSynArgs sa = tail[i].syn;
                sa.params += per_branch * b;
                sa.out = synout + (size_t)b * nout * plane;
                if (int rc = launch_dec_syn(sa, cs)) return rc;
                if (b >= 1) // run_syn (cc-frame-decoder.cpp:1044-1149): blends on 3 planes
                    if (int rc = launch_dec_blend(synout, synout + (size_t)b * nout * plane, 3 * plane,
                                                  f.blend[0], f.blend[b], b == 1, cs))
                        return rc;
            }
            if (int rc = launch_dec_output(synout, f.h, f.w, of[i].bitdepth, of[i].kind, dev + p.out_off, cs)) return rc;
        }
        return CCMI_OK;
    };
    // the decoded bytes of chunk c: headers on the host, payloads copied back on the chunk's
    // own stream right after its tail, so one chunk's download overlaps the other chunk's
    // ARM chains (pinned output buffers make these real DMA copies; pageable ones are staged
    // by the runtime)
    auto download_chunk = [&](int c, hipStream_t cs) -> int {
        for (int i = 0; i < n && outs; ++i) {
            if (chunk_of[i] != c) continue;
            if (of[i].header) memcpy(outs[i], of[i].hdr, of[i].header);
            CCMI_HIP_CHECK(hipMemcpyAsync(outs[i] + of[i].header, dev + pl[i].out_off, of[i].payload,
                                          hipMemcpyDeviceToHost, cs));
        }
        return CCMI_OK;
    };
    // K > 1: streams forked from s after the uploads; each chunk runs ARM -> tail -> download on
    // its stream, and s waits for every chunk before it returns.  The extra streams and the
    // events are leased from the process-wide pool (ccmi_api.cpp) for this call: st[c] for
    // chunks c >= 1 (chunk 0 runs on s), ev[0] fork; per chunk c: [1 + 4c] start, [2 + 4c] ARM
    // done, [3 + 4c] tail done, [4 + 4c] done.
    StreamSetLease lease;
    if (K == 1) {
        if (int rc = launch_chunk(0, s, ev.ok ? ev.e[2] : nullptr)) return rc;
        ev.rec(3, s);
        if (int rc = download_chunk(0, s)) return rc;
    } else {
        lease.set = ccmi_streamset_acquire(K, 1 + 4 * K, true);
        if (!lease.set) return CCMI_ERR_HIP;
        StreamSet &fk = *lease.set;
        // an error after some chunks were queued: s still waits for them before the caller can
        // reuse or free the workspace (the chunks' own streams never outlive it unjoined)
        int started = 0;
        auto join = [&]() {
            for (int c = K - 1; c > K - 1 - started && c >= 1; --c) {
                (void)hipEventRecord(fk.ev[4 + 4 * c], fk.st[c]);
                (void)hipStreamWaitEvent(s, fk.ev[4 + 4 * c], 0);
            }
        };
        CCMI_HIP_CHECK(hipEventRecord(fk.ev[0], s));
        for (int c = K - 1; c >= 0; --c) { // the most expensive chunk first
            hipStream_t cs = c == 0 ? s : fk.st[c];
            if (c > 0) {
                if (hipStreamWaitEvent(cs, fk.ev[0], 0) != hipSuccess) {
                    join();
                    return ccmi_set_error(CCMI_ERR_HIP, "decode: stream fork failed");
                }
                ++started;
            }
            (void)hipEventRecord(fk.ev[1 + 4 * c], cs);
            int rc = launch_chunk(c, cs, fk.ev[2 + 4 * c]);
            if (!rc) {
                (void)hipEventRecord(fk.ev[3 + 4 * c], cs);
                rc = download_chunk(c, cs);
            }
            if (rc) {
                join();
                return rc;
            }
        }
        join();
    }
    ev.rec(4, s);
    for (int i = 0; i < n && lat_out; ++i)
        CCMI_HIP_CHECK(hipMemcpyAsync(lat_out[i], dev + pl[i].lat_off, pl[i].lat_elems * 4, hipMemcpyDeviceToHost, s));
    std::vector<uint32_t> st(n_status);
    CCMI_HIP_CHECK(hipMemcpyAsync(st.data(), status, 4 * n_status, hipMemcpyDeviceToHost, s));
    CCMI_HIP_CHECK(hipStreamSynchronize(s));
    g_last_flags.assign(n, 0u);
    for (int i = 0; i < n; ++i)
        for (int l = 0; l < CCMI_MAX_GRIDS; ++l) g_last_flags[i] |= st[(size_t)i * CCMI_MAX_GRIDS + l];
    for (int i = 0; i < n; ++i)
        for (int l = 0; l < CCMI_MAX_GRIDS; ++l)
            if (st[(size_t)i * CCMI_MAX_GRIDS + l] & CCMI_ARM_FLAG_TIMEOUT)
                // the two waves of a stream lost their hand-off: the latents cannot be trusted
                return ccmi_set_error(CCMI_ERR_HIP,
                                      "decode: stream %d, latent grid %d: the ARM decode's wave hand-off gave up "
                                      "after %d polls; output discarded",
                                      i, l, spin_cap);
    for (int i = 0; i < n && lat_out; ++i)
        for (size_t k = 0; k < pl[i].lat_elems; ++k) lat_out[i][k] >>= kArmPrec;
#if defined(CCMI_ARM_STAMPS)
    {
        std::vector<uint64_t> dbg(16 * all.size());
        CCMI_HIP_CHECK(hipMemcpy(dbg.data(), dev + dbg_off, dbg.size() * 8, hipMemcpyDeviceToHost));
        for (size_t j = 0; j < all.size(); ++j) {
            const size_t k = (size_t)(reinterpret_cast<uint8_t *>(all[j].dbg) - (dev + dbg_off)) / 128;
            fprintf(stderr, "STAMPS stream %zu (%dx%d):", k, all[j].h, all[j].w);
            for (int c = 0; c < 16; ++c) fprintf(stderr, " %llu", (unsigned long long)dbg[16 * k + c]);
            fprintf(stderr, "\n");
        }
    }
#endif
    if (ev.ok) {
        if (K == 1) {
            for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&g_last_ms[k], ev.e[k], ev.e[k + 1]);
        } else {
            // overlapped stages: ARM = the longest chunk's ARM (its start to its ARM end, events
            // of one stream), tail = from the uploads to the last chunk's tail minus that ARM,
            // download = what is left after the last tail (the part not hidden under kernels)
            float span = 0.f, arm = 0.f, all = 0.f;
            (void)hipEventElapsedTime(&g_last_ms[0], ev.e[0], ev.e[1]);
            (void)hipEventElapsedTime(&all, ev.e[1], ev.e[4]);
            const StreamSet &fk = *lease.set;
            for (int c = 0; c < K; ++c) {
                float t = 0.f;
                if (hipEventElapsedTime(&t, fk.ev[1 + 4 * c], fk.ev[2 + 4 * c]) == hipSuccess) arm = std::max(arm, t);
                if (hipEventElapsedTime(&t, ev.e[1], fk.ev[3 + 4 * c]) == hipSuccess) span = std::max(span, t);
            }
            g_last_ms[1] = arm;
            g_last_ms[2] = span - arm;
            g_last_ms[3] = all - span;
            (void)hipGetLastError(); // a timing query that failed must not surface in the next call
        }
    }
    return CCMI_OK;
}

} // namespace

extern "C" int ccmi_decode_last_timing(float *ms4)
{
    if (!ms4) return ccmi_set_error(CCMI_ERR_ARG, "decode_last_timing: null argument");
    for (int k = 0; k < 4; ++k) ms4[k] = g_last_ms[k];
    return CCMI_OK;
}

extern "C" int ccmi_decode_last_arm_flags(uint32_t *flags, int cap, int *n)
{
    if (!n || (cap > 0 && !flags)) return ccmi_set_error(CCMI_ERR_ARG, "decode_last_arm_flags: null argument");
    const int m = std::min(cap, (int)g_last_flags.size());
    for (int i = 0; i < m; ++i) flags[i] = g_last_flags[i];
    *n = (int)g_last_flags.size();
    return CCMI_OK;
}

extern "C" int ccmi_decode_output_size(const uint8_t *stream, size_t len, int out_bitdepth, int out_chroma, int as_yuv,
                                       size_t *size)
{
    if (!stream || !size) return ccmi_set_error(CCMI_ERR_ARG, "decode_output_size: null argument");
    FrameHost f;
    if (int rc = parse_frame_header(stream, len, f)) return rc;
    OutFmt o;
    if (int rc = out_format(f, out_bitdepth, out_chroma, as_yuv, o)) return rc;
    *size = o.header + o.payload;
    return CCMI_OK;
}

extern "C" int ccmi_decode_batch(const uint8_t *const *streams, const size_t *lens, int n, uint8_t *const *out,
                                 const size_t *out_caps, size_t *out_sizes, int out_bitdepth, int out_chroma,
                                 int as_yuv, void *stream)
{
    if (!streams || !lens || !out || !out_caps) return ccmi_set_error(CCMI_ERR_ARG, "decode_batch: null argument");
    return decode_many(streams, lens, n, out, out_caps, out_sizes, out_bitdepth, out_chroma, as_yuv,
                       static_cast<hipStream_t>(stream));
}

extern "C" int ccmi_decode_batch_workspace_bytes(const uint8_t *const *streams, const size_t *lens, int n,
                                                 int out_bitdepth, int out_chroma, int as_yuv, size_t *bytes)
{
    if (!streams || !lens || !bytes) return ccmi_set_error(CCMI_ERR_ARG, "decode_batch_workspace_bytes: null argument");
    return decode_many(streams, lens, n, nullptr, nullptr, nullptr, out_bitdepth, out_chroma, as_yuv, nullptr, nullptr,
                       nullptr, 0, bytes);
}

extern "C" int ccmi_decode_batch_plan(const uint8_t *const *streams, const size_t *lens, int n, int out_bitdepth,
                                      int out_chroma, int as_yuv, size_t *out_sizes, size_t *workspace_bytes)
{
    if (!streams || !lens || !out_sizes || !workspace_bytes) return ccmi_set_error(CCMI_ERR_ARG, "decode_batch_plan: null argument");
    return decode_many(streams, lens, n, nullptr, nullptr, out_sizes, out_bitdepth, out_chroma, as_yuv, nullptr, nullptr,
                       nullptr, 0, workspace_bytes);
}

extern "C" int ccmi_decode_batch_ws(const uint8_t *const *streams, const size_t *lens, int n, uint8_t *const *out,
                                    const size_t *out_caps, size_t *out_sizes, int out_bitdepth, int out_chroma,
                                    int as_yuv, void *workspace, size_t workspace_bytes, void *stream)
{
    if (!streams || !lens || !out || !out_caps || !workspace)
        return ccmi_set_error(CCMI_ERR_ARG, "decode_batch_ws: null argument");
    return decode_many(streams, lens, n, out, out_caps, out_sizes, out_bitdepth, out_chroma, as_yuv,
                       static_cast<hipStream_t>(stream), nullptr, workspace, workspace_bytes);
}

extern "C" int ccmi_decode_latents(const uint8_t *stream, size_t len, int32_t *out, size_t cap, void *hstream)
{
    if (!stream || !out) return ccmi_set_error(CCMI_ERR_ARG, "decode_latents: null argument");
    FrameHost f;
    if (int rc = parse_and_decode_frame(stream, len, f)) return rc;
    size_t n = 0;
    for (int l = 0; l < f.n_layers; ++l) n += (size_t)f.lh[l] * f.lw[l];
    if (cap < n) return ccmi_set_error(CCMI_ERR_ARG, "decode_latents: buffer of %zu ints, need %zu", cap, n);
    size_t osz = 0;
    if (int rc = ccmi_decode_output_size(stream, len, 0, 0, 1, &osz)) return rc;
    std::vector<uint8_t> tmp(osz);
    uint8_t *op = tmp.data();
    return decode_many(&stream, &len, 1, &op, &osz, nullptr, 0, 0, 1, static_cast<hipStream_t>(hstream), &out);
}

static bool ends_with(const std::string &a, const char *b)
{
    const size_t n = strlen(b);
    return a.size() >= n && a.compare(a.size() - n, n, b) == 0;
}

extern "C" int ccmi_decode_file(const char *in_path, const char *out_path, int out_bitdepth, int out_chroma,
                                int verbosity, int device)
{
    if (!in_path) {
        ccmi_set_error(CCMI_ERR_ARG, "decode: no input bitstream");
        return 1;
    }
    FILE *fi = fopen(in_path, "rb");
    if (!fi) {
        ccmi_set_error(CCMI_ERR_IO, "cannot open %s for reading", in_path);
        return 1;
    }
    std::vector<uint8_t> buf;
    {
        fseek(fi, 0, SEEK_END);
        long n = ftell(fi);
        fseek(fi, 0, SEEK_SET);
        buf.resize(n > 0 ? (size_t)n : 0);
        const bool ok = buf.empty() || fread(buf.data(), 1, buf.size(), fi) == buf.size();
        fclose(fi);
        if (!ok) {
            ccmi_set_error(CCMI_ERR_IO, "cannot read %s", in_path);
            return 1;
        }
    }
    if (hipSetDevice(device) != hipSuccess) {
        ccmi_set_error(CCMI_ERR_HIP, "hipSetDevice(%d) failed", device);
        return 1;
    }
    const std::string out = out_path ? out_path : "";
    const int as_yuv = ends_with(out, ".yuv");
    size_t need = 0;
    if (ccmi_decode_output_size(buf.data(), buf.size(), out_bitdepth, out_chroma, as_yuv, &need)) return 1;
    std::vector<uint8_t> res(need);
    const uint8_t *sp = buf.data();
    const size_t ln = buf.size();
    uint8_t *op = res.data();
    size_t got = 0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, nullptr);
    if (decode_many(&sp, &ln, 1, &op, &need, &got, out_bitdepth, out_chroma, as_yuv, nullptr)) return 1;
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (verbosity >= 1) printf("time: all %g\n", ms * 1e-3);
    if (!out.empty()) {
        FILE *fo = fopen(out.c_str(), "wb");
        if (!fo) {
            ccmi_set_error(CCMI_ERR_IO, "cannot open %s for writing", out.c_str());
            return 1;
        }
        const bool ok = fwrite(res.data(), 1, got, fo) == got;
        fclose(fo);
        if (!ok) {
            ccmi_set_error(CCMI_ERR_IO, "cannot write %s", out.c_str());
            return 1;
        }
    }
    return 0;
}
