// dec_api.cpp -- tensor-level C ABI of the fixed-point decoder stages (path B), the
// integer twins of the float entry points: network weights as the decoder's fixed-point
// integers, upsampling and synthesis on caller-owned device buffers.
//
// Reference: cc_frame_decoder::read_arm / read_ups / read_syn (cc-frame-decoder.cpp:201-353,
// decode_weights_qi :157-185, decode_upsweights_qi :188-199), run_ups (:572-679) over
// ups_refine_cpu.hpp:11-79 / ups_upsample_cpu.hpp:12-91, run_syn_branch (:773-1042) over
// synfused_cpu.hpp:17-109 / synlb_cpu.hpp:22-124 / syn_cpu.hpp:21-112.
#include <string.h>

#include "dec_internal.h"

using namespace ccmi;

namespace {

int fill_ups(const ccmi_ups_i32_args *a, DecUpsArgs &u)
{
    if (!a || !a->latent || !a->kernels || !a->out) return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: null argument");
    if (a->n_grids < 1 || a->n_grids > CCMI_MAX_GRIDS) return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: n_grids %d", a->n_grids);
    u = DecUpsArgs{};
    u.lat = a->latent;
    u.n_layers = a->n_grids;
    int off = 0;
    for (int l = 0; l < a->n_grids; ++l) {
        if (a->h[l] < 1 || a->w[l] < 1) return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: grid %d is %dx%d", l, a->h[l], a->w[l]);
        if (l > 0 && (a->h[l] != (a->h[l - 1] + 1) / 2 || a->w[l] != (a->w[l - 1] + 1) / 2))
            return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: grid %d is not ceil(half) of grid %d", l, l - 1);
        u.lh[l] = a->h[l];
        u.lw[l] = a->w[l];
        u.off[l] = off;
        off += a->h[l] * a->w[l];
    }
    u.kernels = a->kernels;
    u.ups_ks = a->ups_k;
    u.n_ups = a->n_ups;
    u.pre_ks = a->pre_k;
    u.n_pre = a->n_pre;
    if (a->n_grids > 1 && (a->n_ups < 1 || a->n_pre < 1)) return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: no kernels");
    u.workspace = static_cast<int32_t *>(a->workspace);
    u.out = a->out;
    return CCMI_OK;
}

int fill_syn(const ccmi_syn_i32_args *a, DecSynArgs &y)
{
    if (!a || !a->in || !a->params || !a->out) return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: null argument");
    if (a->n_layers < 1 || a->n_layers > CCMI_MAX_SYN_LAYERS)
        return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: n_layers must be in [1, %d]", CCMI_MAX_SYN_LAYERS);
    if (a->c_in < 1 || a->h < 1 || a->w < 1) return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: bad input shape");
    y = DecSynArgs{};
    y.in = a->in;
    y.c_in = a->c_in;
    y.h = a->h;
    y.w = a->w;
    y.n_layers = a->n_layers;
    int c = a->c_in;
    for (int l = 0; l < a->n_layers; ++l) {
        const ccmi_syn_layer &L = a->layers[l];
        if (L.n_out < 1 || L.ks < 1 || L.ks % 2 == 0)
            return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: layer %d has n_out=%d ks=%d", l, L.n_out, L.ks);
        if (L.residual && L.n_out != c) return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: residual layer %d needs n_out == n_in", l);
        y.layers[l] = SynLayerDesc{L.n_out, L.ks, L.residual, L.relu};
        c = L.n_out;
    }
    y.params = a->params;
    y.out = a->out;
    y.workspace = static_cast<int32_t *>(a->workspace);
    return CCMI_OK;
}

size_t copy_out(const std::vector<int32_t> &v, int32_t *dst, size_t cap)
{
    if (dst && cap >= v.size() && !v.empty()) memcpy(dst, v.data(), v.size() * 4);
    return v.size();
}

} // namespace

extern "C" int ccmi_decode_weights_i32(const uint8_t *stream, size_t len, int32_t *arm, size_t arm_cap, int32_t *ups,
                                       size_t ups_cap, int32_t *syn, size_t syn_cap, size_t *counts)
{
    if (!stream || !counts) return ccmi_set_error(CCMI_ERR_ARG, "decode_weights_i32: null argument");
    FrameHost f;
    if (int rc = parse_and_decode_frame(stream, len, f)) return rc;
    counts[0] = copy_out(f.arm, arm, arm_cap);
    counts[1] = copy_out(f.ups, ups, ups_cap);
    counts[2] = copy_out(f.syn, syn, syn_cap);
    if ((arm && arm_cap < counts[0]) || (ups && ups_cap < counts[1]) || (syn && syn_cap < counts[2]))
        return ccmi_set_error(CCMI_ERR_ARG, "decode_weights_i32: buffers of %zu / %zu / %zu values, need %zu / %zu / %zu",
                              arm_cap, ups_cap, syn_cap, counts[0], counts[1], counts[2]);
    return CCMI_OK;
}

extern "C" size_t ccmi_ups_workspace_bytes_i32(int n_grids, const int *h, const int *w)
{
    if (!h || !w || n_grids < 1 || n_grids > CCMI_MAX_GRIDS) return 0;
    return 4 * dec_ups_workspace_elems(h, w, n_grids) + 4;
}

extern "C" int ccmi_ups_forward_i32(const ccmi_ups_i32_args *a, void *stream)
{
    DecUpsArgs u;
    if (int rc = fill_ups(a, u)) return rc;
    const size_t need = ccmi_ups_workspace_bytes_i32(a->n_grids, a->h, a->w);
    if (!a->workspace || a->workspace_bytes < need)
        return ccmi_set_error(CCMI_ERR_ARG, "ups_i32: workspace of %zu bytes needed", need);
    return launch_dec_ups(u, static_cast<hipStream_t>(stream));
}

extern "C" size_t ccmi_syn_workspace_bytes_i32(const ccmi_syn_i32_args *a)
{
    if (!a) return 0;
    DecSynArgs y;
    ccmi_syn_i32_args t = *a;
    static int32_t dummy;
    if (!t.in) t.in = &dummy;
    if (!t.params) t.params = &dummy;
    if (!t.out) t.out = &dummy;
    if (fill_syn(&t, y)) return 0;
    return 4 * dec_syn_workspace_elems(y);
}

extern "C" int ccmi_syn_forward_i32(const ccmi_syn_i32_args *a, void *stream)
{
    DecSynArgs y;
    if (int rc = fill_syn(a, y)) return rc;
    const size_t need = 4 * dec_syn_workspace_elems(y);
    if (need && (!a->workspace || a->workspace_bytes < need))
        return ccmi_set_error(CCMI_ERR_ARG, "syn_i32: workspace of %zu bytes needed for this architecture", need);
    return launch_dec_syn(y, static_cast<hipStream_t>(stream));
}
