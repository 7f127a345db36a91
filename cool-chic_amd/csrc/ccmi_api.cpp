// ccmi_api.cpp -- C-ABI entry points of libccmi (declared in include/ccmi.h).
//
// Validation, error reporting (thread-local message, never exit()), stream plumbing.
// The compute lives in the *.hip translation units.
#include <stdarg.h>
#include <stdio.h>

#include <mutex>

#include "ccmi_internal.h"

static thread_local char g_err[512] = "";

int ccmi_set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

static std::mutex g_pool_mu;
static std::vector<StreamSet *> g_pool; // free sets

StreamSet *ccmi_streamset_acquire(int nst, int nev, bool timing)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        ccmi_set_error(CCMI_ERR_HIP, "stream pool: hipGetDevice failed");
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i) {
            StreamSet *s = g_pool[i];
            if (s->device == dev && s->timing == timing && (int)s->st.size() >= nst && (int)s->ev.size() >= nev) {
                g_pool.erase(g_pool.begin() + (long)i);
                return s;
            }
        }
    }
    StreamSet *s = new StreamSet;
    s->device = dev;
    s->timing = timing;
    s->st.assign(nst, nullptr);
    s->ev.assign(nev, nullptr);
    bool ok = true;
    for (auto &x : s->st) ok = ok && hipStreamCreateWithFlags(&x, hipStreamNonBlocking) == hipSuccess;
    for (auto &x : s->ev) ok = ok && (timing ? hipEventCreate(&x) : hipEventCreateWithFlags(&x, hipEventDisableTiming)) == hipSuccess;
    if (!ok) {
        ccmi_set_error(CCMI_ERR_HIP, "stream pool: stream / event creation failed");
        for (auto x : s->st)
            if (x) (void)hipStreamDestroy(x);
        for (auto x : s->ev)
            if (x) (void)hipEventDestroy(x);
        delete s;
        return nullptr;
    }
    return s;
}

void ccmi_streamset_release(StreamSet *set)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.push_back(set);
}

extern "C" const char *ccmi_last_error(void) { return g_err; }

extern "C" int ccmi_version(void) { return 100; }

extern "C" int ccmi_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int check_grids(int n, const int *h, const int *w, const char *who)
{
    if (n < 1 || n > CCMI_MAX_GRIDS) return ccmi_set_error(CCMI_ERR_ARG, "%s: n_grids must be in [1, %d]", who, CCMI_MAX_GRIDS);
    for (int l = 0; l < n; ++l)
        if (h[l] < 1 || w[l] < 1) return ccmi_set_error(CCMI_ERR_ARG, "%s: grid %d has size %dx%d", who, l, h[l], w[l]);
    return CCMI_OK;
}

extern "C" int ccmi_arm_forward_f32(const ccmi_arm_args *a, void *stream)
{
    if (!a || !a->latent || !a->params) return ccmi_set_error(CCMI_ERR_ARG, "arm: null argument");
    if (int rc = check_grids(a->n_grids, a->h, a->w, "arm")) return rc;
    if (a->batch < 1) return ccmi_set_error(CCMI_ERR_ARG, "arm: batch must be >= 1");
    if (a->n_hidden < 0 || a->n_hidden > 4) return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "arm: n_hidden must be in [0, 4]");
    const int64_t need = (int64_t)a->n_hidden * (a->dim_arm * a->dim_arm + a->dim_arm) + 2 * a->dim_arm + 2;
    if (a->param_stride != 0 && a->param_stride < need) return ccmi_set_error(CCMI_ERR_ARG, "arm: param_stride < %lld", (long long)need);
    if (!a->rate && !a->mu && !a->scale && !a->log_scale) return ccmi_set_error(CCMI_ERR_ARG, "arm: no output requested");
    return ccmi_launch_arm_f32(a, static_cast<hipStream_t>(stream));
}

extern "C" int ccmi_ups_forward_f32(const ccmi_ups_args *a, void *stream)
{
    if (!a || !a->latent || !a->params || !a->out) return ccmi_set_error(CCMI_ERR_ARG, "ups: null argument");
    if (int rc = check_grids(a->n_grids, a->h, a->w, "ups")) return rc;
    if (a->batch < 1) return ccmi_set_error(CCMI_ERR_ARG, "ups: batch must be >= 1");
    return ccmi_launch_ups_f32(a, static_cast<hipStream_t>(stream));
}

extern "C" int ccmi_syn_forward_f32(const ccmi_syn_args *a, void *stream)
{
    if (!a || !a->in || !a->params || !a->out) return ccmi_set_error(CCMI_ERR_ARG, "syn: null argument");
    if (a->h < 1 || a->w < 1 || a->c_in < 1 || a->batch < 1) return ccmi_set_error(CCMI_ERR_ARG, "syn: bad shape");
    return ccmi_launch_syn_f32(a, static_cast<hipStream_t>(stream));
}

extern "C" int ccmi_post_f32(const ccmi_post_args *a, void *stream)
{
    if (!a || !a->in || !a->out) return ccmi_set_error(CCMI_ERR_ARG, "post: null argument");
    if (a->h < 1 || a->w < 1 || a->batch < 1) return ccmi_set_error(CCMI_ERR_ARG, "post: bad shape");
    return ccmi_launch_post_f32(a, static_cast<hipStream_t>(stream));
}
