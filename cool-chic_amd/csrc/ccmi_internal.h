// ccmi_internal.h -- shared definitions for the libccmi HIP kernels and the C-ABI layer.
// Not part of the public interface (that is include/ccmi.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/ccmi.h"

#define CCMI_MAX_GRIDS 8

// Geometry of the latent pyramid of one frame: grid l is h[l] x w[l], stored flat
// (row-major) at offset off[l] of the frame's latent vector, as the reference's
// torch.cat of the flattened grids (coolchic.py:360-363).
struct GridGeom {
    int n;
    int h[CCMI_MAX_GRIDS];
    int w[CCMI_MAX_GRIDS];
    int off[CCMI_MAX_GRIDS];
    int total;
};

// Sets the thread-local error string; returns the error code.
int ccmi_set_error(int code, const char *fmt, ...);

#define CCMI_HIP_CHECK(expr)                                                                \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return ccmi_set_error(CCMI_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

static inline int ccmi_div_up(int a, int b) { return (a + b - 1) / b; }

// Stage launchers (return CCMI_OK or an error code; never exit()).
int ccmi_launch_arm_f32(const ccmi_arm_args *a, hipStream_t s);
int ccmi_launch_ups_f32(const ccmi_ups_args *a, hipStream_t s);
int ccmi_launch_syn_f32(const ccmi_syn_args *a, hipStream_t s);
int ccmi_launch_post_f32(const ccmi_post_args *a, hipStream_t s);

// Process-wide pool of side streams and events, one set per concurrent user and device
// (train.hip's ARM side stream, dec_host.cpp's chunk streams).  A set is leased for one call
// and returned to the pool afterwards, so threads that come and go (thread pools) reuse the
// same few streams instead of leaking one per thread; sets are never destroyed (the runtime
// may be gone at process exit).
struct StreamSet {
    int device = -1;
    bool timing = false;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;
};
// A set on the current device with >= nst streams and >= nev events (timing events when
// `timing`), nullptr with the error message set on failure.
StreamSet *ccmi_streamset_acquire(int nst, int nev, bool timing);
void ccmi_streamset_release(StreamSet *set);
struct StreamSetLease {
    StreamSet *set = nullptr;
    StreamSetLease() = default;
    StreamSetLease(const StreamSetLease &) = delete;
    StreamSetLease &operator=(const StreamSetLease &) = delete;
    ~StreamSetLease()
    {
        if (set) ccmi_streamset_release(set);
    }
};
