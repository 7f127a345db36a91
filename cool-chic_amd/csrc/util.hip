// util.hip -- small batched reductions used around the hot path (quantize_model's
// candidate losses, validation): per-row sums and sums of squared differences, with
// double accumulation (loss.py _compute_mse / rate.sum() over ~1e6 terms per row).
#include "ccmi_internal.h"

namespace {

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void row_reduce(const float *__restrict__ a, int64_t as, const float *__restrict__ t,
                                                 int64_t ts, int64_t len, int mode, double *__restrict__ out)
{
    __shared__ double s_red[kT / 64];
    const int b = blockIdx.y;
    const float *ar = a + (int64_t)b * as;
    const float *tr = t ? t + (int64_t)b * ts : nullptr;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < len; i += (int64_t)gridDim.x * kT) {
        const float v = ar[i];
        if (mode == 0) {
            acc += v;
        } else {
            const float d = v - tr[i];
            acc += (double)d * d;
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < kT / 64; ++i) s += s_red[i];
        atomicAdd(&out[b], s);
    }
}

} // namespace

extern "C" int ccmi_row_reduce_f32(const float *a, int64_t a_stride, const float *t, int64_t t_stride, int64_t len,
                                   int batch, int mode, double *out, void *stream)
{
    if (!a || !out || batch < 1 || len < 0 || (mode == 1 && !t) || mode < 0 || mode > 1)
        return ccmi_set_error(CCMI_ERR_ARG, "row_reduce: bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    CCMI_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(double) * batch, s));
    if (len == 0) return CCMI_OK;
    const int64_t blocks = std::min<int64_t>((len + kT - 1) / kT, 256);
    hipLaunchKernelGGL(row_reduce, dim3((unsigned)blocks, batch), dim3(kT), 0, s, a, a_stride, t, t_stride, len, mode,
                       out);
    CCMI_HIP_CHECK(hipGetLastError());
    return CCMI_OK;
}
