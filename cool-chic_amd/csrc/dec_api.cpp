// dec_api.cpp -- path B C-ABI entry points (fixed-point .cool decoder).  Placeholder
// until the HIP decoder lands: every call reports CCMI_ERR_UNSUPPORTED.
#include "ccmi_internal.h"

extern "C" int ccmi_decode_file(const char *, const char *, int, int, int, int)
{
    return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "decode: not implemented yet") ? 1 : 1;
}

extern "C" int ccmi_decode_batch(const uint8_t *const *, const size_t *, int, uint8_t *const *, const size_t *,
                                 size_t *, int, int, int, void *)
{
    return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "decode: not implemented yet");
}

extern "C" int ccmi_decode_output_size(const uint8_t *, size_t, int, int, int, size_t *)
{
    return ccmi_set_error(CCMI_ERR_UNSUPPORTED, "decode: not implemented yet");
}
