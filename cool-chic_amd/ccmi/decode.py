"""Path B (bit-exact .cool decoder) launchers over the C ABI."""

from __future__ import annotations

import ctypes as C
from typing import Sequence

from . import CcmiError, check, lib


def decode_file(inp: str, out: str = "", output_bitdepth: int = 0, output_chroma_format: int = 0,
                verbosity: int = 0, device: int = 0) -> int:
    """Same contract as the reference's cc_decode_cpu (ccdecapi_cpu.cpp:20-30): returns 0 / 1."""
    return lib().ccmi_decode_file(inp.encode(), out.encode(), output_bitdepth, output_chroma_format, verbosity,
                                  device)


def output_size(stream: bytes, output_bitdepth: int = 0, output_chroma_format: int = 0, as_yuv: bool = True) -> int:
    n = C.c_size_t(0)
    buf = C.create_string_buffer(stream, len(stream))
    check(lib().ccmi_decode_output_size(C.cast(buf, C.c_void_p), len(stream), output_bitdepth,
                                        output_chroma_format, int(as_yuv), C.byref(n)))
    return n.value


def decode_batch(streams: Sequence[bytes], output_bitdepth: int = 0, output_chroma_format: int = 0,
                 as_yuv: bool = True, stream_handle: int | None = None) -> list[bytes]:
    """Decode independent intra .cool streams in one batched launch sequence; returns the
    bytes the reference decoder would write for each (YUV planes, or PPM)."""
    n = len(streams)
    bufs = [C.create_string_buffer(s, len(s)) for s in streams]
    sizes = [output_size(s, output_bitdepth, output_chroma_format, as_yuv) for s in streams]
    outs = [C.create_string_buffer(k) for k in sizes]
    sp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    ln = (C.c_size_t * n)(*[len(s) for s in streams])
    op = (C.c_void_p * n)(*[C.cast(o, C.c_void_p) for o in outs])
    cap = (C.c_size_t * n)(*sizes)
    got = (C.c_size_t * n)()
    if stream_handle is None:
        import torch
        stream_handle = torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else None
    check(lib().ccmi_decode_batch(sp, ln, n, op, cap, got, output_bitdepth, output_chroma_format, int(as_yuv),
                                  stream_handle))
    return [o.raw[: got[i]] for i, o in enumerate(outs)]


def decode_latents(stream: bytes, stream_handle: int | None = None) -> list:
    """Integer latents of an intra .cool stream, decoded on the GPU (one np.int32 array
    per grid, row-major)."""
    import numpy as np
    from . import encode
    fr = encode.parse(stream)
    n = sum(h * w for h, w in fr.grid_sizes)
    out = np.zeros(n, dtype=np.int32)
    buf = C.create_string_buffer(stream, len(stream))
    L = lib()
    L.ccmi_decode_latents.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    L.ccmi_decode_latents.restype = C.c_int
    if stream_handle is None:
        import torch
        stream_handle = torch.cuda.current_stream().cuda_stream
    check(L.ccmi_decode_latents(C.cast(buf, C.c_void_p), len(stream), out.ctypes.data, n, stream_handle))
    res, p = [], 0
    for h, w in fr.grid_sizes:
        res.append(out[p: p + h * w].copy())
        p += h * w
    return res


def last_timing() -> dict:
    """Device stage times (ms) of this thread's last decode: upload, arm_cabac, ups_syn_out, download."""
    ms = (C.c_float * 4)()
    check(lib().ccmi_decode_last_timing(ms))
    return dict(zip(("upload", "arm_cabac", "ups_syn_out", "download"), list(ms)))


__all__ = ["last_timing", "decode_latents", "decode_file", "decode_batch", "output_size", "CcmiError"]
