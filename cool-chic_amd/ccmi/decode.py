"""Path B (bit-exact .cool decoder) launchers over the C ABI."""

from __future__ import annotations

import ctypes as C
from typing import Sequence

from . import MAX_GRIDS, MAX_SYN_LAYERS, CcmiError, SynLayer, check, lib


class UpsI32Args(C.Structure):
    _fields_ = [("latent", C.c_void_p), ("n_grids", C.c_int), ("h", C.c_int * MAX_GRIDS), ("w", C.c_int * MAX_GRIDS),
                ("kernels", C.c_void_p), ("ups_k", C.c_int), ("n_ups", C.c_int), ("pre_k", C.c_int), ("n_pre", C.c_int),
                ("out", C.c_void_p), ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t)]


class SynI32Args(C.Structure):
    _fields_ = [("in_", C.c_void_p), ("c_in", C.c_int), ("h", C.c_int), ("w", C.c_int), ("n_layers", C.c_int),
                ("layers", SynLayer * MAX_SYN_LAYERS), ("params", C.c_void_p), ("out", C.c_void_p),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t)]


def _bind():
    L = lib()
    if not getattr(L, "_ccmi_dec_bound", False):
        L.ccmi_decode_weights_i32.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                              C.c_void_p, C.c_size_t, C.c_void_p]
        L.ccmi_ups_workspace_bytes_i32.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
        L.ccmi_ups_workspace_bytes_i32.restype = C.c_size_t
        L.ccmi_ups_forward_i32.argtypes = [C.POINTER(UpsI32Args), C.c_void_p]
        L.ccmi_syn_workspace_bytes_i32.argtypes = [C.POINTER(SynI32Args)]
        L.ccmi_syn_workspace_bytes_i32.restype = C.c_size_t
        L.ccmi_syn_forward_i32.argtypes = [C.POINTER(SynI32Args), C.c_void_p]
        L.ccmi_decode_batch_workspace_bytes.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                        C.c_void_p]
        L.ccmi_decode_batch_ws.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                           C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]
        L.ccmi_decode_batch_plan.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                             C.c_void_p]
        L._ccmi_dec_bound = True
    return L


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


class _PinnedPool:
    """Grow-only pinned host buffer per thread for decode_batch's outputs: the decoder's
    per-chunk downloads are then DMA copies that overlap the rest of the batch, and the
    buffer is reused across calls (hipHostMalloc of a GB-sized buffer costs more than the
    decode).  Like the reference decoder's frame_memory (cc-frame-decoder.cpp:1151), what
    decode_batch(views=True) returns stays valid until the next call on this thread."""

    def __init__(self):
        import threading
        self.tls = threading.local()

    def get(self, nbytes: int):
        import torch
        t = getattr(self.tls, "buf", None)
        if t is None or t.numel() < nbytes:
            self.tls.buf = None
            t = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
            self.tls.buf = t
        return t


_POOL = _PinnedPool()


def decode_batch(streams: Sequence[bytes], output_bitdepth: int = 0, output_chroma_format: int = 0,
                 as_yuv: bool = True, stream_handle: int | None = None, workspace=None, views: bool = False) -> list:
    """Decode independent intra .cool streams in one batched launch sequence; returns the
    bytes the reference decoder would write for each (YUV planes, or PPM).

    One header-only pass sizes the outputs and the device workspace
    (ccmi_decode_batch_plan); the outputs land in a pinned host pool and the device
    workspace comes from torch's caching allocator unless `workspace` (a uint8 CUDA tensor of
    at least decode_batch_workspace_bytes(...) bytes) is given: ccmi_decode_batch_ws, no
    allocation inside the library.  views=True returns memoryviews into the pool (no copy;
    valid until the next call on this thread), otherwise bytes."""
    import torch
    n = len(streams)
    if n < 1:
        raise ValueError("decode_batch: no streams")
    bufs = [C.create_string_buffer(s, len(s)) for s in streams]
    sp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    ln = (C.c_size_t * n)(*[len(s) for s in streams])
    cap = (C.c_size_t * n)()
    need = C.c_size_t(0)
    L = _bind()
    check(L.ccmi_decode_batch_plan(sp, ln, n, output_bitdepth, output_chroma_format, int(as_yuv), cap, C.byref(need)))
    offs, tot = [], 0
    for k in cap:
        offs.append(tot)
        tot += (int(k) + 255) // 256 * 256
    pool = _POOL.get(tot)
    base = pool.data_ptr()
    op = (C.c_void_p * n)(*[base + o for o in offs])
    got = (C.c_size_t * n)()
    dev = torch.device("cuda", torch.cuda.current_device())
    if stream_handle is None:
        stream_handle = torch.cuda.current_stream(dev).cuda_stream
    if workspace is None:
        workspace = torch.empty(max(int(need.value), 256), dtype=torch.uint8, device=dev)
    check(L.ccmi_decode_batch_ws(sp, ln, n, op, cap, got, output_bitdepth, output_chroma_format, int(as_yuv),
                                 workspace.data_ptr(), workspace.numel(), stream_handle))
    mv = memoryview(pool.numpy())
    if views:
        return [mv[o: o + got[i]] for i, o in enumerate(offs)]
    return [bytes(mv[o: o + got[i]]) for i, o in enumerate(offs)]


def decode_batch_workspace_bytes(streams: Sequence[bytes], output_bitdepth: int = 0, output_chroma_format: int = 0,
                                 as_yuv: bool = True) -> int:
    n = len(streams)
    bufs = [C.create_string_buffer(s, len(s)) for s in streams]
    sp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    ln = (C.c_size_t * n)(*[len(s) for s in streams])
    out = C.c_size_t(0)
    check(_bind().ccmi_decode_batch_workspace_bytes(sp, ln, n, output_bitdepth, output_chroma_format, int(as_yuv),
                                                    C.byref(out)))
    return out.value


def weights_i32(stream: bytes):
    """(arm, ups, syn) fixed-point network integers of a stream's intra frame, as the
    decoder uses them (ccmi_decode_weights_i32; cc-frame-decoder.cpp:201-353)."""
    import numpy as np
    L = _bind()
    buf = C.create_string_buffer(stream, len(stream))
    cnt = (C.c_size_t * 3)()
    check(L.ccmi_decode_weights_i32(C.cast(buf, C.c_void_p), len(stream), None, 0, None, 0, None, 0, cnt))
    arr = [np.zeros(max(int(c), 1), dtype=np.int32) for c in cnt]
    check(L.ccmi_decode_weights_i32(C.cast(buf, C.c_void_p), len(stream), arr[0].ctypes.data, arr[0].size,
                                    arr[1].ctypes.data, arr[1].size, arr[2].ctypes.data, arr[2].size, cnt))
    return tuple(a[: int(c)] for a, c in zip(arr, cnt))


def ups_forward_i32(latent, sizes, kernels, ups_k: int, n_ups: int, pre_k: int, n_pre: int):
    """Integer upsampling on the GPU (ccmi_ups_forward_i32): latent int32 [N] (value << 8,
    grids flat in order), kernels int32 (weights_i32()[1]) -> int32 [L, H, W]."""
    import torch
    from . import require_cuda
    require_cuda(latent, kernels)
    L = _bind()
    n = len(sizes)
    h = (C.c_int * MAX_GRIDS)(*[s[0] for s in sizes])
    w = (C.c_int * MAX_GRIDS)(*[s[1] for s in sizes])
    if latent.dtype != torch.int32 or latent.numel() < sum(a * b for a, b in sizes):
        raise ValueError("latent: int32 with sum(h * w) elements expected")
    if kernels.dtype != torch.int32:
        raise ValueError("kernels: int32 expected (weights_i32()[1])")
    latent, kernels = latent.contiguous(), kernels.contiguous()  # held until after the launch
    out = torch.empty(n, sizes[0][0], sizes[0][1], dtype=torch.int32, device=latent.device)
    nws = L.ccmi_ups_workspace_bytes_i32(n, h, w)
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=latent.device)
    a = UpsI32Args(latent=latent.data_ptr(), n_grids=n, h=h, w=w, kernels=kernels.data_ptr(), ups_k=ups_k,
                   n_ups=n_ups, pre_k=pre_k, n_pre=n_pre, out=out.data_ptr(), workspace=ws.data_ptr(), workspace_bytes=nws)
    check(L.ccmi_ups_forward_i32(C.byref(a), torch.cuda.current_stream(latent.device).cuda_stream))
    return out


def syn_forward_i32(x, layers, params):
    """Integer synthesis of one branch on the GPU (ccmi_syn_forward_i32): x int32 [C, H, W]
    at precision 12, layers [(n_out, ks, residual, relu)], params int32 -> int32 [n_out, H, W]."""
    import torch
    from . import require_cuda
    require_cuda(x, params)
    L = _bind()
    c, hh, ww = x.shape
    arr = (SynLayer * MAX_SYN_LAYERS)()
    for i, (n_out, ks, res, relu) in enumerate(layers):
        arr[i] = SynLayer(int(n_out), int(ks), int(res), int(relu))
    if x.dtype != torch.int32 or params.dtype != torch.int32:
        raise ValueError("syn_forward_i32: int32 input and params expected")
    x, params = x.contiguous(), params.contiguous()  # held until after the launch
    out = torch.empty(layers[-1][0], hh, ww, dtype=torch.int32, device=x.device)
    a = SynI32Args(in_=x.data_ptr(), c_in=c, h=hh, w=ww, n_layers=len(layers), layers=arr,
                   params=params.data_ptr(), out=out.data_ptr(), workspace=None, workspace_bytes=0)
    nws = L.ccmi_syn_workspace_bytes_i32(C.byref(a))
    ws = None
    if nws:
        ws = torch.empty(nws, dtype=torch.uint8, device=x.device)
        a.workspace, a.workspace_bytes = ws.data_ptr(), nws
    check(L.ccmi_syn_forward_i32(C.byref(a), torch.cuda.current_stream(x.device).cuda_stream))
    return out


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


# CCMI_ARM_FLAG_* (include/ccmi.h): what the latent decode of a stream did
ARM_FLAG_TIMEOUT, ARM_FLAG_Q32, ARM_FLAG_W32, ARM_FLAG_PRE32, ARM_FLAG_BIG = 1, 2, 4, 8, 16


def last_arm_flags() -> list[int]:
    """Per stream of this thread's last decode call: the OR of its latent grids'
    CCMI_ARM_FLAG_* bits (which multiply forms the ARM kernels ran; TIMEOUT = the call failed)."""
    L = lib()
    n = C.c_int(0)
    check(L.ccmi_decode_last_arm_flags(None, 0, C.byref(n)))
    out = (C.c_uint32 * max(n.value, 1))()
    check(L.ccmi_decode_last_arm_flags(out, n.value, C.byref(n)))
    return [int(v) for v in out[: n.value]]


__all__ = ["last_timing", "last_arm_flags", "decode_latents", "decode_file", "decode_batch", "decode_batch_workspace_bytes", "output_size",
           "weights_i32", "ups_forward_i32", "syn_forward_i32", "CcmiError"]
