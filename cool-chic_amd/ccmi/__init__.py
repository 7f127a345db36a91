"""ctypes binding of libccmi (include/ccmi.h), the MI355X hot-path library.

This module is plumbing: it loads ``cool-chic_amd/lib/libccmi.so`` (built in-tree by
``make -C cool-chic_amd`` / ``__graft_entry__.build()``), mirrors the C structs and
turns torch tensors into raw device pointers.  There is no CPU fallback: if the
library is missing every entry point raises ``CcmiUnavailable``.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("CCMI_LIB", PKG_ROOT / "lib" / "libccmi.so"))

MAX_GRIDS = 8
MAX_SYN_LAYERS = 16

OK, ERR_ARG, ERR_HIP, ERR_UNSUPPORTED, ERR_BITSTREAM, ERR_IO = range(6)

# Public symbols of include/ccmi.h (checked by tests/test_abi.py).
EXPORTED = [
    "ccmi_last_error", "ccmi_version", "ccmi_device_count",
    "ccmi_arm_forward_f32", "ccmi_arm_context_f32", "ccmi_arm_mlp_f32", "ccmi_ups_workspace_bytes", "ccmi_ups_forward_f32",
    "ccmi_syn_workspace_bytes", "ccmi_syn_forward_f32", "ccmi_post_f32", "ccmi_decode_forward_f32",
    "ccmi_decode_file", "ccmi_decode_batch", "ccmi_decode_output_size", "ccmi_decode_last_timing",
    "ccmi_decode_last_arm_flags", "ccmi_decode_latents", "ccmi_decode_batch_workspace_bytes", "ccmi_decode_batch_plan", "ccmi_decode_batch_ws", "ccmi_decode_weights_i32",
    "ccmi_ups_workspace_bytes_i32", "ccmi_ups_forward_i32", "ccmi_syn_workspace_bytes_i32", "ccmi_syn_forward_i32",
    "ccmi_cool_parse", "ccmi_code_wb", "ccmi_decode_wb", "ccmi_code_latent_layer", "ccmi_arm_forward_i32",
    "ccmi_encode_frame", "ccmi_row_reduce_f32", "ccmi_train_param_count", "ccmi_train_workspace_bytes", "ccmi_train_step",
    "ccmi_quantize_f32",
]


class CcmiUnavailable(RuntimeError):
    pass


class CcmiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ccmi error {code}: {msg}")
        self.code = code


class ArmArgs(C.Structure):
    _fields_ = [
        ("latent", C.c_void_p), ("latent_stride", C.c_int64), ("n_grids", C.c_int),
        ("h", C.c_int * MAX_GRIDS), ("w", C.c_int * MAX_GRIDS), ("gain", C.c_float),
        ("quantize", C.c_int), ("dim_arm", C.c_int), ("n_hidden", C.c_int),
        ("params", C.c_void_p), ("param_stride", C.c_int64),
        ("mu", C.c_void_p), ("scale", C.c_void_p), ("log_scale", C.c_void_p), ("rate", C.c_void_p),
        ("out_stride", C.c_int64), ("batch", C.c_int),
    ]


class UpsArgs(C.Structure):
    _fields_ = [
        ("latent", C.c_void_p), ("latent_stride", C.c_int64), ("n_grids", C.c_int),
        ("h", C.c_int * MAX_GRIDS), ("w", C.c_int * MAX_GRIDS), ("gain", C.c_float),
        ("quantize", C.c_int), ("ups_k", C.c_int), ("n_ups", C.c_int), ("pre_k", C.c_int),
        ("n_pre", C.c_int), ("params", C.c_void_p), ("param_stride", C.c_int64),
        ("out", C.c_void_p), ("out_stride", C.c_int64), ("workspace", C.c_void_p),
        ("workspace_bytes", C.c_size_t), ("batch", C.c_int),
    ]


class SynLayer(C.Structure):
    _fields_ = [("n_out", C.c_int), ("ks", C.c_int), ("residual", C.c_int), ("relu", C.c_int)]


class SynArgs(C.Structure):
    _fields_ = [
        ("in_", C.c_void_p), ("in_stride", C.c_int64), ("c_in", C.c_int), ("h", C.c_int), ("w", C.c_int),
        ("n_layers", C.c_int), ("layers", SynLayer * MAX_SYN_LAYERS), ("params", C.c_void_p),
        ("param_stride", C.c_int64), ("out", C.c_void_p), ("out_stride", C.c_int64),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t), ("batch", C.c_int),
    ]


class PostArgs(C.Structure):
    _fields_ = [
        ("in_", C.c_void_p), ("in_stride", C.c_int64), ("h", C.c_int), ("w", C.c_int),
        ("bitdepth", C.c_int), ("yuv420", C.c_int), ("out", C.c_void_p), ("out_stride", C.c_int64),
        ("batch", C.c_int),
    ]


class DecodeArgs(C.Structure):
    _fields_ = [
        ("ups", UpsArgs), ("syn", SynArgs), ("bitdepth", C.c_int), ("yuv420", C.c_int),
        ("out", C.c_void_p), ("out_stride", C.c_int64), ("stages", C.c_int), ("head", C.c_int),
    ]


HEAD_DEFAULT, HEAD_VALU, HEAD_MFMA, HEAD_GENERIC = 0, 1, 2, 3  # ccmi_decode_args.head (CCMI_HEAD_*)


_lib = None


def lib() -> C.CDLL:
    """Load libccmi once; raise CcmiUnavailable (never fall back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).  Load torch
    # first so that the process has ONE HIP runtime, shared by torch tensors / streams and
    # libccmi; loading libccmi first would pull /opt/rocm's runtime under torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise CcmiUnavailable(f"{LIB_PATH} not built: run `make -C cool-chic_amd` (or __graft_entry__.build())")
    L = C.CDLL(str(LIB_PATH))
    L.ccmi_last_error.restype = C.c_char_p
    L.ccmi_version.restype = C.c_int
    L.ccmi_device_count.restype = C.c_int
    for name, st in (("ccmi_arm_forward_f32", ArmArgs), ("ccmi_ups_forward_f32", UpsArgs),
                     ("ccmi_syn_forward_f32", SynArgs), ("ccmi_post_f32", PostArgs),
                     ("ccmi_decode_forward_f32", DecodeArgs)):
        f = getattr(L, name)
        f.argtypes = [C.POINTER(st), C.c_void_p]
        f.restype = C.c_int
    L.ccmi_arm_context_f32.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    L.ccmi_arm_context_f32.restype = C.c_int
    L.ccmi_arm_mlp_f32.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p]
    L.ccmi_arm_mlp_f32.restype = C.c_int
    L.ccmi_ups_workspace_bytes.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]
    L.ccmi_ups_workspace_bytes.restype = C.c_size_t
    L.ccmi_syn_workspace_bytes.argtypes = [C.POINTER(SynArgs)]
    L.ccmi_syn_workspace_bytes.restype = C.c_size_t
    L.ccmi_decode_file.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int]
    L.ccmi_decode_file.restype = C.c_int
    L.ccmi_decode_batch.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int,
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
                                    C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.ccmi_decode_batch.restype = C.c_int
    L.ccmi_decode_output_size.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(C.c_size_t)]
    L.ccmi_decode_output_size.restype = C.c_int
    L.ccmi_decode_last_timing.argtypes = [C.POINTER(C.c_float)]
    L.ccmi_decode_last_timing.restype = C.c_int
    if hasattr(L, "ccmi_decode_last_arm_flags"):  # absent from older builds loaded for A/B runs
        L.ccmi_decode_last_arm_flags.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_int)]
        L.ccmi_decode_last_arm_flags.restype = C.c_int
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != OK:
        raise CcmiError(rc, lib().ccmi_last_error().decode(errors="replace"))


def last_error() -> str:
    return lib().ccmi_last_error().decode(errors="replace")


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    """Device (or host) address of a contiguous tensor; None -> NULL."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("ccmi: tensors must be contiguous")
    return t.data_ptr()


def require_cuda(*ts) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("ccmi: HIP kernels need device tensors (no CPU fallback)")
