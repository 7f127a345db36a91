"""Path B writer (the .cool encoder side) over the C ABI.

Mirrors, on libccmi:
  * ``CCLIB.ccencapi.cc_code_wb_bac`` / ``cc_code_latent_layer_bac`` / ``cc_decode_wb``
    (reference coolchic/cpp/ccencapi.cpp:28-454)            -> ``code_wb``, ``code_latent_layer``,
                                                               ``decode_wb``
  * the integer ARM the encoder runs before CABAC coding (ArmInt pure_int,
    enc/bitstream/armint.py:80-261; encode.py:510-560)       -> ``arm_forward_i32`` (GPU)
  * ``encode_frame`` (enc/bitstream/encode.py:221-623) + headers
    (enc/bitstream/header.py:72-392)                          -> ``encode_frame`` (GPU ARM + host CABAC)
  * the headers read back (cc-bitstream.cpp:58-275)           -> ``parse``
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import check, lib, require_cuda

NN_SLOTS = ("arm_w", "arm_b", "ups_w", "ups_b", "syn_w", "syn_b")


class CoolDesc(C.Structure):
    _fields_ = [
        ("h", C.c_int), ("w", C.c_int), ("bitdepth", C.c_int), ("frame_data_type", C.c_int),
        ("intra_period", C.c_int), ("p_period", C.c_int), ("display_index", C.c_int),
        ("dim_arm", C.c_int), ("n_hidden_arm", C.c_int),
        ("n_ups", C.c_int), ("ups_k", C.c_int), ("n_pre", C.c_int), ("pre_k", C.c_int),
        ("n_branches", C.c_int), ("n_syn_layers", C.c_int),
        ("syn_out", C.c_int * 16), ("syn_ks", C.c_int * 16), ("syn_type", C.c_int * 16),
        ("flow_gain", C.c_int), ("ac_max_val_nn", C.c_int), ("ac_max_val_latent", C.c_int),
        ("hls_sig_blksize", C.c_int),
        ("q_step_index", C.c_int * 6), ("expgol_count", C.c_int * 6), ("n_bytes_nn", C.c_int * 6),
        ("n_grids", C.c_int), ("n_bytes_latent", C.c_int * 8),
        ("nn", C.c_void_p * 6), ("nn_len", C.c_int * 6),
    ]


class ArmI32Args(C.Structure):
    _fields_ = [
        ("latent", C.c_void_p), ("n_grids", C.c_int), ("h", C.c_int * 8), ("w", C.c_int * 8),
        ("dim_arm", C.c_int), ("n_hidden", C.c_int), ("params", C.c_void_p),
        ("mu", C.c_void_p), ("log_scale", C.c_void_p),
    ]


def _bind():
    L = lib()
    if getattr(L, "_ccmi_enc_bound", False):
        return L
    L.ccmi_cool_parse.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(CoolDesc), C.c_void_p, C.c_size_t]
    L.ccmi_code_wb.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                               C.POINTER(C.c_int)]
    L.ccmi_decode_wb.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ccmi_code_latent_layer.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.ccmi_arm_forward_i32.argtypes = [C.POINTER(ArmI32Args), C.c_void_p]
    L.ccmi_encode_frame.argtypes = [C.POINTER(CoolDesc), C.c_void_p, C.c_void_p, C.c_size_t,
                                    C.POINTER(C.c_size_t), C.c_void_p]
    for n in ("ccmi_cool_parse", "ccmi_code_wb", "ccmi_decode_wb", "ccmi_code_latent_layer",
              "ccmi_arm_forward_i32", "ccmi_encode_frame"):
        getattr(L, n).restype = C.c_int
    L._ccmi_enc_bound = True
    return L


def _i32(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.int64).astype(np.int32))


def _grow(call, first_cap: int) -> bytes:
    """Run a C call that writes into (buf, cap, *len); retry once with the size it asks for."""
    n = C.c_size_t(0)
    cap = max(first_cap, 64)
    for _ in range(2):
        buf = C.create_string_buffer(cap)
        rc = call(buf, cap, C.byref(n))
        if rc == 0:
            return buf.raw[: n.value]
        if n.value > cap:
            cap = n.value
            continue
        check(rc)
    check(rc)
    return b""


# ---------------------------------------------------------------- CCLIB.ccencapi surface
def code_wb(x: Sequence[int], use_count: int = -1) -> tuple[bytes, int]:
    """cc_code_wb_bac (ccencapi.cpp:97-177): returns (substream bytes, count used)."""
    L = _bind()
    a = _i32(x)
    used = C.c_int(-1)
    b = _grow(lambda buf, cap, n: L.ccmi_code_wb(a.ctypes.data, a.size, use_count, buf, cap, n, C.byref(used)),
              8 * a.size + 64)
    return b, used.value


def decode_wb(stream: bytes, runs: Sequence[tuple[int, int]]) -> list[np.ndarray]:
    """Decode consecutive runs [(n_weights, count), ...] of one network substream
    (cc_decode_wb::decode_wb_continue, ccencapi.cpp:439-454)."""
    L = _bind()
    ln = np.array([r[0] for r in runs], dtype=np.int32)
    ct = np.array([r[1] for r in runs], dtype=np.int32)
    out = np.zeros(int(ln.sum()) + 1, dtype=np.int32)
    buf = C.create_string_buffer(stream, len(stream))
    check(L.ccmi_decode_wb(C.cast(buf, C.c_void_p), len(stream), len(runs), ln.ctypes.data, ct.ctypes.data,
                           out.ctypes.data))
    res, p = [], 0
    for n in ln:
        res.append(out[p: p + n].copy())
        p += n
    return res


def code_latent_layer(x, mu, log_scale, h: int, w: int, hls_sig_blksize: int) -> bytes:
    """cc_code_latent_layer_bac (ccencapi.cpp:179-410): integer latents of one grid with
    the ARM's mu / log_scale in fixed point (x256)."""
    L = _bind()
    xa, ma, la = _i32(x), _i32(mu), _i32(log_scale)
    if not (xa.size == ma.size == la.size == h * w):
        raise ValueError(f"code_latent_layer: expected {h * w} values per array")
    return _grow(lambda buf, cap, n: L.ccmi_code_latent_layer(xa.ctypes.data, ma.ctypes.data, la.ctypes.data,
                                                              h, w, hls_sig_blksize, buf, cap, n), 4 * h * w + 256)


# ---------------------------------------------------------------- frame level
@dataclass
class CoolFrame:
    """Header fields + quantised network integers of one intra .cool frame."""
    desc: CoolDesc
    nn: dict = field(default_factory=dict)  # slot name -> np.int32 array

    @property
    def grid_sizes(self) -> list[tuple[int, int]]:
        out, h, w = [], self.desc.h, self.desc.w
        for _ in range(self.desc.n_grids):
            out.append((h, w))
            h, w = (h + 1) // 2, (w + 1) // 2
        return out

    def arm_params(self) -> np.ndarray:
        """Decoder-side ARM integers (read_arm, cc-frame-decoder.cpp:201-258)."""
        d, nh = self.desc.dim_arm, self.desc.n_hidden_arm
        sw, sb = self.desc.q_step_index[0], self.desc.q_step_index[1]
        W = self.nn["arm_w"].astype(np.int64) << sw
        B = self.nn["arm_b"].astype(np.int64) << sb
        out, pw, pb = [], 0, 0
        for l in range(nh + 1):
            n_out = d if l < nh else 2
            out += [W[pw: pw + n_out * d], B[pb: pb + n_out]]
            pw += n_out * d
            pb += n_out
        return np.concatenate(out).astype(np.int32)


def parse(stream: bytes) -> CoolFrame:
    """GOP + frame header and the network integers of an intra .cool stream."""
    L = _bind()
    d = CoolDesc()
    cap = 1 << 16
    nn = np.zeros(cap, dtype=np.int32)
    buf = C.create_string_buffer(stream, len(stream))
    check(L.ccmi_cool_parse(C.cast(buf, C.c_void_p), len(stream), C.byref(d), nn.ctypes.data, cap))
    base = nn.ctypes.data
    f = CoolFrame(desc=d)
    for k, name in enumerate(NN_SLOTS):
        n = d.nn_len[k]
        off = ((d.nn[k] or base) - base) // 4
        f.nn[name] = nn[off: off + n].copy()
    return f


def arm_forward_i32(latent, sizes: Sequence[tuple[int, int]], dim_arm: int, n_hidden: int, params):
    """Integer ARM over every latent (device int32 tensors): returns (mu, log_scale), x256."""
    import torch
    require_cuda(latent, params)
    if latent.dtype != torch.int32 or params.dtype != torch.int32:
        raise ValueError("arm_forward_i32: int32 tensors expected")
    n = sum(h * w for h, w in sizes)
    if latent.numel() < n:
        raise ValueError(f"arm_forward_i32: {latent.numel()} latents, grids need {n}")
    mu = torch.empty(n, dtype=torch.int32, device=latent.device)
    ls = torch.empty_like(mu)
    a = ArmI32Args()
    a.latent, a.n_grids = latent.data_ptr(), len(sizes)
    for i, (h, w) in enumerate(sizes):
        a.h[i], a.w[i] = h, w
    a.dim_arm, a.n_hidden, a.params = dim_arm, n_hidden, params.data_ptr()
    a.mu, a.log_scale = mu.data_ptr(), ls.data_ptr()
    check(_bind().ccmi_arm_forward_i32(C.byref(a), torch.cuda.current_stream(latent.device).cuda_stream))
    return mu, ls


def encode_frame(frame: CoolFrame, latent, search_counts: bool = False) -> bytes:
    """Write a whole .cool stream for integer latents (device int32, grids flattened):
    GPU ARM contexts + host CABAC (encode.py:221-623).  search_counts: ignore the frame's
    Exp-Golomb counts and search 0..12 per network slot (use_count = -1)."""
    import torch
    require_cuda(latent)
    if latent.dtype != torch.int32 or not latent.is_contiguous():
        raise ValueError("encode_frame: contiguous int32 device latents expected")
    L = _bind()
    d = CoolDesc.from_buffer_copy(frame.desc)
    keep = []
    for k, name in enumerate(NN_SLOTS):
        a = _i32(frame.nn.get(name, np.zeros(0, np.int32)))
        keep.append(a)
        d.nn[k] = a.ctypes.data if a.size else None
        d.nn_len[k] = a.size
        if search_counts:
            d.expgol_count[k] = -1
    n = sum(h * w for h, w in frame.grid_sizes)
    if latent.numel() < n:
        raise ValueError(f"encode_frame: {latent.numel()} latents given, the frame's grids hold {n}")
    s = torch.cuda.current_stream(latent.device).cuda_stream
    out = _grow(lambda buf, cap, ln: L.ccmi_encode_frame(C.byref(d), latent.data_ptr(), buf, cap, ln, s),
                4 * n + (1 << 16))
    frame.desc = d
    return out


def write_cool(arch, latent, qm, yuv420: bool = True, bitdepth: int = 8, hls_sig_blksize: int = -16) -> bytes:
    """Turn a trained, quantize_model-ed frame into a .cool stream (encode.py:221-623,
    header.py:236-392): latent [N] float (GPU, before gain), qm a ccmi.quantize.QuantizedModel
    with the ccmi.train parameter layout."""
    import torch
    from .quantize import Layout
    lay = Layout.of(arch)
    p = np.asarray(qm.params, dtype=np.float32)

    def sent(idx, q):  # the integers cc_code_wb_bac codes: round(v / q_step), exact here
        return np.round(p[idx] / np.float32(q)).astype(np.int64)

    nn = {
        "arm_w": sent(lay.arm_w, qm.q_step["arm"][0]), "arm_b": sent(lay.arm_b, qm.q_step["arm"][1]),
        "ups_w": sent(lay.ups_w, qm.q_step["upsampling"][0]), "ups_b": np.zeros(0, np.int64),
        "syn_w": sent(lay.syn_w, qm.q_step["synthesis"][0]), "syn_b": sent(lay.syn_b, qm.q_step["synthesis"][1]),
    }
    d = CoolDesc()
    d.h, d.w = arch.sizes[0]
    d.bitdepth, d.frame_data_type = bitdepth, 1 if yuv420 else 0
    d.intra_period = d.p_period = d.display_index = 0
    d.dim_arm, d.n_hidden_arm = arch.dim_arm, arch.n_hidden
    d.n_ups = d.n_pre = arch.n_grids - 1
    d.ups_k, d.pre_k = arch.ups_k, arch.pre_k
    d.n_branches, d.n_syn_layers = 1, len(arch.layers)
    for i, (n, k, res, relu) in enumerate(arch.layers):
        d.syn_out[i], d.syn_ks[i] = int(n), int(k)
        d.syn_type[i] = 16 * int(bool(res)) + int(bool(relu))  # mode index * 16 + non-linearity index
    d.flow_gain = 1
    # get_ac_max_val_nn also counts the (zero) upsampling biases the reference keeps
    d.ac_max_val_nn = int(np.ceil(max(int(np.abs(v).max(initial=0)) for v in nn.values()) + 2))
    yq = torch.round(latent.detach().float() * arch.gain).to(torch.int32).contiguous()
    d.ac_max_val_latent = int(yq.abs().max().item()) + 2
    d.hls_sig_blksize = hls_sig_blksize
    qi = [qm.q_index["arm"][0], qm.q_index["arm"][1], qm.q_index["upsampling"][0], 0,
          qm.q_index["synthesis"][0], qm.q_index["synthesis"][1]]
    ec = [qm.expgol["arm"][0], qm.expgol["arm"][1], qm.expgol["upsampling"][0], 0,
          qm.expgol["synthesis"][0], qm.expgol["synthesis"][1]]
    for k in range(6):
        d.q_step_index[k], d.expgol_count[k] = qi[k], ec[k]
    d.n_grids = arch.n_grids
    return encode_frame(CoolFrame(desc=d, nn=nn), yq)


__all__ = ["CoolDesc", "CoolFrame", "parse", "write_cool", "code_wb", "decode_wb", "code_latent_layer", "arm_forward_i32",
           "encode_frame", "NN_SLOTS"]
