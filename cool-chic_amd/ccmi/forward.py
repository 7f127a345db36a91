"""Path A (float forward) launchers: torch tensors in, torch tensors out.

Each function validates shapes on the host (the kernels trust them), packs the
arguments into the C structs of include/ccmi.h and enqueues the HIP kernels on the
current torch stream.  All tensors must already live on the GPU.
"""

from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import (ArmArgs, DecodeArgs, MAX_GRIDS, MAX_SYN_LAYERS, PostArgs, SynArgs, SynLayer, UpsArgs, check, lib, ptr,
               require_cuda, stream_handle)


def _grid_arrays(sizes: Sequence[tuple[int, int]]):
    if not 1 <= len(sizes) <= MAX_GRIDS:
        raise ValueError(f"1..{MAX_GRIDS} latent grids supported, got {len(sizes)}")
    h = (ctypes.c_int * MAX_GRIDS)()
    w = (ctypes.c_int * MAX_GRIDS)()
    for i, (hh, ww) in enumerate(sizes):
        h[i], w[i] = int(hh), int(ww)
    return h, w


def n_latents(sizes) -> int:
    return sum(int(h) * int(w) for h, w in sizes)


def arm_param_count(dim_arm: int, n_hidden: int) -> int:
    return n_hidden * (dim_arm * dim_arm + dim_arm) + 2 * dim_arm + 2


def pack_arm(layers: Sequence[tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
    """[(W [out,in], b [out]) for each mlp linear] -> flat float32 (ccmi_arm_args.params order)."""
    return torch.cat([t.reshape(-1).float() for wb in layers for t in wb])


def pack_ups(ups: Sequence[torch.Tensor], pre: Sequence[torch.Tensor]) -> torch.Tensor:
    """Full (already symmetric) 1-D kernels -> flat float32 (ccmi_ups_args.params order)."""
    return torch.cat([k.reshape(-1).float() for k in list(ups) + list(pre)])


def pack_syn(layers: Sequence[tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
    return torch.cat([t.reshape(-1).float() for wb in layers for t in wb])


def _as_batch(params: torch.Tensor, B: int):
    """[P] -> shared by every frame (stride 0); [B, P] -> one parameter block per frame."""
    if params.dim() == 1:
        return params.unsqueeze(0), 0
    if params.shape[0] != B:
        raise ValueError(f"params: expected {B} parameter rows, got {params.shape[0]}")
    return params, params.shape[1]


def arm_forward(latent: torch.Tensor, sizes, params: torch.Tensor, dim_arm: int, n_hidden: int,
                gain: float = 16.0, quantize: bool = True, want=("mu", "scale", "log_scale", "rate")) -> dict:
    """latent [B, N] (or [N]) flat grids; params [B, P] (or [P]).  Returns dict of [B, N] tensors."""
    squeeze = latent.dim() == 1
    latent = latent.unsqueeze(0) if squeeze else latent
    B, N = latent.shape
    params, pstride = _as_batch(params, B)
    require_cuda(latent, params)
    if N != n_latents(sizes):
        raise ValueError(f"latent has {N} values, grids hold {n_latents(sizes)}")
    if params.shape[1] < arm_param_count(dim_arm, n_hidden):
        raise ValueError("arm params: expected [B, >=%d]" % arm_param_count(dim_arm, n_hidden))
    latent = latent.float().contiguous()
    params = params.float().contiguous()
    outs = {k: torch.empty(B, N, device=latent.device, dtype=torch.float32) for k in want}
    h, w = _grid_arrays(sizes)
    a = ArmArgs(latent=ptr(latent), latent_stride=N, n_grids=len(sizes), h=h, w=w, gain=float(gain),
                quantize=int(bool(quantize)), dim_arm=dim_arm, n_hidden=n_hidden, params=ptr(params),
                param_stride=pstride, mu=ptr(outs.get("mu")), scale=ptr(outs.get("scale")),
                log_scale=ptr(outs.get("log_scale")), rate=ptr(outs.get("rate")), out_stride=N, batch=B)
    check(lib().ccmi_arm_forward_f32(a, stream_handle(latent.device)))
    if squeeze:
        outs = {k: v[0] for k, v in outs.items()}
    return outs


def ups_forward(latent: torch.Tensor, sizes, params: torch.Tensor, ups_k: int, n_ups: int, pre_k: int, n_pre: int,
                gain: float = 16.0, quantize: bool = True) -> torch.Tensor:
    """latent [B, N] flat grids -> [B, L, H, W] dense synthesis input."""
    squeeze = latent.dim() == 1
    latent = latent.unsqueeze(0) if squeeze else latent
    B, N = latent.shape
    params, pstride = _as_batch(params, B)
    require_cuda(latent, params)
    if N != n_latents(sizes):
        raise ValueError(f"latent has {N} values, grids hold {n_latents(sizes)}")
    if params.shape[1] < n_ups * ups_k + n_pre * pre_k:
        raise ValueError("ups params: wrong shape")
    latent = latent.float().contiguous()
    params = params.float().contiguous()
    L = len(sizes)
    H, W = sizes[0]
    out = torch.empty(B, L, H, W, device=latent.device, dtype=torch.float32)
    h, w = _grid_arrays(sizes)
    nws = lib().ccmi_ups_workspace_bytes(L, h, w, B)
    ws = torch.empty(max(nws, 4), device=latent.device, dtype=torch.uint8)
    a = UpsArgs(latent=ptr(latent), latent_stride=N, n_grids=L, h=h, w=w, gain=float(gain),
                quantize=int(bool(quantize)), ups_k=ups_k, n_ups=n_ups, pre_k=pre_k, n_pre=n_pre,
                params=ptr(params), param_stride=pstride, out=ptr(out), out_stride=L * H * W,
                workspace=ptr(ws), workspace_bytes=nws, batch=B)
    check(lib().ccmi_ups_forward_f32(a, stream_handle(latent.device)))
    return out[0] if squeeze else out


def _syn_args(x, layers, params, out, B, C, H, W, pstride=None):
    if len(layers) > MAX_SYN_LAYERS:
        raise ValueError("too many synthesis layers")
    arr = (SynLayer * MAX_SYN_LAYERS)()
    for i, (n_out, ks, res, relu) in enumerate(layers):
        arr[i] = SynLayer(int(n_out), int(ks), int(bool(res)), int(bool(relu)))
    return SynArgs(in_=ptr(x), in_stride=C * H * W, c_in=C, h=H, w=W, n_layers=len(layers), layers=arr,
                   params=ptr(params), param_stride=params.shape[1] if pstride is None else pstride, out=ptr(out),
                   out_stride=out.shape[1] * H * W, workspace=None, workspace_bytes=0, batch=B)


def syn_param_count(c_in: int, layers) -> int:
    n, c = 0, c_in
    for n_out, ks, _, _ in layers:
        n += n_out * c * ks * ks + n_out
        c = n_out
    return n


def syn_forward(x: torch.Tensor, layers, params: torch.Tensor) -> torch.Tensor:
    """x [B, C, H, W]; layers [(n_out, ks, residual, relu)]; params [B, P] -> [B, n_out_last, H, W]."""
    squeeze = x.dim() == 3
    x = x.unsqueeze(0) if squeeze else x
    B, Cc, H, W = x.shape
    params, pstride = _as_batch(params, B)
    require_cuda(x, params)
    if params.shape[1] < syn_param_count(Cc, layers):
        raise ValueError("syn params: wrong shape")
    x = x.float().contiguous()
    params = params.float().contiguous()
    out = torch.empty(B, int(layers[-1][0]), H, W, device=x.device, dtype=torch.float32)
    a = _syn_args(x, layers, params, out, B, Cc, H, W, pstride)
    nws = lib().ccmi_syn_workspace_bytes(a)
    ws = None
    if nws:
        ws = torch.empty(nws, device=x.device, dtype=torch.uint8)
        a.workspace, a.workspace_bytes = ptr(ws), nws
    check(lib().ccmi_syn_forward_f32(a, stream_handle(x.device)))
    return out[0] if squeeze else out


def post_forward(x: torch.Tensor, bitdepth: int = 8, yuv420: bool = False) -> torch.Tensor:
    """Eval post-processing of FrameEncoder.forward.  yuv420 -> flat [B, H*W + 2*(H/2)*(W/2)]."""
    squeeze = x.dim() == 3
    x = x.unsqueeze(0) if squeeze else x
    require_cuda(x)
    B, Cc, H, W = x.shape
    if Cc != 3:
        raise ValueError("post-processing expects 3 channels")
    x = x.float().contiguous()
    n = H * W + 2 * (H // 2) * (W // 2) if yuv420 else 3 * H * W
    out = torch.empty(B, n, device=x.device, dtype=torch.float32)
    a = PostArgs(in_=ptr(x), in_stride=3 * H * W, h=H, w=W, bitdepth=bitdepth, yuv420=int(bool(yuv420)),
                 out=ptr(out), out_stride=n, batch=B)
    check(lib().ccmi_post_f32(a, stream_handle(x.device)))
    if not yuv420:
        out = out.view(B, 3, H, W)
    return out[0] if squeeze else out


def decode_forward(latent: torch.Tensor, sizes, ups_params: torch.Tensor, ups_k: int, n_ups: int, pre_k: int,
                   n_pre: int, layers, syn_params: torch.Tensor, gain: float = 16.0, quantize: bool = True,
                   bitdepth: int = 8, yuv420: bool = False, head: int = 0, fold: bool = False) -> torch.Tensor:
    """Fused upsampling -> synthesis -> post (ccmi_decode_forward_f32): latent [B, N] ->
    post-processed frames (layout of post_forward), or with bitdepth=0 the raw synthesis
    output [B, C_out, H, W].  head: ccmi.HEAD_* (the 1x1 head on the VALU or on f32 MFMA).
    fold=True also evaluates the level-2 -> 1 upsampling step inside the fused kernel (stages
    bit 3, opt-in: the same values bit for bit, measured slower).
    Raises CcmiError(ERR_UNSUPPORTED) for architectures without a fused kernel (use
    ups_forward / syn_forward / post_forward)."""
    squeeze = latent.dim() == 1
    latent = latent.unsqueeze(0) if squeeze else latent
    B, N = latent.shape
    ups_params, ups_stride = _as_batch(ups_params, B)
    syn_params, syn_stride = _as_batch(syn_params, B)
    require_cuda(latent, ups_params, syn_params)
    if N != n_latents(sizes):
        raise ValueError(f"latent has {N} values, grids hold {n_latents(sizes)}")
    L = len(sizes)
    H, W = sizes[0]
    if ups_params.shape[1] < n_ups * ups_k + n_pre * pre_k:
        raise ValueError("ups params: wrong shape")
    if syn_params.shape[1] < syn_param_count(L, layers):
        raise ValueError("syn params: wrong shape")
    latent = latent.float().contiguous()
    ups_params = ups_params.float().contiguous()
    syn_params = syn_params.float().contiguous()
    n_out = int(layers[-1][0])
    if bitdepth > 0:
        n = H * W + 2 * (H // 2) * (W // 2) if yuv420 else n_out * H * W
    else:
        n = n_out * H * W
    out = torch.empty(B, n, device=latent.device, dtype=torch.float32)
    h, w = _grid_arrays(sizes)
    nws = lib().ccmi_ups_workspace_bytes(L, h, w, B)
    ws = torch.empty(max(nws, 4), device=latent.device, dtype=torch.uint8)
    u = UpsArgs(latent=ptr(latent), latent_stride=N, n_grids=L, h=h, w=w, gain=float(gain),
                quantize=int(bool(quantize)), ups_k=ups_k, n_ups=n_ups, pre_k=pre_k, n_pre=n_pre,
                params=ptr(ups_params), param_stride=ups_stride, out=None, out_stride=0,
                workspace=ptr(ws), workspace_bytes=nws, batch=B)
    y = _syn_args(latent, layers, syn_params, out.view(B, -1, H, W) if (bitdepth == 0 or not yuv420) else out,
                  B, L, H, W, syn_stride)
    y.in_ = None
    a = DecodeArgs(ups=u, syn=y, bitdepth=int(bitdepth), yuv420=int(bool(yuv420)), out=ptr(out), out_stride=n,
                   head=int(head), stages=8 if fold else 0)
    check(lib().ccmi_decode_forward_f32(a, stream_handle(latent.device)))
    if bitdepth == 0 or not yuv420:
        out = out.view(B, n_out, H, W)
    return out[0] if squeeze else out


def split_420(flat: torch.Tensor, H: int, W: int) -> dict:
    """Flat 420 output of post_forward -> {'y': [..,H,W], 'u','v': [..,H/2,W/2]} views."""
    lead = flat.shape[:-1]
    hc, wc = H // 2, W // 2
    y = flat[..., : H * W].reshape(*lead, H, W)
    u = flat[..., H * W: H * W + hc * wc].reshape(*lead, hc, wc)
    v = flat[..., H * W + hc * wc:].reshape(*lead, hc, wc)
    return {"y": y, "u": u, "v": v}


def arm_context(grid: torch.Tensor, dim_arm: int) -> torch.Tensor:
    """_get_neighbor on device: grid [B, H, W] (or [H, W]) -> [B, H*W, dim_arm]."""
    squeeze = grid.dim() == 2
    grid = grid.unsqueeze(0) if squeeze else grid
    require_cuda(grid)
    grid = grid.float().contiguous()
    B, H, W = grid.shape
    out = torch.empty(B, H * W, dim_arm, device=grid.device, dtype=torch.float32)
    check(lib().ccmi_arm_context_f32(ptr(grid), B, H, W, dim_arm, ptr(out), stream_handle(grid.device)))
    return out[0] if squeeze else out


def arm_mlp(ctx: torch.Tensor, params: torch.Tensor, dim_arm: int, n_hidden: int):
    """Arm.forward on device: contexts [..., M, dim_arm] -> (mu, scale, log_scale) [..., M]."""
    require_cuda(ctx, params)
    lead = ctx.shape[:-1]
    flat = ctx.reshape(-1, dim_arm).float().contiguous()
    params = params.float().contiguous()
    m = flat.shape[0]
    mu, sc, ls = (torch.empty(m, device=ctx.device, dtype=torch.float32) for _ in range(3))
    check(lib().ccmi_arm_mlp_f32(ptr(flat), m, dim_arm, n_hidden, ptr(params), ptr(mu), ptr(sc), ptr(ls),
                                 stream_handle(ctx.device)))
    return mu.view(lead), sc.view(lead), ls.view(lead)
