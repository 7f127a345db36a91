"""torch.autograd bridge of the GPU training step: the train-mode CoolChicEncoder forward
(coolchic.py:291-479 with the noisy / soft quantisers) as one torch.autograd.Function whose
forward and backward both run in libccmi (ccmi_train_step with forward_only / grad_raw /
grad_rate), so the reference's own optimisation loop (enc/training/train.py:238-262:
forward -> loss_function -> loss.backward() -> clip_grad_norm_ -> optimizer.step()) drives the
HIP kernels through the mirror modules.

Quantisation noise comes in as a tensor, drawn by the caller with the reference's torch calls
(quantizer.py:188-197), so a given torch RNG state gives the reference's noise.
"""

from __future__ import annotations

import ctypes as C

import torch

from . import check, require_cuda
from .train import NOISE_TYPES, Q_TYPES, Arch, TrainArgs, _bind


def _args(arch: Arch, latent: torch.Tensor, params: torch.Tensor, yuv420: bool) -> TrainArgs:
    from . import SynLayer
    a = TrainArgs()
    B = latent.shape[0]
    a.batch, a.n_grids = B, arch.n_grids
    for i, (h, w) in enumerate(arch.sizes):
        a.h[i], a.w[i] = h, w
    a.dim_arm, a.n_hidden = arch.dim_arm, arch.n_hidden
    a.ups_k, a.n_ups, a.pre_k, a.n_pre = arch.ups_k, arch.n_grids - 1, arch.pre_k, arch.n_grids - 1
    a.n_syn_layers = len(arch.layers)
    for i, (n, k, r, nl) in enumerate(arch.layers):
        a.syn[i] = SynLayer(int(n), int(k), int(r), int(nl))
    a.gain = arch.gain
    a.latent, a.latent_stride = latent.data_ptr(), latent.shape[1]
    a.params, a.param_stride = params.data_ptr(), params.shape[1]
    a.yuv420 = int(yuv420)
    return a


class TrainForward(torch.autograd.Function):
    """(latent [B, N] before gain, params [B, P] in ccmi.train order) -> (raw [B, 3, H, W],
    rate [B, N] bits).  cfg: dict(arch, quantizer, temperature, noise [B, N] | None)."""

    @staticmethod
    def forward(ctx, latent, params, cfg):
        require_cuda(latent, params)
        arch = cfg["arch"]
        lat = latent.detach().float().contiguous()
        prm = params.detach().float().contiguous()
        B, (H, W) = lat.shape[0], arch.sizes[0]
        raw = torch.empty(B, 3, H, W, device=lat.device)
        rate = torch.empty(B, lat.shape[1], device=lat.device)
        noise = cfg.get("noise")
        noise = None if noise is None else noise.detach().float().contiguous()
        TrainForward._run(arch, lat, prm, cfg, noise, raw=raw, rate=rate)
        ctx.save_for_backward(lat, prm)
        ctx.cfg, ctx.noise = cfg, noise
        return raw, rate

    @staticmethod
    def backward(ctx, g_raw, g_rate):
        lat, prm = ctx.saved_tensors
        B, N = lat.shape
        G = torch.zeros(B, N + prm.shape[1], device=lat.device)
        g_raw = torch.zeros(B, 3, *ctx.cfg["arch"].sizes[0], device=lat.device) if g_raw is None else g_raw.contiguous()
        g_rate = torch.zeros(B, N, device=lat.device) if g_rate is None else g_rate.contiguous()
        TrainForward._run(ctx.cfg["arch"], lat, prm, ctx.cfg, ctx.noise, grad=G, g_raw=g_raw, g_rate=g_rate)
        return G[:, :N], G[:, N:], None

    @staticmethod
    def _run(arch, lat, prm, cfg, noise, raw=None, rate=None, grad=None, g_raw=None, g_rate=None):
        L = _bind()
        a = _args(arch, lat, prm, cfg.get("yuv420", False))
        dummy = torch.zeros(1, device=lat.device)
        a.target, a.target_stride = dummy.data_ptr(), 0  # unused: the loss lives in torch
        a.quantizer, a.noise = Q_TYPES[cfg["quantizer"]], NOISE_TYPES["none"]
        a.temperature = float(cfg.get("temperature", 0.3))
        a.noise_param = 1.0
        a.noise_in = None if noise is None else noise.data_ptr()
        a.update, a.step = 0, 1
        if raw is not None:
            a.forward_only, a.raw_out, a.rate_out = 1, raw.data_ptr(), rate.data_ptr()
        else:
            a.grad_out, a.grad_raw, a.grad_rate = grad.data_ptr(), g_raw.data_ptr(), g_rate.data_ptr()
        ws = torch.empty(L.ccmi_train_workspace_bytes(C.byref(a)), dtype=torch.uint8, device=lat.device)
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel()
        check(L.ccmi_train_step(C.byref(a), torch.cuda.current_stream(lat.device).cuda_stream))


class Quantize(torch.autograd.Function):
    """quantize (quantizer.py:116-232) on the GPU: y = Q(x + noise terms), dy/dx from the
    same kernel (ccmi_quantize_f32)."""

    @staticmethod
    def forward(ctx, x, quantizer, temperature, noise):
        require_cuda(x)
        L = _bind()
        if not getattr(L, "_ccmi_q_bound", False):
            L.ccmi_quantize_f32.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p]
            L._ccmi_q_bound = True
        xf = x.detach().float().contiguous()
        y = torch.empty_like(xf)
        dy = torch.empty_like(xf)
        nz = None if noise is None else noise.detach().float().expand_as(xf).contiguous()
        check(L.ccmi_quantize_f32(xf.data_ptr(), xf.numel(), Q_TYPES[quantizer], float(temperature),
                                  None if nz is None else nz.data_ptr(), y.data_ptr(), dy.data_ptr(),
                                  torch.cuda.current_stream(x.device).cuda_stream))
        ctx.save_for_backward(dy)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, gy):
        dy, = ctx.saved_tensors
        return gy * dy, None, None, None


__all__ = ["TrainForward", "Quantize"]
