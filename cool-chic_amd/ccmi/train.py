"""Encoder overfit step on the GPU (ccmi_train_step): the training forward, backward,
clip_grad_norm_ and Adam of enc/training/train.py:238-262, for a batch of independent
frames.  Torch tensors are storage only; every FLOP runs in libccmi's HIP kernels.

Parameter block per frame (float32), in this order:
  ARM      per hidden layer W [d][d] (out, in) then b [d]; W_out [2][d], b_out [2]
           (arm.mlp state_dict order, arm.py:86-101);
  UPS      n_ups half kernels of (ups_k + 1) // 2 taps
           (upsampling.conv_transpose2ds.{i}.parametrizations.weight.original);
  PRE      n_pre half kernels of (pre_k + 1) // 2 taps
           (upsampling.conv2ds.{i}.parametrizations.weight.original);
  SYN      per layer W [n_out][c_in][k][k] then b [n_out] (synthesis.layers.{2i}).
"""

from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Sequence

import torch

from . import MAX_GRIDS, MAX_SYN_LAYERS, SynLayer, check, lib, require_cuda

Q_TYPES = {"none": 0, "softround_alone": 1, "softround": 2, "hardround": 3, "ste": 4, "true_ste": 5}
NOISE_TYPES = {"none": 0, "kumaraswamy": 1, "gaussian": 2}


class TrainArgs(C.Structure):
    _fields_ = [
        ("batch", C.c_int), ("n_grids", C.c_int), ("h", C.c_int * MAX_GRIDS), ("w", C.c_int * MAX_GRIDS),
        ("dim_arm", C.c_int), ("n_hidden", C.c_int), ("ups_k", C.c_int), ("n_ups", C.c_int), ("pre_k", C.c_int),
        ("n_pre", C.c_int), ("n_syn_layers", C.c_int), ("syn", SynLayer * MAX_SYN_LAYERS), ("gain", C.c_float),
        ("latent", C.c_void_p), ("latent_stride", C.c_int64), ("params", C.c_void_p), ("param_stride", C.c_int64),
        ("adam_m", C.c_void_p), ("adam_v", C.c_void_p), ("target", C.c_void_p), ("target_stride", C.c_int64),
        ("yuv420", C.c_int), ("quantizer", C.c_int), ("noise", C.c_int), ("temperature", C.c_float),
        ("noise_param", C.c_float), ("lmbda", C.c_float), ("lr", C.c_float), ("beta1", C.c_float),
        ("beta2", C.c_float), ("eps", C.c_float), ("clip", C.c_float), ("step", C.c_int), ("seed", C.c_uint64),
        ("noise_in", C.c_void_p), ("grad_out", C.c_void_p), ("loss_out", C.c_void_p), ("update", C.c_int),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
    ]


def _bind():
    L = lib()
    if not getattr(L, "_ccmi_train_bound", False):
        L.ccmi_train_step.argtypes = [C.POINTER(TrainArgs), C.c_void_p]
        L.ccmi_train_step.restype = C.c_int
        L.ccmi_train_workspace_bytes.argtypes = [C.POINTER(TrainArgs)]
        L.ccmi_train_workspace_bytes.restype = C.c_size_t
        L.ccmi_train_param_count.argtypes = [C.POINTER(TrainArgs)]
        L.ccmi_train_param_count.restype = C.c_size_t
        L._ccmi_train_bound = True
    return L


@dataclass
class Arch:
    H: int
    W: int
    dim_arm: int = 16
    n_hidden: int = 2
    layers: tuple = ((48, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False))
    n_grids: int = 7
    ups_k: int = 8
    pre_k: int = 7
    gain: float = 16.0

    @property
    def sizes(self):
        s, h, w = [], self.H, self.W
        for _ in range(self.n_grids):
            s.append((h, w))
            h, w = (h + 1) // 2, (w + 1) // 2
        return s

    @property
    def n_latents(self) -> int:
        return sum(h * w for h, w in self.sizes)


def pack_params(arm, ups_half, pre_half, syn) -> torch.Tensor:
    """[(W, b)...], [half...], [half...], [(W, b)...] -> flat float32 parameter block."""
    parts = [t.reshape(-1).float() for wb in arm for t in wb]
    parts += [h.reshape(-1).float() for h in list(ups_half) + list(pre_half)]
    parts += [t.reshape(-1).float() for wb in syn for t in wb]
    return torch.cat(parts)


class Overfitter:
    """GPU state of `batch` frames being overfitted together: latents, parameters and the
    Adam moments live in HBM; step() runs one training iteration for all of them."""

    def __init__(self, arch: Arch, latents: torch.Tensor, params: torch.Tensor, targets: torch.Tensor,
                 yuv420: bool = True, seed: int = 0):
        require_cuda(latents, params, targets)
        self.arch, self.yuv420, self.seed = arch, bool(yuv420), seed
        self.B = latents.shape[0]
        self.latents = latents.float().contiguous()
        self.params = params.float().contiguous()
        self.targets = targets.float().contiguous()
        self.t = 0
        a = self._args()
        L = _bind()
        P = L.ccmi_train_param_count(C.byref(a))
        if P == 0 or self.params.shape[1] != P:
            raise ValueError(f"params: expected [B, {P}] for this architecture, got {tuple(self.params.shape)}")
        if self.latents.shape[1] != arch.n_latents:
            raise ValueError(f"latents: expected [B, {arch.n_latents}]")
        self.P, self.N = P, arch.n_latents
        dev = self.latents.device
        self.m = torch.zeros(self.B, self.N + P, device=dev)
        self.v = torch.zeros(self.B, self.N + P, device=dev)
        self.loss = torch.zeros(self.B, 4, device=dev)
        self.ws = torch.empty(L.ccmi_train_workspace_bytes(C.byref(a)), dtype=torch.uint8, device=dev)

    def _args(self) -> TrainArgs:
        ar = self.arch
        a = TrainArgs()
        a.batch, a.n_grids = self.B, ar.n_grids
        for i, (h, w) in enumerate(ar.sizes):
            a.h[i], a.w[i] = h, w
        a.dim_arm, a.n_hidden = ar.dim_arm, ar.n_hidden
        a.ups_k, a.n_ups, a.pre_k, a.n_pre = ar.ups_k, ar.n_grids - 1, ar.pre_k, ar.n_grids - 1
        a.n_syn_layers = len(ar.layers)
        for i, (n, k, r, nl) in enumerate(ar.layers):
            a.syn[i] = SynLayer(n, k, int(r), int(nl))
        a.gain = ar.gain
        a.latent, a.latent_stride = self.latents.data_ptr(), self.latents.shape[1]
        a.params, a.param_stride = self.params.data_ptr(), self.params.shape[1]
        a.target, a.target_stride = self.targets.data_ptr(), self.targets.shape[1]
        a.yuv420 = int(self.yuv420)
        return a

    def step(self, quantizer_type="softround", quantizer_noise_type="kumaraswamy", soft_round_temperature=0.3,
             noise_parameter=1.0, lmbda=1e-3, lr=1e-2, clip=0.1, update=True, noise=None, grad_out=None):
        """One iteration; returns [B, 4] (loss, mse, rate_bits, grad_norm) of this step's forward."""
        a = self._args()
        if update:
            self.t += 1
        a.adam_m, a.adam_v = self.m.data_ptr(), self.v.data_ptr()
        a.quantizer, a.noise = Q_TYPES[quantizer_type], NOISE_TYPES[quantizer_noise_type]
        a.temperature, a.noise_param, a.lmbda = float(soft_round_temperature), float(noise_parameter), float(lmbda)
        a.lr, a.beta1, a.beta2, a.eps, a.clip = float(lr), 0.9, 0.999, 1e-8, float(clip)
        a.step = max(self.t, 1)
        a.seed = self.seed
        if noise is not None:
            require_cuda(noise)
            noise = noise.float().contiguous()
            a.noise_in = noise.data_ptr()
        if grad_out is not None:
            if grad_out.shape != (self.B, self.N + self.P) or not grad_out.is_contiguous():
                raise ValueError("grad_out: contiguous [B, N + P] expected")
            a.grad_out = grad_out.data_ptr()
        a.loss_out = self.loss.data_ptr()
        a.update = int(update)
        a.workspace, a.workspace_bytes = self.ws.data_ptr(), self.ws.numel()
        check(_bind().ccmi_train_step(C.byref(a), torch.cuda.current_stream(self.latents.device).cuda_stream))
        return self.loss


def cosine_lr(start: float, end: float, it: int, max_it: int, freq: int) -> float:
    """CosineAnnealingLR(T_max = max_itr / freq_valid, eta_min = end) stepped every freq
    iterations (train.py:189-196, :351-352)."""
    T = max_it / freq
    e = it // freq
    return end + (start - end) * (1 + math.cos(math.pi * e / T)) / 2


def linear(a: float, b: float, it: int, max_it: int) -> float:
    """_linear_schedule (train.py)."""
    return a + (b - a) * it / max_it


__all__ = ["Arch", "Overfitter", "pack_params", "cosine_lr", "linear", "Q_TYPES", "NOISE_TYPES"]
