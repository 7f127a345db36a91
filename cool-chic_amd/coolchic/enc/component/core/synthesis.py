"""Synthesis (reference: coolchic/enc/component/core/synthesis.py).

Same layers / state_dict keys as the reference (``layers.{2k}.weight`` / ``.bias``,
odd indices are the non-linearities).  Synthesis.forward runs ccmi_syn_forward_f32:
one fused kernel for 1x1-head + 3x3-tail architectures (all presets), per-layer
kernels otherwise.
"""

import math
from collections import OrderedDict
from typing import List

import torch
from torch import Tensor, nn

from ccmi import forward as _F


class SynthesisConv2d(nn.Module):
    """Conv layer with replicate padding and optional residual (synthesis.py:16-100)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, residual: bool = False):
        super().__init__()
        self.residual = residual
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.pad = int((kernel_size - 1) / 2)
        self.groups = 1
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels))
        self.initialize_parameters()

    def initialize_parameters(self) -> None:
        self.bias = nn.Parameter(torch.zeros_like(self.bias))
        if self.residual:
            self.weight = nn.Parameter(torch.zeros_like(self.weight))
        else:
            out_c, in_c, kh, kw = self.weight.size()
            sqrt_k = math.sqrt(self.groups / (in_c * kh * kw))
            self.weight = nn.Parameter((torch.rand_like(self.weight) - 0.5) * 2 * sqrt_k / (out_c ** 2))

    def forward(self, x: Tensor) -> Tensor:
        raise NotImplementedError("SynthesisConv2d runs inside Synthesis.forward's HIP kernel")


class Synthesis(nn.Module):
    possible_non_linearity = {"none": nn.Identity, "relu": nn.ReLU}
    possible_mode = ["linear", "residual"]

    def __init__(self, input_ft: int, layers_dim: List[str]):
        super().__init__()
        self.input_ft = input_ft
        self.layer_desc = []
        layers = nn.ModuleList()
        for desc in layers_dim:
            out_ft, k_size, mode, non_linearity = desc.split("-")
            out_ft, k_size = int(out_ft), int(k_size)
            assert mode in self.possible_mode, f"Unknown mode {mode}"
            assert non_linearity in self.possible_non_linearity, f"Unknown non linearity {non_linearity}"
            layers.append(SynthesisConv2d(input_ft, out_ft, k_size, residual=mode == "residual"))
            layers.append(self.possible_non_linearity[non_linearity]())
            self.layer_desc.append((out_ft, k_size, mode == "residual", non_linearity == "relu"))
            input_ft = out_ft
        self.layers = nn.Sequential(*layers)

    def packed_params(self) -> Tensor:
        convs = [m for m in self.layers if isinstance(m, SynthesisConv2d)]
        return _F.pack_syn([(m.weight, m.bias) for m in convs])

    def forward(self, x: Tensor, params: Tensor = None) -> Tensor:
        """x [B, C, H, W] -> [B, C_out, H, W] (synthesis.py:264-277)."""
        with torch.no_grad():
            p = self.packed_params().to(x.device) if params is None else params
            return _F.syn_forward(x, self.layer_desc, p)

    def get_param(self) -> "OrderedDict[str, Tensor]":
        return OrderedDict({k: v.detach().clone() for k, v in self.named_parameters()})

    def set_param(self, param) -> None:
        self.load_state_dict(param)

    def reinitialize_parameters(self) -> None:
        for layer in self.layers.children():
            if isinstance(layer, SynthesisConv2d):
                layer.initialize_parameters()
