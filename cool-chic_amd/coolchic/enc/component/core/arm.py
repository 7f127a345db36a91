"""Auto-regressive probability module (reference: coolchic/enc/component/core/arm.py).

Same parameters / state_dict layout as the reference (``mlp.{2k}.weight``,
``mlp.{2k}.bias``); forward passes run the libccmi HIP kernels:
  Arm.forward      -> ccmi_arm_mlp_f32     (arm.py:227-268)
  _get_neighbor    -> ccmi_arm_context_f32 (arm.py:308-352)
CoolChicEncoder.forward does not use these: it runs the fused context + MLP + rate
kernel ccmi_arm_forward_f32 on the whole latent pyramid.
"""

from collections import OrderedDict
from typing import Tuple

import torch
from torch import Tensor, nn

from ccmi import forward as _F

_CTX = {
    8: [13, 22, 30, 31, 32, 37, 38, 39],
    16: [13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39],
    24: [4, 11, 12, 13, 14, 15, 19, 20, 21, 22, 23, 24, 25, 28, 29, 30, 31, 32, 33, 34, 36, 37, 38, 39],
    32: [2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33,
         34, 35, 36, 37, 38, 39],
}


class ArmLinear(nn.Module):
    """Linear layer of the ARM (arm.py:19-101): W [out, in], b [out], optional residual."""

    def __init__(self, in_channels: int, out_channels: int, residual: bool = False):
        super().__init__()
        self.residual = residual
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        self.bias = nn.Parameter(torch.empty(out_channels))
        self.initialize_parameters()

    def initialize_parameters(self) -> None:
        """Biases zero; weights zero if residual else N(0, 1/out^4) (arm.py:65-84)."""
        self.bias = nn.Parameter(torch.zeros_like(self.bias))
        if self.residual:
            self.weight = nn.Parameter(torch.zeros_like(self.weight))
        else:
            self.weight = nn.Parameter(torch.randn_like(self.weight) / self.weight.size(0) ** 2)

    def forward(self, x: Tensor) -> Tensor:
        raise NotImplementedError("ArmLinear is evaluated inside Arm.forward's fused HIP kernel")


class Arm(nn.Module):
    """ARM MLP: residual hidden layers + ReLU, output (mu, log_scale) (arm.py:158-268)."""

    def __init__(self, dim_arm: int, n_hidden_layers_arm: int):
        super().__init__()
        assert dim_arm % 8 == 0, f"ARM context size must be a multiple of 8, found {dim_arm}"
        self.dim_arm = dim_arm
        self.n_hidden_layers_arm = n_hidden_layers_arm
        layers = nn.ModuleList()
        for _ in range(n_hidden_layers_arm):
            layers.append(ArmLinear(dim_arm, dim_arm, residual=True))
            layers.append(nn.ReLU())
        layers.append(ArmLinear(dim_arm, 2, residual=False))
        self.mlp = nn.Sequential(*layers)

    def packed_params(self) -> Tensor:
        """Flat float32 parameters in ccmi_arm_args.params order."""
        lin = [m for m in self.mlp if isinstance(m, ArmLinear)]
        return _F.pack_arm([(m.weight, m.bias) for m in lin])

    def forward(self, x: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        """x [*, M, dim_arm] contexts -> mu, scale = exp(clamp(log_scale - 4, -4.6, 5)), log_scale."""
        with torch.no_grad():
            return _F.arm_mlp(x, self.packed_params().to(x.device), self.dim_arm, self.n_hidden_layers_arm)

    def get_param(self) -> "OrderedDict[str, Tensor]":
        return OrderedDict({k: v.detach().clone() for k, v in self.named_parameters()})

    def set_param(self, param) -> None:
        self.load_state_dict(param)

    def reinitialize_parameters(self) -> None:
        for layer in self.mlp.children():
            if isinstance(layer, ArmLinear):
                layer.initialize_parameters()


def _get_neighbor(x: Tensor, mask_size: int, non_zero_pixel_ctx_idx: Tensor) -> Tensor:
    """x [B, 1, H, W] -> [B, H*W, d] causal contexts, zero padding (arm.py:308-352)."""
    assert x.ndim == 4 and x.shape[1] == 1, "expected [B, 1, H, W]"
    d = int(non_zero_pixel_ctx_idx.numel())
    if mask_size != 9 or d not in _CTX or non_zero_pixel_ctx_idx.tolist() != _CTX[d]:
        raise NotImplementedError("only the reference 9x9 masks of _get_non_zero_pixel_ctx_index are supported")
    B, _, H, W = x.shape
    return _F.arm_context(x.reshape(B, H, W), d)


def _laplace_cdf(x: Tensor, expectation: Tensor, scale: Tensor) -> Tensor:
    """Laplace CDF (arm.py:355-370); elementwise helper, fused into the rate kernel in the hot path."""
    shifted_x = x - expectation
    return 0.5 - 0.5 * shifted_x.sign() * torch.expm1(-shifted_x.abs() / scale)


def _get_non_zero_pixel_ctx_index(dim_arm: int) -> Tensor:
    """Flattened 9x9-mask indices of the causal context pixels (arm.py:373-506)."""
    if dim_arm not in _CTX:
        raise ValueError(f"ARM context size must be 8, 16, 24 or 32. Found {dim_arm}.")
    return torch.tensor(_CTX[dim_arm])
