"""Latent upsampling (reference: coolchic/enc/component/core/upsampling.py).

Same modules, parametrisations and state_dict keys as the reference
(``conv_transpose2ds.{i}.parametrizations.weight.original``, ``conv2ds.{i}...``).
Upsampling.forward in eval mode runs the libccmi pyramid kernels
(ccmi_ups_forward_f32: one launch per pyramid level, all channels).  The training
form (2-D kron kernels, upsampling.py:195-202 / :322-335) is out of this round's scope.
"""

from collections import OrderedDict
from typing import List

import torch
import torch.nn.utils.parametrize as parametrize
from torch import Tensor, nn

from ccmi import forward as _F


class _Parameterization_Symmetric_1d(nn.Module):
    """N-element vector -> 2N (or 2N+1) symmetric kernel (upsampling.py:21-89)."""

    def __init__(self, target_k_size: int):
        super().__init__()
        self.target_k_size = target_k_size
        self.param_size = self.size_param_from_target(target_k_size)

    def forward(self, x: Tensor) -> Tensor:
        return torch.cat([x, torch.flip(x, [0])[self.target_k_size % 2:]])

    @classmethod
    def size_param_from_target(cls, target_k_size: int) -> int:
        return (target_k_size + 1) // 2


class _SymmetricKernelModule(nn.Module):
    def __init__(self, kernel_size: int, init_core: Tensor):
        super().__init__()
        self.target_k_size = kernel_size
        self.param_size = _Parameterization_Symmetric_1d.size_param_from_target(kernel_size)
        self.weight = nn.Parameter(torch.empty(self.param_size))
        self.bias = nn.Parameter(torch.empty(1))  # present in the reference, unused by its forward
        self._init_core = init_core
        self.initialize_parameters()

    def initialize_parameters(self) -> None:
        if parametrize.is_parametrized(self, "weight"):
            parametrize.remove_parametrizations(self, "weight", leave_parametrized=False)
        w = torch.zeros(self.param_size)
        core = self._init_core
        w[self.param_size - core.numel():] = core
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(torch.zeros(1))
        parametrize.register_parametrization(self, "weight", _Parameterization_Symmetric_1d(self.target_k_size),
                                             unsafe=True)

    def forward(self, x: Tensor) -> Tensor:
        raise NotImplementedError("single-filter forward: use Upsampling.forward (fused pyramid kernel)")


class UpsamplingSeparableSymmetricConv2d(_SymmetricKernelModule):
    """Pre-concatenation refine filter, odd kernel, Dirac init (upsampling.py:92-209)."""

    def __init__(self, kernel_size: int):
        assert kernel_size % 2 == 1, f"Upsampling kernel size must be odd, found {kernel_size}."
        super().__init__(kernel_size, torch.tensor([1.0]))


class UpsamplingSeparableSymmetricConvTranspose2d(_SymmetricKernelModule):
    """2x transposed-conv upsampling filter, even kernel, bilinear / bicubic init (upsampling.py:212-355)."""

    def __init__(self, kernel_size: int):
        assert kernel_size >= 4 and not kernel_size % 2, f"Upsampling kernel size shall be even and >=4. Found {kernel_size}"
        core = torch.tensor([1.0 / 4.0, 3.0 / 4.0]) if kernel_size < 8 else \
            torch.tensor([0.0351562, 0.1054687, -0.2617187, -0.8789063])
        super().__init__(kernel_size, core)


class Upsampling(nn.Module):
    """Pyramid upsampling (upsampling.py:358-537)."""

    def __init__(self, ups_k_size: int, ups_preconcat_k_size: int, n_ups_kernel: int, n_ups_preconcat_kernel: int):
        super().__init__()
        self.n_ups_kernel = n_ups_kernel
        self.n_ups_preconcat_kernel = n_ups_preconcat_kernel
        self.ups_k_size = ups_k_size
        self.ups_preconcat_k_size = ups_preconcat_k_size
        self.conv_transpose2ds = nn.ModuleList(
            [UpsamplingSeparableSymmetricConvTranspose2d(ups_k_size) for _ in range(n_ups_kernel)])
        self.conv2ds = nn.ModuleList(
            [UpsamplingSeparableSymmetricConv2d(ups_preconcat_k_size) for _ in range(n_ups_preconcat_kernel)])

    def packed_params(self) -> Tensor:
        """Full symmetric kernels in ccmi_ups_args.params order."""
        return _F.pack_ups([m.weight.detach() for m in self.conv_transpose2ds],
                           [m.weight.detach() for m in self.conv2ds])

    def forward_flat(self, flat: Tensor, sizes, gain: float = 1.0, quantize: bool = False,
                     params: Tensor = None) -> Tensor:
        """Flat latents [B, N] (grid l is sizes[l]) -> [B, L, H, W]; optionally quantising on the fly."""
        p = self.packed_params().to(flat.device) if params is None else params
        return _F.ups_forward(flat, sizes, p, self.ups_k_size, self.n_ups_kernel, self.ups_preconcat_k_size,
                              self.n_ups_preconcat_kernel, gain, quantize)

    def forward(self, decoder_side_latent: List[Tensor]) -> Tensor:
        """List of L tensors [B, 1, H/2^i, W/2^i] -> [B, L, H, W] (upsampling.py:476-506)."""
        if self.training:
            raise NotImplementedError("training-mode upsampling (2-D kron kernels) is not implemented")
        B = decoder_side_latent[0].shape[0]
        if any(t.shape[1] != 1 for t in decoder_side_latent):
            raise NotImplementedError("one feature per latent resolution only (as the reference decoder)")
        sizes = [tuple(t.shape[-2:]) for t in decoder_side_latent]
        flat = torch.cat([t.reshape(B, -1) for t in decoder_side_latent], dim=1)
        with torch.no_grad():
            return self.forward_flat(flat, sizes)

    def get_param(self) -> "OrderedDict[str, Tensor]":
        return OrderedDict({k: v.detach().clone() for k, v in self.named_parameters()})

    def set_param(self, param) -> None:
        self.load_state_dict(param)

    def reinitialize_parameters(self) -> None:
        for m in list(self.conv_transpose2ds) + list(self.conv2ds):
            m.initialize_parameters()
