"""Rate-distortion loss (reference: coolchic/enc/training/loss.py:20-162), the caller of the
training forward in the reference's optimisation loop (train.py:248-256).  Plain torch on
the frame outputs (elementwise + one reduction); the hot path upstream is libccmi's."""

import math
from dataclasses import dataclass, field
from typing import Dict, Optional, Union

import torch
from torch import Tensor


@dataclass(kw_only=True)
class LossFunctionOutput:
    """loss.py:20-51."""
    loss: Optional[Union[float, Tensor]] = None
    mse: Optional[float] = None
    rate_nn_bpp: Optional[float] = None
    rate_latent_bpp: Optional[float] = None
    psnr_db: Optional[float] = field(init=False, default=None)
    total_rate_bpp: Optional[float] = field(init=False, default=None)

    def __post_init__(self):
        if self.mse is not None:
            self.psnr_db = -10.0 * math.log10(self.mse + 1e-10)
        if self.rate_nn_bpp is not None and self.rate_latent_bpp is not None:
            self.total_rate_bpp = self.rate_nn_bpp + self.rate_latent_bpp


def _compute_mse(x: Union[Tensor, Dict[str, Tensor]], y: Union[Tensor, Dict[str, Tensor]]) -> Tensor:
    """loss.py:53-86: plain MSE, or the per-channel MSEs weighted by pixel count (420)."""
    if isinstance(x, Tensor):
        return ((x - y) ** 2).mean()
    total, mse = 0.0, None
    for (_, xc), (_, yc) in zip(x.items(), y.items()):
        n = xc.numel()
        term = torch.pow(xc - yc, 2.0).mean() * n
        mse = term if mse is None else mse + term
        total += n
    return mse / total


def loss_function(decoded_image, rate_latent_bit: Tensor, target_image, lmbda: float = 1e-3,
                  rate_mlp_bit: float = 0.0, compute_logs: bool = False) -> LossFunctionOutput:
    """loss.py:90-162: MSE + lmbda * (latent bits summed per image, averaged over the batch,
    + network bits) / pixels."""
    mse = _compute_mse(decoded_image, target_image)
    ref = decoded_image if isinstance(decoded_image, Tensor) else decoded_image["y"]
    n_pixels = ref.size()[-2] * ref.size()[-1]
    assert rate_latent_bit.ndim == 2, "Rate latent bit should have shape [batch, n_latent]."
    avg_rate_latent_bit = rate_latent_bit.sum(dim=1).mean(dim=0)
    rate_bpp = (avg_rate_latent_bit + rate_mlp_bit) / n_pixels
    loss = mse + lmbda * rate_bpp
    return LossFunctionOutput(
        loss=loss,
        mse=mse.detach().item() if compute_logs else None,
        rate_nn_bpp=rate_mlp_bit / n_pixels if compute_logs else None,
        rate_latent_bpp=avg_rate_latent_bit.detach().item() / n_pixels if compute_logs else None,
    )
