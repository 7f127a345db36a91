"""Quantizer (reference: coolchic/enc/component/core/quantizer.py:16-232).

Every (quantizer_type, quantizer_noise_type) pair of the reference, on the GPU:
  * the noise is drawn exactly as the reference draws it (torch.rand_like / randn_like on
    the input, quantizer.py:188-197; Kumaraswamy reparameterisation :60-102), so the same
    torch RNG state gives the same noise;
  * the rounding / soft-rounding and its derivative run in libccmi's quantiser kernel
    (ccmi_quantize_f32, the kernel the training step uses) as a torch.autograd.Function:
    softround (:16-41), softround + noise + softround, "ste" (hard round forward, softround
    derivative), "true_ste" (identity derivative), "hardround" (zero derivative), "none".
CPU tensors raise: there is no CPU path.
"""

from typing import Literal, Optional

import torch
from torch import Tensor

POSSIBLE_QUANTIZATION_NOISE_TYPE = Literal["kumaraswamy", "gaussian", "none"]
POSSIBLE_QUANTIZER_TYPE = Literal["softround_alone", "softround", "hardround", "ste", "none", "true_ste"]


def generate_kumaraswamy_noise(uniform_noise: Tensor, kumaraswamy_param) -> Tensor:
    """quantizer.py:60-102: Kumaraswamy(a, b(a)) noise with its mode at 1/2, shifted to
    (-1/2, 1/2)."""
    a = kumaraswamy_param
    b = (2 ** a * (a - 1) + 1) / a
    return (1 - (1 - uniform_noise) ** (1 / b)) ** (1 / a) - 0.5


def draw_noise(x: Tensor, quantizer_noise_type: str, noise_parameter) -> Optional[Tensor]:
    """The additive noise of quantizer.py:188-197, drawn with the reference's torch calls."""
    if quantizer_noise_type == "none":
        return None
    if quantizer_noise_type == "gaussian":
        return torch.randn_like(x, requires_grad=False) * noise_parameter
    if quantizer_noise_type == "kumaraswamy":
        assert noise_parameter is not None, "noise_parameter must be provided"
        return generate_kumaraswamy_noise(torch.rand_like(x, requires_grad=False), noise_parameter)
    raise ValueError(f"unknown quantizer_noise_type {quantizer_noise_type}")


def quantize(x: Tensor, quantizer_noise_type: POSSIBLE_QUANTIZATION_NOISE_TYPE = "kumaraswamy",
             quantizer_type: POSSIBLE_QUANTIZER_TYPE = "softround", soft_round_temperature: Optional[Tensor] = None,
             noise_parameter: Optional[Tensor] = None) -> Tensor:
    """quantizer.py:116-232 (same arguments, same semantics)."""
    from ccmi.autograd import Quantize
    if quantizer_type in ("softround_alone", "softround", "ste"):
        assert soft_round_temperature is not None, "soft_round_temperature must be provided"
    noise = draw_noise(x, quantizer_noise_type, noise_parameter)
    if quantizer_type in ("none", "softround") and noise is None:
        noise = torch.zeros_like(x)  # the reference adds a noise tensor here; "none" noise = 0
    t = float(soft_round_temperature) if soft_round_temperature is not None else 1.0
    return Quantize.apply(x, quantizer_type, t, noise)
