"""Quantizer (reference: coolchic/enc/component/core/quantizer.py:116-232).

Eval mode only: ``hardround`` with no noise is ``torch.round`` (quantizer.py:231-232);
inside CoolChicEncoder.forward it is fused into the ARM and upsampling kernels.
"""

from typing import Literal, Optional

import torch
from torch import Tensor

POSSIBLE_QUANTIZATION_NOISE_TYPE = Literal["kumaraswamy", "gaussian", "none"]
POSSIBLE_QUANTIZER_TYPE = Literal["softround_alone", "softround", "hardround", "ste", "none", "true_ste"]


def quantize(x: Tensor, quantizer_noise_type: POSSIBLE_QUANTIZATION_NOISE_TYPE = "kumaraswamy",
             quantizer_type: POSSIBLE_QUANTIZER_TYPE = "softround", soft_round_temperature: Optional[Tensor] = None,
             noise_parameter: Optional[Tensor] = None) -> Tensor:
    if quantizer_noise_type == "none" and quantizer_type == "hardround":
        return torch.round(x)
    raise NotImplementedError(
        f"quantizer ({quantizer_noise_type}, {quantizer_type}): training-time quantisers are not part of the "
        "decode hot path implemented here (eval uses 'none'/'hardround')")
