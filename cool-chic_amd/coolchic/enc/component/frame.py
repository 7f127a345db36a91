"""FrameEncoder (reference: coolchic/enc/component/frame.py), intra frames.

forward() = CoolChicEncoder.forward + the eval post-processing of frame.py:175-183
(rounding to the output bitdepth, optional 444 -> 420 nearest, clamp).  In eval mode the
whole decode tail is ccmi_decode_forward_f32 (coolchic.decoded_batch: one fused kernel
for the last upsampling step, the synthesis and the post-processing); the staged
ccmi_ups / ccmi_syn / ccmi_post path remains for architectures without a fused kernel
and for train mode.  Inter coding (warping, frame.py:165-170) is disabled in the reference
and not part of this hot path.
"""

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

import torch
from torch import Tensor, nn

from ccmi import ERR_UNSUPPORTED, CcmiError
from ccmi import forward as _F
from coolchic.enc.component.coolchic import CoolChicEncoder, CoolChicEncoderParameter, decoded_batch


@dataclass
class FrameEncoderOutput:
    decoded_image: Union[Tensor, Dict[str, Tensor]]
    rate: Tensor
    additional_data: Dict[str, Any] = field(default_factory=dict)


class FrameEncoder(nn.Module):
    def __init__(self, coolchic_encoder_param: CoolChicEncoderParameter, frame_type: str = "I",
                 frame_data_type: str = "rgb", bitdepth: int = 8):
        super().__init__()
        if frame_type != "I":
            raise NotImplementedError("only intra frames are part of the decode hot path")
        self.coolchic_encoder_param = coolchic_encoder_param
        self.frame_type = frame_type
        self.frame_data_type = frame_data_type
        self.bitdepth = bitdepth
        self.coolchic_encoder = CoolChicEncoder(coolchic_encoder_param)

    def forward(self, reference_frames: Optional[List[Tensor]] = None, quantizer_noise_type: str = "kumaraswamy",
                quantizer_type: str = "softround", soft_round_temperature: Optional[float] = 0.3,
                noise_parameter: Optional[float] = 1.0, AC_MAX_VAL: int = -1,
                flag_additional_outputs: bool = False) -> FrameEncoderOutput:
        if not self.training:
            # eval: the raw synthesis output is not part of FrameEncoderOutput, so the decode
            # tail runs as one fused kernel (pyramid, last upsampling step, synthesis and this
            # post-processing); architectures without a fused kernel take the staged path
            yuv420 = self.frame_data_type == "yuv420"
            try:
                out, rate, add = decoded_batch([self.coolchic_encoder], self.bitdepth, yuv420, AC_MAX_VAL,
                                               flag_additional_outputs)
            except CcmiError as e:
                if e.code != ERR_UNSUPPORTED:
                    raise
            else:
                if yuv420:
                    H, W = self.coolchic_encoder.grid_sizes[0]
                    out = {k: v.unsqueeze(1) for k, v in _F.split_420(out, H, W).items()}
                return FrameEncoderOutput(out, rate, add if flag_additional_outputs else {})
        raw, rate, add = self.coolchic_encoder.forward(quantizer_noise_type, quantizer_type, soft_round_temperature,
                                                       noise_parameter, AC_MAX_VAL, flag_additional_outputs)
        return FrameEncoderOutput(self.post_process(raw), rate, add if flag_additional_outputs else {})

    def post_process(self, raw: Tensor):
        if self.training:
            # frame.py:175-183 in train mode: no rounding; 444 -> 420 nearest (even rows /
            # columns, yuv.py:275-299); clamp to [0, 1] -- differentiable torch ops
            if self.frame_data_type == "yuv420":  # F.interpolate(scale 0.5, nearest): floor(H / 2) rows
                h2, w2 = 2 * (raw.shape[-2] // 2), 2 * (raw.shape[-1] // 2)
                return {"y": raw[:, 0:1].clamp(0.0, 1.0), "u": raw[:, 1:2, 0:h2:2, 0:w2:2].clamp(0.0, 1.0),
                        "v": raw[:, 2:3, 0:h2:2, 0:w2:2].clamp(0.0, 1.0)}
            return raw.clamp(0.0, 1.0)
        H, W = raw.shape[-2:]
        if self.frame_data_type == "yuv420":
            out = _F.post_forward(raw, self.bitdepth, True)
            d = _F.split_420(out, H, W)
            return {k: v.unsqueeze(1) for k, v in d.items()}
        return _F.post_forward(raw, self.bitdepth, False)
